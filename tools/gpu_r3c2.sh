#!/bin/bash
# round 3 study: C2 (N = 50 000, additive only) — the replay beside the band or before it, deferral on/off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c2; mkdir -p $O
run() {  # <label> <env...>
  local l=$1; shift
  env "$@" NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --n-org 50000 --additive-only > $O/$l.json 2> $O/$l.err || { tail $O/$l.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$l', round(d['ms_per_step'],3), s['band_ms'], s['count_ms'], s['schedule_ms'], d['roofline'].get('kernel'))"
  grep "nldsc debug" $O/$l.err | tail -1
}
for k in 1 2; do
run base_$k X=1
run serial_$k NLDSC_REPLAY_OVERLAP=0
run nodefer_$k NLDSC_DEFER_REP=0
run exact_$k NLDSC_REPLAY_OVERLAP=0 NLDSC_DEFER_REP=0
done
