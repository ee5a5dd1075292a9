#!/bin/bash
# round 3: shards forced into round launches kept in the single-block kernel — parity tests of the band launch
# paths, then 1/8 shards with and without missing calls and a 1/4 shard (round launches from 1 round, default, vs 4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3mf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_torchrun.py -m gpu -x -q --timeout 300 --timeout-method thread -k "round or ksplit or quad or t2 or split or deferred or rccl or torchrun" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # <label> <round_min> <args>
  local l=$1 rm=$2; shift 2
  NLDSC_ROUND_MIN=$rm timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 "$@" > $O/$l.json 2> $O/e.err || { tail $O/e.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$l', round(d['ms_per_step'],3), s['band_ms'], s['count_ms'], d['roofline'].get('kernel','')[:50])"
}
for k in 1 2; do
  run mf8_rm1_$k 1 --missing 0 --rehearse 0/8 || exit 1
  run mf8_rm4_$k 4 --missing 0 --rehearse 0/8 || exit 1
  run m8_rm1_$k 1 --rehearse 0/8 || exit 1
  run m4_rm1_$k 1 --rehearse 1/4 || exit 1
done
