#!/bin/bash
# round 3 study: the K-split factor of a 1/8 shard of C3 (bench --rehearse 3/8), the cost model's choice vs forced P
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ks; mkdir -p $O
for P in 0 1 3 4 5 6 8 0 3 8; do
  NLDSC_KSPLIT_P=$P NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 3/8 > $O/p$P.json 2> $O/p$P.err || { tail $O/p$P.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/p$P.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('P=$P', round(d['ms_per_step'],3), s['band_ms'], s['count_ms'], s['schedule_ms'])"
  grep "nldsc debug" $O/p$P.err | tail -2
done
