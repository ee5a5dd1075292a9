#!/bin/bash
# short runs (C2, the 1/8 shard) where the schedule and the small kernels between the count and the band are on the
# critical path: the previous commit's library against the working tree's, same process; then the GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-short}; mkdir -p $O
timeout -k 10 400 python tools/ab_libs.py --libs prev=ab_libs/r4_prev.so cur=ab_libs/r4_cur.so --workload c2 c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3))"
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 0/8 > $O/r0_$i.json 2> $O/r0_$i.err || { tail $O/r0_$i.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/r0_$i.json').read().strip().splitlines()[-1]); print('shard', round(d['ms_per_step'],3), d['stages_ms'])"
done
[ "$2" = "ab-only" ] && exit 0
bash tools/gpu_tests.sh $1/t
