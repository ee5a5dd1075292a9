#!/bin/bash
# the schedule's window-edge search beside the count (00f4bb2: LDS-staged, count first) against before it (the
# working tree), C2 and rank 0's 1/8 shard of C3, with a third engine between the two builds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ord}; mkdir -p $O
timeout -k 10 500 python tools/ab_libs.py --libs beside=ab_libs/r4_00f.so pad=ab_libs/r4_dummy.so before=ab_libs/r4_cur.so --workload c2 c3r0of8 --runs 10 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3), x['stages_ms_median'])"
