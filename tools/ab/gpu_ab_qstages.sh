#!/bin/bash
# quad kernel (C5 slice, missing-free 4 x 4 super-items): LDS ring of 3 / 4 (base) / 6 two-chunk stages, same process
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-qs}; mkdir -p $O
timeout -k 10 800 python tools/ab_libs.py --libs base=ab_libs/r4_base.so s3=ab_libs/r4_qs3.so s6=ab_libs/r4_qs6.so --workload c5 --c5-snp 300000 --runs 5 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3))"
