#!/bin/bash
# the epilogue's share of the single-block fp4 band (verdict r03 item 5): a study build with the epilogue compiled out
# (outputs wrong, timing only) against the build, C2 and C3, a third engine between them
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-noepi}; mkdir -p $O
timeout -k 10 500 python tools/ab_libs.py --no-check --libs cur=ab_libs/r4_cur.so pad=ab_libs/r4_pad.so noepi=ab_libs/r4_noepi.so --workload c2 c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3))"
