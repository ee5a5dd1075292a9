#!/bin/bash
# pack_table's pair-count sums: one atomic pair per workgroup (working tree) against per wave (HEAD), C2 and C3, a third
# engine between the two builds; then the tests that read the pair counts
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pack}; mkdir -p $O
timeout -k 10 500 python tools/ab_libs.py --libs cur=ab_libs/r4_cur.so pad=ab_libs/r4_dummy.so prev=ab_libs/r4_prev.so --workload c2 c3 --runs 10 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "torchrun or pairs or device or bench or issued" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
