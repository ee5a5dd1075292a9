#!/bin/bash
# the balanced (stream-K) K-split of a band's partial last round against the P-piece split: K-split tests, then a
# same-process A/B (a third engine between the two builds) on rank 0's 1/8 shard of C3 and on C3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-bal}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "ksplit or round or schedule or split_halo or issued" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python tools/ab_libs.py --libs bal=ab_libs/r4_bal.so pad=ab_libs/r4_pad.so pre=ab_libs/r4_prebal.so --workload c3r0of8 c3 --runs 10 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3))"
