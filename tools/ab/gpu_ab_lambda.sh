#!/bin/bash
# Same-process A/B: round-4 HEAD library, the working tree (band kernel body in a forced-inline lambda), and the working
# tree with the round-4 form of that kernel (ab_libs/r5_nolambda.so): C3 / C2, with the L2 deltas between builds
# (gpurun --timeout 900 -- bash tools/ab/gpu_ab_lambda.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abl}; mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py --libs head=ab_libs/r5_head.so new=nldsc_amd/libnldsc_amd.so nolambda=ab_libs/r5_nolambda.so --workload c3 c2 --runs 10 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3),x['max_abs_dl2_vs_first'],x['stages_ms_median'])"
