#!/bin/bash
# Same-process A/B: round-4 HEAD library vs the working tree, default and with the persistent round kernel
# (option band_persist), C2 / C3 / rank 0 of 8 (gpurun --timeout 900 -- bash tools/ab/gpu_ab_persist.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abp}; mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py --libs head=ab_libs/r5_head.so new=nldsc_amd/libnldsc_amd.so persist=nldsc_amd/libnldsc_amd.so,band_persist=1 --workload c3 c2 c3r0of8 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3),x['stages_ms_median'])"
