#!/bin/bash
# band-edge items on 16 x 16 sub-tiles: the working tree's library (edge) against HEAD's (ab_libs/r4_head.so) and the
# study builds r4_e1 (edge code compiled, never taken) and r4_e2 (no edge code), C3 and C2
# (gpurun --timeout 900 -- bash tools/ab/gpu_ab_edge.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-edge}; mkdir -p $O
timeout -k 10 800 python tools/ab_libs.py --libs head=ab_libs/r4_head.so edge=nldsc_amd/libnldsc_amd.so e1=ab_libs/r4_e1.so e2=ab_libs/r4_e2.so --workload c3 c2 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3))"
