#!/bin/bash
# the single-block fp4 band with WG waves per workgroup (study builds ab_libs/r4_wg<W>.so; plan items of mostly one row
# block per workgroup share the row strip through L1) against one wave per workgroup
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wg}; mkdir -p $O
timeout -k 10 900 python tools/ab_libs.py --libs head=ab_libs/r4_head.so wg1=nldsc_amd/libnldsc_amd.so wg2=ab_libs/r4_wg2.so wg4=ab_libs/r4_wg4.so --workload c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3))"
