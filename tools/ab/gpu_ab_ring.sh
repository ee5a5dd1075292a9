#!/bin/bash
# the single-block fp4 band's per-wave LDS ring (study builds ab_libs/r4_ring<S>.so) against the register prefetch
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ring}; mkdir -p $O
timeout -k 10 900 python tools/ab_libs.py --libs base=nldsc_amd/libnldsc_amd.so ring3=ab_libs/r4_ring3.so ring4=ab_libs/r4_ring4.so ring5=ab_libs/r4_ring5.so --workload c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),round(x['band_ms_min'],3))"
