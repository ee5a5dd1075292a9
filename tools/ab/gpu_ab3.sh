#!/bin/bash
# same-process A/B of two builds with a third engine between them (ab_libs.py's second engine in a process pays ~1 ms
# of host time per C2 run whatever its build: profiles/r04_ab_engine_position.json)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab3}; mkdir -p $O
timeout -k 10 500 python tools/ab_libs.py --libs cur=ab_libs/r4_cur.so pad=ab_libs/r4_dummy.so prev=ab_libs/r4_prev.so --workload c2 c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3), x['stages_ms_median'])"
