#!/bin/bash
# C2 host-path check: the bench line with and without NLDSC_DEBUG_TIMING, and the same-process A/B against HEAD~ builds
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c2c}; mkdir -p $O
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu --no-file --steps 10 --n-org 50000 --additive-only > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
NLDSC_DEBUG_TIMING=1 timeout -k 10 120 python bench.py --no-cpu --no-file --steps 10 --n-org 50000 --additive-only > $O/d$i.json 2> $O/d$i.err || { tail $O/d$i.err; exit 1; }
done
for f in b1 d1 b2 d2; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), d['stages_ms'])"; done
timeout -k 10 300 python tools/ab_libs.py --libs prev=ab_libs/r4_a7.so cur=ab_libs/r4_cur.so intree=nldsc_amd/libnldsc_amd.so --workload c2 c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3))"
