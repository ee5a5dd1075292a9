#!/bin/bash
# round 3: plan stream priority — wall-time breakdown and the A/B (one process, interleaved)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3w; mkdir -p $O
NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python tools/run_lib.py --runs 6 --n-org 50000 --additive-only > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
grep "nldsc debug" $O/c2.log | tail -3
timeout -k 10 400 python tools/ab_libs.py --libs prio=nldsc_amd/libnldsc_amd.so noprio=nldsc_amd/libnldsc_amd.so,NLDSC_PLAN_PRIORITY=0 --workload c2 c3 --runs 10 \
  > $O/ab_prio.json 2> $O/ab_prio.err || { tail $O/ab_prio.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/ab_prio.json'))['ab']
for w,v in d.items(): print(w, {k:(round(x['total_ms_median'],3), round(x['band_ms_median'],3)) for k,x in v.items()})"
