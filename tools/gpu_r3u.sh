#!/bin/bash
# round 3: where a run's wall time goes (NLDSC_DEBUG_TIMING), C3 and C2, one engine per process
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3u; mkdir -p $O
NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python tools/run_lib.py --runs 6 > $O/c3.log 2>&1 || { tail $O/c3.log; exit 1; }
NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python tools/run_lib.py --runs 6 --n-org 50000 --additive-only > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
grep "count\|band " $O/c3.log | tail -4; grep "count\|band " $O/c2.log | tail -4
