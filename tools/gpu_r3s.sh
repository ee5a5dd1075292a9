#!/bin/bash
# round 3: deferred rare-variant items — the rare-variant GPU tests, then the C2 A/B (defer vs KC launch)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3s; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "rare or deferred or column_block or ksplit or round_launch" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/ab_libs.py --libs defer=nldsc_amd/libnldsc_amd.so kc=nldsc_amd/libnldsc_amd.so,NLDSC_DEFER_REP=0 --workload c2 --runs 10 \
  > $O/ab_defer.json 2> $O/ab_defer.err || { tail $O/ab_defer.err; exit 1; }
cat $O/ab_defer.json
