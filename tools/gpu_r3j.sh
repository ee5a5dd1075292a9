#!/bin/bash
# round 3: the parity tests (file 1 of the GPU suite), then the tiled-row-layout study A/B (same box, interleaved)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3j; mkdir -p $O
echo "[$(date +%H:%M:%S)] parity tests"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "round_launch or ksplit_equals" --timeout 400 --timeout-method thread > $O/gpu_tests_parity.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests_parity.log; exit 1; }
tail -2 $O/gpu_tests_parity.log
echo "[$(date +%H:%M:%S)] tiled A/B"
timeout -k 10 300 python tools/ab_libs.py --libs new=nldsc_amd/libnldsc_amd.so tiled=ab_libs/tiled.so --workload c3 c2 c5 --runs 8 \
  > $O/ab_tiled.json 2> $O/ab_tiled.err || { tail $O/ab_tiled.err; exit 1; }
cat $O/ab_tiled.json
echo "[$(date +%H:%M:%S)] done"
