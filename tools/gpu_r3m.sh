#!/bin/bash
# round 3: additive-only quad super-items with missing calls — the routing / bitwise tests, then the C2 A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3m; mkdir -p $O
echo "[$(date +%H:%M:%S)] tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "round_launch" --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo "[$(date +%H:%M:%S)] A/B"
timeout -k 10 300 python tools/ab_libs.py --libs quad_add=nldsc_amd/libnldsc_amd.so single=nldsc_amd/libnldsc_amd.so,NLDSC_QUAD_ADD=0 --workload c2 --runs 10 \
  > $O/ab_quad_add.json 2> $O/ab_quad_add.err || { tail $O/ab_quad_add.err; exit 1; }
cat $O/ab_quad_add.json
echo "[$(date +%H:%M:%S)] done"
echo "[$(date +%H:%M:%S)] A/B add+dom 32x64 tiles (study)"
timeout -k 10 300 python tools/ab_libs.py --libs base=nldsc_amd/libnldsc_amd.so nc2dom=nldsc_amd/libnldsc_amd.so,NLDSC_F4_NC2_DOM=1 --workload c3 --runs 8 \
  > $O/ab_nc2dom.json 2> $O/ab_nc2dom.err || { tail $O/ab_nc2dom.err; exit 1; }
cat $O/ab_nc2dom.json
