#!/bin/bash
# round 3: block-interleaved resident layout — smoke, the whole GPU parity file, then the A/B against the row-major
# build of HEAD (ab_libs/rowmajor.so) on C3, C2, C5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[$(date +%H:%M:%S)] parity tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests_parity.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests_parity.log; exit 1; }
tail -2 $O/gpu_tests_parity.log
echo "[$(date +%H:%M:%S)] A/B"
timeout -k 10 300 python tools/ab_libs.py --libs tiled=nldsc_amd/libnldsc_amd.so rowmajor=ab_libs/rowmajor.so --workload c3 c2 c5 --runs 8 \
  > $O/ab_layout.json 2> $O/ab_layout.err || { tail $O/ab_layout.err; exit 1; }
cat $O/ab_layout.json
echo "[$(date +%H:%M:%S)] done"
