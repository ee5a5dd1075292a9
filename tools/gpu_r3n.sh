#!/bin/bash
# round 3: the parallel file loader (GPU tests that load .bed files, the bench's wall clock from a file), then the
# checkpoint's PMC phase (tools/gpu_round3.sh <tag> skip-tests pmc)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ck; mkdir -p $O
echo "[$(date +%H:%M:%S)] file-loading tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_torchrun.py -m gpu -x -v -k "pybind or golden or torchrun or cli or sharded" --timeout 300 --timeout-method thread > $O/gpu_tests_files.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests_files.log; exit 1; }
tail -2 $O/gpu_tests_files.log
echo "[$(date +%H:%M:%S)] bench"
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench failed; tail $O/bench_c3.err; exit 1; }
tail -c 600 $O/bench_c3.json
bash tools/gpu_round3.sh r3ck skip-tests pmc
