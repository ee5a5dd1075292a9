#!/bin/bash
# round 3: the rest of the GPU suite (C4 genome, torchrun / RCCL), smoke, then the checkpoint bench + rocprof stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ck; mkdir -p $O
echo "[$(date +%H:%M:%S)] c4 + torchrun tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_torchrun.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests_rest.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests_rest.log; exit 1; }
tail -2 $O/gpu_tests_rest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_round3.sh r3ck skip-tests bench
