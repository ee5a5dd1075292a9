#!/bin/bash
# GPU parity tests + smoke on the GPU box (first half of a round checkpoint; tools/gpu_round.sh <tag> skip-tests
# is the second).  Usage: gpurun --timeout 1200 -- bash tools/gpu_tests.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-run}
mkdir -p $O
echo "[$(date +%H:%M:%S)] tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[$(date +%H:%M:%S)] done"
