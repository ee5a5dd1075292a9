#!/bin/bash
# Round checkpoint on the GPU box: GPU parity tests, smoke, default bench (with the CPU baseline),
# rocprofv3 kernel statistics of the same bench.  Usage (from this container):
#   gpurun --timeout 900 -- bash tools/gpu_round.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-run}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 bench.py --no-cpu --steps 5 > $O/prof_bench.json 2> $O/prof.err \
  || { echo rocprof failed; tail $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cat $O/kernel_stats.csv | cut -c1-200
