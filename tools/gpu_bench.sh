#!/bin/bash
# GPU parity tests, default bench (C3, with CPU baseline), C5 slice bench, rocprof kernel stats of the C3 bench.
#   gpurun --timeout 1200 -- bash tools/gpu_bench.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-run}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 bench.py --no-cpu --steps 5 > $O/prof_bench.json 2> $O/prof.err \
  || { echo rocprof failed; tail $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -c1-150 $O/kernel_stats.csv
timeout -k 10 400 python bench.py --workload c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
