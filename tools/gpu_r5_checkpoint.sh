#!/bin/bash
# Round-5 checkpoint, second half (after tools/gpu_tests.sh): the default bench line (C3, with the CPU baseline and the
# file wall clock), rocprofv3 kernel statistics and a kernel trace of the same bench, the C2 / C5 bench lines, PMC
# passes for C3 / C2 / C5 (tools/gpu_round.sh pmc) and the quad kernel's stall buckets
# (gpurun --timeout 1200 -- bash tools/gpu_r5_checkpoint.sh <tag> [bench|pmc])
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r5cp}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
PH=${2:-bench}
if [ "$PH" = bench ]; then
  step bench c3
  timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench failed; tail $O/bench_c3.err; exit 1; }
  tail -c 300 $O/bench_c3.json
  step rocprof stats
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 bench.py --no-cpu --no-file --no-extra --steps 5 > $O/prof_bench.json 2> $O/prof.err \
    || { echo rocprof failed; tail $O/prof.err; exit 1; }
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c3.csv \;
  find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace_c3.csv \;
  step bench c2 c5
  timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --n-org 50000 --additive-only > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
  timeout -k 10 400 python bench.py --no-cpu --no-file --steps 2 --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
  step rehearse
  timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --rehearse 0/8 > $O/rehearse_r0of8.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
  step force-dist
  timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --force-dist > $O/bench_force_dist.json 2> $O/force_dist.err || { tail $O/force_dist.err; exit 1; }
  step done
  exit 0
fi
step pmc
timeout -k 10 1100 bash tools/gpu_round.sh $T skip-tests pmc-only > $O/pmc.txt 2>&1 || { tail -20 $O/pmc.txt; exit 1; }
tail -5 $O/pmc.txt
step stall c5
timeout -k 10 400 bash tools/ab/gpu_stall_probe.sh $T/stall "c5:NLDSC_NONE=0:--workload c5 --no-extra" > $O/stall.txt 2>&1 || { tail $O/stall.txt; exit 1; }
tail -c 1200 $O/stall.txt
step done
