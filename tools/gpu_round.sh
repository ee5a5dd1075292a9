#!/bin/bash
# Round checkpoint on the GPU box : GPU parity tests, smoke, the default bench (C3, file wall clock + CPU
# baseline), rocprofv3 kernel statistics of the same bench, PMC passes (HBM traffic, MFMA busy, clock, L2) of the
# current kernels for C3, C2 and the C5 slice, their bench lines, a per-rank rehearsal of 8-GPU strong scaling and a
# 2-rank gloo run of `bench.py --gpus 2` (the bench starting its own ranks).  Every step has its own time limit and
# the script stops at the first failure.  gpurun's limit (1200 s) takes it in three calls (from this container):
#   gpurun --timeout 1200 -- bash tools/gpu_tests.sh <tag>                       (the GPU suite + smoke)
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag> skip-tests bench      (bench, rocprof stats)
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag> skip-tests pmc        (PMC passes, C2 / C5, scaling)
#   (phase pmc-only: the PMC passes alone)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-run}
O=gpurun_out/$T
mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
if [ "$2" != "skip-tests" ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo smoke failed; cat $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
PH=${3:-all}
if [ "$PH" = all ] || [ "$PH" = bench ]; then
step bench
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench failed; tail $O/bench_c3.err; exit 1; }
tail -c 400 $O/bench_c3.json
step rocprof stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 > $O/prof_bench.json 2> $O/prof.err \
  || { echo rocprof failed; tail $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c3.csv \;
[ "$PH" = bench ] && { step done; exit 0; }
fi
pmc() {  # <label> <workload string> <alg-bytes spec> <bench args>
  local label=$1 wl=$2 alg=$3; shift 3
  local B="python3 bench.py --no-cpu --no-file --no-extra --steps 1 --warmup 0 $*" P=$O/pmc_$label
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o f --output-format csv -- $B > /dev/null 2> $P.f.err && \
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o w --output-format csv -- $B > /dev/null 2> $P.w.err && \
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace -d $P/sq -o s --output-format csv -- $B > /dev/null 2> $P.s.err && \
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $P/l2 -o l --output-format csv -- $B > /dev/null 2> $P.l.err \
    || { echo "pmc $label failed"; tail $P.*.err; return 1; }
  if [ -n "$LDS_PASS" ]; then
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d $P/lds -o d --output-format csv -- $B > /dev/null 2> $P.d.err \
      || { echo "pmc $label lds failed"; tail $P.d.err; return 1; }
  fi
  python3 tools/pmc_summary.py $P --workload "$wl" --alg-bytes $alg > $O/pmc_$label.json
}
step pmc c3
pmc c3 "C3 bench: N=315599 M=80000 missing=0.01 add+dom 1 cM" band_f4_kernel=6312960000 || exit 1
step pmc c2
pmc c2 "C2 bench: N=50000 M=80000 missing=0.01 additive-only 1 cM" band_f4_kernel=1003520000 --n-org 50000 --additive-only || exit 1
step pmc c5
LDS_PASS=1 pmc c5 "C5 slice bench: N=315599 M=1250000 missing=0 add+dom 1000 kb" band_f4_q_kernel=98640000000 --workload c5 || exit 1
[ "$PH" = pmc-only ] && { step done; exit 0; }
step bench c2 c5
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --n-org 50000 --additive-only > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu --no-file --steps 2 --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
step rehearse
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --rehearse 0/8 > $O/rehearse_r0of8.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
step gloo2
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --no-cpu --no-file --steps 5 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo gloo2 failed; tail $O/bench_gloo2.err; exit 1; }
tail -c 300 $O/bench_gloo2.json
step done
