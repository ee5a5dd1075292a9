#!/bin/bash
# Round checkpoint on the GPU box: GPU parity tests, smoke, default bench (file wall clock + CPU baseline),
# rocprofv3 kernel statistics of the same bench, PMC passes (HBM traffic of the current kernels), and a
# 2-rank gloo rehearsal of the strong-scaling bench on the one GPU.  Usage (from this container):
#   gpurun --timeout 1500 -- bash tools/gpu_round.sh <tag> [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-run}
O=gpurun_out/$T
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo smoke failed; cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 > $O/prof_bench.json 2> $O/prof.err \
  || { echo rocprof failed; tail $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -c1-160 $O/kernel_stats.csv | head -12
B="python3 bench.py --no-cpu --no-file --steps 1 --warmup 0"
P=$O/pmc
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o f --output-format csv -- $B > /dev/null 2> $O/pmc_f.err && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o w --output-format csv -- $B > /dev/null 2> $O/pmc_w.err && \
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace -d $P/sq -o s --output-format csv -- $B > /dev/null 2> $O/pmc_s.err && \
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $P/l2 -o l --output-format csv -- $B > /dev/null 2> $O/pmc_l.err \
  || { echo pmc failed; tail $O/pmc_*.err; exit 1; }
python3 tools/pmc_summary.py $P --workload "C3 bench: N=315599 M=80000 missing=0.01 add+dom 1 cM" \
  --alg-bytes band_f4_kernel=6312960000 > $O/pmc.json && python3 - $O/pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if k.startswith("band"):
        print(k, {x: v.get(x) for x in ("traffic_bytes", "mfma_busy_frac_per_simd", "effective_clock_ghz", "l2_hit_rate")})
PY
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --backend gloo --steps 3 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo gloo2 failed; tail $O/bench_gloo2.err; exit 1; }
tail -1 $O/bench_gloo2.json
echo done
