#!/bin/bash
# Measurement round on the GPU box: default bench (C3 + CPU baseline), rocprofv3 kernel stats, PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ/GRBM, TCC hit/miss) of the C3 bench, C4 whole-genome bench, and a 2-rank
# gloo rehearsal of the multi-GPU bench path.   gpurun --timeout 1200 -- bash tools/gpu_measure.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-run}; O=gpurun_out/$T; mkdir -p $O
B="python3 bench.py --no-cpu --steps 1 --warmup 0"
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 bench.py --no-cpu --steps 5 > $O/prof_bench.json 2> $O/prof.err \
  || { echo rocprof failed; tail $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/fetch -o f --output-format csv -- $B > /dev/null 2> $O/pmc_f.err \
  && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc/write -o w --output-format csv -- $B > /dev/null 2> $O/pmc_w.err \
  && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace -d $O/pmc/sq -o s --output-format csv -- $B > /dev/null 2> $O/pmc_s.err \
  && timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/pmc/l2 -o l --output-format csv -- $B > /dev/null 2> $O/pmc_l.err \
  || { echo pmc failed; tail $O/pmc_*.err; exit 1; }
find $O/pmc -name "*.db" -delete 2>/dev/null
timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail $O/bench_c4.err; exit 1; }
cat $O/bench_c4.json
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --no-cpu > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo gloo2 failed; tail $O/bench_gloo2.err; exit 1; }
cat $O/bench_gloo2.json
