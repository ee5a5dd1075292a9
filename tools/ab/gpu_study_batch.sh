#!/bin/bash
# One lease, several measurements (each step its own time limit; the script stops at the first failure):
#   genome  - the 22-autosome whole genome from .bed files (tools/e2e_genome.py --autosomes)
#   c2      - C2 bench + SQ instruction-mix / wait counters of its band kernel (verdict r03 item 5)
#   f32     - the fp32 MFMA GEMM path on C3 (north_star's GEMM) + its rocprofv3 kernel statistics (item 7)
#   gpurun --timeout 1200 -- bash tools/ab/gpu_study_batch.sh <tag> genome c2 f32
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-batch}; shift
mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
for what in "$@"; do
case $what in
genome)
  step genome
  timeout -k 10 600 python -u tools/e2e_genome.py --autosomes --fit --out $O/e2e_genome_c4.json > $O/e2e.log 2>&1 || { echo e2e failed; tail -30 $O/e2e.log; exit 1; }
  tail -c 600 $O/e2e.log ;;
c2)
  step c2
  timeout -s KILL 60 rocprofv3 --list-avail > $O/counters_avail.txt 2>&1 || true
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 --n-org 50000 --additive-only > $O/c2_bench.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
  B="python3 bench.py --no-cpu --no-file --steps 1 --warmup 1 --n-org 50000 --additive-only"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace -d $O/c2_sq -o s --output-format csv -- $B > /dev/null 2> $O/c2_sq.err || { tail $O/c2_sq.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-trace -d $O/c2_inst -o i --output-format csv -- $B > /dev/null 2> $O/c2_inst.err || { tail $O/c2_inst.err; echo "inst pass failed (continuing)"; }
  tail -c 300 $O/c2_bench.json ;;
f32)
  step f32
  timeout -k 10 300 python bench.py --no-cpu --no-file --steps 3 --path f32 > $O/f32_bench.json 2> $O/f32.err || { tail $O/f32.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/f32_prof -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 3 --path f32 > /dev/null 2> $O/f32_prof.err || { tail $O/f32_prof.err; exit 1; }
  find $O/f32_prof -name "*kernel_stats.csv" -exec cp {} $O/f32_kernel_stats.csv \;
  tail -c 300 $O/f32_bench.json ;;
esac
done
step done
