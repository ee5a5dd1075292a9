#!/bin/bash
# PMC + kernel-stats passes of the C3 bench (run on the GPU box from the repo root; see tools/pmc_summary.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --no-cpu --steps 1 --warmup 0"
D=gpurun_out/pmc_f4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/stats -o k --output-format csv -- python3 bench.py --no-cpu --steps 5 > $D.bench.json 2> $D.stats.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o f --output-format csv -- $B > /dev/null 2> $D.f.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o w --output-format csv -- $B > /dev/null 2> $D.w.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace -d $D/sq -o s --output-format csv -- $B > /dev/null 2> $D.s.err && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $D/l2 -o l --output-format csv -- $B > /dev/null 2> $D.l.err
echo rc=$?
