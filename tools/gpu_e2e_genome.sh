#!/bin/bash
# Whole genome from .bed files on one GPU (verdict r03 item 2): the 22 C4 autosomes (N = 315 599, sum M ~ 600 k,
# ~47 GB) written to $TMPDIR, then the CLI timed cold / warm and per stage.   gpurun --timeout 1200 -- bash tools/gpu_e2e_genome.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-e2e}
mkdir -p $O
df -h $TMPDIR > $O/df.txt; free -g >> $O/df.txt; nproc >> $O/df.txt; cat $O/df.txt
timeout -k 10 1100 python -u tools/e2e_genome.py --autosomes --fit --out $O/e2e_genome_c4.json > $O/e2e.log 2>&1 || { echo e2e failed; tail -30 $O/e2e.log; exit 1; }
tail -c 1500 $O/e2e.log
