#!/bin/bash
# End-to-end CLI wall clock (C2- and C3-sized files) on the GPU box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/e2e_cli.py --n-org 50000 --n-snp 80000 --dir /tmp/nldsc_e2e --out gpurun_out/e2e_c2.json \
  || { echo c2 failed; exit 1; }
timeout -k 10 400 python tools/e2e_cli.py --n-org 315599 --n-snp 80000 --dir /tmp/nldsc_e2e --out gpurun_out/e2e_c3.json \
  || { echo c3 failed; exit 1; }
