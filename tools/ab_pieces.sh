#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/pieces_ab.py --rounds 5 --pieces 1,2,3,4 --out gpurun_out/ab_pieces.json > gpurun_out/ab_pieces.log 2>&1 \
  || { tail -20 gpurun_out/ab_pieces.log; exit 1; }
cat gpurun_out/ab_pieces.log
timeout -k 10 300 bash tools/ab_c4conc.sh
