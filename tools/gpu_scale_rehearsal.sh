#!/bin/bash
# The metric's multi-GPU commands rehearsed on the one-GPU box (verdict r03 item 1): `bench.py --gpus 8` and
# `--gpus 4` at the full C3 size with gloo ranks sharing GPU 0 (the bench starts its own ranks), then the per-rank
# cost of an 8-GPU run (--rehearse R/8 for the first and a middle rank).   gpurun --timeout 1200 -- bash tools/gpu_scale_rehearsal.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-scale}
mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step gloo8
timeout -k 10 500 python bench.py --gpus 8 --backend gloo --no-cpu --no-file --steps 3 > $O/bench_gloo8.json 2> $O/bench_gloo8.err || { echo gloo8 failed; tail -30 $O/bench_gloo8.err; exit 1; }
tail -c 600 $O/bench_gloo8.json
step gloo4
timeout -k 10 400 python bench.py --gpus 4 --backend gloo --no-cpu --no-file --steps 3 > $O/bench_gloo4.json 2> $O/bench_gloo4.err || { echo gloo4 failed; tail -30 $O/bench_gloo4.err; exit 1; }
tail -c 300 $O/bench_gloo4.json
step rehearse
for r in 0 3 7; do
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 --rehearse $r/8 > $O/rehearse_r${r}of8.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
done
step one
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 > $O/bench_c3_one.json 2> $O/bench_c3_one.err || { tail $O/bench_c3_one.err; exit 1; }
step done
