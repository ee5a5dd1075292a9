#!/bin/bash
# Runtime + kernel + copy trace of a few C2 runs (what each GPU command of a run is, in API order)
# (gpurun --timeout 600 -- bash tools/ab/gpu_trace_c2.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-trc2}; mkdir -p $O
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace -d $O/c2 -o t --output-format csv -- python3 bench.py --no-cpu --no-file --steps 3 --n-org 50000 --additive-only > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu --no-file --steps 20 --n-org 50000 --additive-only > $O/c2b.json 2> $O/c2b.err || { tail $O/c2b.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu --no-file --steps 10 > $O/c3b.json 2> $O/c3b.err || { tail $O/c3b.err; exit 1; }
ls -R $O | head -30
