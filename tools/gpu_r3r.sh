#!/bin/bash
# round 3: stall counters of the C3 / C2 band kernels, the RCCL one-rank tests (device assembly), quad-round test,
# and the 1/8 rehearsal with a one-rank RCCL group (gather + device assembly timed)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_torchrun.py tests/test_gpu_parity.py -m gpu -x -v -k "rccl or force_dist or quad_round" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --force-dist > $O/bench_forcedist.json 2> $O/bench_forcedist.err || { tail $O/bench_forcedist.err; exit 1; }
tail -c 700 $O/bench_forcedist.json
bash tools/gpu_stall_probe.sh r3r/stall "c3::" "c2::--n-org 50000 --additive-only"
