#!/bin/bash
# Loader source reads as unaligned 16-byte vector loads: the load / orientation / file / large-image GPU tests, the
# golden sets, then the bench line (oneshot_gpu_ms: the load from a device image) and an A/B of the run
# (gpurun --timeout 900 -- bash tools/ab/gpu_r5_load.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5l}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "golden or files or halo or orientation or past_2p32 or full_size or rare" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step bench
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c3', round(d['ms_per_step'],3), d['stages_ms'], 'frac', round(r['frac'],4), 'pipe', round(r['mfma_pipe_frac'],3), 'oneshot', d.get('oneshot_gpu_ms'))"
step done
