#!/bin/bash
# Three rotating chunk buffers in the single-block fp4 K loop (four K steps of load distance): bitwise tests, then a
# same-box A/B against the previous build, C3 / C2 / rank 0 of 8, two orders
# (gpurun --timeout 900 -- bash tools/ab/gpu_r5_fence.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5fe}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "round_launch or 2x2 or column_block or full_size or c2_shape or golden or ksplit" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
k=0
for order in "new=ab_libs/r5_k3.so prev=ab_libs/r5_fence.so" "prev=ab_libs/r5_fence.so new=ab_libs/r5_k3.so"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 c3r0of8 --runs 10 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step done
