#!/bin/bash
# Quad kernel variant (see the tag): quad / routing GPU tests, then a same-box C5
# A/B against the fenced build (r5_fence), two orders
# (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_qset.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5qs}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c5_shape or routing or issued or 2x2 or quad" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
k=0
for order in "new=ab_libs/r5_q2set.so prev=ab_libs/r5_fence.so" "prev=ab_libs/r5_fence.so new=ab_libs/r5_q2set.so"; do
  k=$((k+1)); step ab $k
  timeout -k 10 400 python tools/ab_libs.py --libs $order --workload c5 --c5-snp 600000 --runs 3 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.1f/%.1f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step done
