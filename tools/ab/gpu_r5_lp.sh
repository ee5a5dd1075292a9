#!/bin/bash
# Loader at ~64 k workgroups with its count parts folded at load: load / count GPU tests, the load probe, and a run
# A/B against the previous build (the run's tail kernel now reads one part), C3 / C2, two orders
# (gpurun --timeout 900 -- bash tools/ab/gpu_r5_lp.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5lp}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "golden or files or halo or orientation or past_2p32 or full_size or rare or c5_shape or c2_shape or split" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step loads
timeout -k 10 200 python tools/ab/load_probe.py --loads 9 --libs prev=ab_libs/r5_fence.so new=ab_libs/r5_lp.so > $O/load.txt 2>&1 || { tail $O/load.txt; exit 1; }
tail -2 $O/load.txt
k=0
for order in "new=ab_libs/r5_lp.so prev=ab_libs/r5_fence.so" "prev=ab_libs/r5_fence.so new=ab_libs/r5_lp.so"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 --runs 10 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f cnt %.4f' % (n, x['total_ms_median'], x['band_ms_median'], x['stages_ms_median']['count_ms']) for n, x in v.items()))"
done
step done
