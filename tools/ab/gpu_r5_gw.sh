#!/bin/bash
# Two-wave workgroups for the single-block fp4 kernels (option band_gw): bitwise tests, then a same-box A/B against
# one-wave workgroups (same library), C3 / C2 / rank 0 of 8, two orders; then the loader stage sizes (load_probe)
# (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_gw.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5gw}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "two_wave or round_launch" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
L=ab_libs/r5_gw.so
k=0
for order in "gw2=$L,band_gw=2 gw1=$L,band_gw=1" "gw1=$L,band_gw=1 gw2=$L,band_gw=2"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 c3r0of8 --runs 8 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step loads
timeout -k 10 200 python tools/ab/load_probe.py --loads 9 --libs ua=ab_libs/r5_ua.so sc8=ab_libs/r5_sc8.so sc16=ab_libs/r5_sc16.so sc32=ab_libs/r5_sc32.so > $O/load.txt 2>&1 || { tail $O/load.txt; exit 1; }
tail -4 $O/load.txt
step done
