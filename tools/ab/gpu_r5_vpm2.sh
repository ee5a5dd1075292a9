#!/bin/bash
# VALU per MFMA of the full 8-product step (F4_VPM 3 / 4 / 5) on the fenced-load K loop: C3 and rank 0 of 8, two orders
# (gpurun --timeout 900 -- bash tools/ab/gpu_r5_vpm2.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5vpm2}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
k=0
for order in "v4=ab_libs/r5_fence.so v3=ab_libs/r5_vpm3.so v5=ab_libs/r5_vpm5.so" "v5=ab_libs/r5_vpm5.so v3=ab_libs/r5_vpm3.so v4=ab_libs/r5_fence.so"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c3r0of8 --runs 10 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step done
