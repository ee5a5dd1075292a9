#!/bin/bash
# Additive-only fp4 loop: the VALU-per-MFMA interleave of its steps (4, 5, 6, or the formula's 7) with the m plane's
# decode as an explicit v_bitop3 (b3*) or as written (nb*: a v_not per word beside it); C2, two orders
# (gpurun --timeout 900 -- bash tools/ab/gpu_r5_vpm.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5vpm}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
A="nb=ab_libs/r5_sc16.so b3=ab_libs/r5_b3.so b3v4=ab_libs/r5_b3v4.so b3v5=ab_libs/r5_b3v5.so b3v6=ab_libs/r5_b3v6.so nbv4=ab_libs/r5_nbv4.so nbv5=ab_libs/r5_nbv5.so nbv6=ab_libs/r5_nbv6.so"
B="nbv6=ab_libs/r5_nbv6.so nbv5=ab_libs/r5_nbv5.so nbv4=ab_libs/r5_nbv4.so b3v6=ab_libs/r5_b3v6.so b3v5=ab_libs/r5_b3v5.so b3v4=ab_libs/r5_b3v4.so b3=ab_libs/r5_b3.so nb=ab_libs/r5_sc16.so"
k=0
for order in "$A" "$B"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c2 --runs 10 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step done
