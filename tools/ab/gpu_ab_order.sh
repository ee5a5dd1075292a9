#!/bin/bash
# Position bias check of the interleaved A/B (the same builds in permuted orders) and the additive decode without the
# v_not (opaque w >> 2): C3 and C2 (gpurun --timeout 900 -- bash tools/ab/gpu_ab_order.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abo}; mkdir -p $O
k=0
for order in "head=ab_libs/r5_head.so cur=ab_libs/r5_cur.so opq=nldsc_amd/libnldsc_amd.so" "opq=nldsc_amd/libnldsc_amd.so cur=ab_libs/r5_cur.so head=ab_libs/r5_head.so" "nolambda=ab_libs/r5_nolambda.so opq=nldsc_amd/libnldsc_amd.so"; do
  k=$((k+1))
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 --runs 8 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
