#!/bin/bash
# A/B of the fp4 decode / VALU-interleave variants (ab_libs/*.so built by tools/build_variant.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=${1:-"h5=ab_libs/h5.so:f4:xcd,o4=ab_libs/o4.so:f4:xcd,n4=ab_libs/n4.so:f4:xcd,n3=ab_libs/n3.so:f4:xcd,h5b=ab_libs/h5.so:f4:xcd,n4b=ab_libs/n4.so:f4:xcd"}
timeout -k 10 400 python tools/band_ab.py --rounds 3 --n-snp 80000 --length-cm 280 \
  --variants "$V" --out gpurun_out/ab_vpm.json > gpurun_out/ab_vpm.log 2>&1 || { tail gpurun_out/ab_vpm.log; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_vpm.json'))['summary']
for k,v in d.items(): print(f"{k:6s} band {v['band_ms_median']:.3f} total {v['total_ms_median']:.3f}")
PY
