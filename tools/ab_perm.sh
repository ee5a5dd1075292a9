#!/bin/bash
# MFMA issue order of the 8 products in the fp4 K loop (study builds -DNLDSC_F4_PERM=...) vs the default
#   bash tools/ab_perm.sh 01426357 03472156 ...   (ab_libs/p<perm>.so from tools/build_variant.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V="base=f4:xcd"
for p in "$@"; do V="$V,p$p=ab_libs/p$p.so:f4:xcd"; done
V="$V,base2=f4:xcd"
timeout -k 10 400 python tools/band_ab.py --rounds 4 --n-snp 80000 --length-cm 280 --variants "$V" \
  --out gpurun_out/ab_perm.json > gpurun_out/ab_perm.log 2>&1 || { tail gpurun_out/ab_perm.log; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_perm.json'))['summary']
for k,v in d.items(): print(f"{k:10s} band {v['band_ms_median']:.3f} min {v['band_ms_min']:.3f} total {v['total_ms_median']:.3f} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
