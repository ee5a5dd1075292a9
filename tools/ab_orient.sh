#!/bin/bash
# Allele orientation A/B on C3 with PLINK's usual coding (A2 = major: --major swaps 00 <-> 11 in every SNP)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/band_ab.py --rounds 4 --n-snp 80000 --length-cm 280 --major \
  --variants "ori=f4:xcd,file=f4:xcd:noori,ori2=f4:xcd,file2=f4:xcd:noori" \
  --out gpurun_out/ab_orient.json > gpurun_out/ab_orient.log 2>&1 || { tail gpurun_out/ab_orient.log; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_orient.json'))['summary']
for k,v in d.items(): print(f"{k:6s} band {v['band_ms_median']:.3f} total {v['total_ms_median']:.3f} items {v['items']} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
