#!/bin/bash
# Item order A/B: diagonal block pairs last in every XCD run (dl) vs the plan order, on C3 and on a C5-density slice
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd,dl=f4:xcd:dl,base2=f4:xcd,dl2=f4:xcd:dl" \
  --out gpurun_out/ab_diaglast_c3.json > gpurun_out/ab_diaglast_c3.log 2>&1 || { tail gpurun_out/ab_diaglast_c3.log; exit 1; }
timeout -k 10 400 python tools/band_ab.py --rounds 2 --n-snp 400000 --length-cm 115200000 --window 1000000 \
  --variants "base=f4:xcd,dl=f4:xcd:dl" \
  --out gpurun_out/ab_diaglast_c5.json > gpurun_out/ab_diaglast_c5.log 2>&1 || { tail gpurun_out/ab_diaglast_c5.log; exit 1; }
python - <<'PY'
import json
for w in ("c3", "c5"):
    d=json.load(open(f'gpurun_out/ab_diaglast_{w}.json'))['summary']
    for k,v in d.items(): print(f"{w} {k:6s} band {v['band_ms_median']:.3f} min {v['band_ms_min']:.3f} total {v['total_ms_median']:.3f} items {v['items']} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
