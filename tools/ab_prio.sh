#!/bin/bash
# s_setprio over the MFMA groups of the fp4 K loop (study builds) vs the default build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd,prio1=ab_libs/prio1.so:f4:xcd,prio3=ab_libs/prio3.so:f4:xcd,base2=f4:xcd,prio1b=ab_libs/prio1.so:f4:xcd" \
  --out gpurun_out/ab_prio.json > gpurun_out/ab_prio.log 2>&1 || { tail gpurun_out/ab_prio.log; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_prio.json'))['summary']
for k,v in d.items(): print(f"{k:6s} band {v['band_ms_median']:.3f} min {v['band_ms_min']:.3f} total {v['total_ms_median']:.3f} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
