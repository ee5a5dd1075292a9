#!/bin/bash
# pinned positions upload + pinned result landing (new) vs pageable copies (ab_libs/head.so): engine wall time per run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/band_ab.py --rounds 6 --n-snp 80000 --length-cm 280 \
  --variants "new=f4:xcd,old=ab_libs/head.so:f4:xcd,new2=f4:xcd,old2=ab_libs/head.so:f4:xcd" \
  --out gpurun_out/ab_pinned.json > gpurun_out/ab_pinned.log 2>&1 || { tail gpurun_out/ab_pinned.log; exit 1; }
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_pinned.json'))['summary']
for k,v in d.items(): print(f"{k:6s} band {v['band_ms_median']:.3f} total {v['total_ms_median']:.3f} count {v['count_ms_median']:.3f} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
