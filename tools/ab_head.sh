#!/bin/bash
# GPU parity of the current build, then interleaved A/B on C3 against the HEAD build (ab_libs/head.so).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "head=ab_libs/head.so:f4:xcd,cur=f4:xcd,head2=ab_libs/head.so:f4:xcd,cur2=f4:xcd" \
  --out gpurun_out/ab_head.json > gpurun_out/ab_head.log 2>&1
rc=$?
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_head.json'))['summary']
for k,v in d.items(): print(f"{k:8s} band {v['band_ms_median']:.3f} total {v['total_ms_median']:.3f} count {v['count_ms_median']:.3f} items {v['items']} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
exit $rc
