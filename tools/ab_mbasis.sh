#!/bin/bash
# GPU parity of the current build, then A/B against the HEAD build (o-basis) on C3
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "head=ab_libs/head.so:f4:xcd,mb=f4:xcd,mbr=f4:xcd:round-1,head2=ab_libs/head.so:f4:xcd,mb2=f4:xcd" \
  --out gpurun_out/ab5.json > gpurun_out/ab5.log 2>&1
rc=$?
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab5.json'))['summary']
for k,v in d.items(): print(k, round(v['band_ms_median'],3), round(v['issued_tflops']), v['items'], v['max_abs_l2_vs_first'], v['ws_equal'])
PY
exit $rc
