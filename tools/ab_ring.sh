#!/bin/bash
# A/B: register-staged fp4 loop vs per-wave LDS ring (LDS-DMA) of depth 3/4/5
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd:round-1,ring3=f4:xcd:ring3,ring4=f4:xcd:ring4,ring5=f4:xcd:ring5,ring4r=f4:xcd:ring4:round-1,grp0=f4:xcd:grp0,base1=f4:xcd" \
  --out gpurun_out/ab4.json > gpurun_out/ab4.log 2>&1
rc=$?
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab4.json'))['summary']
for k,v in d.items(): print(k, round(v['band_ms_median'],3), round(v['issued_tflops']), v['items'], v['max_abs_l2_vs_first'], v['ws_equal'])
PY
exit $rc
