#!/bin/bash
# A/B: one wave per block pair vs 4-wave workgroups of skewed 2x2 tiles (barrier period 0/1/2/8)
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd:round-1,grp0=f4:xcd:grp0,grp1=f4:xcd:grp1,grp2=f4:xcd:grp2,grp8=f4:xcd:grp8,grp2r=f4:xcd:grp2:round-1,grp1r=f4:xcd:grp1:round-1" \
  --out gpurun_out/ab3.json > gpurun_out/ab3.log 2>&1
rc=$?
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab3.json'))['summary']
for k,v in d.items(): print(k, round(v['band_ms_median'],3), round(v['issued_tflops']), v['items'], v['max_abs_l2_vs_first'], v['ws_equal'])
PY
exit $rc
