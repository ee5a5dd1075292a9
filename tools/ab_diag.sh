#!/bin/bash
# Diagnostic A/B of the fp4 band kernel: L2-resident operands (same), no decode VALU (nodec), both
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd:round-1,same=ab_libs/same.so:f4:xcd:round-1,nodec=ab_libs/nodec.so:f4:xcd:round-1,both=ab_libs/both.so:f4:xcd:round-1,nc2=f4nc2:xcd" \
  --out gpurun_out/ab2.json > gpurun_out/ab2.log 2>&1
rc=$?
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab2.json'))['summary']
for k,v in d.items(): print(k, round(v['band_ms_median'],3), round(v['issued_tflops']), v['items'])
PY
exit $rc
