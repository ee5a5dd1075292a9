#!/bin/bash
# fp4 band kernel on A2-minor (synthetic default) vs A2-major coded genotypes
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 --variants "minor=f4:xcd,head=ab_libs/head.so:f4:xcd" --out gpurun_out/ab6a.json > gpurun_out/ab6a.log 2>&1 && \
timeout -k 10 300 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 --major --variants "major=f4:xcd,headmajor=ab_libs/head.so:f4:xcd" --out gpurun_out/ab6b.json > gpurun_out/ab6b.log 2>&1
rc=$?
python - <<'PY'
import json
for f in ['gpurun_out/ab6a.json','gpurun_out/ab6b.json']:
    d=json.load(open(f))['summary']
    for k,v in d.items(): print(k, round(v['band_ms_median'],3), round(v['issued_tflops']), v['items'], v['max_abs_l2_vs_first'], v['ws_equal'])
PY
exit $rc
