#!/bin/bash
# Cost of running the diagonal block pairs in a launch of their own (the shape of a count-fused first phase)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/band_ab.py --rounds 5 --n-snp 80000 --length-cm 280 \
  --variants "base=f4:xcd,dsplit=f4:xcd:dsplit,base2=f4:xcd,dsplit2=f4:xcd:dsplit" \
  --out gpurun_out/ab_dsplit_c3.json > gpurun_out/ab_dsplit_c3.log 2>&1 || { tail gpurun_out/ab_dsplit_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dsplit -o k --output-format csv -- python3 tools/band_ab.py --rounds 2 --n-snp 80000 --length-cm 280 --variants "dsplit=f4:xcd:dsplit" > gpurun_out/prof_dsplit.log 2>&1 || { tail gpurun_out/prof_dsplit.log; exit 1; }
find gpurun_out/prof_dsplit -name "*kernel_stats.csv" -exec cp {} gpurun_out/dsplit_kernel_stats.csv \;
find gpurun_out/prof_dsplit -name "*kernel_trace.csv" -exec cp {} gpurun_out/dsplit_kernel_trace.csv \;
rm -rf gpurun_out/prof_dsplit
python - <<'PY'
import json
d=json.load(open('gpurun_out/ab_dsplit_c3.json'))['summary']
for k,v in d.items(): print(f"c3 {k:8s} band {v['band_ms_median']:.3f} min {v['band_ms_min']:.3f} total {v['total_ms_median']:.3f} count {v['count_ms_median']:.3f} items {v['items']} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
