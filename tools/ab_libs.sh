#!/bin/bash
# Interleaved A/B of alternate builds ab_libs/<name>.so (tools/build_variant.sh) against the default build on C3:
#   bash tools/ab_libs.sh <out-tag> name1 name2 ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
V="base=f4:xcd"
for p in "$@"; do V="$V,$p=ab_libs/$p.so:f4:xcd"; done
V="$V,base2=f4:xcd"
timeout -k 10 400 python tools/band_ab.py --rounds 4 --n-snp 80000 --length-cm 280 --variants "$V" \
  --out gpurun_out/ab_$T.json > gpurun_out/ab_$T.log 2>&1 || { tail gpurun_out/ab_$T.log; exit 1; }
python - "$T" <<'PY'
import json, sys
d=json.load(open(f'gpurun_out/ab_{sys.argv[1]}.json'))['summary']
for k,v in d.items(): print(f"{k:10s} band {v['band_ms_median']:.3f} min {v['band_ms_min']:.3f} total {v['total_ms_median']:.3f} dl2 {v['max_abs_l2_vs_first']:.2e} ws {v['ws_equal']}")
PY
