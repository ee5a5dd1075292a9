#!/bin/bash
# Bench lines of every BASELINE config the repo measures on one GPU, on the current kernels:
#   gpurun --timeout 1200 -- bash tools/ab/gpu_sweep.sh <tag>   ->  gpurun_out/<tag>/<name>.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-sweep}
O=gpurun_out/$T
mkdir -p $O
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py --no-cpu --no-file "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python - $O/$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.2f" % d["ms_per_step"], "band_ms=%s" % (d.get("stages_ms") or {}).get("band_ms"),
      "frac=%s" % r.get("frac"), flush=True)
PY
}
run c2 200 --steps 10 --n-org 50000 --additive-only
run c3_missing0 200 --steps 10 --missing 0
run c3_i8 300 --steps 5 --path i8
run c4 400 --workload c4 --steps 3
run c5_slice 600 --workload c5 --steps 1 --warmup 1
run c3_fp32 400 --steps 2 --warmup 1 --path f32
echo done
