#!/bin/bash
# One GPU session: GPU parity tests, smoke, then bench variants named on the command line
# (each "label:args" pair runs `bench.py <args>` into gpurun_out/<tag>/bench_<label>.json).
#   gpurun --timeout 1200 -- bash tools/gpu_probe.sh <tag> [tests] "c3:" "c3m0:--missing 0" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-probe}; shift
O=gpurun_out/$T
mkdir -p $O
if [ "$1" = "tests" ]; then
  shift
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo smoke failed; cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
for v in "$@"; do
  label=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py $args > $O/bench_$label.json 2> $O/bench_$label.err \
    || { echo "bench $label failed"; tail $O/bench_$label.err; exit 1; }
  python - "$O/bench_$label.json" "$label" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.2f" % d["ms_per_step"], "band_ms=%s" % r.get("avg_launch_ms"),
      "frac=%s" % r.get("frac"), "stages=%s" % d.get("stages_ms"))
PY
done
echo done
