#!/bin/bash
# A/B of engine environment knobs on one box: each "label:ENV=VAL:bench args" runs bench.py with that
# variable set, into gpurun_out/<tag>/bench_<label>.json.
#   gpurun --timeout 900 -- bash tools/ab/gpu_ab_env.sh <tag> "c3on:NLDSC_REPLAY_OVERLAP=1:" "c3off:NLDSC_REPLAY_OVERLAP=0:" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-ab}; shift
O=gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  label=${v%%:*}; rest=${v#*:}; kv=${rest%%:*}; args=${rest#*:}
  env ${kv//,/ } timeout -k 10 300 python bench.py --no-cpu --no-file $args > $O/bench_$label.json 2> $O/bench_$label.err \
    || { echo "bench $label failed"; tail $O/bench_$label.err; exit 1; }
  python - "$O/bench_$label.json" "$label" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value=%.4g" % d["value"], "ms/step=%.3f" % d["ms_per_step"], "stages=%s" % d.get("stages_ms"))
PY
done
echo done
