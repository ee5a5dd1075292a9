#!/bin/bash
# Where the band kernels' wave cycles go (SQ buckets: waits, issue stalls, active) with MFMA busy and the clock, for one
# or more bench workloads: a 1-step bench under one rocprofv3 --pmc pass per workload (counters in their own run).
#   gpurun --timeout 600 -- bash tools/gpu_stall_probe.sh <tag> "c3:" "c2:--n-org 50000 --additive-only" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-stall}; shift
O=gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  label=${v%%:*}; args=${v#*:}
  B="python3 bench.py --no-cpu --no-file --no-extra --steps 1 --warmup 1 $args"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-trace -d $O/${label}_sq -o s --output-format csv -- $B > /dev/null 2> $O/${label}_sq.err \
    || { echo "sq pass $label failed"; tail $O/${label}_sq.err; exit 1; }
  python3 - $O $label <<'PY'
import csv, glob, json, sys
from collections import defaultdict
O, label = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(float)); dur = defaultdict(float)
for f in glob.glob(f"{O}/{label}_sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nldsc::", "")
        if not n.startswith("band"):
            continue
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            dur[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
out = {"label": label}
for n, c in acc.items():
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    g = c.get("GRBM_GUI_ACTIVE", 0)
    out[n] = {"wait_any": c.get("SQ_WAIT_ANY", 0) / w, "wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / w,
              "active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / w,
              "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(g / 8 * 1024, 1),
              "clock_ghz": g / 8 / dur[n] / 1e9 if dur[n] > 0 else None, "pmc_ms": dur[n] * 1e3,
              "valu_insts": c.get("SQ_INSTS_VALU", 0)}
print(json.dumps(out))
PY
done
echo done
