#!/bin/bash
# Where the band kernel's cycles go, per engine variant: for each "label:ENV=VAL:bench args" a timed bench
# (--steps 10) and two rocprofv3 --pmc passes of a 1-step bench (SQ wave-cycle buckets + MFMA busy + clock;
# FETCH_SIZE), each pass in its own run.  Output: gpurun_out/<tag>/<label>_{bench.json,sq,fetch}.
#   gpurun --timeout 900 -- bash tools/ab/gpu_stall_probe.sh <tag> "c3:NLDSC_T2=1:" "c3all:NLDSC_T2=2:" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-stall}; shift
O=gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  label=${v%%:*}; rest=${v#*:}; kv=${rest%%:*}; args=${rest#*:}
  export "$kv"
  timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 $args > $O/${label}_bench.json 2> $O/${label}_bench.err \
    || { echo "bench $label failed"; tail $O/${label}_bench.err; exit 1; }
  B="python3 bench.py --no-cpu --no-file --steps 1 --warmup 1 $args"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-trace -d $O/${label}_sq -o s --output-format csv -- $B > /dev/null 2> $O/${label}_sq.err \
    || { echo "sq pass $label failed"; tail $O/${label}_sq.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/${label}_fetch -o f --output-format csv -- $B > /dev/null 2> $O/${label}_f.err \
    || { echo "fetch pass $label failed"; tail $O/${label}_f.err; exit 1; }
  unset "${kv%%=*}"
  python3 - $O $label <<'PY'
import csv, glob, json, sys
from collections import defaultdict
O, label = sys.argv[1], sys.argv[2]
b = json.loads(open(f"{O}/{label}_bench.json").read().strip().splitlines()[-1])
acc = defaultdict(lambda: defaultdict(float)); dur = defaultdict(float)
for part in ("sq", "fetch"):
    for f in glob.glob(f"{O}/{label}_{part}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nldsc::", "")
            if not n.startswith("band"):
                continue
            acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
out = {"label": label, "ms_per_step": b["ms_per_step"], "band_ms": b["stages_ms"]["band_ms"]}
for n, c in acc.items():
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    g = c.get("GRBM_GUI_ACTIVE", 0)
    out[n] = {"wait_any": c.get("SQ_WAIT_ANY", 0) / w, "wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / w,
              "active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0) / w,
              "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(g / 8 * 1024, 1),
              "clock_ghz": g / 8 / dur[n] / 1e9 if dur[n] > 0 else None, "pmc_ms": dur[n] * 1e3,
              "fetch_gb_x2": 2 * c.get("FETCH_SIZE", 0) * 1024 / 1e9, "valu_insts": c.get("SQ_INSTS_VALU", 0)}
print(json.dumps(out))
PY
done
echo done
