#!/bin/bash
# Counter passes over one bench workload, each pass in its own rocprofv3 run (rocprofv3 does not split counters
# over passes: at most 8 SQ / 4 TCC / 2 GRBM per pass).  Output: gpurun_out/<tag>/<label>_p<k>/ (+ a per-kernel sum).
#   gpurun --timeout 900 -- bash tools/ab/gpu_pmc_probe.sh <tag> <label> "<bench args>" "<counters pass 1>" ["<pass 2>" ...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; label=$2; args=$3; shift 3
O=gpurun_out/$T
mkdir -p $O
B="python3 bench.py --no-cpu --no-file --steps 1 --warmup 1 $args"
k=0
for ctrs in "$@"; do
  k=$((k + 1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -d $O/${label}_p$k -o p --output-format csv -- $B \
    > $O/${label}_p$k.out 2> $O/${label}_p$k.err || { echo "pass $k ($ctrs) failed"; tail $O/${label}_p$k.err; exit 1; }
  echo "pass $k done"
done
python3 - $O $label <<'PY'
import csv, glob, json, sys
from collections import defaultdict
O, label = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(int); dur = defaultdict(float)
for f in glob.glob(f"{O}/{label}_p*/**/*counter_collection.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nldsc::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r.get("Dispatch_Id"), k)
        if r["Counter_Name"].startswith("GRBM_GUI_ACTIVE") and key not in seen:
            seen.add(key)
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
out = {k: dict(v, pmc_seconds=dur.get(k)) for k, v in acc.items() if k.startswith("band") or k.startswith("count")}
json.dump(out, open(f"{O}/{label}_summary.json", "w"), indent=1)
print(json.dumps(out)[:3000])
PY
echo done
