#!/bin/bash
# round 3: split halo runs (boundary pairs once) — the torchrun tests, then the 1/8 rehearsal split vs duplicate
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_torchrun.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 0/8 > $O/reh_dup_$k.json 2> $O/reh.err || { tail $O/reh.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 0/8 --split-halo > $O/reh_split_$k.json 2> $O/reh.err || { tail $O/reh.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 3/8 > $O/reh3_dup_$k.json 2> $O/reh.err || { tail $O/reh.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 3/8 --split-halo > $O/reh3_split_$k.json 2> $O/reh.err || { tail $O/reh.err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r3y/reh*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"], 3), d["stages_ms"]["band_ms"], d["per_rank"][0]["pairs"])
PY
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --no-cpu --no-file --steps 5 > $O/gloo2.json 2> $O/gloo2.err || { tail $O/gloo2.err; exit 1; }
tail -c 500 $O/gloo2.json
