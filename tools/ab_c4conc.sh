#!/bin/bash
# C4 whole genome on one GPU: chromosomes one at a time vs 2 / 3 at once (host threads, one stream each)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 1 2 3 1 2; do
  timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --concurrent $c > gpurun_out/c4_conc$c.json 2> gpurun_out/c4_conc$c.err \
    || { echo "c4 concurrent $c failed"; tail gpurun_out/c4_conc$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_conc$c.json')); print('concurrent $c', round(d['ms_per_step'],2), 'ms', round(d['value']/1e9,3), 'G pairs/s')"
done
