#!/bin/bash
# The round-end driver's N = 1 bench command on the final tree.   gpurun --timeout 600 -- bash tools/gpu_r6_driver_like.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6drv; mkdir -p $O
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['ms_per_step'],3), round(d['value']/1e9,3), round(r['frac'],4), r['traffic'], r['traffic_source'], d['cpu_baseline']['value'])"
