#!/bin/bash
# round 3: the GPU suite + smoke on round launches from one round on, then the shard rehearsals and C3 (defaults)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3v; mkdir -p $O
bash tools/gpu_tests.sh r3v || exit 1
for r in 0/8 3/8 1/4; do
  l=${r/\//of}
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse $r > $O/reh_$l.json 2> $O/reh.err || { tail $O/reh.err; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
for f in reh_0of8 reh_3of8 reh_1of4 c3; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$f', round(d['ms_per_step'],3), s['band_ms'], s['count_ms'], d['roofline'].get('work_items'))"; done
