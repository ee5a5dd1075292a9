#!/bin/bash
# round end, after the PMC summaries of the current kernels are committed under profiles/: the default bench line
# (C3, file wall clock + CPU baseline), its rocprofv3 kernel statistics, and the C2 / C5-slice bench lines, each of
# which reads its traffic from those summaries.   gpurun --timeout 1200 -- bash tools/gpu_bench_final.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r3b}
bash tools/gpu_round.sh $T skip-tests bench || exit 1
O=gpurun_out/$T
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --n-org 50000 --additive-only > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu --no-file --steps 2 --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 --rehearse 0/8 > $O/rehearse_r0of8.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
for f in bench_c3 bench_c2 bench_c5 rehearse_r0of8; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['ms_per_step'],3), d['stages_ms'].get('band_ms'), round(r['frac'],4), r.get('traffic'))"; done
