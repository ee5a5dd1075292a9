#!/bin/bash
# Round 5 checkpoint of the run-overhead changes: same-process A/B against HEAD's library (ab_libs/r5_head.so), the
# benches, then the GPU suite (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_check.sh <tag> [skip-tests])
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5c}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step ab
timeout -k 10 400 python tools/ab_libs.py --libs head=ab_libs/r5_head.so new=nldsc_amd/libnldsc_amd.so --workload c2 c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  for n,x in v.items(): print(w,n,round(x['total_ms_median'],3),round(x['band_ms_median'],3),x['stages_ms_median'])"
step bench
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 20 --n-org 50000 --additive-only > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
python3 -c "
import json
for w in ('c2','c3'):
  d=json.loads(open('$O/'+w+'.json').read().strip().splitlines()[-1]); print(w, round(d['ms_per_step'],3), d['stages_ms'])"
[ "$2" = skip-tests ] && exit 0
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
step done
