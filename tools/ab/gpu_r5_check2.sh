#!/bin/bash
# GPU suite first (new load kernels), then A/B vs HEAD of round 4, the benches and the host-path probe
# (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_check2.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5d}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step ab
timeout -k 10 300 python tools/ab_libs.py --libs head=ab_libs/r5_head.so new=nldsc_amd/libnldsc_amd.so --workload c2 c3 --runs 8 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
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
  d=json.loads(open('$O/'+w+'.json').read().strip().splitlines()[-1]); print(w, round(d['ms_per_step'],3), d['stages_ms'], {k: d.get(k) for k in ('fp32_path','oneshot_gpu_ms')})"
step probe
timeout -k 10 300 python tools/hostpath_probe.py --runs 4 > $O/probe.txt 2>&1 || { tail -30 $O/probe.txt; exit 1; }
grep -E "^c[23] " $O/probe.txt
step done
