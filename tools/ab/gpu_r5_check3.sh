#!/bin/bash
# Load-time genotype counts (no per-run count pass): GPU suite, then A/B against round 4's library and the previous
# round-5 build, C3 / C2 / rank 0 of 8, two orders, and the bench (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_check3.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5h}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step ab
k=0
for order in "head=ab_libs/r5_head.so prev=ab_libs/r5_cur.so new=nldsc_amd/libnldsc_amd.so" "new=nldsc_amd/libnldsc_amd.so prev=ab_libs/r5_cur.so head=ab_libs/r5_head.so"; do
  k=$((k+1))
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 c3r0of8 --runs 8 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step bench
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 20 --n-org 50000 --additive-only > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
python3 -c "
import json
for w in ('c2','c3'):
  d=json.loads(open('$O/'+w+'.json').read().strip().splitlines()[-1]); print(w, round(d['ms_per_step'],3), d['stages_ms'], d.get('oneshot_gpu_ms',{}).get('load'), d.get('fp32_path',{}).get('frac'), d.get('fp32_path',{}).get('vs_default_path'))"
step done
