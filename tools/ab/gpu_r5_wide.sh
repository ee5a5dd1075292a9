#!/bin/bash
# The wide copy of the rows (option band4): its bitwise and round-launch GPU tests, then a same-box A/B of the
# single-block fp4 kernels on the wide rows against the 2-bit rows (same library, band4 0) and the previous build,
# C3 / C2 / rank 0 of 8, two orders, and the C3 bench line
# (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_wide.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5w}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "wide or round_launch or full_size or c2_shape or golden" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
L=nldsc_amd/libnldsc_amd.so
k=0
for order in "w4=$L w2=$L,band4=0 prev=ab_libs/r5_q2.so" "prev=ab_libs/r5_q2.so w2=$L,band4=0 w4=$L"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 c3r0of8 --runs 8 > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step bench
timeout -k 10 300 python bench.py --no-cpu --no-file --steps 10 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c3', round(d['ms_per_step'],3), d['stages_ms'], 'frac', round(r['frac'],4), 'pipe', round(r['mfma_pipe_frac'],3), 'oneshot', d.get('oneshot_gpu_ms',{}).get('load'), d.get('oneshot_gpu_ms',{}).get('total'))"
step done
