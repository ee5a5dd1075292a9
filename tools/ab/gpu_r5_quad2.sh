#!/bin/bash
# Quad super-items in tile order without null padding: the quad / routing GPU tests, C5 A/B against round 4's library
# and the previous round-5 build, then the C3 band kernel's stall buckets (tools/ab/gpu_stall_probe.sh)
# (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_quad2.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5q2}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "c5_shape or routing or issued or 2x2 or quad or round_launches" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step ab c5
timeout -k 10 500 python tools/ab_libs.py --libs new=nldsc_amd/libnldsc_amd.so head=ab_libs/r5_head.so prev=ab_libs/r5_cur.so \
  --workload c5 --c5-snp 600000 --runs 3 > $O/ab_c5.json 2> $O/ab_c5.err || { tail $O/ab_c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab_c5.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items(): print(w, ' '.join('%s %.1f/%.1f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
step stall c3
timeout -k 10 600 bash tools/ab/gpu_stall_probe.sh ${1:-r5q2}/stall "c3:NLDSC_NONE=0:--no-extra" > $O/stall.txt 2>&1 || { tail $O/stall.txt; exit 1; }
tail -c 1500 $O/stall.txt
step done
