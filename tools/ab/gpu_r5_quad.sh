#!/bin/bash
# Quad super-items in groups of 32 per XCD slot: the quad / routing GPU tests, C5 A/B against round 4's library and the
# previous round-5 build (ungrouped), and the C5 slice's HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
# (gpurun --timeout 1200 -- bash tools/ab/gpu_r5_quad.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5q}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "c5_shape or routing or issued or 2x2 or quad or round_launches" > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step ab c5
timeout -k 10 500 python tools/ab_libs.py --libs head=ab_libs/r5_head.so prev=ab_libs/r5_cur.so new=nldsc_amd/libnldsc_amd.so \
  --workload c5 --c5-snp 600000 --runs 3 > $O/ab_c5.json 2> $O/ab_c5.err || { tail $O/ab_c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab_c5.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items(): print(w, ' '.join('%s %.1f/%.1f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
step pmc c5
B="python3 bench.py --no-cpu --no-file --no-extra --steps 1 --warmup 0 --workload c5"
P=$O/pmc_c5
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o f --output-format csv -- $B > /dev/null 2> $P.f.err && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o w --output-format csv -- $B > /dev/null 2> $P.w.err && \
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace -d $P/sq -o s --output-format csv -- $B > /dev/null 2> $P.s.err \
  || { echo "pmc failed"; tail $P.*.err; exit 1; }
python3 tools/pmc_summary.py $P --workload "C5 slice bench: N=315599 M=1250000 missing=0 add+dom 1000 kb" --alg-bytes band_f4_q_kernel=98640000000 > $O/pmc_c5.json
python3 -c "
import json; d=json.load(open('$O/pmc_c5.json'))
k=d.get('kernels',d)
for n,v in k.items():
  if 'q_kernel' in n: print(n, {a:b for a,b in v.items() if not isinstance(b,(list,dict))})"
step done
