#!/bin/bash
# The fused small-slice plan: its schedule tests, then same-box A/B against the previous build (ab_libs/base.so) on a
# 1/8 shard of C3 and C2.   gpurun --timeout 900 -- bash tools/gpu_r6_plan.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-plan}; mkdir -p $O
echo "[$(date +%H:%M:%S)] tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "schedule or sharded or ksplit or round_launches or issued or device_table or halo or heavy_maf" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "[$(date +%H:%M:%S)] ab"
timeout -k 10 400 python tools/ab_libs.py --libs base=ab_libs/base.so new=nldsc_amd/libnldsc_amd.so --workload c3r0of8 c3 --runs 12 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read())['ab']
for wl,v in d.items():
    for k,x in v.items(): print(wl, k, round(x['band_ms_median'],4), round(x['total_ms_median'],4), x['stages_ms_median'])"
for r in 0 3 7; do
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 10 --rehearse $r/8 > $O/rehearse_r${r}of8.json 2> $O/rehearse.err || { tail $O/rehearse.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rehearse_r${r}of8.json').read().strip().splitlines()[-1]); print('rehearse $r/8', round(d['ms_per_step'],4), d['stages_ms'])"
done
echo "[$(date +%H:%M:%S)] done"
