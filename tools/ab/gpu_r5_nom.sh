#!/bin/bash
# Study: does the 8-product loop's decode VALU count hold the C3 band?  The working-tree library against a build whose
# decode leaves the m plane zero (7 VALU per code word instead of 9; wrong results, --no-check), two orders; then the
# C5 slice's HBM traffic for the quad kernel's tile order (FETCH_SIZE pass)
# (gpurun --timeout 900 -- bash tools/ab/gpu_r5_nom.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5nom}; mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
k=0
for order in "cur=ab_libs/r5_q2.so nom=ab_libs/r5_nom.so" "nom=ab_libs/r5_nom.so cur=ab_libs/r5_q2.so"; do
  k=$((k+1)); step ab $k
  timeout -k 10 300 python tools/ab_libs.py --libs $order --workload c3 c2 --runs 8 --no-check > $O/ab$k.json 2> $O/ab$k.err || { tail $O/ab$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab$k.json').read().strip().splitlines()[-1])['ab']
for w,v in d.items():
  print('order $k', w, ' '.join('%s %.3f/%.3f' % (n, x['total_ms_median'], x['band_ms_median']) for n, x in v.items()))"
done
step pmc c5 fetch
B="python3 bench.py --no-cpu --no-file --no-extra --steps 1 --warmup 0 --workload c5"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/c5fetch -o f --output-format csv -- $B > /dev/null 2> $O/c5fetch.err || { tail $O/c5fetch.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/c5fetch/**/*counter_collection.csv', recursive=True)[0]
tot = 0; n = set()
for r in csv.DictReader(open(f)):
    if 'band_f4_q_kernel<true, 4, false>' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE':
        tot += float(r['Counter_Value']); n.add(r['Dispatch_Id'])
print('c5 quad fetch per run (x2 corrected): %.3f TB over %d launches' % (tot * 1024 * 2 / 1e12, len(n)))
PY
step done
