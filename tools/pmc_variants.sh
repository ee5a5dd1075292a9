#!/bin/bash
# FETCH_SIZE + GRBM_GUI_ACTIVE (effective clock) of fp4 band-kernel variants, one rocprofv3 pass each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/pmcv
mkdir -p $D
for v in "base=f4:xcd" "grp1=f4:xcd:grp1" "same=ab_libs/same.so:f4:xcd" "r1=f4:xcd:round-1"; do
  n=${v%%=*}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d $D/$n -o p --output-format csv -- \
    python3 tools/band_ab.py --rounds 1 --n-snp 80000 --length-cm 280 --variants "$v" > $D/$n.log 2>&1 || { echo "fail $n"; tail -5 $D/$n.log; exit 1; }
done
python3 - <<'PY'
import glob, csv, collections
for d in sorted(glob.glob('gpurun_out/pmcv/*/')):
    rows = collections.defaultdict(lambda: collections.defaultdict(float)); dur = {}
    for f in glob.glob(d + '**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'band' not in r['Kernel_Name']: continue
            rows[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
            dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    for k in sorted(rows, key=int):
        f = rows[k].get('FETCH_SIZE', 0) * 1024 * 2; g = rows[k].get('GRBM_GUI_ACTIVE', 0)
        print(d.split('/')[-2], k, 'fetch_GB %.2f' % (f / 1e9), 'dur_ms %.3f' % (dur[k] * 1e3), 'clk_GHz %.3f' % (g / 8 / dur[k] / 1e9))
PY
