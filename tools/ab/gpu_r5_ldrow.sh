#!/bin/bash
# Row loader variants (ab_libs/r5_<name>.so): C3 loads from a device image, one engine per process, kernels under
# rocprofv3, the list then its reverse (gpurun --timeout 600 -- bash tools/ab/gpu_r5_ldrow.sh <tag> base ld32 ld64)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5lr}; shift; mkdir -p $O
L="$*"; R=$(echo $L | tr ' ' '\n' | tac | tr '\n' ' ')
pass=0
for l in $L $R; do
  pass=$((pass + 1))
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p$pass$l -o k --output-format csv -- python3 tools/ab/load_probe.py --loads 6 --libs $l=ab_libs/r5_$l.so > $O/s$pass$l.log 2>&1 || { tail $O/s$pass$l.log; exit 1; }
  python3 -c "
import csv
for r in csv.reader(open('$O/p$pass$l/k_kernel_stats.csv')):
    if 'load_tiled' in r[0]: print('$pass $l', 'load_tiled avg', round(float(r[3])/1e3, 1), 'min', round(float(r[5])/1e3, 1), 'us')"
done
