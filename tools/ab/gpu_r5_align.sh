#!/bin/bash
# The row loader's source alignment: C3 loads from a device image whose rows start 3 mod 16 (a .bed image's rows follow
# its 3-byte header) and from the same image placed 13 bytes in (rows 16-byte aligned), kernels under rocprofv3
# (gpurun --timeout 600 -- bash tools/ab/gpu_r5_align.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5al}; mkdir -p $O
for s in 0 13 1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p$s -o k --output-format csv -- python3 tools/ab/load_probe.py --loads 6 --shift $s > $O/s$s.log 2>&1 || { tail $O/s$s.log; exit 1; }
  tail -2 $O/s$s.log
  f=$(find $O/p$s -name '*kernel_stats.csv' | head -1); grep -E "load_(tiled|orient)" $f | awk -F'","' '{print substr($1,1,30), $2, $3}' | cut -c1-120
done
