#!/bin/bash
# Where a run's wall time goes outside the band: the debug_timing engine option's stage lines and a kernel-trace timeline of the C2
# and C3 benches (gpurun --timeout 600 -- bash tools/gpu_timeline.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tl}; mkdir -p $O
for w in c2 c3; do
  A=""; [ $w = c2 ] && A="--n-org 50000 --additive-only"
  timeout -k 10 200 python bench.py --no-cpu --no-file --steps 5 --option debug_timing=1 $A > $O/${w}_dbg.json 2> $O/${w}_dbg.err || { tail $O/${w}_dbg.err; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/${w}_tr -o t --output-format csv -- python3 bench.py --no-cpu --no-file --steps 3 $A > /dev/null 2> $O/${w}_tr.err || { tail $O/${w}_tr.err; exit 1; }
done
grep "nldsc debug" $O/c2_dbg.err | tail -3; grep "nldsc debug" $O/c3_dbg.err | tail -3
