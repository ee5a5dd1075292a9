#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace) of short runs: a 1/8 shard of C3 (one rank of the 8-GPU run) and C2, to
# see where a run's time goes between and around the band launches.  gpurun --timeout 600 -- bash tools/gpu_r6_traces.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tr}; mkdir -p $O
for w in shard c2; do
  A="--rehearse 0/8"; [ $w = c2 ] && A="--n-org 50000 --additive-only"
  echo "[$(date +%H:%M:%S)] $w"
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${w}_tr -o t --output-format csv -- python3 bench.py --no-cpu --no-file --no-extra --steps 5 $A > $O/${w}.json 2> $O/${w}.err || { tail $O/${w}.err; exit 1; }
done
echo "[$(date +%H:%M:%S)] done"
