#!/bin/bash
# gpurun --timeout 300 -- bash tools/gpu_r6_host_probe.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-hp}; mkdir -p $O
timeout -k 10 200 python tools/host_overhead_probe.py > $O/host_probe.json 2> $O/host_probe.err || { tail $O/host_probe.err; exit 1; }
cat $O/host_probe.json
