#!/bin/bash
# Host-result path of a run, pinned vs ordinary arrays: debug stage lines + a kernel/copy trace of C2
# (gpurun --timeout 600 -- bash tools/ab/gpu_hostpath.sh <tag>)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-hp}; mkdir -p $O
timeout -k 10 300 python tools/hostpath_probe.py > $O/probe.txt 2>&1 || { tail -30 $O/probe.txt; exit 1; }
grep -v "^\[nldsc debug\] super" $O/probe.txt | tail -60
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tr -o t --output-format csv -- python3 tools/hostpath_probe.py --runs 4 > /dev/null 2> $O/tr.err || { tail $O/tr.err; exit 1; }
echo traced
