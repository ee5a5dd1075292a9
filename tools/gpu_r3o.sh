#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3o; mkdir -p $O
timeout -k 10 600 python tools/c5_rows_probe.py 1250000 > $O/c5_rows.log 2> $O/c5_rows.err || { tail -20 $O/c5_rows.err; cat $O/c5_rows.log; exit 1; }
cat $O/c5_rows.log
