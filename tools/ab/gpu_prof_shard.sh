#!/bin/bash
# kernel statistics of one rank's shard of the 8-GPU strong-scaling run (bench.py --rehearse R/8)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ps}; mkdir -p $O
for r in 0 3; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$r -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 --rehearse $r/8 > $O/r$r.json 2> $O/r$r.err || { tail $O/r$r.err; exit 1; }
find $O/p$r -name "*kernel_stats.csv" -exec cp {} $O/stats_r$r.csv \;
find $O/p$r -name "*kernel_trace.csv" -exec cp {} $O/trace_r$r.csv \;
done
