#!/bin/bash
# C5 slice (imputed: no missing calls) and C3 with 0% missing vs the default 1%, current engine
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 400 python3 bench.py --workload c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 200 python3 bench.py --no-cpu --missing 0 > $O/bench_c3_nomiss.json 2> $O/bench_c3_nomiss.err || { echo c3 nomiss failed; tail $O/bench_c3_nomiss.err; exit 1; }
cat $O/bench_c3_nomiss.json
