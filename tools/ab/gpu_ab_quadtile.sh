#!/bin/bash
# quad super-items in 4 x 8 (I, J) tiles vs the 16 x 16 (I, d) tiles: the quad tests, then a same-process A/B on the
# C5 shape (ab_libs/r4_pre_qtile.so built from the previous commit) and the C5-slice bench with its PMC traffic pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-qtile}
mkdir -p $O
step() { echo "[$(date +%H:%M:%S)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "2x2_workgroups or quad or column_block_pairs or c5_shape or issued" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
step ab
timeout -k 10 500 python tools/ab_libs.py --libs new=nldsc_amd/libnldsc_amd.so old=ab_libs/r4_pre_qtile.so --workload c5 --c5-snp 400000 --runs 6 > $O/ab_c5.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
tail -c 1200 $O/ab_c5.json
step bench c5
timeout -k 10 400 python bench.py --no-cpu --no-file --steps 2 --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
tail -c 400 $O/bench_c5.json
B="python3 bench.py --no-cpu --no-file --steps 1 --warmup 0 --workload c5"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc/fetch -o f --output-format csv -- $B > /dev/null 2> $O/pmc_f.err || { tail $O/pmc_f.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/pmc/l2 -o l --output-format csv -- $B > /dev/null 2> $O/pmc_l.err || { tail $O/pmc_l.err; exit 1; }
step done
