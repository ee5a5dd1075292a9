#!/bin/bash
# round 3: the large-image load fix — its test, then the C5 slice bench and its PMC passes again
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ck; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests_large.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests_large.log; exit 1; }
tail -2 $O/gpu_tests_large.log
timeout -k 10 400 python bench.py --no-cpu --no-file --steps 2 --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
tail -c 400 $O/bench_c5.json
B="python3 bench.py --no-cpu --no-file --steps 1 --warmup 0 --workload c5"
P=$O/pmc_c5
rm -rf $P
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o f --output-format csv -- $B > /dev/null 2> $P.f.err && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o w --output-format csv -- $B > /dev/null 2> $P.w.err && \
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace -d $P/sq -o s --output-format csv -- $B > /dev/null 2> $P.s.err && \
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $P/l2 -o l --output-format csv -- $B > /dev/null 2> $P.l.err && \
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --kernel-trace -d $P/lds -o d --output-format csv -- $B > /dev/null 2> $P.d.err \
  || { echo "pmc c5 failed"; tail $P.*.err; exit 1; }
python3 tools/pmc_summary.py $P --workload "C5 slice bench: N=315599 M=1250000 missing=0 add+dom 1000 kb" --alg-bytes band_f4_q_kernel=98640000000 > $O/pmc_c5.json
echo done
