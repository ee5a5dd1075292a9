cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a; mkdir -p $O
echo "[$(date +%H:%M:%S)] new tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3_full.py tests/test_gpu_parity.py -k "c3_full or pinned or full_size or golden" -m gpu -x -v --timeout 400 --timeout-method thread > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -60 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
echo "[$(date +%H:%M:%S)] bench"
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench failed; tail $O/bench_c3.err; exit 1; }
tail -c 600 $O/bench_c3.json
echo "[$(date +%H:%M:%S)] done"
