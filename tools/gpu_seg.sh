cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/seg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "segmented or f4_gram or full_size or missing_free or golden" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 200 python bench.py --no-cpu > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
cat $O/c3.json | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu --n-org 1100003 > $O/big_f4.json 2> $O/big_f4.err || { tail $O/big_f4.err; exit 1; }
cat $O/big_f4.json | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu --path i8 --n-org 1100003 > $O/big_i8.json 2> $O/big_i8.err || { tail $O/big_i8.err; exit 1; }
cat $O/big_i8.json | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu --n-org 1100003 --additive-only > $O/big_f4_add.json 2> $O/big_f4_add.err || { tail $O/big_f4_add.err; exit 1; }
cat $O/big_f4_add.json | cut -c1-300
