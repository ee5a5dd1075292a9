cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d64; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c2_shape or column_block or additive or deferred or golden or random_small" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python tools/ab_libs.py --libs base=ab_libs/base.so tree=nldsc_amd/libnldsc_amd.so --workload c2 c3 --runs 12 > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read())['ab']
for wl,v in d.items():
    for k,x in v.items(): print(wl, k, round(x['band_ms_median'],4), round(x['total_ms_median'],4), x['max_abs_dl2_vs_first'])"
