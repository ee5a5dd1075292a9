# round 3: column-block pair items (NLDSC_F4_NC2) — bitwise tests, then C2 A/B; the routing / 2x2 / issued tests
# on the new default (quad)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "column_block_pairs or 2x2 or issued or routing or round_launches or device_table" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" $O/tests.log | head -80; exit 1; }
L=nldsc_amd/libnldsc_amd.so
summ() { python3 -c "import json; d=json.load(open('$1'))['ab']; print('$1', {w: {k: (round(v['band_ms_median'],3), round(v['band_ms_min'],3), round(v['total_ms_median'],3)) for k,v in x.items()} for w,x in d.items()})"; }
timeout -k 10 500 python tools/ab_libs.py --libs nc1=$L nc2=$L,NLDSC_F4_NC2=1 --workload c2 --runs 10 > $O/ab_nc2.json 2> $O/ab_nc2.err || { tail $O/ab_nc2.err; exit 1; }
summ $O/ab_nc2.json
