# round 3: targeted GPU tests, the routing host-wait probe, pairwise interleaved A/B on C3 / C5 / C2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "2x2 or issued or device_table or replayed_rare or round_launches or ksplit or gpu_schedule or routing or rare_variants or golden" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
NLDSC_DEBUG_TIMING=1 timeout -k 10 200 python tools/run_lib.py --runs 3 > $O/debug.log 2>&1 || { tail $O/debug.log; exit 1; }
grep "nldsc debug" $O/debug.log | tail -3
L=nldsc_amd/libnldsc_amd.so
for pair in "new=$L old=ab_libs/r2base.so" "new=$L nocompact=$L,NLDSC_COMPACT=0"; do
  tag=$(echo $pair | sed 's/=[^ ]*//g; s/ /_/g')
  timeout -k 10 400 python tools/ab_libs.py --libs $pair --workload c3 --runs 8 > $O/ab_$tag.json 2> $O/ab_$tag.err || { tail $O/ab_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/ab_$tag.json'))['ab']['c3']; print('$tag', {k: (round(v['band_ms_median'],3), round(v['band_ms_min'],3), round(v['total_ms_median'],3)) for k,v in d.items()})"
done
timeout -k 10 400 python tools/ab_libs.py --libs quad=$L,NLDSC_T2=3 quadnc=$L,NLDSC_T2=3,NLDSC_COMPACT=0 --workload c5 c3m0 --runs 4 > $O/ab_quad.json 2> $O/ab_quad.err || { tail $O/ab_quad.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ab_quad.json'))['ab']; print({w: {k: (round(v['band_ms_median'],3), round(v['total_ms_median'],3)) for k,v in x.items()} for w,x in d.items()})"
