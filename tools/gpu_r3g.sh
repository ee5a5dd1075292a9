# round 3: default-kernel choice (NLDSC_T2=1 vs 3) and the parity-grouped decode variant, same-box interleaved A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3g; mkdir -p $O
L=nldsc_amd/libnldsc_amd.so
summ() { python3 -c "import json; d=json.load(open('$1'))['ab']; print('$1', {w: {k: (round(v['band_ms_median'],3), round(v['band_ms_min'],3), round(v['total_ms_median'],3)) for k,v in x.items()} for w,x in d.items()})"; }
timeout -k 10 500 python tools/ab_libs.py --libs t2=$L,NLDSC_T2=1 quad=$L,NLDSC_T2=3 --workload c3 c2 c3m0 c5 --runs 6 > $O/ab_t2_quad.json 2> $O/ab_t2_quad.err || { tail $O/ab_t2_quad.err; exit 1; }
summ $O/ab_t2_quad.json
timeout -k 10 500 python tools/ab_libs.py --libs base=$L parity=ab_libs/parity.so --workload c3 c2 --runs 8 > $O/ab_parity.json 2> $O/ab_parity.err || { tail $O/ab_parity.err; exit 1; }
summ $O/ab_parity.json
# two band streams, one engine per process (the A/B harness's several engines alias HW queues)
for k in 1 2 3; do for s in 1 2; do
  NLDSC_BAND_STREAMS=$s timeout -k 10 200 python tools/run_lib.py --runs 12 > $O/streams_${s}_$k.log 2>&1 || { tail $O/streams_${s}_$k.log; exit 1; }
done; done
python3 - <<'PY'
import glob, re, statistics as st
for s in (1, 2):
    v = [float(re.search(r"band ([\d.]+)", l).group(1)) for f in sorted(glob.glob(f"gpurun_out/r3g/streams_{s}_*.log"))
         for l in open(f).read().splitlines()[2:] if l.startswith("band")]
    print("band_streams", s, "median", round(st.median(v), 3), "min", round(min(v), 3), "n", len(v))
PY
timeout -k 10 500 python tools/ab_libs.py --libs new=$L old=ab_libs/r2base.so --workload c2 c3m0 --runs 8 > $O/ab_new_old_c2.json 2> $O/ab_new_old_c2.err || { tail $O/ab_new_old_c2.err; exit 1; }
summ $O/ab_new_old_c2.json
