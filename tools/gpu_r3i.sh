# round 3: C2 single-engine timing, NLDSC_F4_NC2=0 vs 1, alternating processes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3i; mkdir -p $O
for k in 1 2 3; do for s in 0 1; do
  NLDSC_F4_NC2=$s timeout -k 10 200 python tools/run_lib.py --runs 12 --n-org 50000 --additive-only > $O/nc2_${s}_$k.log 2>&1 || { tail $O/nc2_${s}_$k.log; exit 1; }
done; done
python3 - <<'PY'
import glob, re, statistics as st
for s in (0, 1):
    rows = [l for f in sorted(glob.glob(f"gpurun_out/r3i/nc2_{s}_*.log")) for l in open(f).read().splitlines()[2:] if l.startswith("band")]
    keys = ["band", "total", "count_ms", "stats_ms", "schedule_ms", "finalize_ms"]
    vals = {k: [float(re.search(k + r" ([\d.]+)", l).group(1)) for l in rows] for k in keys}
    print("nc2", s, {k: round(st.median(v), 3) for k, v in vals.items()}, "n", len(rows))
PY
# C3 tail K-split pieces: model (0) vs forced P, alternating processes
for k in 1 2; do for P in 0 1 3 5 7; do
  NLDSC_TAIL_KSPLIT=$P timeout -k 10 200 python tools/run_lib.py --runs 12 > $O/tail_${P}_$k.log 2>&1 || { tail $O/tail_${P}_$k.log; exit 1; }
done; done
python3 - <<'PY'
import glob, re, statistics as st
for P in (0, 1, 3, 5, 7):
    v = [float(re.search(r"band ([\d.]+)", l).group(1)) for f in sorted(glob.glob(f"gpurun_out/r3i/tail_{P}_*.log"))
         for l in open(f).read().splitlines()[2:] if l.startswith("band")]
    print("tail P", P, "band median", round(st.median(v), 3), "min", round(min(v), 3), "n", len(v))
PY
