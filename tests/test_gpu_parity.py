"""GPU parity: the HIP path (through the C ABI / the pybind11 drop-in) against the oracle.

Tolerances are those of conftest.TOL.  Integer outputs (window sizes) and
MAF are exact; NaN patterns are exact.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO, TOL_F32, assert_ld_close, golden_sets, load_set, max_errors, progress, record, tol_for
from oracle import oracle as O

pytestmark = pytest.mark.gpu
SETS = sorted(golden_sets())


@pytest.fixture(scope="module")
def engine():
    # torch bundles its own libamdhip64.so.7; initialise it before libnldsc_amd.so pulls in ROCm's copy so
    # the process has ONE HIP runtime (the full-size test allocates through torch)
    import torch
    torch.cuda.init()
    from nldsc_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def run_set(engine, name, flags=0, own=None):
    bed, pos, meta, orc, f64 = load_set(name)
    engine.load_bed_bytes(bed, meta["n_snp"], meta["n_org"])
    got = engine.run(meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos, flags=flags, own=own)
    return got, meta, orc, f64, pos, bed


MODES = {"f32": 8, "i8": 4, "f4": 16}  # _lib.FLAG_FP32, _lib.FLAG_EXACT_I8, _lib.FLAG_EXACT_F4
EXACT = ("i8", "f4")  # integer Gram paths: exact up to the fp64 epilogue


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("name", SETS)
def test_golden_sets_vs_oracle_and_f64(engine, name, mode):
    """Default run (rare variants' residuals replayed in the reference's fp32 arithmetic) against the oracle;
    FLAG_EXACT_RARE run against the fp64 truth, tightly."""
    ref, meta, orc, f64, _, bed = run_set(engine, name, flags=MODES[mode])
    got, *_ = run_set(engine, name, flags=MODES[mode] | _lib_flag("FLAG_EXACT_RARE"))
    record(f"golden_{name}_{mode}", dict(vs_oracle=max_errors(ref, orc), vs_f64=max_errors(got, f64)))
    # MAF: the same fp32 formula from integer counts -> bit-exact
    np.testing.assert_array_equal(got["maf"], f64["maf"])
    np.testing.assert_array_equal(ref["maf"], orc["maf"])
    assert_ld_close(got, f64, tol=tol_for(mode), label=f"{name} vs f64")
    assert_ld_close(ref, orc, tol=tol_for(mode), label=f"{name} vs oracle")
    cnt = O.code_counts(bed, meta["n_snp"], meta["n_org"])
    rep = (cnt[:, [0, 2, 3]].min(1) <= 16) & ~np.isnan(orc["residuals_std"])
    assert rep.any()
    np.testing.assert_array_equal(ref["residuals_std"][rep], orc["residuals_std"][rep])
    # tighter against the fp64 restatement: the GPU path differs only by fp32 lookup values and
    # 2048-sample fp32 MFMA chains
    m = ~np.isnan(f64["l2"])
    assert np.max(np.abs(got["l2"][m] - f64["l2"][m]), initial=0) < 5e-5
    m = ~np.isnan(f64["l2d"])
    assert np.max(np.abs(got["l2d"][m] - f64["l2d"][m]), initial=0) < 5e-6
    m = ~np.isnan(f64["residuals_std"])
    np.testing.assert_allclose(got["residuals_std"][m], f64["residuals_std"][m], rtol=1e-12)
    if mode == "i8":  # exact integer Gram + fp64 epilogue: equal to the fp64 restatement to rounding
        for k in ("l2", "l2d"):
            m = ~np.isnan(f64[k])
            assert np.max(np.abs(got[k][m] - f64[k][m]), initial=0) < 1e-9, k
        for k in ("l2_ws", "l2d_ws", "l2d_wse"):
            np.testing.assert_array_equal(got[k], f64[k])


@pytest.mark.parametrize("name", ["n1001", "n1003"])
def test_sharded_runs_assemble_to_full(engine, name):
    full, meta, _, _, pos, _ = run_set(engine, name)
    M = meta["n_snp"]
    cuts = [0, 17, 400, 401, 777, M]
    parts = {k: np.full_like(v, np.nan if v.dtype.kind == "f" else -7) for k, v in full.items()}
    for a, b in zip(cuts[:-1], cuts[1:]):
        engine.run(meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos, own=(a, b), out=parts)
    for k in full:
        if full[k].dtype.kind == "i":
            np.testing.assert_array_equal(parts[k], full[k], err_msg=k)
        else:
            np.testing.assert_allclose(parts[k], full[k], rtol=1e-12, atol=3e-12, err_msg=k)


def test_strict_plink_order(engine):
    from nldsc_amd import _lib
    name = "n1003"
    got, meta, _, _, pos, bed = run_set(engine, name, flags=_lib.FLAG_STRICT_PLINK_ORDER)
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(meta["n_snp"], -1)
    exp = O.run_f64(rows, meta["n_org"], meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos,
                    strict=True)
    assert_ld_close(got, exp, label="strict")
    ref, *_ = run_set(engine, name)
    assert not np.allclose(np.nan_to_num(ref["l2"]), np.nan_to_num(got["l2"]))  # N%4=3: the order matters


def test_additive_only(engine):
    from nldsc_amd import _lib
    full, *_ = run_set(engine, "n1002")
    got, *_ = run_set(engine, "n1002", flags=_lib.FLAG_ADDITIVE_ONLY)
    np.testing.assert_allclose(got["l2"], full["l2"], rtol=1e-12, atol=3e-12)
    np.testing.assert_array_equal(got["l2_ws"], full["l2_ws"])
    assert np.isnan(got["l2d"]).all()
    assert (got["l2d_ws"] == -1).all() and (got["l2d_wse"] == -1).all()


def test_pybind_calculate_on_files():
    from nldsc_amd.ldscore import _ldscore as lds
    for name in ("n1000", "allmiss"):
        _, pos, meta, orc, f64 = load_set(name)
        p = lds.LDScoreParams(os.path.join(GOLDEN, name + ".bed"), n_snp=meta["n_snp"], n_org=meta["n_org"],
                              ld_wind=meta["ld_wind"], maf=meta["maf"], std_thr=meta["std_thr"],
                              rsq_thr=meta["rsq_thr"], positions=pos.tolist())
        r = lds.calculate(p)
        got = {k: np.asarray(getattr(r, k), dtype=orc[k].dtype) for k in orc}
        assert_ld_close(got, orc, label=name)


def test_pybind_errors(tmp_path):
    from nldsc_amd.ldscore import _ldscore as lds
    bad = tmp_path / "bad.bed"
    bad.write_bytes(b"\x6c\x1b\x00" + b"\x00" * 100)
    p = lds.LDScoreParams(str(bad), n_snp=4, n_org=100, ld_wind=1.0, maf=0.01, std_thr=1e-5, rsq_thr=0.01,
                          positions=[0.0, 0.1, 0.2, 0.3])
    with pytest.raises(ValueError, match="Invalid PLINK magic number"):
        lds.calculate(p)
    short = tmp_path / "short.bed"
    short.write_bytes(b"\x6c\x1b\x01" + b"\x00" * 50)  # 4 SNPs x 25 B needed
    p.bedfile = str(short)
    with pytest.raises(RuntimeError, match="too short"):
        lds.calculate(p)


def test_cli_end_to_end(tmp_path):
    out = tmp_path / "n1000.L2"
    cmd = [sys.executable, "-m", "nldsc_amd", "ld", "--bfile", os.path.join(GOLDEN, "n1000"), "--ld-wind-cm", "1",
           "-maf", "0.01", "--std-thr", "1e-5", "--extra", "--write-m", "--out", str(out)]
    subprocess.run(cmd, check=True, cwd=REPO, capture_output=True, timeout=300)
    import pandas as pd
    got = pd.read_csv(out, sep="\t")
    ref = pd.read_csv(os.path.join(GOLDEN, "n1000.ref.L2"), sep="\t")  # reference formatting of the oracle
    assert list(got.columns) == list(ref.columns)
    for c in ("CHR", "SNP", "BP", "WSA", "WSD", "WSDE", "MAF"):
        assert got[c].equals(ref[c]) or np.allclose(got[c], ref[c], equal_nan=True), c
    for c, tol in (("L2", 2e-5), ("L2D", 2e-5), ("RSTD", 2e-5)):
        assert np.allclose(got[c], ref[c], atol=tol, equal_nan=True), c
    mfile = tmp_path / "n1000.M"
    m = pd.read_csv(mfile, sep="\t")
    sc = ref.sort_values(by=["CHR", "BP"]).dropna().drop_duplicates(subset="SNP")
    assert int(m["M"][0]) == len(sc)
    assert int(m["MD"][0]) == int(len(sc) * (sc["WSDE"] / sc["WSA"]).mean())


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("seed", range(12))
def test_random_small_configs_vs_f64(engine, seed, mode):
    """Ragged sizes: N from 3 (tiny K) to 700, M from 1 to 260, windows from a few SNPs to all."""
    from nldsc_amd import synth
    rng = np.random.default_rng(1000 + seed)
    N = int(rng.choice([3, 4, 5, 7, 33, 64, 127, 255, 256, 511, 700]))
    M = int(rng.integers(1, 260))
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=float(rng.uniform(0.5, 20)), seed=seed,
                           missing=float(rng.choice([0.0, 0.01, 0.2])))
    if M > 10:
        spec.negative_pos = [int(rng.integers(0, M))]
    g = synth.genotypes(spec)
    rows = synth.pack_bed_rows(g)
    pos = synth.positions_cm(spec)
    w = float(rng.choice([0.05, 0.5, 1.0, 100.0]))
    maf, std_thr, rsq = float(rng.choice([0.0, 0.01, 0.05])), float(rng.choice([0.0, 1e-5])), 0.5 / max(M, 11)
    engine.load_bed_bytes(synth.bed_bytes(rows), M, N)
    # tiny N % 4 == 0 cohorts often have SNPs without hom-A1 calls: compared with the exact truth, so the
    # exact residual (test_rare_variants_reference_residual covers the reference's fp32 one)
    got = engine.run(w, maf, std_thr, rsq, pos, flags=MODES[mode] | _lib_flag("FLAG_EXACT_RARE"))
    exp = O.run_f64(rows, N, w, maf, std_thr, rsq, pos)
    tol = dict(l2=(1e-4, 1e-5), l2d=(1e-5, 1e-5), residuals_std=(1e-12, 1e-10), maf=(0.0, 0.0))
    if mode in EXACT:
        tol.update(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12))
    assert_ld_close(got, exp, tol=tol, wse_budget=0.02, label=f"seed{seed} N{N} M{M}")


def c3_targets(M):
    """>= 64 SNPs of a full-size slice: both edges of every 32-SNP block in a band of 16 blocks (j mod 32 in
    {0, 1, 30, 31}: first/last rows and columns of the diagonal blocks and of their neighbours), plus the
    chromosome ends, where the windows are one-sided."""
    t = {0, 1, 31, 32, M - 33, M - 2, M - 1}
    for b in range(20, 36):
        t.update(32 * b + k for k in (0, 1, 30, 31))
    return np.array(sorted(x for x in t if 0 <= x < M), np.int32)


C3_RSQ = 1.0 / 80_000  # the headline chromosome's rsq_thr (1/M, M = 80 000): r2adj is dense around it at this N


@pytest.fixture(scope="module")
def c3_slice(engine):
    """N = 315 599 (N % 4 = 3, BASELINE.json configs[2]) on a 2 000-SNP chr1-density slice generated on the
    GPU, with the oracle (fp32, the reference's structure) over the WHOLE slice (~1.1 M pairs), the exact fp64
    truth at c3_targets, and the exact per-pair r2adj of any SNP on demand (the WSDE tie audit)."""
    from nldsc_amd import synth
    N, M = 315_599, 2000
    buf, pos = synth.device_bed(M, N, seed=3, length_cm=7.0)
    bed = buf.cpu().numpy().tobytes()
    args = (1.0, 1e-4, 1e-5, C3_RSQ)
    t = c3_targets(M)
    progress("c3 fixture: oracle, all 2000 SNPs")
    exp = O.run_c(bed, M, N, *args, pos, flags=O.NO_COPIES)
    progress("c3 fixture: fp64 truth")
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    truth = O.run_f64_targets(rows, N, *args, pos, t, bed=bed)
    cache = {}

    def pairs(js):  # exact per-pair r2adj (cached across the modes)
        need = [int(j) for j in js if int(j) not in cache]
        if need:
            for j, p in zip(need, O.pair_r2_f64(rows, N, *args[:3], pos, need, bed=bed)):
                cache[j] = p
        return [cache[int(j)] for j in js]
    progress("c3 fixture: done")
    yield dict(buf=buf, pos=pos, N=N, M=M, args=args, t=t, exp=exp, truth=truth, pairs=pairs)


@pytest.mark.parametrize("mode", sorted(MODES))
def test_full_size_slice_vs_oracle(engine, c3_slice, mode):
    """C3 shape at full N, the whole 2 000-SNP slice against the oracle's full run: WSA / WSD / MAF / NaN pattern
    exact, L2 / L2D / RSTD within conftest.TOL at every SNP, and every WSDE difference audited — a pair of that SNP
    must sit within 1e-6 of rsq_thr in exact arithmetic, and the exact paths must equal the exact count there.  71
    targets (every block edge in a band of 16 blocks, both sides of each diagonal block, the chromosome ends) also
    against the exact fp64 truth; integer outputs reproducible run to run."""
    from conftest import wsde_tie_audit
    d = c3_slice
    buf, pos, N, M, t = d["buf"], d["pos"], d["N"], d["M"], d["t"]
    engine.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    got = engine.run(*d["args"], pos, flags=MODES[mode])
    sub = {k: v[t] for k, v in got.items()}
    exp, truth = d["exp"], d["truth"]
    esub = {k: v[t] for k, v in exp.items()}
    audit = wsde_tie_audit(got["l2d_wse"], exp["l2d_wse"], d["pairs"], C3_RSQ, label=f"{mode} vs oracle",
                           exact="a" if mode in EXACT else None)
    record(f"full_size_{mode}", dict(n_org=N, n_snp=M, rsq_thr=C3_RSQ, targets=t.tolist(),
                                     gpu_vs_oracle_all=max_errors(got, exp), gpu_vs_truth=max_errors(sub, truth),
                                     oracle_vs_truth=max_errors(esub, truth), wsde_vs_oracle=audit))
    assert len(t) >= 64
    assert_ld_close(sub, truth, wse_budget=None, label="N=315599 vs fp64 truth")
    wsde_tie_audit(sub["l2d_wse"], truth["l2d_wse"], lambda js: d["pairs"](t[js]), C3_RSQ,
                   label=f"{mode} vs truth", exact="b")
    if mode in EXACT:
        for k in ("l2", "l2d"):
            assert np.max(np.abs(sub[k] - truth[k])) < 1e-8, k
        for k in ("l2_ws", "l2d_ws", "l2d_wse"):
            np.testing.assert_array_equal(sub[k], truth[k], err_msg=k)
    np.testing.assert_array_equal(got["maf"], exp["maf"])
    assert_ld_close(got, exp, wse_budget=None, label="N=315599 whole slice")
    assert (got["l2_ws"] > 100).all() and np.isfinite(got["l2"]).all()
    # bit-reproducible: per-SNP sums across items are fixed-point integer atomics (order-independent)
    again = engine.run(*d["args"], pos, flags=MODES[mode])
    for k in got:
        np.testing.assert_array_equal(again[k], got[k], err_msg=k)


@pytest.fixture(scope="module")
def c5_slice(engine):
    """C5 shape (BASELINE.json configs[4], imputed genome): N = 315 599, no missing calls (hard calls), bp
    positions at 288 bp per SNP (2.88 Gb / 10 M SNPs, duplicates from integer rounding), --ld-wind-kb 1000:
    ~6 900 neighbours per SNP, so the plan's tiled wide-band item order and the missing-free 3-of-8 fp4
    products run at full N.  12 000 SNPs (3.5 Mb); oracle + fp64 truth at 40 targets (each one's window is
    ~14 000 fp32 dots of 315 599 samples in the oracle)."""
    from nldsc_amd import synth
    N, M = 315_599, 12_000
    buf, pos = synth.device_bed(M, N, seed=21, length_cm=288.0 * M, missing=0.0)
    pos = np.round(pos)
    bed = buf.cpu().numpy().tobytes()
    args = (1.0e6, 1e-4, 1e-5, 1.0 / M)
    t = set()
    for b in range(180, 186):  # mid-chromosome band, full windows: both edges of 6 blocks
        t.update(32 * b + k for k in (0, 1, 30, 31))
    t.update({0, 1, 31, 32})                             # left end: one-sided windows
    t.update({M - 1, M - 2, M - 32, M - 33})             # right end
    for k in range(8):
        t.add(4000 + 331 * k)                            # interior SNPs at various block offsets
    t = np.array(sorted(t), np.int32)
    progress(f"c5 fixture: oracle at {len(t)} targets")
    exp = O.run_c(bed, M, N, *args, pos, targets=t, flags=O.NO_COPIES)
    progress("c5 fixture: fp64 truth")
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    truth = O.run_f64_targets(rows, N, *args, pos, t, bed=bed)
    progress("c5 fixture: done")
    yield dict(buf=buf, pos=pos, N=N, M=M, args=args, t=t, exp=exp, truth=truth)


@pytest.mark.parametrize("mode", ["f4", "i8", "f32"])
def test_c5_shape_1000kb_vs_oracle(engine, c5_slice, mode):
    d = c5_slice
    buf, pos, N, M, t = d["buf"], d["pos"], d["N"], d["M"], d["t"]
    engine.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    got = engine.run(*d["args"], pos, flags=MODES[mode])
    tim = engine.timings()
    sub = {k: v[t] for k, v in got.items()}
    exp, truth = d["exp"], d["truth"]
    record(f"c5_shape_{mode}", dict(n_org=N, n_snp=M, targets=t.tolist(), band_items=tim["band_items"],
                                    mean_window=float(got["l2_ws"].mean()), gpu_vs_oracle=max_errors(sub, exp),
                                    gpu_vs_truth=max_errors(sub, truth), oracle_vs_truth=max_errors(exp, truth)))
    assert len(t) >= 40
    assert got["l2_ws"][M // 2] > 6000  # ~6 900 neighbours mid-chromosome
    assert_ld_close(sub, truth, label="C5 shape vs fp64 truth")
    assert_ld_close(sub, exp, label="C5 shape vs oracle")
    if mode in EXACT:
        for k in ("l2", "l2d"):
            assert np.max(np.abs(sub[k] - truth[k])) < 1e-8, k
        for k in ("l2_ws", "l2d_ws", "l2d_wse"):
            np.testing.assert_array_equal(sub[k], truth[k], err_msg=k)
    assert np.isfinite(got["l2"]).all() and (got["l2_ws"] > 2000).all()
    again = engine.run(*d["args"], pos, flags=MODES[mode])
    for k in got:  # bit-reproducible run to run
        np.testing.assert_array_equal(again[k], got[k], err_msg=k)


@pytest.fixture(scope="module")
def c2_slice(engine):
    """C2 shape (BASELINE.json configs[1]): N = 50 000 (N % 4 = 0), chr1 SNP density (80 000 SNPs over
    280 cM: ~570 neighbours at 1 cM), 1 % missing calls, additive scores only.  3 000 SNPs: the whole
    chromosome slice against the full oracle run, 160 SNPs against the fp64 truth."""
    from nldsc_amd import synth
    N, M = 50_000, 3000
    buf, pos = synth.device_bed(M, N, seed=8, length_cm=280.0 * M / 80_000)
    bed = buf.cpu().numpy().tobytes()
    args = (1.0, 1e-4, 1e-5, 1.0 / M)
    exp = O.run_c(bed, M, N, *args, pos, flags=O.NO_COPIES)
    t = np.unique(np.concatenate([np.arange(0, M, 32), np.arange(31, M, 32)])[::2]).astype(np.int32)
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    truth = O.run_f64_targets(rows, N, *args, pos, t, bed=bed)
    yield dict(buf=buf, pos=pos, N=N, M=M, args=args, t=t, exp=exp, truth=truth)


@pytest.mark.parametrize("mode", ["f4", "i8", "f32"])
def test_c2_shape_additive_only_vs_oracle(engine, c2_slice, mode):
    from nldsc_amd import _lib
    d = c2_slice
    buf, pos, N, M, t = d["buf"], d["pos"], d["N"], d["M"], d["t"]
    engine.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    got = engine.run(*d["args"], pos, flags=MODES[mode] | _lib.FLAG_ADDITIVE_ONLY)
    exp, truth = d["exp"], d["truth"]
    record(f"c2_shape_{mode}", dict(n_org=N, n_snp=M, mean_window=float(got["l2_ws"].mean()),
                                    gpu_vs_oracle=max_errors(got, exp), gpu_vs_truth_targets=max_errors(
                                        {k: v[t] for k, v in got.items()}, truth)))
    assert np.isnan(got["l2d"]).all() and (got["l2d_ws"] == -1).all() and (got["l2d_wse"] == -1).all()
    assert got["l2_ws"].mean() > 450
    add_only = dict(l2=exp["l2"], maf=exp["maf"], residuals_std=exp["residuals_std"], l2_ws=exp["l2_ws"])
    for k in ("l2_ws", "maf"):
        np.testing.assert_array_equal(got[k], add_only[k], err_msg=k)
    tol = {k: v for k, v in __import__("conftest").TOL.items()}
    for k in ("l2", "residuals_std"):
        atol, rtol = tol[k]
        np.testing.assert_allclose(got[k], add_only[k], rtol=rtol, atol=atol, err_msg=f"{k} vs oracle")
    sub = {k: v[t] for k, v in got.items()}
    np.testing.assert_array_equal(sub["l2_ws"], truth["l2_ws"])
    np.testing.assert_allclose(sub["l2"], truth["l2"], rtol=1e-4, atol=1e-3)
    if mode in EXACT:  # exact vectors for the rare variants too (by default they are the reference's fp32 ones)
        ex = engine.run(*d["args"], pos, flags=MODES[mode] | _lib.FLAG_ADDITIVE_ONLY | _lib.FLAG_EXACT_RARE)
        assert np.max(np.abs(ex["l2"][t] - truth["l2"])) < 1e-9


def test_f4_gram_is_bitwise_the_int8_gram(engine):
    """The fp4 path's fp32 accumulators hold the same exact integers as the int8 path's int32 ones
    (N < 2^20), and the fp64 epilogue is the same code: integer outputs, MAF and residual std are
    identical, and L2 / L2D differ only by the order of the fp64 atomic sums (two runs of one path
    differ the same way; one wrong Gram entry would move r2 by ~1e-6) — at N = 315 599 and on ragged
    small cases (tiny K, padding slots, missing calls)."""
    from nldsc_amd import synth
    N, M = 315_599, 1200
    buf, pos = synth.device_bed(M, N, seed=5, length_cm=4.0)
    engine.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    args = (1.0, 1e-4, 1e-5, 1.0 / M, pos)
    a, b = engine.run(*args, flags=MODES["i8"]), engine.run(*args, flags=MODES["f4"])
    assert engine.timings()["path"] == "f4"
    same_gram(a, b, "N=315599")
    rng = np.random.default_rng(77)
    for N in (3, 5, 64, 129, 1001):
        M = int(rng.integers(40, 200))
        spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=3.0, seed=N, missing=0.05)
        rows = synth.pack_bed_rows(synth.genotypes(spec))
        pos = synth.positions_cm(spec)
        engine.load_bed_bytes(synth.bed_bytes(rows), M, N)
        args = (1.0, 0.0, 0.0, 0.01, pos)
        a, b = engine.run(*args, flags=MODES["i8"]), engine.run(*args, flags=MODES["f4"])
        same_gram(a, b, f"N={N}")


@pytest.mark.parametrize("N", [524_292, 1_100_003])
def test_segmented_f4_gram_is_bitwise_the_int8_gram(engine, N):
    """Rows longer than one fp32-exact segment (N > 2^19: 4 096 chunks of 128 samples) run the segmented
    fp4 kernel, which folds its fp32 accumulators into int32 after every segment (ld_kernels.hip
    band_f4_body, SEG > 0).  N = 524 292 has a final segment of 2 chunks; N = 1 100 003 > 2^20 (which used
    to fall back to the int8 path) has three segments.  Same exactness check as above, against the int8
    path, plus the diagonal transpose and missing-call products (1 % missing calls)."""
    from nldsc_amd import synth
    M = 600
    buf, pos = synth.device_bed(M, N, seed=11, length_cm=3.0)
    engine.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    for args in ((1.0, 1e-4, 1e-5, 1.0 / M, pos), (0.4, 0.01, 1e-5, 0.05, pos)):
        a = engine.run(*args, flags=MODES["i8"])
        b = engine.run(*args, flags=MODES["f4"])
        assert engine.timings()["path"] == "f4"
        assert (b["l2_ws"] > 10).all()
        same_gram(a, b, f"N={N}")
        c = engine.run(*args, flags=MODES["f4"] | _lib_flag("FLAG_ADDITIVE_ONLY"))
        np.testing.assert_array_equal(c["l2_ws"], a["l2_ws"])
        np.testing.assert_allclose(c["l2"], a["l2"], rtol=1e-13, atol=3e-12)


def same_gram(a, b, label):
    for k in ("maf", "residuals_std", "l2_ws", "l2d_ws", "l2d_wse"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"{label} {k}")
    for k in ("l2", "l2d"):
        np.testing.assert_array_equal(np.isnan(a[k]), np.isnan(b[k]), err_msg=f"{label} {k}")
        # the per-item partial sums enter the per-SNP totals in 2^-44 fixed point: <= ~40 quanta apart
        np.testing.assert_allclose(a[k], b[k], rtol=1e-13, atol=3e-12, equal_nan=True, err_msg=f"{label} {k}")


@pytest.mark.parametrize("order", ["sorted", "unsorted"])
def test_heavy_maf_failure_both_schedule_paths(engine, order):
    """Sorted positions take the no-sync path (all-pass schedule + device left pointers), unsorted ones
    the sequential host replay; both must match the fp64 truth with a third of the SNPs failing MAF and
    some unused (pos < 0)."""
    from nldsc_amd import synth
    rng = np.random.default_rng(91)
    N, M = 200, 240
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=6.0, seed=91, missing=0.02)
    spec.negative_pos = [int(x) for x in rng.integers(0, M, 6)]
    g = synth.genotypes(spec)
    rows = synth.pack_bed_rows(g)
    pos = synth.positions_cm(spec)
    if order == "unsorted":
        k = rng.permutation(M)[:20]
        pos[k] = pos[k[::-1]]
    engine.load_bed_bytes(synth.bed_bytes(rows), M, N)
    exp = O.run_f64(rows, N, 1.0, 0.2, 1e-5, 0.01, pos)
    assert np.isnan(exp["l2"]).sum() > M // 5  # many SNPs fail MAF 0.2
    for mode in EXACT:
        got = engine.run(1.0, 0.2, 1e-5, 0.01, pos, flags=MODES[mode] | _lib_flag("FLAG_EXACT_RARE"))
        assert_ld_close(got, exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10),
                                           maf=(0.0, 0.0)), label=f"{order} {mode}")


def test_resident_image_survives_alternating_orders(engine):
    """The resident rows are counted in place and each run rewrites their last byte from the saved original
    for its own sample order, so compat / strict / compat runs on one loaded image equal fresh loads."""
    for name in ("n1001", "n1003"):
        bed, pos, meta, orc, f64 = load_set(name)
        args = (meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos)
        engine.load_bed_bytes(bed, meta["n_snp"], meta["n_org"])
        a = engine.run(*args)
        s1 = engine.run(*args, flags=_lib_flag("FLAG_STRICT_PLINK_ORDER"))
        b = engine.run(*args)
        engine.load_bed_bytes(bed, meta["n_snp"], meta["n_org"])
        s2 = engine.run(*args, flags=_lib_flag("FLAG_STRICT_PLINK_ORDER"))
        same_gram(a, b, name)
        same_gram(s1, s2, name + " strict")
        assert not np.array_equal(a["l2_ws"], s1["l2_ws"]) or not np.allclose(a["l2"], s1["l2"], equal_nan=True)


def _lib_flag(name):
    from nldsc_amd import _lib
    return getattr(_lib, name)


def test_halo_loaded_shards_assemble_to_full(engine, tmp_path):
    """Position sharding as the torchrun driver runs it: each rank loads only its halo range of the .bed
    file (nldsc_engine_load_bed_file_range) and computes its owned SNPs; the assembled table equals the
    single-GPU run on the whole file."""
    from nldsc_amd import distributed as D
    from nldsc_amd import synth
    N, M = 1003, 900
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=12.0, seed=44, missing=0.02)
    synth.write_plink(str(tmp_path / "c"), spec)
    pos = synth.positions_cm(spec)
    args = (1.0, 0.01, 1e-5, 1.0 / M)
    engine.load_bed_file(str(tmp_path / "c.bed"), M, N)
    full = engine.run(*args, pos)
    run = D.engine_runner(str(tmp_path / "c.bed"), M, N, *args, pos, device=0)
    got = D.empty_result(M)
    for own in D.shard_ranges(pos, 1.0, 4):
        a, b = D.halo_range(pos, 1.0, own)
        assert b - a < M
        part = run(own)
        for k in got:
            got[k][own[0]:own[1]] = part[k][own[0]:own[1]]
    for k in ("l2_ws", "l2d_ws", "l2d_wse", "maf", "residuals_std"):
        np.testing.assert_array_equal(got[k], full[k], err_msg=k)
    for k in ("l2", "l2d"):
        np.testing.assert_allclose(got[k], full[k], rtol=1e-12, atol=3e-12, equal_nan=True, err_msg=k)


@pytest.mark.parametrize("seed", range(6))
def test_gpu_schedule_matches_host_schedule(engine, seed):
    """Non-negative sorted positions take the GPU schedule (window edges by binary search, the drifting
    right pointer as a prefix max, tile-ordered items by a prefix sum); engine option gpu_plan 0 forces the host
    replay.  Same block pairs, same scores, for whole runs and owned sub-ranges, narrow and wide bands."""
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    rng = np.random.default_rng(500 + seed)
    N = int(rng.choice([64, 301, 1003]))
    M = int(rng.integers(50, 1500))
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=float(rng.uniform(1.0, 40.0)), seed=seed, missing=0.02)
    rows = synth.pack_bed_rows(synth.genotypes(spec))
    pos = synth.positions_cm(spec)
    if seed % 3 == 0:
        pos = np.round(pos, 1)  # duplicate positions and exact window ties
    w = float(rng.choice([0.5, 1.0, 5.0]))
    args = (w, 0.01, 1e-5, 1.0 / M, pos)
    owns = [(0, M), (M // 3, 2 * M // 3), (M - 1, M), (0, 1)]
    # odd seeds additive-only: the GPU plan pairs column blocks (items (I, J, 2))
    flags = MODES["f4"] | _lib_flag("FLAG_EXACT_RARE") | (_lib_flag("FLAG_ADDITIVE_ONLY") if seed % 2 else 0)
    out = {}
    # the GPU schedule in one fused launch (slices <= 32 768 SNPs: every case here), as the kernel chain of long
    # slices (plan_fused 0), and the host replay (gpu_plan 0)
    for g, opts in (("fused", {}), ("chain", {"plan_fused": 0}), ("host", {"gpu_plan": 0})):
        with Engine(0, options=opts) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            out[g] = [(e.run(*args, own=o, flags=flags), e.timings()["band_items"]) for o in owns]
    for g, h in (("fused", "host"), ("chain", "host"), ("fused", "chain")):
        for o, (a, na), (b, nb) in zip(owns, out[g], out[h]):
            # (additive-only: the host plan keeps single block pairs, so only the two GPU plans count alike)
            assert na == nb or (seed % 2 and h == "host"), (g, h, o, na, nb)
            sub = {k: v[o[0]:o[1]] for k, v in a.items()}
            ref = {k: v[o[0]:o[1]] for k, v in b.items()}
            same_gram(sub, ref, f"{g} vs {h} own {o}")
    if seed % 2:
        return
    exp = O.run_f64(rows, N, *args)
    assert_ld_close(out["fused"][0][0], exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12),
                                                       residuals_std=(1e-12, 1e-10), maf=(0.0, 0.0)),
                    label=f"gpu plan seed {seed}")


def _swap_alleles(rows, which):
    """Swap hom-A1 (00) and hom-A2 (11) codes of the SNPs in `which` (as if .bim A1/A2 were exchanged)."""
    rows = rows.copy()
    sub = rows[which].astype(np.uint32)
    t = ~(sub ^ (sub >> 1)) & 0x55
    rows[which] = (sub ^ (t | (t << 1))).astype(np.uint8)
    return rows


@pytest.mark.parametrize("name", ["n1001", "n1003", "allmiss"])
def test_allele_orientation_is_invisible(name):
    """The engine stores every SNP minor-homozygote-as-00 (rows with more 11 than 00 calls are swapped at
    load).  On a file whose alleles are swapped for half of the SNPs (A2 = major, PLINK's usual order), the
    scores equal the fp64 truth of that file, and equal a run that keeps the file coding (engine option orient 0)."""
    import torch
    torch.cuda.init()
    from nldsc_amd.engine import Engine
    bed, pos, meta, _, _ = load_set(name)
    N, M = meta["n_org"], meta["n_snp"]
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    swapped = _swap_alleles(rows, np.arange(0, M, 2))
    args = (meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos)
    exp = O.run_f64(swapped, N, *args)
    out = {}
    for o in ("1", "0"):
        for mode in ("f4", "i8", "f32"):
            with Engine(0, options={"orient": int(o)}) as e:  # swapped rare SNPs may lack hom-A1 calls: exact residuals
                e.load_bed_bytes(b"\x6c\x1b\x01" + swapped.tobytes(), M, N)
                out[o, mode] = e.run(*args, flags=MODES[mode] | _lib_flag("FLAG_EXACT_RARE"))
    exact = dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10), maf=(0.0, 0.0))
    for mode in ("f4", "i8"):
        assert_ld_close(out["1", mode], exp, tol=exact, label=f"{name} oriented {mode}")
        same_gram(out["1", mode], out["0", mode], f"{name} {mode}")
    assert_ld_close(out["1", "f32"], exp, tol=TOL_F32, label=f"{name} oriented f32")


@pytest.mark.parametrize("N", [301, 1003, 4096])
def test_missing_free_blocks_skip_m_products(engine, N):
    """32-SNP blocks without any missing call have an all-zero missing-indicator plane, and the fp4 kernel
    skips every product with it (3 of 8 MFMAs left when both blocks are missing-free, 5 when one is).
    Blocks alternate between no missing calls, 2 % missing and a single missing call; results equal the
    int8 kernel (which always computes all 8 products) and the fp64 truth."""
    from nldsc_amd import synth
    M = 600
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=8.0, seed=N, missing=0.02)
    g = synth.genotypes(spec)
    clean = synth.genotypes(synth.SynthSpec(n_org=N, n_snp=M, length_cm=8.0, seed=N, missing=0.0))
    blk = np.arange(M) // 32
    g[blk % 3 == 0] = clean[blk % 3 == 0]       # missing-free blocks
    one = (blk % 3 == 1) & (np.arange(M) % 32 == 5)
    g[blk % 3 == 1] = clean[blk % 3 == 1]
    g[one, N // 2] = -1                           # blocks with a single missing call
    rows = synth.pack_bed_rows(g)
    pos = synth.positions_cm(spec)
    args = (1.0, 0.01, 1e-5, 1.0 / M, pos)
    engine.load_bed_bytes(synth.bed_bytes(rows), M, N)
    xr = _lib_flag("FLAG_EXACT_RARE")
    f4 = engine.run(*args, flags=MODES["f4"] | xr)
    i8 = engine.run(*args, flags=MODES["i8"] | xr)
    same_gram(f4, i8, f"N={N}")
    exp = O.run_f64(rows, N, *args)
    assert_ld_close(f4, exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10),
                                      maf=(0.0, 0.0)), label=f"missing-free blocks N={N}")


@pytest.mark.parametrize("strict", [False, True])
@pytest.mark.parametrize("t2", ["1", "3"])
def test_routing_reads_this_runs_individual_slots(engine, strict, t2):
    """The routing predicate (blk_miss, from the load-time per-row missing flags of both sample orders) must equal the
    band kernels' own (a missing call among this run's individual slots): a missing-free super-item runs the
    missing-free decode.  N % 4 = 3: a 01 call in the last byte's low pair (PLINK's sample 1000) is an individual for
    the PLINK order only, one in the high pair (padding for PLINK) for the reference's order only; everything else
    is missing-free.  Bitwise the single-block kernel's results and the fp64 truth in both orders."""
    from nldsc_amd import _lib, synth
    from nldsc_amd.engine import Engine
    N, M = 1003, 640
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=6.0, seed=91, missing=0.0)
    rows = synth.pack_bed_rows(synth.genotypes(spec)).copy()
    nb = rows.shape[1]
    rows[5, nb - 1] = (rows[5, nb - 1] & 0xFC) | 0x01     # PLINK sample 1000 missing (low pair)
    rows[200, nb - 1] = (rows[200, nb - 1] & 0x3F) | 0x40  # the padding pair (high) reads 01
    pos = synth.positions_cm(spec)
    flags = MODES["f4"] | _lib_flag("FLAG_EXACT_RARE") | (_lib.FLAG_STRICT_PLINK_ORDER if strict else 0)
    args = (1.0, 0.01, 1e-5, 1.0 / M, pos)

    def fresh():
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            return e.run(*args, flags=flags)
    got = _opt_run("ksplit", 0, lambda: _opt_run("t2", t2, fresh))
    ref = _opt_run("ksplit", 0, lambda: _opt_run("t2", 0, fresh))
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    exp = O.run_f64(rows, N, *args, strict=strict)
    assert_ld_close(got, exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10),
                                       maf=(0.0, 0.0)), label=f"routing strict={strict}")


@pytest.mark.parametrize("t2", ["0", "1", "3"])
@pytest.mark.parametrize("dom", [True, False])
def test_issued_products_counted_per_item(engine, t2, dom):
    """flop_issued (the bench's mfma_pipe_frac) counts what each kernel issues per work item: fp4 single-block items
    1 + cm + rm + rm cm + dom (2 + rm + cm) 32x32 block products over all K, less the transposed ones of diagonal
    blocks; items the routing sends to the 2 x 2 kernel (missing-free super-items) 1 + 2 dom; int8 4 + dom (2 + 2
    !diag); fp32 1 + dom (2 - diag); with the quad kernel (option t2 = 3) every wave of a routed 4 x 4 super-item that
    needs one of its four block pairs issues all four (4 (1 + 2 dom)).  Groups of four blocks alternate between
    missing-free, one missing call and 2 % missing."""
    from nldsc_amd import _lib, synth
    from nldsc_amd.engine import Engine
    N, M = 1003, 800
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=8.0, seed=77, missing=0.02)
    g = synth.genotypes(spec)
    clean = synth.genotypes(synth.SynthSpec(n_org=N, n_snp=M, length_cm=8.0, seed=77, missing=0.0))
    grp = np.arange(M) // 128
    g[grp % 3 != 2] = clean[grp % 3 != 2]
    g[(grp % 3 == 1) & (np.arange(M) % 128 == 5), N // 2] = -1
    rows = synth.pack_bed_rows(g)
    pos = synth.positions_cm(spec)
    nblk = (M + 31) // 32
    miss = np.array([(g[32 * b:32 * b + 32] < 0).any() for b in range(nblk)], int)
    _, _, items = _lib.plan_band(pos, np.ones(M, np.uint8), 1.0, max_nc=1)
    I, J = items[:, 0], items[:, 1]
    rm, cm, nd = miss[I], miss[J], (I != J).astype(int)
    f4 = 1 + cm + rm * nd + rm * cm + (1 + nd + rm + cm * nd if dom else 0)
    mb = lambda b: miss[np.minimum(b, nblk - 1)]  # noqa: E731
    if t2 == "1":  # super-items whose four (clamped) blocks are missing-free run in the 2 x 2 kernel
        routed = ~(mb(I & ~1) | mb((I & ~1) + 1) | mb(J & ~1) | mb((J & ~1) + 1)).astype(bool)
        assert routed.any() and not routed.all()
        f4 = np.where(routed, 1 + (2 if dom else 0), f4)
    if t2 == "3":  # 4 x 4 super-items whose eight blocks are missing-free run in the quad kernel
        free = ~np.any([mb(4 * (I >> 2) + k) | mb(4 * (J >> 2) + k) for k in range(4)], axis=0).astype(bool)
        assert free.any() and not free.all()
        routed = free
        needed = set(zip(I.tolist(), J.tolist()))
        quad = 0
        for I4, J4 in sorted(set(zip((I[routed] >> 2).tolist(), (J[routed] >> 2).tolist()))):
            for w in range(4):
                pairs = [(4 * I4 + 2 * (w >> 1) + a, 4 * J4 + 2 * (w & 1) + b) for a in (0, 1) for b in (0, 1)]
                quad += 4 * (3 if dom else 1) if any(p in needed for p in pairs) else 0
        f4 = np.append(np.where(routed, 0, f4), quad)
    i8 = 4 + (2 + 2 * nd if dom else 0 * nd)
    f32 = 1 + (1 + nd if dom else 0 * nd)
    expect = {"f4": int(f4.sum()), "i8": int(i8.sum()), "f32": int(f32.sum())}
    row_bytes = -(-((N + 3) // 4) // 64) * 64
    flags = _lib_flag("FLAG_EXACT_RARE") | (0 if dom else _lib_flag("FLAG_ADDITIVE_ONLY"))

    def run():
        out = {}
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            for mode in MODES:
                e.run(1.0, 0.01, 1e-5, 1.0 / M, pos, flags=flags | MODES[mode])
                out[mode] = e.timings()["flop_issued"] / (2.0 * 32 * 32 * 4 * row_bytes)
        return out
    got = _opt_run("ksplit", 0, lambda: _opt_run("t2", t2, run))
    assert got == {k: float(v) for k, v in expect.items()}, (got, expect)


def test_device_table_equals_host_run(engine):
    """nldsc_engine_run_device (the multi-GPU gather's source) writes the owned slice of the score table into a
    device [7, width] block — columns past the slice NaN — equal to the host run's arrays, with the same pair
    count; an empty owned range gives an all-NaN block."""
    import torch
    from nldsc_amd.distributed import RESULT_KEYS
    bed, pos, meta, _, _ = load_set("n1003")
    M = meta["n_snp"]
    engine.load_bed_bytes(bed, M, meta["n_org"])
    args = (meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos)
    for own in [(0, M), (17, 400), (M - 1, M), (400, 400)]:
        host = engine.run(*args, own=own)
        th = engine.timings()
        n = own[1] - own[0]
        tab = torch.full((7, n + 9), 123.0, dtype=torch.float64, device="cuda:0")
        engine.run_device(*args, tab, own=own)
        td = engine.timings()
        arr = tab.cpu().numpy()
        for k, key in enumerate(RESULT_KEYS):
            np.testing.assert_array_equal(arr[k, :n], host[key][own[0]:own[1]].astype(np.float64),
                                          err_msg=f"{own} {key}")
        assert np.isnan(arr[:, n:]).all()
        assert td["pairs"] == th["pairs"] and td["flop_issued"] == th["flop_issued"], (td, th)


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("n_org,strict", [(50_000, False), (50_001, True), (50_001, False), (315_599, False)])
def test_rare_variants_reference_residual(engine, mode, n_org, strict):
    """Rare variants (<= 16 calls in a genotype class): by default the engine replays the reference's fp32
    residual (reference_residual_kernel), so their residual std is bit-identical to the oracle's and the
    noise-dominated residuals enter WSD / L2D as in the reference — in particular SNPs with het + hom-A2
    calls only (A1 minor, no hom-minor call: an exactly constant residual the reference reports as noise),
    which exist at N % 4 == 0 or in the strict order (the reference's order at N % 4 != 0 reads a hom-A1
    padding pair in every row).  With FLAG_EXACT_RARE the engine reports the exact residual and equals
    the fp64 truth."""
    from conftest import rare_variant_set
    from nldsc_amd import _lib
    rows, pos = rare_variant_set(n_org)
    M = rows.shape[0]
    bed = b"\x6c\x1b\x01" + rows.tobytes()
    oflags = O.NO_COPIES | (O.STRICT_ORDER if strict else 0)
    args = (1.0, 1e-5, 1e-5, 1.0 / M, pos)
    orc = O.run_c(bed, M, n_org, *args, flags=oflags)
    cnt = O.code_counts(bed, M, n_org, strict=strict)
    passed = ~np.isnan(orc["residuals_std"])
    constant = (cnt[:, 0] == 0) & (cnt[:, 2] > 0) & (cnt[:, 3] > 0) & passed
    replayed = (cnt[:, [0, 2, 3]].min(1) <= 16) & passed
    assert (constant.sum() > 50) == (n_org % 4 == 0 or strict) and replayed.sum() > 90
    base = MODES[mode] | (_lib.FLAG_STRICT_PLINK_ORDER if strict else 0)
    engine.load_bed_bytes(bed, M, n_org)
    got = engine.run(*args, flags=base)
    stats_ms = engine.timings()["stats_ms"]  # includes the replay kernel
    record(f"rare_{n_org}_{'strict' if strict else 'compat'}_{mode}",
           dict(constant_residual=int(constant.sum()), replayed=int(replayed.sum()), stats_ms=stats_ms,
                constant_above_std_thr=int((orc["residuals_std"][constant] > 1e-5).sum()),
                gpu_vs_oracle=max_errors(got, orc)))
    np.testing.assert_array_equal(got["residuals_std"][replayed], orc["residuals_std"][replayed])
    assert_ld_close(got, orc, tol=tol_for(mode), label=f"rare N={n_org} {mode}")
    exact = engine.run(*args, flags=base | _lib.FLAG_EXACT_RARE)
    truth = O.run_f64(rows, n_org, *args, strict=strict)
    assert (exact["residuals_std"][constant] == 0).all()
    tol = dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10), maf=(0.0, 0.0)) \
        if mode in EXACT else TOL_F32
    assert_ld_close(exact, truth, tol=tol, label=f"rare exact N={n_org} {mode}")
    if constant.any():
        assert (got["l2d_ws"] != exact["l2d_ws"]).any()  # the noise residuals are counted by default


@pytest.mark.parametrize("N,M,dom", [(20_001, 1500, True), (20_001, 1500, False), (4096, 700, True)])
def test_ksplit_equals_single_pass(engine, N, M, dom):
    """Launches too small to fill the GPU (a rank's shard) split every item's K loop into P pieces whose exact
    integer Gram tiles are summed by an epilogue kernel: every output is bitwise the single-pass one
    (option ksplit 0), and both equal the fp64 truth.  Additive-only bands pair column blocks by default
    (option f4_nc2), which takes no K-split: those runs here use single-block items (option f4_nc2 0)."""
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=6.0, seed=N + M, missing=0.02)
    rows = synth.pack_bed_rows(synth.genotypes(spec))
    pos = synth.positions_cm(spec)
    flags = MODES["f4"] | _lib_flag("FLAG_EXACT_RARE") | (0 if dom else _lib_flag("FLAG_ADDITIVE_ONLY"))
    args = (1.0, 0.01, 1e-5, 1.0 / M, pos)

    def fresh(split):
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            r = e.run(*args, flags=flags)
            assert (e.timings()["ksplit"] > 1) == split
            return r

    def both():
        return fresh(True), _opt_run("ksplit", 0, lambda: fresh(False))
    got, ref = both() if dom else _opt_run("f4_nc2", 0, both)
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    exp = O.run_f64(rows, N, *args)
    if not dom:
        exp = dict(exp, l2d=np.full(M, np.nan), l2d_ws=np.full(M, -1, np.int32), l2d_wse=np.full(M, -1, np.int32))
    assert_ld_close(got, exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10),
                                       maf=(0.0, 0.0)), label=f"ksplit N={N}")


def missing_free_blocks(rows, n_org):
    """32-SNP blocks without a missing call (code 01) among the individual slots the reference reads — every pair
    of the bytes before the last, the last byte's high n_org % 4 pairs (stream.h:55-66) — as the engine counts them
    at load (row_missing_kernel, free_blocks) to gate the super-item kernels."""
    rows = np.asarray(rows, np.uint8)
    M, nb = rows.shape
    miss = np.stack([((rows >> (2 * k)) & 3) == 1 for k in range(4)], axis=-1)  # [M, nb, pair k = bits 2k+1:2k]
    r = n_org % 4
    keep = [k >= 4 - r for k in range(4)] if r else [True] * 4
    row_miss = miss[:, :nb - 1, :].any(axis=(1, 2)) | miss[:, nb - 1, keep].any(axis=1)
    return int(sum(not row_miss[32 * b:32 * b + 32].any() for b in range((M + 31) // 32)))


def _opt_run(name, value, fn):
    """fn() with engine option `name` = value on every engine it creates (Engine.default_options; C ABI
    nldsc_engine_set_option)."""
    from nldsc_amd.engine import Engine
    had, old = name in Engine.default_options, Engine.default_options.get(name)
    Engine.default_options[name] = int(value)
    try:
        return fn()
    finally:
        if had:
            Engine.default_options[name] = old
        else:
            Engine.default_options.pop(name, None)


@pytest.mark.parametrize("mode", ["f32", "i8", "f4"])
def test_band_mode_option_selects_the_default_path(mode):
    """Engine option band_mode (nldsc_engine_set_option) picks the path a run without a path flag takes: the same
    path and the same results as that path's flag (include/nldsc_ld.h, FLAG_EXACT_F4 / EXACT_I8 / FP32)."""
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 1003, 300
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=3.0, seed=5, missing=0.01)
    rows, pos = synth.pack_bed_rows(synth.genotypes(spec)), synth.positions_cm(spec)
    args = (1.0, 0.01, 1e-5, 1.0 / M, pos)

    def run(flags):
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            return e.run(*args, flags=flags), e.timings()["path"]
    got, path = _opt_run("band_mode", {"f32": 0, "i8": 1, "f4": 2}[mode], lambda: run(0))
    ref, ref_path = run(MODES[mode])
    assert path == ref_path == mode
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


T2_CASES = {
    # (N, M, length cM, window cM, missing, dom, own, rare): odd block counts, narrow and wide bands, missing-free
    # blocks (3 products) beside blocks with missing calls, an owned sub-range, additive only, replayed rare
    # variants (the KC launch)
    "odd_blocks_narrow": (4099, 990, 30.0, 0.3, 0.02, True, None, False),
    "wide_band": (2053, 1500, 4.0, 1.0, 0.01, True, None, False),
    "missing_free": (6000, 1100, 8.0, 1.0, 0.0, True, None, False),
    "additive_only": (4096, 1025, 8.0, 1.0, 0.02, False, None, False),
    "owned_range": (3001, 1400, 10.0, 1.0, 0.02, True, (333, 1001), False),
    "rare_replay": (50_001, 400, None, 1.0, None, True, None, True),
    # missing calls in every third block only: the routed default splits the band between both kernels
    "mixed_blocks": (5003, 1300, 8.0, 1.0, "mixed", True, None, False),
    # ... in every third group of four blocks: the quad kernel's 4 x 4 super-items beside single-block items
    "mixed_groups": (5003, 1700, 8.0, 1.0, "mixed4", True, None, False),
    # missing-free: a block count not a multiple of four (clamped strips), an owned range, additive only
    "missing_free_odd": (4099, 1090, 12.0, 0.5, 0.0, True, None, False),
    "missing_free_owned": (3001, 1400, 10.0, 1.0, 0.0, True, (333, 1001), False),
    "missing_free_additive": (4096, 1025, 8.0, 1.0, 0.0, False, None, False),
    # additive-only with missing calls (T2=3: every super-item in the quad kernel, 4 products per pair): an owned
    # range, odd blocks, replayed rare variants (the KC launch), blocks with and without missing calls
    "additive_owned": (3001, 1400, 10.0, 1.0, 0.02, False, (333, 1001), False),
    "additive_odd_narrow": (4099, 990, 30.0, 0.3, 0.02, False, None, False),
    "additive_rare_replay": (50_001, 400, None, 1.0, None, False, None, True),
    "additive_mixed_groups": (5003, 1700, 8.0, 1.0, "mixed4", False, None, False),
}


@pytest.mark.parametrize("t2", ["2", "1", "3"])
@pytest.mark.parametrize("case", sorted(T2_CASES))
def test_2x2_workgroups_bitwise_single_block(engine, case, t2):
    """The 2 x 2 block-pair workgroups (LDS-shared strips) — for every super-item (option t2 = 2) or for the
    missing-free ones with the rest routed to the single-block kernel (t2 = 1), and the 4 x 4 quad workgroups for the
    missing-free 4 x 4 super-items (t2 = 3, the default) — give bitwise the single-block kernel's results (t2 = 0):
    each wave forms its block pair's partial sums exactly as the
    single-block kernel does; both match the fp64 truth."""
    from conftest import rare_variant_set
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M, length, wind, missing, dom, own, rare = T2_CASES[case]
    if rare:
        rows, pos = rare_variant_set(N)
        M = len(pos)
    else:
        spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=length, seed=N + M,
                               missing=0.0 if isinstance(missing, str) else missing)
        g = synth.genotypes(spec)
        if isinstance(missing, str):  # "mixed": every third block; "mixed4": every third group of four blocks
            rng = np.random.default_rng(M)
            span = 128 if missing == "mixed4" else 32
            for b in range(0, (M + span - 1) // span, 3):
                j = span * b + rng.integers(0, min(span, M - span * b))
                g[j, rng.choice(N, 20, replace=False)] = -1
        rows = synth.pack_bed_rows(g)
        pos = synth.positions_cm(spec)
    # (the fp64-truth comparison needs the exact rare-variant residuals; the rare case keeps the replay: KC launch)
    flags = MODES["f4"] | (0 if dom else _lib_flag("FLAG_ADDITIVE_ONLY")) | (0 if rare else _lib_flag("FLAG_EXACT_RARE"))
    args = (wind, 1e-5, 1e-5, 1.0 / M, pos)

    def fresh(kernel):  # (engine options apply to the engines made here); small enough launches for the K-split
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            r = e.run(*args, flags=flags, own=own)
            # with routing (t2 1, 3) a run takes the super-item kernels only when one of its 32-SNP blocks is
            # missing-free (the engine's free_blocks gate), else it is the single-block run (the gate
            # checked against the data, not inferred from the case name)
            got_kernel = e.timings()["band_kernel"]
            want = kernel if t2 == "2" or free > 0 else "f4"
            assert got_kernel == want, (got_kernel, want, free)
            return r
    free = missing_free_blocks(rows, N)
    got = _opt_run("ksplit", 0, lambda: _opt_run("t2", t2, lambda: fresh(
        {"2": "f4_2x2", "1": "f4_routed", "3": "f4_quad"}[t2])))
    ref = _opt_run("ksplit", 0, lambda: _opt_run("t2", 0, lambda: fresh("f4")))
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{case} {k}")
    if rare:
        return  # the replayed residuals are the reference's fp32 ones, not the fp64 truth
    exp = O.run_f64(rows, N, *args)
    if own is not None:
        lo, hi = own
        exp = {k: v[lo:hi] for k, v in exp.items()}
        got = {k: v[lo:hi] for k, v in got.items()}
    if not dom:
        n = len(next(iter(exp.values())))
        exp = dict(exp, l2d=np.full(n, np.nan), l2d_ws=np.full(n, -1, np.int32), l2d_wse=np.full(n, -1, np.int32))
    assert_ld_close(got, exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10),
                                       maf=(0.0, 0.0)), label=f"2x2 {case} T2={t2}")


NC2_CASES = {
    # additive-only: (T2_CASES key, option t2); pairs with one column block routed to a super-item kernel, diagonal
    # pairs, odd last items of a row, owned ranges, the KC launch of replayed rare variants
    "additive_single": ("additive_only", "0"),
    "additive_routed": ("additive_only", "1"),
    "mixed_blocks_routed": ("mixed_blocks", "1"),
    "mixed_groups_quad": ("mixed_groups", "3"),
    "missing_free_quad": ("missing_free_additive", "3"),
    "owned_range": ("owned_range", "1"),
    "odd_blocks_narrow": ("odd_blocks_narrow", "0"),
    "rare_replay": ("rare_replay", "1"),
}


@pytest.mark.parametrize("case", sorted(NC2_CASES))
def test_f4_column_block_pairs_bitwise_single_blocks(engine, case):
    """Additive-only fp4 items of two column blocks (option f4_nc2 1: 32 x 64 tiles, the row strip decoded once for
    both; a block the super-item routing takes is dropped from its item) give bitwise the single-block items' results
    and the same issued-product count."""
    from conftest import rare_variant_set
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    key, t2 = NC2_CASES[case]
    N, M, length, wind, missing, _, own, rare = T2_CASES[key]
    if rare:
        rows, pos = rare_variant_set(N)
        M = len(pos)
    else:
        spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=length, seed=N + M,
                               missing=0.0 if isinstance(missing, str) else missing)
        g = synth.genotypes(spec)
        if isinstance(missing, str):
            rng = np.random.default_rng(M)
            span = 128 if missing == "mixed4" else 32
            for b in range(0, (M + span - 1) // span, 3):
                j = span * b + rng.integers(0, min(span, M - span * b))
                g[j, rng.choice(N, 20, replace=False)] = -1
        rows = synth.pack_bed_rows(g)
        pos = synth.positions_cm(spec)
    flags = MODES["f4"] | _lib_flag("FLAG_ADDITIVE_ONLY") | (0 if rare else _lib_flag("FLAG_EXACT_RARE"))
    args = (wind, 1e-5, 1e-5, 1.0 / M, pos)

    def fresh():
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            r = e.run(*args, flags=flags, own=own)
            return r, e.timings()
    # (the quad kernel keeps only the missing-free super-items, so the pairs run here)
    run = lambda nc2: _opt_run("ksplit", 0, lambda: _opt_run("t2", t2, lambda: _opt_run("f4_nc2", nc2, fresh)))  # noqa
    (got, tg), (ref, tr) = run("1"), run("0")
    assert tg["band_items"] < tr["band_items"], (tg["band_items"], tr["band_items"])  # the plan paired them
    assert tg["flop_issued"] == tr["flop_issued"], (tg["flop_issued"], tr["flop_issued"])
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{case} {k}")


ROUND_CASES = {
    # (N, M, length cM, dom, tail K-split required): ~9 400-9 700 items in 2 048-item rounds; the cost model K-splits
    # the partial last round at both lengths (N = 131 101: 1 025 K chunks; N = 315 599: C3 rows)
    "n131k_dom": (131_101, 12_000, 15.0, True, False),
    "n131k_add": (131_101, 12_000, 15.0, False, False),
    "n315k_dom_tail": (315_599, 12_000, 15.0, True, True),
}


@pytest.mark.parametrize("case", sorted(ROUND_CASES))
def test_band_round_launches_bitwise_one_launch(engine, case):
    """The single-block fp4 band in launches of one round of the wave slots each (the default for long rows,
    N >= 2^17, when the band has at least one round of items), with the partial last round K-split when the cost
    model prefers it, gives bitwise the results of one launch of all items (option band_rounds 0): the per-SNP sums
    are order-independent fixed point, the K-split partial Gram tiles are exact integers, and every item runs once.
    12 000 SNPs at 800 per cM, 1 % missing; a few SNPs against the exact truth.  The additive-only case runs
    single-block items (f4_nc2 0)."""
    if not ROUND_CASES[case][3]:
        return _opt_run("f4_nc2", 0, lambda: _round_launch_case(case))
    return _round_launch_case(case)


def _round_launch_case(case):
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M, length, dom, tail = ROUND_CASES[case]
    buf, pos = synth.device_bed(M, N, seed=31, length_cm=length, missing=0.01)
    flags = MODES["f4"] | _lib_flag("FLAG_EXACT_RARE") | (0 if dom else _lib_flag("FLAG_ADDITIVE_ONLY"))
    args = (1.0, 1e-4, 1e-5, 1.0 / M, pos)

    def fresh(rounds):
        with Engine(0) as e:
            e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
            r = e.run(*args, flags=flags)
            t = e.timings()
            assert (t["band_round_items"] > 0) == rounds, t
            if rounds:
                assert t["band_items"] >= t["band_round_items"], t
                assert t["band_tail_ksplit"] > 1 or not tail, t
            return r
    got = fresh(True)
    ref = _opt_run("band_rounds", 0, lambda: fresh(False))
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert (got["l2_ws"] > 100).all() and np.isfinite(got["l2"]).all()
    targets = np.array([0, 31, 32, 4095, 4096, 6000, M - 33, M - 1], np.int32)
    bed = buf.cpu().numpy().tobytes()
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    exp = O.run_f64_targets(rows, N, *args, targets, bed=bed)
    sub = {k: v[targets] for k, v in got.items()}
    if not dom:
        exp = dict(exp, l2d=np.full(len(targets), np.nan), l2d_ws=np.full(len(targets), -1, np.int32),
                   l2d_wse=np.full(len(targets), -1, np.int32))
    assert_ld_close(sub, exp, tol=dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12), residuals_std=(1e-12, 1e-10),
                                       maf=(0.0, 0.0)), label=f"rounds {case}")


def test_round_launches_with_replayed_rare_variants_in_the_tail(engine):
    """The default CLI path in full: rare variants replayed in the reference's fp32 arithmetic (no
    FLAG_EXACT_RARE), the band in round launches, and the partial last round K-split — where the KC epilogue of
    the tail reads the partial Gram tiles the main launch wrote.  Rare SNPs (<= 16 calls in a genotype class) sit in
    the last row blocks (whose items end the tile-ordered plan: the K-split tail) and mid-chromosome.  Bitwise equal
    to one launch (option band_rounds 0) and to the KC launch of the deferred rare-variant items (defer_rep 0); the
    replayed SNPs' residual std equals the oracle's bit for bit and their scores
    pass the bar against it."""
    import torch
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 315_599, 12_000
    buf, pos = synth.device_bed(M, N, seed=33, length_cm=15.0, missing=0.01)
    nb = (N + 3) // 4
    img = buf.cpu().numpy().copy()
    del buf
    rows = img[3:].reshape(M, nb)
    rng = np.random.default_rng(7)
    rare = np.array(sorted({M - 1, M - 5, M - 40, M - 70, M - 130, 6001, 6002, 300}), np.int64)
    for j in rare:  # 100 het, 8 hom-A2 calls, 1 % missing: MAF 1.8e-4 passes 1e-4; 8 calls in a class: replayed
        g = np.zeros(N, np.int8)
        pick = rng.choice(N, 108, replace=False)
        g[pick[:100]], g[pick[100:]] = 1, 2
        g[rng.random(N) < 0.01] = -1
        rows[j] = synth.pack_bed_rows(g[None])[0]
    dev = torch.from_numpy(img).to("cuda:0")
    flags = MODES["f4"]
    args = (1.0, 1e-4, 1e-5, 1.0 / M, pos)

    def fresh(rounds):
        with Engine(0) as e:
            e.load_bed_device(dev.data_ptr(), dev.numel(), M, N)
            r = e.run(*args, flags=flags)
            t = e.timings()
            assert (t["band_round_items"] > 0) == rounds, t
            if rounds:
                assert t["band_tail_ksplit"] > 1, t
            return r
    got = fresh(True)
    for var, value, rounds in (("band_rounds", 0, False), ("defer_rep", 0, True)):
        ref = _opt_run(var, value, lambda: fresh(rounds))
        for k in got:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{var}={value} {k}")
    bed = img.tobytes()
    t = np.array(sorted(set(rare.tolist()) | {M - 2, M - 33, 6000, 5990}), np.int32)
    exp = O.run_c(bed, M, N, *args, targets=t, flags=O.NO_COPIES)
    sub = {k: v[t] for k, v in got.items()}
    is_rare = np.isin(t, rare)
    assert np.isfinite(exp["residuals_std"][is_rare]).all()
    np.testing.assert_array_equal(sub["residuals_std"][is_rare], exp["residuals_std"][is_rare])
    assert_ld_close(sub, exp, label="rounds + replayed rare tail vs oracle")


def test_quad_round_launches_bitwise_one_launch(engine):
    """Missing-free bands of many 4 x 4 super-items (a C5-shaped slice: 1000 kb windows, 288 bp per SNP) run the quad
    kernel in launches of one workgroup per CU (option q_rounds, from 16 such rounds): bitwise the one-launch results
    (option q_rounds 0) — the per-SNP sums are order-independent fixed point."""
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 2053, 150_000
    buf, pos = synth.device_bed(M, N, seed=5, length_cm=288.0 * M, missing=0.0)
    args = (1.0e6, 1e-4, 1e-5, 1.0 / M, pos)

    def fresh():
        with Engine(0) as e:
            e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
            r = e.run(*args)
            assert e.timings()["band_kernel"] == "f4_quad"
            return r
    got = fresh()
    ref = _opt_run("q_rounds", 0, fresh)
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert (got["l2_ws"] > 3000).all()  # (a half window at the chromosome ends)


@pytest.mark.parametrize("dom", [False, True])
def test_deferred_rare_variant_items_bitwise_kc_launch(engine, dom):
    """Items holding a replayed rare variant run their K loops in the main single-block launch and their epilogues
    after the replay from stored Gram tiles (option defer_rep, the default): bitwise the separate KC launch
    (option defer_rep 0).  Additive-only: a rare variant only in the second column block of a column-block pair item
    (block 1 of item (0, 0, 2)) — that pair must take the ka terms too — and equal to single-block items
    (option f4_nc2 0)."""
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 50_000, 320
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=2.0, seed=91, missing=0.01)
    g = synth.genotypes(spec)
    rng = np.random.default_rng(3)
    for j in (40, 41, 200):  # rare: 100 het, 8 hom-A2 calls (<= 16 in a class: replayed), 1 % missing
        r = np.zeros(N, np.int8)
        r[rng.choice(N, 108, replace=False)[:100]] = 1
        r[rng.choice(np.flatnonzero(r == 0), 8, replace=False)] = 2
        r[rng.random(N) < 0.01] = -1
        g[j] = r
    rows = synth.pack_bed_rows(g)
    pos = synth.positions_cm(spec)
    flags = MODES["f4"] | (0 if dom else _lib_flag("FLAG_ADDITIVE_ONLY"))
    args = (1.0, 1e-4, 1e-5, 1.0 / M, pos)

    def fresh():
        with Engine(0) as e:
            e.load_bed_bytes(synth.bed_bytes(rows), M, N)
            return e.run(*args, flags=flags)
    ksplit_off = lambda fn: _opt_run("ksplit", 0, fn)  # noqa: E731  (small launch: no whole-band K-split)
    got = ksplit_off(fresh)
    refs = {"kc_launch": ksplit_off(lambda: _opt_run("defer_rep", 0, fresh))}
    if not dom:
        refs["single_blocks"] = ksplit_off(lambda: _opt_run("f4_nc2", 0, fresh))
    for name, ref in refs.items():
        for k in got:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{name} {k}")
    exp = O.run_c(synth.bed_bytes(rows), M, N, *args)
    if not dom:
        exp = dict(exp, l2d=np.full(M, np.nan), l2d_ws=np.full(M, -1, np.int32), l2d_wse=np.full(M, -1, np.int32))
    assert_ld_close(got, exp, label=f"deferred rare dom={dom}")


def test_deferred_rare_items_capped_on_wide_bands_with_missing_calls(engine):
    """A wide band (1000 kb windows at 288 bp per SNP: ~3 500 neighbours) of data with missing calls keeps nearly every
    item in the single-block kernel; the deferred rare-variant Gram tiles would need 32 KiB per item (~140
    GB at the C5 slice with 1 % missing).  Past 2^16 items the engine runs the rare-variant items in the KC launch
    instead: bitwise the KC launch (option defer_rep 0), and the exact integer outputs of a few SNPs equal the oracle's."""
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 2053, 90_000
    buf, pos = synth.device_bed(M, N, seed=41, length_cm=288.0 * M, missing=0.01)
    args = (1.0e6, 1e-4, 1e-5, 1.0 / M, pos)

    def fresh():
        with Engine(0) as e:
            e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
            r = e.run(*args)
            t = e.timings()
            assert t["band_items"] > (1 << 16) and t["band_kernel"] in ("f4", "f4_quad"), t
            return r
    got = fresh()
    ref = _opt_run("defer_rep", 0, fresh)
    for k in got:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    t = np.array([0, 31, 32, 45_000, M - 1], np.int32)
    bed = buf.cpu().numpy().tobytes()
    exp = O.run_c(bed, M, N, *args, targets=t, flags=O.NO_COPIES)
    sub = {k: v[t] for k, v in got.items()}
    assert_ld_close(sub, exp, label="wide band, missing calls, replayed rare variants vs oracle")
