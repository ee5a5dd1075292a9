"""The oracle against the committed golden vectors, the fp64 restatement and the reference's
documented quirks (CPU only)."""
import os

import numpy as np
import pytest

from conftest import assert_ld_close, golden_sets, load_set
from oracle import oracle as O

SETS = sorted(golden_sets())


@pytest.mark.parametrize("name", SETS)
def test_c_oracle_reproduces_golden(name):
    bed, pos, meta, orc, _ = load_set(name)
    got = O.run_c(bed, meta["n_snp"], meta["n_org"], meta["ld_wind"], meta["maf"], meta["std_thr"],
                  meta["rsq_thr"], pos, threads=1)
    for k in orc:
        np.testing.assert_array_equal(got[k], orc[k], err_msg=f"{name}:{k}")


@pytest.mark.parametrize("name", SETS)
def test_f64_restatement_reproduces_golden(name):
    bed, pos, meta, _, f64 = load_set(name)
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(meta["n_snp"], -1)
    got = O.run_f64(rows, meta["n_org"], meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"], pos)
    for k in f64:
        np.testing.assert_allclose(got[k], f64[k], rtol=1e-12, atol=1e-12, err_msg=f"{name}:{k}")


@pytest.mark.parametrize("name", SETS)
def test_c_oracle_matches_f64_restatement(name):
    """Two independent formulations of the reference's algorithm agree within fp32 noise."""
    _, _, _, orc, f64 = load_set(name)
    assert_ld_close(orc, f64, label=name)


@pytest.mark.parametrize("name", ["n1001", "n1003"])
def test_targets_mode_equals_full_mode(name):
    bed, pos, meta, orc, _ = load_set(name)
    t = np.arange(0, meta["n_snp"], 13, dtype=np.int32)
    got = O.run_c(bed, meta["n_snp"], meta["n_org"], meta["ld_wind"], meta["maf"], meta["std_thr"],
                  meta["rsq_thr"], pos, targets=t, threads=1)
    for k in orc:
        np.testing.assert_array_equal(got[k], orc[k][t], err_msg=k)


def test_unpack_order_reference_vs_plink():
    """stream.h:55-66: high bit pair first; the last byte keeps its high N%4 pairs."""
    row = np.array([[0b11_10_01_00, 0b00_00_10_11]], np.uint8)  # byte 0 codes (PLINK low->high) 0,1,2,3
    ref = O.unpack_codes(row, 7)
    assert ref.tolist() == [[3, 2, 1, 0, 0, 0, 2]]  # reference: high pairs first, then 3 high pairs of byte 1
    strict = O.unpack_codes(row, 7, strict=True)
    assert strict.tolist() == [[0, 1, 2, 3, 3, 2, 0]]  # PLINK order


def test_all_missing_snp_poisons_windows():
    _, _, _, orc, _ = load_set("allmiss")
    j = 50
    assert np.isnan(orc["maf"][j]) and np.isnan(orc["l2"][j])
    in_win = np.flatnonzero(np.isnan(orc["l2"]))
    assert j in in_win and len(in_win) > 100  # every window containing SNP 50
    # L2D is NaN only for the SNP itself (its residual std is NaN, so it is never a dominance neighbour)
    assert np.flatnonzero(np.isnan(orc["l2d"])).tolist() == [j]


def test_all_missing_with_padding_pair_fails_maf():
    _, _, _, orc, _ = load_set("allmiss_pad")
    assert orc["maf"][50] == 0.0 and np.isnan(orc["l2"][50]) and orc["l2_ws"][50] == -1


def test_unused_and_maf_failed_snps():
    _, pos, meta, orc, _ = load_set("n1003")
    for j in (103, 1199):  # position -1
        assert pos[j] < 0 and np.isnan(orc["maf"][j]) and np.isnan(orc["l2"][j]) and orc["l2_ws"][j] == -1
    j = 8  # monomorphic: MAF reported, no scores
    assert orc["maf"][j] == 0.0 and np.isnan(orc["l2"][j]) and np.isnan(orc["residuals_std"][j])
    j = 20  # hom-A1/het only: residual std exactly 0 -> never a dominance neighbour
    assert orc["residuals_std"][j] == 0.0 and orc["l2d_ws"][j] >= 0


def test_window_tie_is_inclusive():
    bed, pos, meta, orc, _ = load_set("n1000")
    a = 200
    b = int(np.flatnonzero(pos == pos[a] + meta["ld_wind"])[0])
    nb = O.replay_windows(pos, np.ones(len(pos), bool), meta["ld_wind"])
    assert nb[0][b] <= a  # a is inside b's window: |pos_b - pos_a| == w counts (tools.h:41-49)


def test_bad_magic_raises_value_error():
    bed, pos, meta, _, _ = load_set("n1001")
    with pytest.raises(ValueError):
        O.run_c(b"\x00" + bed[1:], meta["n_snp"], meta["n_org"], 1.0, 0.01, 1e-5, 0.001, pos)


@pytest.mark.parametrize("name", ["n1003", "allmiss"])
def test_f64_targets_contingency_truth(name):
    bed, pos, meta, _, f64 = load_set(name)
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(meta["n_snp"], -1)
    t = np.arange(0, meta["n_snp"], 29)
    got = O.run_f64_targets(rows, meta["n_org"], meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"],
                            pos, t)
    for k in got:
        np.testing.assert_allclose(got[k], f64[k][t], rtol=1e-12, atol=1e-12, err_msg=k)


def _openblas_arch():
    try:
        from threadpoolctl import threadpool_info
        import scipy.linalg  # noqa: F401  (loads scipy's OpenBLAS)
    except ImportError:
        return None
    for d in threadpool_info():
        if d.get("internal_api") == "openblas" and "scipy" in os.path.basename(d.get("filepath", "")):
            return d.get("architecture"), d.get("version")
    return None


@pytest.mark.skipif(_openblas_arch() is None or _openblas_arch()[0] != "SkylakeX",
                    reason="needs scipy's OpenBLAS with its SkylakeX sdot kernel (this container's CPU)")
def test_dot_matches_openblas_sdot():
    """The oracle's arma::dot -> BLAS sdot (n > 32) is OpenBLAS's own arithmetic: bit-identical to the
    single-threaded sdot of the OpenBLAS that scipy ships (0.3.28, SkylakeX kernel) — the library the
    survey's probe of the reference linked — on lengths around every kernel boundary (32-element tail,
    64-element main step) and at the BASELINE sizes."""
    import ctypes

    from scipy.linalg import blas
    from threadpoolctl import threadpool_limits
    L = O.lib()
    L.oracle_sdot.restype = ctypes.c_float
    fp = ctypes.POINTER(ctypes.c_float)
    rng = np.random.default_rng(9)
    with threadpool_limits(1):
        for n in list(range(33, 140)) + [1000, 4097, 10001, 50_000, 315_599]:
            for kind in range(2):
                x = rng.standard_normal(n).astype(np.float32)
                y = (rng.standard_normal(n) if kind else rng.integers(0, 3, n) - 0.7).astype(np.float32)
                got = L.oracle_sdot(x.ctypes.data_as(fp), y.ctypes.data_as(fp), n)
                assert np.float32(got) == np.float32(blas.sdot(x, y)), n


@pytest.mark.parametrize("n_org", [50_000, 50_001])
def test_rare_variant_residual_noise(n_org):
    """SNPs whose read samples hold het + hom-A2 calls only have an exactly constant residual (truth: std 0),
    but the reference computes it in fp32 and reports rounding noise (oracle: the reference's arithmetic,
    sdot pinned to OpenBLAS).  Recorded: at N % 4 == 0 all 96 of them pass std-thr 1e-5 here (so the
    reference counts them in WSD / L2D); at N % 4 != 0 none exist, because the reference reads a hom-A1
    padding pair in every row.  The engine replays this arithmetic by default (tests/test_gpu_parity.py)."""
    from conftest import rare_variant_set
    rows, pos = rare_variant_set(n_org)
    bed = b"\x6c\x1b\x01" + rows.tobytes()
    M = rows.shape[0]
    orc = O.run_c(bed, M, n_org, 1.0, 1e-5, 1e-5, 1.0 / M, pos, flags=O.NO_COPIES)
    cnt = O.code_counts(bed, M, n_org)
    flagged = (cnt[:, 0] == 0) & (cnt[:, 2] > 0) & (cnt[:, 3] > 0) & ~np.isnan(orc["residuals_std"])
    noisy = flagged & (orc["residuals_std"] > 1e-5)
    record_path = os.path.join(os.path.dirname(__file__), "..", "gpurun_out")
    if os.path.isdir(record_path):
        import json
        json.dump(dict(n_org=n_org, flagged=int(flagged.sum()), noisy=int(noisy.sum()),
                       max_noise=float(orc["residuals_std"][flagged].max(initial=0))),
                  open(os.path.join(record_path, f"rare_noise_{n_org}.json"), "w"))
    if n_org % 4 == 0:
        assert flagged.sum() > 50 and noisy.sum() >= 0.5 * flagged.sum()
    else:
        assert flagged.sum() == 0
    # SNPs with <= 2 genotypes of any other kind: the reference's fp32 residual is exactly 0 as well
    two = ((cnt[:, [0, 2, 3]] > 0).sum(1) <= 2) & ~flagged & ~np.isnan(orc["residuals_std"])
    assert two.sum() > 20 and (orc["residuals_std"][two] == 0).all()


@pytest.mark.parametrize("name", ["n1000", "n1003"])
def test_pair_r2_f64_sums_to_the_truth(name):
    """oracle.pair_r2_f64 (the WSDE tie audit's per-pair exact r2adj) agrees with the fp64 truth it is cut from: its
    pairs sum to L2 - 1 and L2D, count WSA / WSD, and its pairs above rsq_thr count WSDE, on every SNP."""
    bed, pos, meta, _, f64 = load_set(name)
    M, N = meta["n_snp"], meta["n_org"]
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    js = np.arange(M)
    pairs = O.pair_r2_f64(rows, N, meta["ld_wind"], meta["maf"], meta["std_thr"], pos, js, bed=bed)
    for j, p in zip(js, pairs):
        if p is None:
            assert f64["l2_ws"][j] == -1
            continue
        ks, r2a, kds, r2d = p
        assert len(ks) == f64["l2_ws"][j] and len(kds) == f64["l2d_ws"][j]
        assert int((r2d > meta["rsq_thr"]).sum()) == f64["l2d_wse"][j]
        np.testing.assert_allclose(1.0 + r2a.sum(), f64["l2"][j], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(r2d.sum(), f64["l2d"][j], rtol=1e-10, atol=1e-10)


def test_wsde_tie_audit_rules():
    """conftest.wsde_tie_audit: a difference is accepted only on a SNP holding a pair within 1e-6 of rsq_thr, by at most
    1, and the side named exact must equal the exact count there."""
    from conftest import wsde_tie_audit
    thr = 1e-3
    exact_pairs = {0: (None, None, None, np.array([thr + 5e-7, 0.5])),   # a tie: 2 pairs above
                   1: (None, None, None, np.array([thr + 1e-3, 0.5]))}   # no tie
    pairs = lambda js: [exact_pairs[int(j)] for j in js]  # noqa: E731
    rec = wsde_tie_audit(np.array([1, 5]), np.array([2, 5]), pairs, thr, exact="b")
    assert rec["flips"] == 1 and rec["snps"] == [0] and rec["ties_1e6"] == [1]
    with pytest.raises(AssertionError, match="no pair within"):
        wsde_tie_audit(np.array([3, 4]), np.array([3, 5]), pairs, thr)
    with pytest.raises(AssertionError, match="more than 1"):
        wsde_tie_audit(np.array([0, 5]), np.array([2, 5]), pairs, thr)
    with pytest.raises(AssertionError, match="exact WSDE"):
        wsde_tie_audit(np.array([1, 5]), np.array([2, 5]), pairs, thr, exact="a")
    assert wsde_tie_audit(np.array([1, 5]), np.array([1, 5]), pairs, thr)["flips"] == 0
