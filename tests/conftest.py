import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def golden_sets():
    with open(os.path.join(GOLDEN, "sets.json")) as fh:
        return json.load(fh)


def load_set(name):
    """(bed bytes, positions, meta, oracle result, f64 result) of a committed fixture."""
    import pandas as pd
    meta = golden_sets()[name]
    bed = open(os.path.join(GOLDEN, name + ".bed"), "rb").read()
    bim = pd.read_csv(os.path.join(GOLDEN, name + ".bim"), sep="\t", header=None)
    pos = (bim[2] if meta["metric"] == "cm" else bim[3]).to_numpy(dtype=np.float64)
    orc = dict(np.load(os.path.join(GOLDEN, name + ".oracle.npz")))
    f64 = dict(np.load(os.path.join(GOLDEN, name + ".f64.npz")))
    return bed, pos, meta, orc, f64


# Tolerances: integer window counts exact; MAF exact;
# residual std relative 1e-4 (the reference accumulates means and variances in fp32: measured 4e-5
# relative at N = 315 599, 1.4e-7 at N = 1 000); L2 |d| <= 1e-3 + 1e-4 |L2|; L2D |d| <= 3e-6 + 1e-4 |L2D|
# (round 6: was 1e-5, above a C3 SNP's mean L2D of 2.8e-5; the exact paths measured <= 1.2e-6 from the oracle
# at N = 315 599, 2e-7 at N = 1 000); WSDE +-1 where a pair's exact r2adj lies within 1e-6 of rsq_thr (small
# cases: a budget of 0.1 % of SNPs; full-N cases audit every difference: WSDE_TIE).
TOL = dict(l2=(1e-3, 1e-4), l2d=(3e-6, 1e-4), residuals_std=(0.0, 1e-4), maf=(0.0, 0.0))
# The fp32 MFMA path (FLAG_FP32) at small N: its standardised vectors are rounded to fp32 before the dot products,
# so its L2D is up to 4.3e-6 from the oracle's at N = 1 000 .. 50 001 (itself fp32): the round-5 bar for it.
TOL_F32 = dict(TOL, l2d=(1e-5, 1e-4))
WSDE_TIE = 1e-6  # |r2adj - rsq_thr| of a pair whose side of the threshold may differ between fp32 and exact sums


def tol_for(mode: str) -> dict:
    return TOL_F32 if mode == "f32" else TOL


def max_errors(got: dict, exp: dict) -> dict:
    out = {}
    for k in ("l2", "l2d", "residuals_std"):
        m = ~np.isnan(exp[k]) & ~np.isnan(got[k])
        d = np.abs(got[k][m] - exp[k][m])
        out[k] = dict(max_abs=float(d.max(initial=0)),
                      max_rel=float((d / np.maximum(np.abs(exp[k][m]), 1e-300)).max(initial=0)))
    for k in ("l2_ws", "l2d_ws", "l2d_wse"):
        out[k] = dict(mismatches=int((got[k] != exp[k]).sum()))
    return out


def progress(msg: str) -> None:
    """Append a line to gpurun_out/progress.log (GPU boxes): long fixtures show they are alive."""
    d = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(d):
        import time
        with open(os.path.join(d, "progress.log"), "a") as fh:
            fh.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def record(name: str, payload: dict) -> None:
    """Write measured parity numbers to gpurun_out/ when it exists (GPU box runs)."""
    d = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, f"parity_{name}.json"), "w") as fh:
            json.dump(payload, fh, indent=1)


def assert_ld_close(got: dict, exp: dict, *, tol=TOL, wse_budget=0.001, label="", skip=None):
    skip = np.zeros(len(exp["l2"]), bool) if skip is None else skip
    keep = ~skip
    for k in ("l2_ws", "l2d_ws"):
        bad = np.flatnonzero((got[k] != exp[k]) & keep)
        assert bad.size == 0, f"{label} {k} differs at {bad[:10]}: got {got[k][bad[:10]]} exp {exp[k][bad[:10]]}"
    d = np.abs(got["l2d_wse"].astype(np.int64) - exp["l2d_wse"]) * keep
    # (wse_budget None: the caller audits every difference against the exact per-pair r2adj: wsde_tie_audit)
    assert d.max(initial=0) <= 1 and (wse_budget is None or (d > 0).sum() <= max(1, int(wse_budget * len(d)))), \
        f"{label} l2d_wse differs at {np.flatnonzero(d)[:10]}"
    for k, (atol, rtol) in tol.items():
        g, e = got[k][keep], exp[k][keep]
        nan_g, nan_e = np.isnan(g), np.isnan(e)
        bad = np.flatnonzero(nan_g != nan_e)
        assert bad.size == 0, f"{label} {k} NaN pattern differs at {np.flatnonzero(keep)[bad[:10]]}"
        m = ~nan_e
        err = np.abs(g[m] - e[m])
        lim = atol + rtol * np.abs(e[m])
        bad = np.flatnonzero(err > lim)
        assert bad.size == 0, (f"{label} {k}: {bad.size} out of tolerance, worst |d|={err.max():.3g} "
                               f"at {np.flatnonzero(keep)[np.flatnonzero(m)[bad[:5]]]}")


def wsde_tie_audit(a_wse, b_wse, pairs, rsq_thr, *, label="", exact=None) -> dict:
    """Every SNP j whose WSDE differs between two results (`r2d > rsq_thr` counted per pair, ldscalc.h:41-47) must
    hold at least |a_j - b_j| pairs whose exact r2adj lies within WSDE_TIE of rsq_thr: the two sides rounded a
    tie differently.  `pairs(js)` returns the exact per-pair values (oracle.pair_r2_f64) of those SNPs.  `exact`
    ("a" or "b"): that side must equal the exact count at every audited SNP.  Returns the audit record."""
    a, b = np.asarray(a_wse, np.int64), np.asarray(b_wse, np.int64)
    flips = np.flatnonzero(a != b)
    rec = dict(n=int(a.size), flips=int(flips.size), rate=float(flips.size / max(a.size, 1)), snps=flips.tolist(),
               diff=(a - b)[flips].tolist(), min_gap=[], ties_1e6=[])
    if flips.size == 0:
        return rec
    assert np.abs(a - b).max() <= 1, f"{label}: WSDE differs by more than 1 at {flips[:10]}"
    for j, p in zip(flips, pairs(flips)):
        assert p is not None, f"{label}: SNP {j} not computed in the exact restatement"
        gap = np.abs(p[3] - rsq_thr)
        ties = int((gap < WSDE_TIE).sum())
        rec["min_gap"].append(float(gap.min(initial=np.inf)))
        rec["ties_1e6"].append(ties)
        assert ties >= 1, f"{label}: SNP {j}: WSDE {a[j]} vs {b[j]} with no pair within {WSDE_TIE} of rsq_thr " \
                          f"(closest {gap.min(initial=np.inf):.3g})"
        if exact is not None:
            want = int((p[3] > rsq_thr).sum())
            assert (a if exact == "a" else b)[j] == want, f"{label}: SNP {j}: exact WSDE {want}"
    return rec


def rare_variant_set(n_org: int, n_snp: int = 400, seed: int = 5):
    """PLINK rows + cM positions of a chromosome where every other SNP is rare (MAF 1e-4 .. 3e-3, most
    without a hom-minor call) and a quarter of the SNPs have A1 as the minor allele (PLINK's default): at
    N % 4 == 0 those have het + hom-A2 calls only — a constant dominance coding whose fp32 residual in the
    reference is rounding noise."""
    from nldsc_amd import synth
    rng = np.random.default_rng(seed)
    M, N = n_snp, n_org
    maf = np.where(np.arange(M) % 2 == 0, 10 ** rng.uniform(-4, np.log10(3e-3), M), rng.uniform(0.05, 0.5, M))
    g = np.empty((M, N), np.int8)
    for j in range(M):
        a = (rng.random(N) < maf[j]).astype(np.int8) + (rng.random(N) < maf[j]).astype(np.int8)
        if j % 4 == 0:
            a = 2 - a  # minor allele = A1
        a[rng.random(N) < 0.01] = -1
        g[j] = a
    pos = np.cumsum(rng.exponential(0.05, M))
    return synth.pack_bed_rows(g), pos
