"""The headline chromosome at full size (BASELINE.json configs[2]: N = 315 599, M = 80 000, 1 cM, add + dom), and the
zero-copy host-result path the bench measures it through.

* The fp32 MFMA path (north star's GEMM, FLAG_FP32) against the default exact path over all 80 000 SNPs: window
  counts and MAF equal, L2 / L2D within conftest.TOL, and every WSDE difference audited against the exact per-pair
  r2adj (oracle.pair_r2_f64: integer contingency tables, binary64) — each must sit on a pair within 1e-6 of rsq_thr,
  and the exact path must equal the exact count there (ldscalc.h:41-47).
* Results written straight into nldsc_host_alloc arrays: bitwise the ordinary-array run, entries outside
  the owned range untouched, the pair count the same, for full, middle, last-SNP and empty ranges and a mixed case
  (one array ordinary: the landing buffer).
"""
import numpy as np
import pytest

from conftest import TOL, assert_ld_close, progress, record, wsde_tie_audit
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FP32, F4 = 8, 16  # _lib.FLAG_FP32, _lib.FLAG_EXACT_F4


@pytest.fixture(scope="module")
def engine():
    import torch
    torch.cuda.init()
    from nldsc_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def test_fp32_path_wsde_flips_are_ties_at_full_c3(engine):
    import torch

    from nldsc_amd import synth
    N, M = 315_599, 80_000
    buf, pos = synth.device_bed(M, N, seed=7, length_cm=280.0)  # bench.py's C3 image (rank 0)
    args = (1.0, 1e-4, 1e-5, 1.0 / M)
    engine.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    progress("c3 full: runs")
    exact = engine.run(*args, pos, flags=F4)
    f32 = engine.run(*args, pos, flags=FP32)
    bed = buf.cpu().numpy().tobytes()
    del buf
    torch.cuda.empty_cache()
    for k in ("l2_ws", "l2d_ws", "maf", "residuals_std"):
        np.testing.assert_array_equal(f32[k], exact[k], err_msg=k)
    assert_ld_close(f32, exact, wse_budget=None, label="fp32 path vs exact path, C3")
    rows = np.frombuffer(bed, np.uint8, offset=3).reshape(M, -1)
    progress("c3 full: tie audit")
    audit = wsde_tie_audit(f32["l2d_wse"], exact["l2d_wse"],
                           lambda js: O.pair_r2_f64(rows, N, *args[:3], pos, js, bed=bed), args[3],
                           label="fp32 path vs exact path, C3", exact="b")
    ok = exact["l2_ws"] > 0
    record("c3_full_fp32_audit", dict(
        n_org=N, n_snp=M, rsq_thr=args[3], wsde=audit,
        l2_max_abs=float(np.max(np.abs(f32["l2"][ok] - exact["l2"][ok]))),
        l2d_max_abs=float(np.nanmax(np.abs(f32["l2d"][ok] - exact["l2d"][ok])))))
    progress("c3 full: done")
    assert audit["flips"] > 0  # r2adj is dense around 1/M at this N: some pairs round to the other side in fp32
    assert np.isfinite(exact["l2"]).all() and (exact["l2_ws"] > 100).all()


def _sentinel(arrs):
    for k, v in arrs.items():
        v.fill(12345.5 if v.dtype == np.float64 else -7)


@pytest.mark.parametrize("flags", [F4, FP32])
def test_pinned_results_written_in_place(engine, flags):
    """nldsc_engine_run into nldsc_host_alloc arrays (finalize_out_kernel writes the caller's mapped pinned memory, the
    per-workgroup pair counts read from host memory) against ordinary numpy arrays (the landing buffer)."""
    from nldsc_amd import _lib, synth
    N, M = 20_001, 1500
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=6.0, seed=17, missing=0.01)
    rows = synth.pack_bed_rows(synth.genotypes(spec))
    pos_np = synth.positions_cm(spec)
    pos_pin = _lib.pinned_empty(M, np.float64)
    pos_pin[:] = pos_np
    args = (1.0, 1e-4, 1e-5, 1.0 / M)
    engine.load_bed_bytes(synth.bed_bytes(rows), M, N)
    for own in [(0, M), (301, 977), (M - 1, M), (640, 640)]:
        ref = _lib.alloc_result(M)[0]
        _sentinel(ref)
        engine.run(*args, pos_np, own=own, flags=flags, out=ref)
        t_ref = engine.timings()
        assert t_ref["result_direct"] == (0 if own[0] < own[1] else -1)
        for mixed in (False, True):
            pin = _lib.alloc_result(M, pinned=True)[0]
            if mixed:  # one ordinary array: the whole result goes through the landing buffer
                pin["l2d_wse"] = np.empty(M, np.int32)
            _sentinel(pin)
            engine.run(*args, pos_pin, own=own, flags=flags, out=pin)
            t = engine.timings()
            assert t["result_direct"] == (-1 if own[0] == own[1] else 0 if mixed else 1), (own, mixed)
            assert t["pairs"] == t_ref["pairs"], (own, mixed)
            for k in ref:
                np.testing.assert_array_equal(pin[k], ref[k], err_msg=f"{k} own={own} mixed={mixed}")
            outside = np.ones(M, bool)
            outside[own[0]:own[1]] = False
            for k, v in pin.items():
                assert (v[outside] == (12345.5 if v.dtype == np.float64 else -7)).all(), (k, own, mixed)
            if own[0] < own[1]:
                assert (pin["l2_ws"][own[0]:own[1]] >= 0).all() and np.isfinite(pin["maf"][own[0]:own[1]]).all()
    full = _lib.alloc_result(M, pinned=True)[0]
    engine.run(*args, pos_pin, flags=flags | _lib.FLAG_EXACT_RARE, out=full)  # (exact residuals: the fp64 truth)
    exp = O.run_f64(rows, N, *args, pos_np)
    tol = dict(TOL, l2d=(1e-5, 1e-4)) if flags == FP32 else dict(l2=(1e-9, 1e-12), l2d=(1e-9, 1e-12),
                                                                  residuals_std=(1e-12, 1e-10), maf=(0.0, 0.0))
    assert_ld_close(full, exp, tol=tol, wse_budget=0.01, label="pinned results vs fp64 truth")
