"""The C-ABI library and the pybind11 drop-in load, export what include/nldsc_ld.h declares and
mirror the reference's binding (nldsc/ldscore/_ldscore/ldscore.cpp:17-54).  No compute calls."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO


def header_functions():
    text = open(os.path.join(REPO, "include", "nldsc_ld.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nldsc_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_bound_entry_points():
    from nldsc_amd import _lib
    assert header_functions() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    from nldsc_amd import _lib
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    L = _lib.lib()
    for f in header_functions():
        assert getattr(L, f) is not None
    assert L.nldsc_version().decode() == "0.1.0"


def test_library_is_gfx950_code_object():
    from nldsc_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"band_kernel" in data


def test_pybind_module_mirrors_reference_binding():
    from nldsc_amd.ldscore import _ldscore as lds
    p = lds.LDScoreParams("x.bed", n_snp=2, n_org=5, ld_wind=1.0, maf=0.01, std_thr=1e-5, rsq_thr=0.01,
                          positions=[0.5, 1.5])
    assert (p.bedfile, p.n_snp, p.n_org, p.ld_wind, p.maf, p.std_thr, p.rsq_thr, p.positions) == \
        ("x.bed", 2, 5, 1.0, 0.01, 1e-5, 0.01, [0.5, 1.5])
    with pytest.raises(TypeError):  # keyword-only after bfile (ldscore.cpp:24-33)
        lds.LDScoreParams("x.bed", 2, 5, 1.0, 0.01, 1e-5, 0.01, [0.5, 1.5])
    q = lds.LDScoreParams()
    q.bedfile = "y.bed"
    q.positions = [1, 2, 3]
    assert q.positions == [1.0, 2.0, 3.0]
    r = lds.LDScoreResult()
    for k in ("l2", "l2d", "maf", "residuals_std", "l2_ws", "l2d_ws", "l2d_wse"):
        assert getattr(r, k) == []
    r.l2_ws = [1, 2]
    assert r.l2_ws == [1, 2]
    assert callable(lds.calculate)


def test_calculate_without_gpu_fails_loudly(monkeypatch):
    """No CPU fallback: with no HIP device `calculate` raises (never silently computes on the host)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from nldsc_amd.ldscore import _ldscore as lds
    p = lds.LDScoreParams("x.bed", n_snp=1, n_org=5, ld_wind=1.0, maf=0.01, std_thr=1e-5, rsq_thr=0.01,
                          positions=[0.5])
    with pytest.raises(RuntimeError, match="no HIP device"):
        lds.calculate(p)
    from nldsc_amd import engine
    with pytest.raises(RuntimeError):
        engine.Engine(0)


def test_product_never_imports_the_oracle():
    for root, _, files in os.walk(os.path.join(REPO, "nldsc_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(root, f), errors="replace").read()
                assert "oracle" not in re.sub(r"(#|//).*", "", text).lower().replace("oracle-free", ""), f


def test_legacy_environment_knobs_are_reported():
    """The round 1-4 environment knobs are engine options now (nldsc_engine_set_option); setting one warns once on
    stderr when an engine is created (with or without a GPU) instead of being ignored silently."""
    import sys
    code = ("from nldsc_amd import engine\n"
            "for _ in range(2):\n"
            "    try:\n        engine.Engine(0).close()\n    except RuntimeError:\n        pass\n")
    env = dict(os.environ, NLDSC_T2="1", NLDSC_BAND_MODE="0")
    p = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stderr.count('$NLDSC_T2 is no longer read; use the engine option "t2"') == 1, p.stderr
    assert p.stderr.count('"band_mode"') == 1, p.stderr
