"""ctypes binding of libnldsc_amd.so (C ABI: include/nldsc_ld.h).

This is the product path's only route to the GPU engine besides the pybind11 `_ldscore`
module.  There is no CPU fallback: if the library is missing, or no HIP device is visible,
calls raise.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libnldsc_amd.so")

OK = 0
E_BAD_MAGIC, E_IO, E_SIZE, E_ARG, E_HIP, E_OOM, E_NODEV = -1, -2, -3, -4, -5, -6, -7
FLAG_STRICT_PLINK_ORDER = 1
FLAG_ADDITIVE_ONLY = 2
FLAG_EXACT_I8 = 4
FLAG_FP32 = 8
FLAG_EXACT_F4 = 16
FLAG_EXACT_RARE = 32

# every symbol include/nldsc_ld.h declares (tests check the library exports all of them)
EXPORTED = (
    "nldsc_ld_calculate", "nldsc_version", "nldsc_device_count", "nldsc_engine_create",
    "nldsc_engine_destroy", "nldsc_engine_load_bed_file", "nldsc_engine_load_bed_host",
    "nldsc_engine_load_bed_device", "nldsc_engine_run", "nldsc_engine_timings",
    "nldsc_synth_bed_device", "nldsc_engine_path", "nldsc_plan_band", "nldsc_engine_load_bed_file_range",
    "nldsc_format_scores", "nldsc_engine_ksplit", "nldsc_engine_band_kernel", "nldsc_engine_band_round_items",
    "nldsc_engine_band_tail_ksplit", "nldsc_engine_run_device", "nldsc_engine_run_device_split",
    "nldsc_engine_run_device_finish", "nldsc_engine_set_option", "nldsc_host_alloc", "nldsc_host_free",
    "nldsc_engine_result_direct",
)


class Params(ctypes.Structure):
    _fields_ = [("bedfile", ctypes.c_char_p), ("n_snp", ctypes.c_int32), ("n_org", ctypes.c_int32),
                ("ld_wind", ctypes.c_double), ("positions", ctypes.POINTER(ctypes.c_double)),
                ("maf", ctypes.c_double), ("std_thr", ctypes.c_double), ("rsq_thr", ctypes.c_double),
                ("flags", ctypes.c_uint32), ("device", ctypes.c_int32)]


class Result(ctypes.Structure):
    _fields_ = [("l2", ctypes.POINTER(ctypes.c_double)), ("l2d", ctypes.POINTER(ctypes.c_double)),
                ("maf", ctypes.POINTER(ctypes.c_double)), ("residuals_std", ctypes.POINTER(ctypes.c_double)),
                ("l2_ws", ctypes.POINTER(ctypes.c_int32)), ("l2d_ws", ctypes.POINTER(ctypes.c_int32)),
                ("l2d_wse", ctypes.POINTER(ctypes.c_int32))]


class NLDSCError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


_libs: dict = {}


def lib(path: str | None = None) -> ctypes.CDLL:
    """The engine library (default: the in-tree build; `path` loads another build of the same ABI,
    e.g. for interleaved A/B timing of kernel variants in one process)."""
    path = path or LIB_PATH
    if path not in _libs:
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same soname as ROCm's). If
        # torch is already imported, make sure its runtime is initialised before ours binds to it.
        if "torch" in sys.modules:
            try:
                sys.modules["torch"].cuda.init()
            except Exception:  # no device: our own calls will report it
                pass
        if not os.path.exists(path):
            raise ImportError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (make -C nldsc_amd/csrc). nldsc_amd has no CPU fallback.")
        L = ctypes.CDLL(path)
        c_err = [ctypes.c_char_p, ctypes.c_size_t]
        vp = ctypes.c_void_p
        L.nldsc_version.restype = ctypes.c_char_p
        L.nldsc_version.argtypes = []
        L.nldsc_device_count.restype = ctypes.c_int
        L.nldsc_device_count.argtypes = []
        L.nldsc_ld_calculate.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(Result)] + c_err
        L.nldsc_engine_create.argtypes = [ctypes.c_int32, ctypes.POINTER(vp)] + c_err
        L.nldsc_engine_destroy.argtypes = [vp]
        L.nldsc_engine_destroy.restype = None
        L.nldsc_engine_load_bed_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32] + c_err
        L.nldsc_engine_load_bed_host.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32] + c_err
        L.nldsc_engine_load_bed_device.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32] + c_err
        L.nldsc_engine_run.argtypes = [vp, ctypes.POINTER(Params), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.POINTER(Result)] + c_err
        L.nldsc_engine_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int32)]
        L.nldsc_plan_band.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, vp, vp, vp, ctypes.c_int32]
        L.nldsc_engine_path.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]
        if hasattr(L, "nldsc_engine_ksplit"):
            L.nldsc_engine_ksplit.argtypes = [vp]
        if hasattr(L, "nldsc_engine_band_kernel"):
            L.nldsc_engine_band_kernel.argtypes = [vp]
        if hasattr(L, "nldsc_engine_band_round_items"):
            L.nldsc_engine_band_round_items.argtypes = [vp]
        if hasattr(L, "nldsc_engine_band_tail_ksplit"):
            L.nldsc_engine_band_tail_ksplit.argtypes = [vp]
        if hasattr(L, "nldsc_engine_result_direct"):
            L.nldsc_engine_result_direct.argtypes = [vp]
        if hasattr(L, "nldsc_engine_run_device"):
            L.nldsc_engine_run_device.argtypes = [vp, ctypes.POINTER(Params), ctypes.c_int32, ctypes.c_int32, vp,
                                                  ctypes.c_int32] + c_err
        if hasattr(L, "nldsc_engine_run_device_split"):
            L.nldsc_engine_run_device_split.argtypes = [vp, ctypes.POINTER(Params), ctypes.c_int32, ctypes.c_int32, vp,
                                                        ctypes.c_int32, vp, ctypes.c_int32,
                                                        ctypes.POINTER(ctypes.c_int32)] + c_err
            L.nldsc_engine_run_device_finish.argtypes = [vp, vp, ctypes.c_int32] + c_err
        # entry points newer builds add (an older build loaded for A/B timing may lack them)
        if path == LIB_PATH or hasattr(L, "nldsc_engine_load_bed_file_range"):
            L.nldsc_engine_load_bed_file_range.argtypes = [vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                                           ctypes.c_int32, ctypes.c_int32] + c_err
        if hasattr(L, "nldsc_engine_set_option"):
            L.nldsc_engine_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64] + c_err
        if hasattr(L, "nldsc_host_alloc"):
            L.nldsc_host_alloc.restype = vp
            L.nldsc_host_alloc.argtypes = [ctypes.c_size_t]
            L.nldsc_host_free.restype = None
            L.nldsc_host_free.argtypes = [vp]
        L.nldsc_synth_bed_device.argtypes = [ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_float), ctypes.c_float, ctypes.c_float,
                                             ctypes.c_uint64] + c_err
        for name in EXPORTED:
            if name not in ("nldsc_version", "nldsc_device_count", "nldsc_engine_destroy", "nldsc_host_alloc",
                            "nldsc_host_free") and hasattr(L, name):
                getattr(L, name).restype = ctypes.c_int
        if hasattr(L, "nldsc_format_scores"):
            L.nldsc_format_scores.restype = ctypes.c_int64
            L.nldsc_format_scores.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int32] + [vp] * 7 + \
                [ctypes.c_int32, vp, ctypes.c_int64]  # out: any writable buffer address
        _libs[path] = L
    return _libs[path]


def check(rc: int, err) -> None:
    if rc != OK:
        msg = err.value.decode(errors="replace") if err is not None else f"error {rc}"
        if rc == E_BAD_MAGIC:
            raise ValueError(msg)
        raise NLDSCError(rc, msg)


def errbuf():
    return ctypes.create_string_buffer(1024)


class _Pinned:
    """Owner of one nldsc_host_alloc buffer (freed with the last numpy view of it)."""

    def __init__(self, L, ptr: int, nbytes: int):
        self._L, self.ptr, self.nbytes = L, ptr, nbytes

    def __del__(self):
        if self.ptr:
            self._L.nldsc_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = 0


def pinned_empty(n: int, dtype) -> np.ndarray:
    """An uninitialised numpy array in page-locked, device-mapped host memory (nldsc_host_alloc).  Result arrays
    there are written by the GPU directly (no landing buffer, no host copy) and positions there are read by DMA in
    place.  Falls back to an ordinary array when the library cannot allocate one (no HIP device)."""
    dt = np.dtype(dtype)
    nbytes = max(int(n), 1) * dt.itemsize
    L = lib()
    ptr = L.nldsc_host_alloc(nbytes) if hasattr(L, "nldsc_host_alloc") else None
    if not ptr:
        return np.empty(n, dt)
    owner = _Pinned(L, ptr, nbytes)
    raw = (ctypes.c_char * nbytes).from_address(ptr)
    raw._owner = owner  # the ctypes view keeps the buffer alive; numpy keeps the view alive (its .base)
    return np.frombuffer(raw, dtype=dt, count=int(n))


def alloc_result(n: int, pinned: bool = False):
    """numpy arrays + the C struct pointing at them (pinned: in nldsc_host_alloc memory, see pinned_empty)."""
    if pinned:
        arrs = {k: pinned_empty(n, np.float64) for k in ("l2", "l2d", "maf", "residuals_std")}
        arrs.update({k: pinned_empty(n, np.int32) for k in ("l2_ws", "l2d_ws", "l2d_wse")})
        for k, v in arrs.items():
            v.fill(np.nan if v.dtype == np.float64 else -1)
    else:
        arrs = dict(l2=np.full(n, np.nan), l2d=np.full(n, np.nan), maf=np.full(n, np.nan),
                    residuals_std=np.full(n, np.nan), l2_ws=np.full(n, -1, np.int32),
                    l2d_ws=np.full(n, -1, np.int32), l2d_wse=np.full(n, -1, np.int32))
    d, i = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
    res = Result(arrs["l2"].ctypes.data_as(d), arrs["l2d"].ctypes.data_as(d), arrs["maf"].ctypes.data_as(d),
                 arrs["residuals_std"].ctypes.data_as(d), arrs["l2_ws"].ctypes.data_as(i),
                 arrs["l2d_ws"].ctypes.data_as(i), arrs["l2d_wse"].ctypes.data_as(i))
    return arrs, res


def make_params(n_snp, n_org, ld_wind, maf, std_thr, rsq_thr, positions, *, bedfile=None, flags=0, device=-1):
    pos = np.ascontiguousarray(positions, dtype=np.float64)
    if pos.shape != (n_snp,):
        raise ValueError(f"positions must have n_snp={n_snp} elements, got {pos.shape}")
    p = Params(bedfile.encode() if bedfile else None, int(n_snp), int(n_org), float(ld_wind),
               pos.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), float(maf), float(std_thr), float(rsq_thr),
               int(flags), int(device))
    return p, pos  # keep `pos` alive while p is used


def plan_band(positions, pass_flags, ld_wind, own=None, max_nc=1):
    """Host-only schedule (C ABI nldsc_plan_band): returns (L, R, items[k, 4])."""
    pos = np.ascontiguousarray(positions, dtype=np.float64)
    n = len(pos)
    fl = np.ascontiguousarray(pass_flags, dtype=np.uint8)
    own = (0, n) if own is None else own
    L_ = np.empty(n, np.int32)
    R_ = np.empty(n, np.int32)
    args = (pos.ctypes.data, fl.ctypes.data, n, float(ld_wind), int(own[0]), int(own[1]), int(max_nc),
            L_.ctypes.data, R_.ctypes.data)
    k = lib().nldsc_plan_band(*args, None, 0)
    if k < 0:
        raise ValueError(f"nldsc_plan_band error {k}")
    items = np.zeros((max(k, 1), 4), np.int32)
    k2 = lib().nldsc_plan_band(*args, items.ctypes.data, len(items))
    assert k2 == k
    return L_, R_, items[:k]
