"""Python handle on the GPU engine (C ABI `nldsc_engine_*`, include/nldsc_ld.h).

`Engine` keeps a .bed image resident in HBM and runs the LD-score hot path over it; it is
what the benchmark, the GPU parity tests and the multi-GPU driver use.  `calculate` is the
one-shot equivalent of the reference's `_ldscore.calculate(params)`
(nldsc/ldscore/_ldscore/ldscalc.h:8-65).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

# nldsc_engine_band_kernel codes (include/nldsc_ld.h NLDSC_BAND_*)
BAND_KERNELS = {0: "f32", 1: "i8", 2: "f4", 3: "f4_seg", 4: "f4_ksplit", 5: "f4_2x2", 6: "f4_routed",
                7: "f4_quad"}


def _torch_ready(*tensors):
    """Device tensors handed to the engine were written on torch's current stream (fills, copies, collectives:
    with RCCL, `req.wait()` only orders torch's stream); the engine runs on its own non-blocking HIP stream, so
    the host waits for torch's stream first."""
    import torch
    for d in {t.device for t in tensors if t is not None and t.is_cuda}:
        torch.cuda.current_stream(d).synchronize()


class Engine:
    # Engine options (C ABI nldsc_engine_set_option) applied to every new engine before `options`: test and study
    # knobs of the schedule and kernel choice (all paths give the same results: the GPU tests compare them), empty by
    # default.  See nldsc_amd/csrc/ld_engine.cpp nldsc_engine_set_option for the names.
    default_options: dict = {}

    def __init__(self, device: int = -1, lib_path: str | None = None, options: dict | None = None):
        self._L = L = _lib.lib(lib_path)
        self._h = ctypes.c_void_p()
        err = _lib.errbuf()
        _lib.check(L.nldsc_engine_create(int(device), ctypes.byref(self._h), err, len(err)), err)
        self.n_snp = 0
        self.n_org = 0
        for name, value in {**Engine.default_options, **(options or {})}.items():
            self.set_option(name, value)

    def set_option(self, name: str, value: int):
        """One engine option (nldsc_engine_set_option); "orient" applies from the next load."""
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_set_option(self._h, name.encode(), int(value), err, len(err)), err)

    def close(self):
        if self._h:
            self._L.nldsc_engine_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- loading ------------------------------------------------------------------------
    def load_bed_file(self, path: str, n_snp: int, n_org: int):
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_load_bed_file(self._h, path.encode(), n_snp, n_org, err, len(err)), err)
        self.n_snp, self.n_org = n_snp, n_org

    def load_bed_file_range(self, path: str, n_snp_file: int, n_org: int, begin: int, end: int):
        """Rows [begin, end) of a .bed file of n_snp_file SNPs (position sharding: own range + halo)."""
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_load_bed_file_range(self._h, path.encode(), n_snp_file, n_org, int(begin),
                                                               int(end), err, len(err)), err)
        self.n_snp, self.n_org = int(end) - int(begin), n_org

    def load_bed_bytes(self, bed, n_snp: int, n_org: int):
        """`bed`: the whole .bed content (bytes / uint8 numpy array), magic included."""
        buf = np.frombuffer(bed, dtype=np.uint8) if isinstance(bed, (bytes, bytearray)) else np.ascontiguousarray(bed, np.uint8)
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_load_bed_host(self._h, buf.ctypes.data, buf.nbytes, n_snp, n_org, err,
                                                         len(err)), err)
        self.n_snp, self.n_org = n_snp, n_org

    def load_bed_device(self, ptr: int, nbytes: int, n_snp: int, n_org: int):
        """Copy a .bed image that already lives in this device's memory (e.g. a torch tensor)."""
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_load_bed_device(self._h, ctypes.c_void_p(ptr), nbytes, n_snp, n_org, err,
                                                           len(err)), err)
        self.n_snp, self.n_org = n_snp, n_org

    # ---- compute ------------------------------------------------------------------------
    def run(self, ld_wind, maf, std_thr, rsq_thr, positions, *, own=None, flags=0, out=None):
        """LD scores for owned SNPs [own[0], own[1]) (default all).  Returns dict of numpy arrays
        (entries outside the owned range are NaN / -1, or whatever `out` held)."""
        n = self.n_snp
        own = (0, n) if own is None else own
        p, _keep = _lib.make_params(n, self.n_org, ld_wind, maf, std_thr, rsq_thr, positions, flags=flags)
        if out is None:
            arrs, res = _lib.alloc_result(n)
        else:
            arrs = out
            d, i = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
            res = _lib.Result(*(arrs[k].ctypes.data_as(d if arrs[k].dtype == np.float64 else i)
                                for k in ("l2", "l2d", "maf", "residuals_std", "l2_ws", "l2d_ws", "l2d_wse")))
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_run(self._h, ctypes.byref(p), int(own[0]), int(own[1]),
                                               ctypes.byref(res), err, len(err)), err)
        return arrs

    def run_device(self, ld_wind, maf, std_thr, rsq_thr, positions, table, *, own=None, flags=0):
        """As `run`, but the owned slice of the score table stays on the device: `table` is a float64 device
        tensor of shape (7, width) on this engine's GPU (rows l2, l2d, maf, residuals_std, l2_ws, l2d_ws, l2d_wse;
        column c = SNP own[0] + c; NaN past the slice), written when this returns (C ABI nldsc_engine_run_device)."""
        n = self.n_snp
        own = (0, n) if own is None else own
        if table.dim() != 2 or table.shape[0] != 7 or not table.is_cuda or str(table.dtype) != "torch.float64" \
                or not table.is_contiguous():
            raise ValueError("table must be a contiguous float64 CUDA tensor of shape (7, width)")
        p, _keep = _lib.make_params(n, self.n_org, ld_wind, maf, std_thr, rsq_thr, positions, flags=flags)
        _torch_ready(table)
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_run_device(self._h, ctypes.byref(p), int(own[0]), int(own[1]),
                                                      ctypes.c_void_p(table.data_ptr()), int(table.shape[1]), err,
                                                      len(err)), err)
        return table

    def run_device_split(self, ld_wind, maf, std_thr, rsq_thr, positions, table, export, *, own, flags=0) -> int:
        """First half of a split run (C ABI nldsc_engine_run_device_split): the loaded slice is the owned SNPs
        [own[0], own[1]) and the right halo after them; computes the pairs whose lower SNP is owned and writes the
        halo's accumulator rows into `export` (contiguous int64 device tensor of >= 6 * halo elements).  Returns the
        number of halo SNPs exported; finish with run_device_finish."""
        n = self.n_snp
        if table.dim() != 2 or table.shape[0] != 7 or not table.is_cuda or str(table.dtype) != "torch.float64" \
                or not table.is_contiguous():
            raise ValueError("table must be a contiguous float64 CUDA tensor of shape (7, width)")
        if not export.is_cuda or str(export.dtype) != "torch.int64" or not export.is_contiguous():
            raise ValueError("export must be a contiguous int64 CUDA tensor")
        p, _keep = _lib.make_params(n, self.n_org, ld_wind, maf, std_thr, rsq_thr, positions, flags=flags)
        cnt = ctypes.c_int32(0)
        _torch_ready(table, export)
        err = _lib.errbuf()
        _lib.check(self._L.nldsc_engine_run_device_split(
            self._h, ctypes.byref(p), int(own[0]), int(own[1]), ctypes.c_void_p(table.data_ptr()),
            int(table.shape[1]), ctypes.c_void_p(export.data_ptr()), int(export.numel() // 6), ctypes.byref(cnt),
            err, len(err)), err)
        return int(cnt.value)

    def run_device_finish(self, imported=None, n: int = 0):
        """Second half: add the left neighbour's exported block (int64 device tensor laid out [6][n]) into the
        first n owned SNPs, finalize and write the table given to run_device_split."""
        err = _lib.errbuf()
        ptr = ctypes.c_void_p(imported.data_ptr()) if (imported is not None and n > 0) else None
        if ptr is not None:
            _torch_ready(imported)
        _lib.check(self._L.nldsc_engine_run_device_finish(self._h, ptr, int(n), err, len(err)), err)

    def timings(self) -> dict:
        ms = (ctypes.c_double * 6)()
        flop, issued, pairs = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        nl = ctypes.c_int32()
        self._L.nldsc_engine_timings(self._h, ms, ctypes.byref(flop), ctypes.byref(issued), ctypes.byref(pairs),
                                        ctypes.byref(nl))
        keys = ("count_ms", "stats_ms", "schedule_ms", "band_ms", "finalize_ms", "total_ms")
        d = {k: ms[i] for i, k in enumerate(keys)}
        d.update(flop_alg=flop.value, flop_issued=issued.value, pairs=pairs.value, band_items=nl.value)
        ex, ops = ctypes.c_int32(), ctypes.c_double()
        self._L.nldsc_engine_path(self._h, ctypes.byref(ex), ctypes.byref(ops))
        L = self._L  # (an older build loaded for A/B timing may lack the newer entry points)
        d.update(exact_i8=ex.value > 0, path={0: "f32", 1: "i8", 2: "f4"}[ex.value], ops_alg_i8=ops.value,
                 ksplit=L.nldsc_engine_ksplit(self._h) if hasattr(L, "nldsc_engine_ksplit") else 1,
                 band_kernel=(BAND_KERNELS.get(L.nldsc_engine_band_kernel(self._h), "?")
                              if hasattr(L, "nldsc_engine_band_kernel") else "?"),
                 band_round_items=(self._L.nldsc_engine_band_round_items(self._h)
                                   if hasattr(self._L, "nldsc_engine_band_round_items") else 0),
                 band_tail_ksplit=(self._L.nldsc_engine_band_tail_ksplit(self._h)
                                   if hasattr(self._L, "nldsc_engine_band_tail_ksplit") else 1),
                 result_direct=(self._L.nldsc_engine_result_direct(self._h)
                                if hasattr(self._L, "nldsc_engine_result_direct") else -1))
        return d


def calculate(bedfile: str, n_snp, n_org, ld_wind, maf, std_thr, rsq_thr, positions, *, flags=0, device=-1) -> dict:
    """One-shot C-ABI call `nldsc_ld_calculate` (file -> GPU -> results)."""
    p, _keep = _lib.make_params(n_snp, n_org, ld_wind, maf, std_thr, rsq_thr, positions, bedfile=bedfile,
                                flags=flags, device=device)
    arrs, res = _lib.alloc_result(n_snp)
    err = _lib.errbuf()
    _lib.check(_lib.lib().nldsc_ld_calculate(ctypes.byref(p), ctypes.byref(res), err, len(err)), err)
    return arrs


def device_count() -> int:
    return int(_lib.lib().nldsc_device_count())


def synth_bed_device(device: int, ptr: int, n_snp: int, n_org: int, thr: np.ndarray, rho: float = 0.9,
                     missing: float = 0.01, seed: int = 7):
    t = np.ascontiguousarray(thr, dtype=np.float32)
    err = _lib.errbuf()
    _lib.check(_lib.lib().nldsc_synth_bed_device(int(device), ctypes.c_void_p(ptr), n_snp, n_org,
                                                 t.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), float(rho),
                                                 float(missing), int(seed), err, len(err)), err)
