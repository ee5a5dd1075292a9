"""`estimate_lds` — the caller of the hot path (behaviour of nldsc/ldscore/routine.py:15-102).

Parses .bed/.bim/.fam, validates parameters, builds `_ldscore.LDScoreParams`, runs
`_ldscore.calculate` on the GPU, optionally prints the summary, and writes the TSV
`CHR SNP BP L2 L2D [MAF WSA WSD WSDE RSTD]` (tab-separated, `%.5f`, NaN as empty field)
to `out`.  Additions: `write_m` writes the `M`/`MD` file the h2 reader looks for
(nldsc/h2/common.py:115-132,142-144) with exactly the values its fallback would compute.
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import pandas as pd

from ..core.common import elapsed_time
from ..core.logger import log
from . import _ldscore as lds
from .common import BIMFile, LDWindow, MAF, PLINKFile, ResidualsSTDThreshold, RSQThreshold

__all__ = ["estimate_lds", "make_output", "format_scores", "write_scores", "show_summary", "m_values", "write_m_file"]


def show_summary(ld) -> None:
    import click
    pd.set_option("display.precision", 3)
    data = pd.DataFrame({"L2": list(ld.l2), "L2D": list(ld.l2d), "MAF": list(ld.maf)})
    click.echo("=" * 62)
    click.echo("L2/L2D/MAF Correlation matrix\n" + str(data.corr()))
    description = data.describe().drop("count")
    click.echo(f"\nShort summary:\n"
               f"- Number of additive non-null LD: {data['L2'].count()}\n"
               f"- Number of non-additive non-null LD: {data['L2D'].count()}\n"
               + str(description))
    click.echo("=" * 62)


def make_output(bim: BIMFile, ld, *, extra: bool = False) -> pd.DataFrame:
    cols = {"CHR": bim.chr.reset_index(drop=True), "SNP": bim.snp.reset_index(drop=True),
            "BP": bim.bp.reset_index(drop=True), "L2": pd.Series(list(ld.l2)), "L2D": pd.Series(list(ld.l2d))}
    if extra:
        cols.update(MAF=pd.Series(list(ld.maf)), WSA=pd.Series(list(ld.l2_ws)), WSD=pd.Series(list(ld.l2d_ws)),
                    WSDE=pd.Series(list(ld.l2d_wse)), RSTD=pd.Series(list(ld.residuals_std)))
    return pd.DataFrame(cols)


HEADER = ("CHR", "SNP", "BP", "L2", "L2D")
HEADER_EXTRA = ("MAF", "WSA", "WSD", "WSDE", "RSTD")


def format_scores(bim: BIMFile, ld, *, extra: bool = False) -> bytes:
    """The bytes `make_output(bim, ld, extra=extra).to_csv(path, sep="\t", index=False, float_format="%.5f")`
    writes (routine.py:94-101 of the reference), formatted by the native writer (nldsc_format_scores):
    ~20x faster than pandas on the float columns.  CHR / SNP / BP are printed as pandas prints the parsed
    .bim columns (int64 -> decimal, object -> the text); any other column type goes through pandas."""
    import ctypes

    from .. import _lib
    cols = (bim.chr.reset_index(drop=True), bim.snp.reset_index(drop=True), bim.bp.reset_index(drop=True))
    n = len(cols[0])
    # pandas prints a null object cell (e.g. a SNP id read as NaN: 'NA', 'NULL') as an empty field, str() as 'nan'
    if any(c.dtype.kind not in "iuO" or c.isna().any() for c in cols) or len(ld.l2) != n:
        buf = make_output(bim, ld, extra=extra).to_csv(sep="\t", index=False, float_format="%.5f")
        return buf.encode()
    text = [list(map(str, c.tolist())) for c in cols]  # what pandas prints for int64 / object cells
    f64 = lambda v: np.ascontiguousarray(v, dtype=np.float64)  # noqa: E731
    i32 = lambda v: np.ascontiguousarray(v, dtype=np.int32)  # noqa: E731
    arrs = [f64(ld.l2), f64(ld.l2d)]
    if extra:
        arrs += [f64(ld.maf), i32(ld.l2_ws), i32(ld.l2d_ws), i32(ld.l2d_wse), f64(ld.residuals_std)]
    lib, parts, chunk = _lib.lib(), [], 16384
    out = np.empty(0, np.uint8)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        prefix = "\n".join(map("\t".join, zip(text[0][a:b], text[1][a:b], text[2][a:b]))).encode()
        need = len(prefix) + (b - a) * (16 + 7 * 400) + 1  # worst case of the numeric fields
        if out.size < need:
            out = np.empty(need, np.uint8)
        ptrs = [v[a:].ctypes.data for v in arrs] + [None] * (7 - len(arrs))
        got = lib.nldsc_format_scores(prefix, len(prefix), b - a, *ptrs, int(bool(extra)), out.ctypes.data,
                                      out.size)
        if got < 0:
            raise RuntimeError(f"nldsc_format_scores failed ({got})")
        parts.append(out[:got].tobytes())
    head = "\t".join(HEADER + (HEADER_EXTRA if extra else ())) + "\n"
    return head.encode() + b"".join(parts)


def write_scores(path: str, bim: BIMFile, ld, *, extra: bool = False) -> None:
    with open(path, "wb") as fh:
        fh.write(format_scores(bim, ld, extra=extra))


def m_values(bim: BIMFile, ld) -> tuple[int, int]:
    """M, MD as LDScoreReader derives them without an .M file (h2/common.py:128-130): rows
    surviving dropna + SNP de-duplication, and M * mean(WSDE / WSA)."""
    df = make_output(bim, ld, extra=True).sort_values(by=["CHR", "BP"]).dropna().drop_duplicates(subset="SNP")
    m = len(df["L2"])
    md = m * (df["WSDE"] / df["WSA"]).mean()
    return int(m), int(md)


def write_m_file(path: str, m: int, md: int) -> None:
    pd.DataFrame({"M": [m], "MD": [md]}).to_csv(path, sep="\t", index=False)


class _Result:
    """LDScoreResult-shaped holder for tables assembled from several ranks."""

    def __init__(self, d: dict):
        for k, v in d.items():
            setattr(self, k, v.tolist())


def _backend() -> str:
    """Collectives backend of the torchrun path: RCCL ("nccl", one GPU per rank) unless $NLDSC_DIST_BACKEND
    says "gloo" (CPU collectives; ranks may then share GPUs, e.g. a 2-rank rehearsal on one GPU)."""
    return os.environ.get("NLDSC_DIST_BACKEND", "nccl")


def _split_halo() -> bool:
    """$NLDSC_SPLIT_HALO=1: boundary pairs computed once across ranks (right halo's sums sent point to point); by
    default each rank loads a two-sided halo and computes them itself (the same band time at C3/8, no exchange)."""
    return os.environ.get("NLDSC_SPLIT_HALO", "0") != "0"


def _local_device() -> int:
    import torch
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return local if _backend() == "nccl" else local % max(1, torch.cuda.device_count())


def _process_group():
    """The torch.distributed module when launched by torchrun with WORLD_SIZE > 1, else None."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        dev = _local_device()
        torch.cuda.set_device(dev)
        if _backend() == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(_backend())
    return dist


def _calculate_sharded(dist, params):
    from .. import distributed as D
    dev = _local_device()
    pos = np.asarray(params.positions, dtype=np.float64)
    plan = D.split_plan(pos, params.ld_wind, dist.get_world_size()) if _split_halo() else None
    if plan is not None:  # boundary pairs once: halo sums sent to the next rank (point to point)
        full = D.calculate_sharded_split(params.bedfile, params.n_snp, params.n_org, params.ld_wind, params.maf,
                                         params.std_thr, params.rsq_thr, pos, plan, flags=params.flags, device=dev)
    elif _backend() == "nccl":  # the owned slices stay in device memory and are gathered over RCCL
        full = D.calculate_sharded_device(params.bedfile, params.n_snp, params.n_org, params.ld_wind, params.maf,
                                          params.std_thr, params.rsq_thr, pos, flags=params.flags, device=dev)
    else:  # gloo: host result arrays, CPU collectives
        run = D.engine_runner(params.bedfile, params.n_snp, params.n_org, params.ld_wind, params.maf,
                              params.std_thr, params.rsq_thr, pos, flags=params.flags, device=dev)
        full = D.calculate_sharded(run, pos, params.ld_wind, params.n_snp)
    return None if full is None else _Result(full)


@elapsed_time
def estimate_lds(bfile: str, ld_wind: float, wind_metric: str, maf_thr: float = 1e-5, std_thr: float = 1e-5,
                 rsq_thr: float | None = None, *, out: str | None = None, extra: bool = False, summary: bool = False,
                 verbose: int = 0, write_m: bool = False, flags: int = 0, device: int | None = None,
                 progress: bool | None = None):
    bed_, bim_, fam_ = PLINKFile.parse(bfile)
    ld_wind_ = LDWindow(ld_wind, metric=wind_metric)
    maf_thr_ = MAF(maf_thr)
    std_thr_ = ResidualsSTDThreshold(std_thr)
    if rsq_thr is None:
        rsq_thr = 1.0 / bim_.n_snp
    rsq_thr_ = RSQThreshold(rsq_thr)
    log.info(f"Input: {bed_.data}, size: (M={bim_.n_snp}, N={fam_.n_org})")

    params = lds.LDScoreParams(
        bfile=bed_.data, n_snp=bim_.n_snp, n_org=fam_.n_org, ld_wind=ld_wind_.data, maf=maf_thr_.data,
        std_thr=std_thr_.data, rsq_thr=rsq_thr_.data,
        positions=np.asarray(getattr(bim_, ld_wind_.metric), dtype=np.float64).tolist())
    params.flags = int(flags)
    if device is not None:
        params.device = int(device)
    log.info("Running the estimator. It may take a long time.")
    from ..core.progress import Progress
    bar = Progress(bim_.n_snp, "SNPs", enabled=progress)
    bar.update(0, "reading the .bed and computing on the GPU", force=True)
    dist = _process_group()
    if dist is None:
        ld = lds.calculate(params)
    else:  # torchrun: position-sharded over the ranks' GPUs, tables gathered on rank 0
        ld = _calculate_sharded(dist, params)
        if ld is None:
            return None
    ws = np.asarray(ld.l2_ws)
    bar.close(f"{int(ws[ws > 0].sum()):,} SNP pairs")
    log.info("Estimation completed")

    if summary:
        show_summary(ld)
    if out:
        log.info("Writing data to disk...")
        write_scores(out, bim_, ld, extra=extra)
        if write_m:
            m, md = m_values(bim_, ld)
            write_m_file(str(Path(out).with_suffix(".M")), m, md)
        log.info(f"Completed. File: {out}")
        return None
    return make_output(bim_, ld, extra=extra)
