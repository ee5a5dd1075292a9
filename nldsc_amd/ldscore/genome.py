"""Whole-genome `nldsc ld`: one invocation over per-chromosome PLINK sets.

`--bfile chr@` expands `@` to the chromosome numbers whose `.bed/.bim/.fam` exist (1..22, then X/Y/MT).
Every chromosome is an independent unit (the reference accepts one chromosome per file,
nldsc/ldscore/common.py:114-117, and windows never cross chromosomes).  Under torchrun the units are
assigned to GPUs by longest-processing-time first on their estimated pair count; each rank writes the
outputs of its own chromosomes (`--out` must contain `@` too), so nothing crosses GPUs.  On each GPU
the next chromosome's `.bed` is read by a host thread while the current one is computed.
"""
from __future__ import annotations

import os
import threading
import time
from pathlib import Path

import numpy as np

from ..core.common import NLDSCParameterError, elapsed_time
from ..core.logger import log
from .common import FAMFile, BIMFile, LDWindow, MAF, ResidualsSTDThreshold, RSQThreshold
from .routine import m_values, make_output, write_m_file, write_scores

CHROMS = [str(c) for c in range(1, 23)] + ["X", "Y", "XY", "MT"]


def expand_bfile(pattern: str) -> list[tuple[str, str]]:
    """[(chromosome, prefix)] for a pattern with '@' whose three PLINK files exist."""
    if "@" not in pattern:
        raise NLDSCParameterError("a whole-genome --bfile needs '@' in place of the chromosome number")
    p = pattern[:-4] if pattern.endswith((".bed", ".bim", ".fam")) else pattern
    out = []
    for c in CHROMS:
        stem = p.replace("@", c)
        if all(os.path.exists(stem + ext) for ext in (".bed", ".bim", ".fam")):
            out.append((c, stem))
    if not out:
        raise FileNotFoundError(f'No PLINK file set matches "{pattern}"')
    return out


class _Prefetch:
    """Reads a .bed file on a host thread (the read releases the GIL)."""

    def __init__(self, path: str):
        self.path, self.data, self.err = path, None, None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        try:
            self.data = np.fromfile(self.path, dtype=np.uint8)
        except Exception as ex:  # noqa: BLE001
            self.err = ex

    def get(self) -> np.ndarray:
        self.t.join()
        if self.err is not None:
            raise self.err
        return self.data


def _readahead(path: str) -> None:
    """Ask the kernel to start reading `path` into the page cache (asynchronous readahead)."""
    try:
        fd = os.open(path, os.O_RDONLY)
        try:
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_WILLNEED)
        finally:
            os.close(fd)
    except (OSError, AttributeError):
        pass


def _default_runner(device: int):
    """The GPU engine, fed by its own file reader (file -> pinned slots -> pitched H2D copies overlapping
    the reads, ~20 GB/s from the page cache) instead of a host array copied from pageable memory."""
    from ..engine import Engine
    eng = Engine(device)

    def run(bed_path: str, n_snp: int, n_org: int, ld_wind, maf, std_thr, rsq_thr, positions, flags):
        eng.load_bed_file(bed_path, n_snp, n_org)
        return eng.run(ld_wind, maf, std_thr, rsq_thr, positions, flags=flags), eng.timings()
    run.wants_path = True
    return run


@elapsed_time
def estimate_lds_genome(bfile: str, ld_wind: float, wind_metric: str, maf_thr: float = 1e-5,
                        std_thr: float = 1e-5, rsq_thr: float | None = None, *, out: str | None = None,
                        extra: bool = False, write_m: bool = False, flags: int = 0, device: int | None = None,
                        runner=None, rank: int | None = None, world: int | None = None,
                        progress: bool | None = None) -> dict:
    """Returns {chromosome: output DataFrame (None when written to `out`)} for the chromosomes this rank
    processed."""
    units = expand_bfile(bfile)
    if out is not None and "@" not in out:
        raise NLDSCParameterError("a whole-genome run needs '@' in --out (one output per chromosome)")
    ld_wind_ = LDWindow(ld_wind, metric=wind_metric)
    maf_thr_, std_thr_ = MAF(maf_thr), ResidualsSTDThreshold(std_thr)
    if rank is None or world is None:
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    # cheap host pass: .bim/.fam of every unit, pair-work estimate for the assignment
    from ..distributed import assign_units, window_work
    meta = []
    for chrom, stem in units:
        bim, fam = BIMFile(stem + ".bim"), FAMFile(stem + ".fam")
        pos = np.asarray(getattr(bim, ld_wind_.metric), dtype=np.float64)
        meta.append(dict(chrom=chrom, stem=stem, bim=bim, n_org=fam.n_org, pos=pos,
                         work=float(window_work(pos, ld_wind_.data).sum()) * fam.n_org))
    mine = assign_units([m["work"] for m in meta], world)[rank]
    log.info(f"[rank {rank}/{world}] {len(mine)} of {len(units)} chromosomes: "
             f"{', '.join(meta[u]['chrom'] for u in mine)}")
    if runner is None:
        if device is None:  # torchrun: one rank per GPU (ranks beyond the visible GPUs share them round-robin)
            from .. import _lib
            local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, _lib.lib().nldsc_device_count())
        else:
            local = int(device)
        runner = _default_runner(local)
    from ..core.progress import Progress
    total_snp = sum(meta[u]["bim"].n_snp for u in mine)
    bar = Progress(total_snp, "SNPs", label=f"ld rank {rank}" if world > 1 else "ld", enabled=progress,
                   any_rank=True)
    done_snp = 0
    results = {}
    # a path-fed runner (the engine's own reader) gets the next file read ahead into the page cache;
    # other runners get the bytes, read by a host thread while the current chromosome computes
    by_path = getattr(runner, "wants_path", False)
    pre = None
    if mine and not by_path:
        pre = _Prefetch(meta[mine[0]]["stem"] + ".bed")
    for k, u in enumerate(mine):
        m = meta[u]
        nxt = meta[mine[k + 1]]["stem"] + ".bed" if k + 1 < len(mine) else None
        if by_path:
            bed = m["stem"] + ".bed"
            if nxt is not None:
                threading.Thread(target=_readahead, args=(nxt,), daemon=True).start()
        else:
            bed = pre.get()
            pre = _Prefetch(nxt) if nxt is not None else None
        n_snp = m["bim"].n_snp
        rsq = RSQThreshold(1.0 / n_snp if rsq_thr is None else rsq_thr).data
        t0 = time.perf_counter()
        res, tim = runner(bed, n_snp, m["n_org"], ld_wind_.data, maf_thr_.data, std_thr_.data, rsq, m["pos"], flags)
        ld = _Res(res)
        df = make_output(m["bim"], ld, extra=extra) if out is None else None
        if out is not None:
            path = out.replace("@", m["chrom"])
            write_scores(path, m["bim"], ld, extra=extra)
            if write_m:
                mm, md = m_values(m["bim"], ld)
                write_m_file(str(Path(path).with_suffix(".M")), mm, md)
        results[m["chrom"]] = df
        log.info(f"[rank {rank}] chr{m['chrom']}: M={n_snp} N={m['n_org']} "
                 f"in {time.perf_counter() - t0:.2f} s")
        done_snp += n_snp
        bar.update(done_snp, f"{k + 1}/{len(mine)} chromosomes, chr{m['chrom']} done")
    bar.close(f"{len(mine)} chromosomes")
    return results


class _Res:
    def __init__(self, d: dict):
        for k, v in d.items():
            setattr(self, k, list(v))
