"""Position sharding of the LD-score computation over GPUs (one process per GPU, torch.distributed).

SURVEY.md §8(e): windows are local (1 cM), so a chromosome splits into contiguous SNP ranges with
no exchange on the hot path.  Rank g owns SNPs [lo_g, hi_g) and computes every pair that touches an
owned SNP (the engine recomputes the pairs it shares with the neighbouring ranges — a halo of about
one window — instead of exchanging partial sums).  The per-SNP score tables are then gathered to
rank 0 in one collective (RCCL over xGMI with the "nccl" backend, gloo on CPU).

Whole-genome runs (several chromosome files) assign chromosome units to ranks by longest-processing-
time-first on the estimated pair count (`assign_units`).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np

RESULT_KEYS = ("l2", "l2d", "maf", "residuals_std", "l2_ws", "l2d_ws", "l2d_wse")


def window_work(positions: np.ndarray, ld_wind: float) -> np.ndarray:
    """Estimated in-window neighbours per SNP (two-pointer sweep over sorted used positions)."""
    pos = np.asarray(positions, dtype=np.float64)
    used = pos >= 0
    p = pos[used]
    lo = np.searchsorted(p, p - ld_wind, side="left")
    hi = np.searchsorted(p, p + ld_wind, side="right")
    w = np.zeros(len(pos))
    w[used] = (hi - lo - 1).clip(min=0) + 1.0  # + per-SNP fixed cost
    return w


def shard_ranges(positions: np.ndarray, ld_wind: float, world: int) -> list[tuple[int, int]]:
    """Contiguous SNP ranges with about equal estimated pair work."""
    n = len(positions)
    if world <= 1 or n == 0:
        return [(0, n)]
    c = np.concatenate([[0.0], np.cumsum(window_work(positions, ld_wind))])
    cuts = [0] + [int(np.searchsorted(c, c[-1] * g / world, side="left")) for g in range(1, world)] + [n]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]


def halo_range(positions: np.ndarray, ld_wind: float, own: tuple[int, int]) -> tuple[int, int]:
    """SNP rows [a, b) a GPU loads to compute its owned range [lo, hi): the owned SNPs plus every SNP
    within one window of them.  Exact only when every position is non-negative and
    sorted — then the reference's neighbours of SNP j are exactly the MAF-passing SNPs with
    |pos_k - pos_j| <= w (its ChunkwiseReader pointers, stream.h:131-155,182-197, never lag or stop
    early).  Anything else (unused SNPs with pos < 0, unsorted positions) needs the reference's
    sequential pointer history: load the whole chromosome, (0, n)."""
    pos = np.asarray(positions, dtype=np.float64)
    n = len(pos)
    lo, hi = own
    if hi <= lo:
        return lo, lo
    # `not (pos >= 0)` also catches NaN positions, which the reference treats as unused (is_used: pos >= 0)
    if n == 0 or not (pos >= 0).all() or (np.diff(pos) < 0).any():
        return 0, n
    # a few ulps of slack: the kernels test |pos_k - pos_j| <= w, not pos_k >= pos_j - w (extra rows are harmless)
    eps = 8.0 * np.finfo(np.float64).eps * (float(pos[-1]) + abs(ld_wind))
    a = int(np.searchsorted(pos, pos[lo] - ld_wind - eps, side="left"))
    b = int(np.searchsorted(pos, pos[hi - 1] + ld_wind + eps, side="right"))
    return min(a, lo), max(b, hi)


def empty_result(n_snp: int) -> dict:
    return {k: (np.full(n_snp, np.nan) if k in RESULT_KEYS[:4] else np.full(n_snp, -1, np.int32))
            for k in RESULT_KEYS}


def assign_units(work: Sequence[float], world: int) -> list[list[int]]:
    """LPT: unit indices per rank, heaviest units first onto the least loaded rank."""
    load = np.zeros(world)
    out: list[list[int]] = [[] for _ in range(world)]
    for u in sorted(range(len(work)), key=lambda k: -work[k]):
        g = int(np.argmin(load))
        out[g].append(u)
        load[g] += work[u]
    return out


def gather_spans(own: tuple[int, int], *, device=None) -> list[tuple[int, int]]:
    """Every rank's owned range (one small all_gather; constant for a given sharding, so callers that gather
    repeatedly compute it once)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    span = torch.tensor([own[0], own[1]], dtype=torch.int64, device=device)
    spans = torch.empty(world * 2, dtype=torch.int64, device=device)  # flat: gloo's shape rule
    dist.all_gather_into_tensor(spans, span)
    return [(int(a), int(b)) for a, b in spans.view(world, 2).cpu().tolist()]


def table_width(spans: list[tuple[int, int]]) -> int:
    """Columns of the per-rank score table block: the widest owned range."""
    return max(max((b - a for a, b in spans), default=1), 1)


def assemble(arr: np.ndarray, spans: list[tuple[int, int]], n_snp: int) -> dict:
    """The full result table from the gathered [world, 7, width] block (rank g's columns = its owned SNPs)."""
    full = empty_result(n_snp)
    for g, (a, b) in enumerate(spans):
        for k, key in enumerate(RESULT_KEYS):
            v = arr[g, k, : b - a]
            full[key][a:b] = v if full[key].dtype.kind == "f" else v.astype(np.int32)
    return full


_ASSEMBLY: dict = {}


def _assemble_device(blocks, spans: list[tuple[int, int]], n_snp: int, raw: bool = False, slot: int = 0,
                     sync: bool = True):
    """Rank 0 with RCCL: the gathered [world, 7, width] device block -> the [7, n_snp] table in device memory (one
    strided copy per rank), then one copy into a pinned host buffer (both buffers reused across calls; `slot` picks
    one of several such pairs), so only the table itself crosses PCIe, not every rank's padded block, and no per-key
    host copies follow.  sync=False (raw only): the copies stay queued on the current stream."""
    import torch
    key = (blocks.device, n_snp, slot)
    if key not in _ASSEMBLY:
        for k in [k for k in _ASSEMBLY if k[:2] != key[:2]]:
            del _ASSEMBLY[k]
        _ASSEMBLY[key] = (torch.empty((len(RESULT_KEYS), n_snp), dtype=torch.float64, device=blocks.device),
                          torch.empty((len(RESULT_KEYS), n_snp), dtype=torch.float64, pin_memory=True))
    full, host = _ASSEMBLY[key]
    covered = 0
    for g, (a, b) in enumerate(spans):
        if b > a:
            full[:, a:b].copy_(blocks[g, :, : b - a])
            covered += b - a
    if covered != n_snp:  # (shard_ranges covers every SNP; other span sets leave the rest as not computed)
        own = np.zeros(n_snp, bool)
        for a, b in spans:
            own[a:b] = True
        idx = torch.from_numpy(np.flatnonzero(~own)).to(full.device)
        full[:4, idx] = float("nan")
        full[4:, idx] = -1.0
    host.copy_(full, non_blocking=True)
    if not sync:
        if not raw:
            raise ValueError("sync=False needs raw=True")
        return host.numpy()  # (complete once the current stream has run the copies)
    torch.cuda.current_stream(full.device).synchronize()
    h = host.numpy()
    if raw:  # the [7, n_snp] table itself (a view of the pinned buffer the next gather reuses)
        return h
    # copies: the pinned buffer is reused by the next gather (a caller keeping this dict must not see it change)
    return {k: (h[i].copy() if i < 4 else h[i].astype(np.int32)) for i, k in enumerate(RESULT_KEYS)}


def gather_table(table, spans: list[tuple[int, int]], n_snp: int, *, out=None, raw: bool = False, slot: int = 0,
                 sync: bool = True):
    """One all_gather of every rank's [7, width] fp64 table block (torch tensor; with RCCL it stays in device
    memory and rank 0 assembles the table there before one copy to pinned host memory); the full result dict on
    rank 0, None elsewhere.  `out`: a reusable flat buffer of world * 7 * width elements on the table's device.
    (Rank 0's arrays are its own: the pinned staging buffer reused by the next call is copied out.)  raw (RCCL, rank 0):
    the assembled [7, n_snp] fp64 table as a view of that pinned buffer instead — no host copies per call (the
    strong-scaling bench gathers every step), valid until the next call with the same `slot`.  sync=False (RCCL, raw):
    everything stays queued on the current stream — the caller synchronises it before reading the table (the
    strong-scaling bench gathers step k on a side stream while step k + 1 computes)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    if out is None:
        out = torch.empty(world * table.numel(), dtype=table.dtype, device=table.device)  # flat: gloo's shape rule
    dist.all_gather_into_tensor(out, table.reshape(-1))
    if rank != 0:
        return None
    blocks = out.view((world,) + tuple(table.shape))
    if blocks.is_cuda:
        return _assemble_device(blocks, spans, n_snp, raw=raw, slot=slot, sync=sync)
    return assemble(blocks.numpy(), spans, n_snp)


def gather_ranges(local: dict, own: tuple[int, int], n_snp: int, *, device=None,
                  spans: list[tuple[int, int]] | None = None) -> dict | None:
    """Gather every rank's owned slice of host result arrays; the full table on rank 0, None elsewhere.
    One all_gather of a [world, 7, width] fp64 block (RCCL over xGMI with device tensors, gloo on CPU)."""
    import torch
    spans = gather_spans(own, device=device) if spans is None else spans
    lo, hi = own
    tab = np.full((len(RESULT_KEYS), table_width(spans)), np.nan)
    for k, key in enumerate(RESULT_KEYS):
        tab[k, :hi - lo] = np.asarray(local[key][lo:hi], dtype=np.float64)
    t = torch.from_numpy(tab)
    if device is not None:
        t = t.to(device, non_blocking=False)
    return gather_table(t, spans, n_snp)


def calculate_sharded(load_and_run: Callable[[tuple[int, int]], dict], positions: np.ndarray, ld_wind: float,
                      n_snp: int, *, device=None) -> dict | None:
    """Run `load_and_run(own_range) -> result dict` on this rank's range and gather to rank 0."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    own = shard_ranges(positions, ld_wind, world)[rank]
    local = load_and_run(own)
    return gather_ranges(local, own, n_snp, device=device)


def calculate_sharded_device(bed_path: str, n_snp: int, n_org: int, ld_wind: float, maf: float, std_thr: float,
                             rsq_thr: float, positions: np.ndarray, *, flags: int = 0, device: int = 0) -> dict | None:
    """The RCCL path of `calculate_sharded` + `engine_runner`: this rank's engine reads its halo_range of the .bed,
    writes its owned slice of the score table straight into a device block (nldsc_engine_run_device), and the
    blocks are gathered device to device; only rank 0's gathered table crosses to the host."""
    import torch
    import torch.distributed as dist
    from .engine import Engine
    world, rank = dist.get_world_size(), dist.get_rank()
    pos = np.asarray(positions, dtype=np.float64)
    own = shard_ranges(pos, ld_wind, world)[rank]
    dev = torch.device(f"cuda:{device}")
    spans = gather_spans(own, device=dev)
    tab = torch.full((len(RESULT_KEYS), table_width(spans)), float("nan"), dtype=torch.float64, device=dev)
    lo, hi = own
    if hi > lo:
        a, b = halo_range(pos, ld_wind, own)
        with Engine(device) as e:
            e.load_bed_file_range(bed_path, n_snp, n_org, a, b)
            e.run_device(ld_wind, maf, std_thr, rsq_thr, pos[a:b], tab, own=(lo - a, hi - a), flags=flags)
    return gather_table(tab, spans, n_snp)


def split_plan(positions: np.ndarray, ld_wind: float, world: int) -> list[tuple[int, int, int]] | None:
    """Per rank (lo, hi, b) for split runs — the owned range [lo, hi) and the loaded slice [lo, b), its right halo
    one window past hi — when each boundary pair can be computed once, by the rank owning its lower SNP: positions
    non-negative and sorted (so the windows are the reference's neighbour sets) and every right halo inside the next
    rank's owned range (it then receives the halo's sums).  None otherwise (the ranks then load a two-sided halo and
    compute boundary pairs twice)."""
    pos = np.asarray(positions, dtype=np.float64)
    n = len(pos)
    if world <= 1 or n == 0 or not (pos >= 0).all() or (np.diff(pos) < 0).any():
        return None
    ranges = shard_ranges(pos, ld_wind, world)
    out = []
    for g, (lo, hi) in enumerate(ranges):
        if hi <= lo:
            return None
        b = halo_range(pos, ld_wind, (lo, hi))[1]
        if g + 1 < world and b > ranges[g + 1][1]:
            return None
        out.append((lo, hi, b))
    return out


def exchange_halo(export, n_send: int, imported, n_recv: int):
    """Send this rank's exported halo block ([6][n_send] int64) to the next rank and receive the previous rank's
    ([6][n_recv]) — point to point (RCCL over xGMI with device tensors; gloo with CPU tensors: a device export is
    staged through the host)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    send, recv = export[: 6 * n_send], imported[: 6 * n_recv]
    host = dist.get_backend() == "gloo"
    if host:
        send, recv_h = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)
    ops = []
    if rank + 1 < world and n_send > 0:
        ops.append(dist.P2POp(dist.isend, send, rank + 1))
    if rank > 0 and n_recv > 0:
        ops.append(dist.P2POp(dist.irecv, recv_h if host else recv, rank - 1))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if host and rank > 0 and n_recv > 0:
        recv.copy_(recv_h)
    if recv.is_cuda:
        # with RCCL, wait() only makes torch's current stream wait for the receive; the engine reads `imported` on
        # its own stream, so the host waits here (also done by Engine.run_device_finish)
        torch.cuda.current_stream(recv.device).synchronize()


def calculate_sharded_split(bed_path: str, n_snp: int, n_org: int, ld_wind: float, maf: float, std_thr: float,
                            rsq_thr: float, positions: np.ndarray, plan: list[tuple[int, int, int]], *, flags: int = 0,
                            device: int = 0) -> dict | None:
    """The sharded CLI run with each boundary pair computed once (`split_plan`): this rank loads [lo, b) of the .bed,
    runs the first half of a split run, sends its right halo's sums to the next rank, adds the previous rank's, and
    finishes; the score-table blocks are then gathered as in calculate_sharded_device."""
    import torch
    import torch.distributed as dist
    from .engine import Engine
    world, rank = dist.get_world_size(), dist.get_rank()
    pos = np.asarray(positions, dtype=np.float64)
    lo, hi, b = plan[rank]
    n_recv = plan[rank - 1][2] - plan[rank - 1][1] if rank > 0 else 0
    dev = torch.device(f"cuda:{device}")
    coll = dev if dist.get_backend() != "gloo" else None
    spans = gather_spans((lo, hi), device=coll)
    tab = torch.full((len(RESULT_KEYS), table_width(spans)), float("nan"), dtype=torch.float64, device=dev)
    export = torch.empty(6 * max(b - hi, 1), dtype=torch.int64, device=dev)
    imported = torch.empty(6 * max(n_recv, 1), dtype=torch.int64, device=dev)
    with Engine(device) as e:
        e.load_bed_file_range(bed_path, n_snp, n_org, lo, b)
        n_send = e.run_device_split(ld_wind, maf, std_thr, rsq_thr, pos[lo:b], tab, export, own=(0, hi - lo),
                                    flags=flags)
        exchange_halo(export, n_send, imported, n_recv)
        e.run_device_finish(imported, n_recv)
    return gather_table(tab if coll is not None else tab.cpu(), spans, n_snp)


def engine_runner(bed_path: str, n_snp: int, n_org: int, ld_wind: float, maf: float, std_thr: float,
                  rsq_thr: float, positions: np.ndarray, *, flags: int = 0, device: int = 0):
    """`load_and_run` for calculate_sharded backed by this rank's GPU engine: the rank reads only its
    `halo_range` of the .bed (one window around its owned SNPs) and computes the owned SNPs on that
    slice; rsq_thr stays the whole chromosome's (1/M)."""
    pos = np.asarray(positions, dtype=np.float64)

    def run(own):
        from .engine import Engine
        res = empty_result(n_snp)
        lo, hi = own
        if hi <= lo:
            return res
        a, b = halo_range(pos, ld_wind, own)
        with Engine(device) as e:
            e.load_bed_file_range(bed_path, n_snp, n_org, a, b)
            part = e.run(ld_wind, maf, std_thr, rsq_thr, pos[a:b], own=(lo - a, hi - a), flags=flags)
        for k in RESULT_KEYS:
            res[k][lo:hi] = part[k][lo - a:hi - a]
        return res
    return run
