"""Position sharding + gather over torch.distributed (gloo on CPU, world sizes 2 and 3).

The per-rank compute is the C oracle restricted to the rank's owned SNPs (the GPU engine takes its
place on the GPU box); what is tested here is the partition, the ownership contract and the gather.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import load_set


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from nldsc_amd import distributed as D
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bed, pos, meta, orc, _ = load_set(name)
        M = meta["n_snp"]

        def run(own):
            t = np.arange(own[0], own[1], dtype=np.int32)
            part = O.run_c(bed, M, meta["n_org"], meta["ld_wind"], meta["maf"], meta["std_thr"], meta["rsq_thr"],
                           pos, targets=t, threads=1)
            full = {k: (np.full(M, np.nan) if v.dtype.kind == "f" else np.full(M, -1, np.int32))
                    for k, v in part.items()}
            for k in part:
                full[k][own[0]:own[1]] = part[k]
            return full

        res = D.calculate_sharded(run, pos, meta["ld_wind"], M)
        if rank == 0:
            ok = all(np.array_equal(res[k], orc[k], equal_nan=True) for k in orc)
            with open(os.path.join(outdir, "ok"), "w") as fh:
                fh.write("1" if ok else "0")
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "n1001"), (3, "n1003")])
def test_sharded_gather_equals_single_process(world, name):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), name, d), nprocs=world, join=True)
        assert open(os.path.join(d, "ok")).read() == "1"


def test_shard_ranges_cover_and_balance():
    from nldsc_amd import distributed as D
    _, pos, meta, _, _ = load_set("n1000")
    for world in (1, 2, 3, 8):
        r = D.shard_ranges(pos, meta["ld_wind"], world)
        assert r[0][0] == 0 and r[-1][1] == len(pos)
        assert all(a[1] == b[0] for a, b in zip(r[:-1], r[1:]))
        w = D.window_work(pos, meta["ld_wind"])
        loads = [w[a:b].sum() for a, b in r]
        assert max(loads) <= 1.1 * (sum(loads) / world) + w.max()


def test_assign_units_lpt():
    from nldsc_amd import distributed as D
    work = [9, 8, 7, 6, 5, 4, 3, 2, 1]
    a = D.assign_units(work, 3)
    assert sorted(sum(a, [])) == list(range(9))
    loads = [sum(work[u] for u in us) for us in a]
    assert max(loads) <= 4 / 3 * sum(work) / 3  # LPT bound


def test_halo_range_bounds():
    from nldsc_amd import distributed as D
    pos = np.array([0.0, 0.5, 1.0, 1.0, 2.0, 3.5, 4.0, 4.4, 6.0])
    assert D.halo_range(pos, 1.0, (4, 6)) == (2, 8)   # [1.0, 4.5] around owned 2.0 .. 3.5, ties included
    assert D.halo_range(pos, 1.0, (0, 1)) == (0, 4)
    assert D.halo_range(pos, 1.0, (3, 3)) == (3, 3)   # empty owned range: nothing to load
    neg = pos.copy(); neg[5] = -1.0
    assert D.halo_range(neg, 1.0, (4, 6)) == (0, len(pos))  # unused SNP: the reference's pointers need it all
    uns = pos[::-1].copy()
    assert D.halo_range(uns, 1.0, (4, 6)) == (0, len(pos))
    nan = pos.copy(); nan[7] = np.nan  # NaN position: unused for the reference (pos >= 0 is false)
    assert D.halo_range(nan, 1.0, (4, 6)) == (0, len(pos))


@pytest.mark.parametrize("world", [2, 3, 5])
def test_halo_slices_reproduce_full_run(world):
    """What a rank computes on its halo slice (rows [a, b), positions[a:b]) equals the full chromosome's
    result on its owned SNPs — checked with the C oracle, which replays the reference's ChunkwiseReader
    exactly, on sorted non-negative positions (cM, with ties at window edges) and the kb metric."""
    from nldsc_amd import distributed as D
    from nldsc_amd import synth
    from oracle import oracle as O
    N, M = 301, 400
    spec = synth.SynthSpec(n_org=N, n_snp=M, length_cm=9.0, seed=31, missing=0.02, tie_pairs=[50, 220],
                           monomorphic=[7, 300], hom1_het_only=[111])
    rows = synth.pack_bed_rows(synth.genotypes(spec))
    pos = synth.positions_cm(spec)
    bed = synth.bed_bytes(rows)
    args = (1.0, 0.01, 1e-5, 1.0 / M)
    full = O.run_c(bed, M, N, args[0], args[1], args[2], args[3], pos, threads=1)
    for own in D.shard_ranges(pos, args[0], world):
        a, b = D.halo_range(pos, args[0], own)
        assert b - a < M  # a real slice
        part = O.run_c(synth.bed_bytes(rows[a:b]), b - a, N, args[0], args[1], args[2], args[3], pos[a:b],
                       threads=1)
        lo, hi = own
        for k in full:
            np.testing.assert_array_equal(part[k][lo - a:hi - a], full[k][lo:hi], err_msg=f"{own} {k}")


def _halo_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from nldsc_amd import distributed as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sizes = [5, 0, 7, 3][:world]  # halo SNPs each rank sends to the next (the last rank sends none)
        n_send = sizes[rank] if rank + 1 < world else 0
        n_recv = sizes[rank - 1] if rank > 0 else 0
        export = torch.arange(6 * max(n_send, 1), dtype=torch.int64) + 1000 * rank
        imported = torch.full((6 * max(n_recv, 1),), -1, dtype=torch.int64)
        D.exchange_halo(export, n_send, imported, n_recv)
        exp = (torch.arange(6 * n_recv, dtype=torch.int64) + 1000 * (rank - 1)) if n_recv else None
        ok = exp is None or torch.equal(imported[: 6 * n_recv], exp)
        with open(os.path.join(outdir, f"ok{rank}"), "w") as fh:
            fh.write("1" if ok else "0")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_halo_exchange_point_to_point(world):
    """exchange_halo: each rank's exported block reaches the next rank (gloo; an empty send is skipped on both
    sides)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_halo_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        assert all(open(os.path.join(d, f"ok{r}")).read() == "1" for r in range(world))


def test_split_plan_halo_within_next_owned_range():
    """split_plan: owned ranges cover every SNP once, each slice is the owned range plus one window on the right,
    inside the next rank's owned range; unsorted or negative positions (and one-rank runs) give no plan."""
    from nldsc_amd import distributed as D
    rng = np.random.default_rng(1)
    pos = np.cumsum(rng.exponential(0.01, 20_000))
    for world in (2, 3, 8):
        plan = D.split_plan(pos, 1.0, world)
        assert plan is not None and plan[0][0] == 0 and plan[-1][1] == len(pos) == plan[-1][2]
        for g, (lo, hi, b) in enumerate(plan):
            assert lo < hi <= b
            assert b == np.searchsorted(pos, pos[hi - 1] + 1.0 + 1e-9, side="right") or b == hi
            if g + 1 < world:
                assert plan[g + 1][0] == hi and b <= plan[g + 1][1]
    assert D.split_plan(pos, 1.0, 1) is None
    assert D.split_plan(pos[::-1], 1.0, 2) is None
    bad = pos.copy(); bad[10] = -1.0
    assert D.split_plan(bad, 1.0, 2) is None
    assert D.split_plan(pos, 150.0, 8) is None  # windows longer than a rank's range
