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
