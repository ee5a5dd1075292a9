"""The torchrun paths of the CLI on the GPU: two ranks, each with its own engine on its
GPU share (both on GPU 0 when the box has one: $NLDSC_DIST_BACKEND=gloo), the one chromosome position-sharded
(halo reads, owned ranges) and the table gathered on rank 0; and the whole-genome mode with chromosome units
over the ranks.  Compared with the single-process run of the same command.  Exercises the import order of
the torchrun path (torch before _ldscore, nldsc_amd/ldscore/__init__.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ld(args, *, ranks=1, env_extra=None, timeout=300):
    env = dict(os.environ, NLDSC_DIST_BACKEND="gloo", **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    if ranks > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "nldsc_amd", "ld"] + args
    else:
        cmd = [sys.executable, "-m", "nldsc_amd", "ld"] + args
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0 and "crashed" not in p.stderr, p.stderr[-3000:]
    return p


def _same_table(a, b):
    x, y = pd.read_csv(a, sep="\t"), pd.read_csv(b, sep="\t")
    assert list(x.columns) == list(y.columns) and len(x) == len(y)
    for c in x.columns:
        if x[c].dtype.kind in "iuO":
            assert x[c].equals(y[c]), c
        else:  # the fp64 sums differ only in addition order: %.5f text equal up to a rounding tie
            np.testing.assert_allclose(x[c], y[c], atol=1.1e-5, rtol=0, equal_nan=True, err_msg=c)


@pytest.mark.parametrize("name", ["n1001", "n1003"])
def test_torchrun_one_chromosome_two_ranks(tmp_path, name):
    common = ["--bfile", os.path.join(GOLDEN, name), "--ld-wind-cm", "1", "-maf", "0.01", "--extra", "--write-m"]
    _ld(common + ["--out", str(tmp_path / "one.L2")])
    p = _ld(common + ["--out", str(tmp_path / "two.L2")], ranks=2)
    _same_table(tmp_path / "one.L2", tmp_path / "two.L2")
    assert (tmp_path / "two.M").read_text() == (tmp_path / "one.M").read_text()
    assert "SNP pairs" in p.stderr  # progress line (rank 0)


def test_torchrun_whole_genome_two_ranks(tmp_path):
    from nldsc_amd import synth
    for c, (m, n) in {1: (900, 1003), 2: (700, 1003), 3: (500, 1003)}.items():
        synth.write_plink(str(tmp_path / f"chr{c}"), synth.SynthSpec(n_org=n, n_snp=m, length_cm=6.0, seed=c),
                          chrom=c)
    common = ["--bfile", str(tmp_path / "chr@"), "--ld-wind-cm", "1", "-maf", "0.01", "--extra"]
    _ld(common + ["--out", str(tmp_path / "one_@.L2")])
    p = _ld(common + ["--out", str(tmp_path / "two_@.L2")], ranks=2)
    for c in (1, 2, 3):
        _same_table(tmp_path / f"one_{c}.L2", tmp_path / f"two_{c}.L2")
    assert "ld rank 0" in p.stderr and "ld rank 1" in p.stderr  # each rank reports its own chromosomes


RCCL_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {repo!r})
import numpy as np
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
from nldsc_amd import distributed as D
from nldsc_amd.ldscore import _ldscore as lds
from nldsc_amd.ldscore.common import PLINKFile
bed, bim, fam = PLINKFile.parse({bfile!r})
pos = np.asarray(bim.cm, dtype=np.float64)
full = D.calculate_sharded_device(bed.data, bim.n_snp, fam.n_org, 1.0, 0.01, 1e-5, 1.0 / bim.n_snp, pos, device=0)
p = lds.LDScoreParams(bed.data, n_snp=bim.n_snp, n_org=fam.n_org, ld_wind=1.0, maf=0.01, std_thr=1e-5,
                      rsq_thr=1.0 / bim.n_snp, positions=pos.tolist())
one = lds.calculate(p)
out = {{}}
for k in D.RESULT_KEYS:
    a, b = np.asarray(full[k], dtype=np.float64), np.asarray(getattr(one, k), dtype=np.float64)
    out[k] = bool(np.array_equal(a, b, equal_nan=True))
print(json.dumps(out), flush=True)
dist.destroy_process_group()
'''


def test_rccl_device_gather_one_rank(tmp_path):
    """The RCCL ("nccl") branch of the sharded CLI path, which the 2-rank tests above (gloo: ranks share the one GPU)
    do not reach: a process group of one over RCCL, the owned score-table block written on the device
    (nldsc_engine_run_device), gather_spans / all_gather_into_tensor on device tensors, rank 0's copy to the host.
    Equal bit for bit to the single-process `calculate` (one rank owns every SNP)."""
    import json
    script = tmp_path / "rccl1.py"
    script.write_text(RCCL_SCRIPT.format(repo=REPO, bfile=os.path.join(GOLDEN, "n1003")))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert all(d.values()), d


def test_bench_force_dist_rccl_one_rank():
    """`bench.py --force-dist`: the strong-scaling bench's N-GPU code (process group, owned range + halo, device
    table, RCCL gather every step, max-over-ranks timing) run as a group of one on the one GPU.  The line records the
    RCCL group it saw (rccl_world) and, in the overlapped mode, each step's gather timed with HIP events on its side
    stream (gather_ms: the all-gather, assembly and D2H on the GPU), the host's wait for an earlier gather and the
    enqueue time apart (verdict r04: gather_ms used to time the enqueue only)."""
    import json
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    def bench(*extra):
        p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu", "--no-file", "--steps", "3",
                            "--warmup", "1", "--n-snp", "6000", "--n-org", "20000", "--length-cm", "21", "--no-extra",
                            *extra],
                           cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    d = bench("--force-dist")
    assert d["n_gpus"] == 1 and d["value"] > 0 and "RCCL" in d["config"]["parallelism"], d
    assert "side stream" in d["config"]["parallelism"], d  # each step's gather beside the next step's compute
    assert d["stages_ms"]["gather_ms"] > 0 and d["per_rank"][0]["owned_snps"] == 6000
    r0 = d["per_rank"][0]
    assert d["rccl_world"] == 1 and d["collectives_backend"] == "nccl", d
    assert r0["gather_ms"] > 0 and r0["gather_enqueue_ms"] > 0 and r0["gather_wait_ms"] >= 0 and "gather_note" in d, r0
    # the overlapped gather, the sequential one and the one-process run: the same table
    seq, one = bench("--force-dist", "--no-gather-overlap"), bench()
    assert "side stream" not in seq["config"]["parallelism"], seq
    assert d["table_digest"] == seq["table_digest"] == one["table_digest"], (d["table_digest"], seq["table_digest"],
                                                                              one["table_digest"])


def test_bench_default_line_records_and_rehearsal():
    """The default one-GPU bench line carries its extra records after the timed region (fp32_path: the fp32 MFMA
    path on the same rows, its window counts equal to the default path's; oneshot_gpu_ms: load + run), and a
    rehearsal of one rank of 8 (`--rehearse 0/8`, a split run whose host result is the owned slice alone) skips them."""
    import json
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    def bench(*extra):
        p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu", "--no-file", "--steps", "2",
                            "--warmup", "1", "--n-snp", "6000", "--n-org", "20000", "--length-cm", "21", *extra],
                           cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-3000:]
        return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    d = bench()
    f = d["fp32_path"]
    assert f["band_ms"] > 0 and 0 < f["frac"] < 1 and f["vs_default_path"]["l2_ws_equal"], f
    assert f["vs_default_path"]["l2d_ws_equal"] and f["vs_default_path"]["l2_max_abs_diff"] < 1e-3, f
    o = d["oneshot_gpu_ms"]
    assert o["load"] > 0 and o["run"] > 0 and abs(o["total"] - o["load"] - o["run"]) < 0.01, o
    r = bench("--rehearse", "0/8")
    assert "fp32_path" not in r and "oneshot_gpu_ms" not in r and r["value"] > 0, r


SPLIT_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {repo!r})
import numpy as np
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("gloo")
from nldsc_amd import distributed as D
from nldsc_amd.ldscore import _ldscore as lds
from nldsc_amd.ldscore.common import PLINKFile
bed, bim, fam = PLINKFile.parse({bfile!r})
pos = np.asarray(bim.cm, dtype=np.float64)
M, N, w = bim.n_snp, fam.n_org, 1.0
args = (bed.data, M, N, w, 1e-4, 1e-5, 1.0 / M)
plan = D.split_plan(pos, w, dist.get_world_size())
assert plan is not None
split = D.calculate_sharded_split(*args, pos, plan, device=0)
dup = D.calculate_sharded(D.engine_runner(*args, pos, device=0), pos, w, M)
if dist.get_rank() == 0:
    p = lds.LDScoreParams(bed.data, n_snp=M, n_org=N, ld_wind=w, maf=1e-4, std_thr=1e-5, rsq_thr=1.0 / M,
                          positions=pos.tolist())
    one = lds.calculate(p)
    out = dict(plan=plan)
    for k in D.RESULT_KEYS:
        a = np.asarray(split[k], dtype=np.float64)
        refs = (np.asarray(dup[k], dtype=np.float64), np.asarray(getattr(one, k), dtype=np.float64))
        if k in ("l2", "l2d"):  # fp64 partial sums per work item: the block grid is relative to each slice
            out[k] = [bool(np.allclose(a, r, rtol=1e-12, atol=1e-12, equal_nan=True)) for r in refs]
        else:
            out[k] = [bool(np.array_equal(a, r, equal_nan=True)) for r in refs]
    print(json.dumps(out), flush=True)
dist.destroy_process_group()
'''


@pytest.mark.parametrize("ranks", [2, 3])
def test_split_halo_equals_duplicate_halo_and_one_process(tmp_path, ranks):
    """Boundary pairs computed once (split runs: each rank loads its owned range + right halo, sends the halo's
    fixed-point sums to the next rank, point to point) give the two-sided-halo results and the one-process `calculate`:
    the window counts, MAF and residual std bitwise, L2 / L2D to 1e-12 (each work item's fp64 partial sums group the
    pairs by the 32-SNP block grid, which starts at each rank's slice; gloo ranks sharing the one GPU; N = 20 011,
    6 000 SNPs over 9 cM, 1 % missing)."""
    import json
    from nldsc_amd import synth
    synth.write_plink(str(tmp_path / "chr1"), synth.SynthSpec(n_org=20_011, n_snp=6000, length_cm=9.0, seed=17,
                                                                missing=0.01), chrom=1)
    script = tmp_path / "split.py"
    script.write_text(SPLIT_SCRIPT.format(repo=REPO, bfile=str(tmp_path / "chr1")))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert len(d.pop("plan")) == ranks
    assert all(a and b for a, b in d.values()), d


EIGHT_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {repo!r})
import numpy as np
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("gloo")
from nldsc_amd import distributed as D
from nldsc_amd.ldscore import _ldscore as lds
from nldsc_amd.ldscore.common import PLINKFile
bed, bim, fam = PLINKFile.parse({bfile!r})
pos = np.asarray(bim.cm, dtype=np.float64)
M, N, w = bim.n_snp, fam.n_org, 1.0
args = (bed.data, M, N, w, 1e-4, 1e-5, 1.0 / M)
own = D.shard_ranges(pos, w, dist.get_world_size())[dist.get_rank()]
full = D.calculate_sharded(D.engine_runner(*args, pos, device=0), pos, w, M)
owned = [torch.zeros(2, dtype=torch.int64) for _ in range(dist.get_world_size())]
dist.all_gather(owned, torch.tensor(own, dtype=torch.int64))
if dist.get_rank() == 0:
    p = lds.LDScoreParams(bed.data, n_snp=M, n_org=N, ld_wind=w, maf=1e-4, std_thr=1e-5, rsq_thr=1.0 / M,
                          positions=pos.tolist())
    one = lds.calculate(p)
    out = dict(spans=[t.tolist() for t in owned])
    for k in D.RESULT_KEYS:
        a, r = np.asarray(full[k], dtype=np.float64), np.asarray(getattr(one, k), dtype=np.float64)
        if k in ("l2", "l2d"):  # each rank's 32-SNP block grid starts at its halo slice: fp64 sums regrouped
            out[k] = bool(np.allclose(a, r, rtol=1e-12, atol=1e-12, equal_nan=True))
        else:
            out[k] = bool(np.array_equal(a, r, equal_nan=True))
    print(json.dumps(out), flush=True)
dist.destroy_process_group()
'''


def test_eight_gloo_ranks_gathered_table_equals_one_process(tmp_path):
    """The metric's largest rank count (8) through the sharded path on one GPU (gloo ranks sharing it): each rank
    loads its owned range + halo from the .bed, computes its owned SNPs, the table is gathered on rank 0 and equals
    the one-process `calculate` (window counts, MAF, residual std bitwise; L2 / L2D to 1e-12); the 8 owned ranges
    tile [0, M).  N = 20 011, 6 000 SNPs over 9 cM, 1 % missing."""
    import json
    from nldsc_amd import synth
    synth.write_plink(str(tmp_path / "chr1"), synth.SynthSpec(n_org=20_011, n_snp=6000, length_cm=9.0, seed=23,
                                                                missing=0.01), chrom=1)
    script = tmp_path / "eight.py"
    script.write_text(EIGHT_SCRIPT.format(repo=REPO, bfile=str(tmp_path / "chr1")))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    spans = d.pop("spans")
    assert len(spans) == 8 and spans[0][0] == 0 and spans[-1][1] == 6000
    assert all(spans[g][1] == spans[g + 1][0] for g in range(7)) and all(b > a for a, b in spans), spans
    assert all(d.values()), d


def _bench(args, timeout=600):
    import json
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def test_bench_eight_gloo_ranks_equals_one_gpu():
    """`bench.py --gpus 8` (the metric's 8-GPU command, its ranks started by bench.py itself) rehearsed with 8 gloo
    ranks on the one GPU: n_gpus 8, one per_rank entry per rank, owned SNPs tiling the chromosome, and the gathered
    score table equal to the 1-GPU run of the same synthetic chromosome (window counts bitwise, L2 / L2D sums to
    1e-9 relative)."""
    small = ["--no-cpu", "--no-file", "--steps", "2", "--warmup", "1", "--n-snp", "6000", "--n-org", "20000",
             "--length-cm", "21"]
    one = _bench(["--gpus", "1"] + small)
    eight = _bench(["--gpus", "8", "--backend", "gloo"] + small)
    assert eight["n_gpus"] == 8 and eight["scaling"] == "strong" and eight["value"] > 0, eight
    pr = eight["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8)) and sum(r["owned_snps"] for r in pr) == 6000, pr
    a, b = one["table_digest"], eight["table_digest"]
    assert a["counts_sha16"] == b["counts_sha16"] and a["n_snp"] == b["n_snp"] == 6000, (a, b)
    for k in ("l2_sum", "l2d_sum"):
        assert abs(a[k] - b[k]) <= 1e-9 * abs(a[k]), (k, a[k], b[k])
