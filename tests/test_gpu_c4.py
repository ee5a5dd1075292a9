"""C4 (BASELINE.json configs[3]) at full N: 22 autosome PLINK sets of N = 315 599 individuals through the
whole-genome driver (`--bfile chr@`, nldsc_amd/ldscore/genome.py), the reference's one-chromosome-per-file
contract (nldsc/ldscore/common.py:114-117) repeated over the genome by its caller's logic
(nldsc/ldscore/routine.py:51-102, ldscalc.h:34-54 per chromosome).

M_c is proportional to each autosome's genetic length (200-400 SNPs per file, 1 % missing calls) at C4's SNP
density (600 000 SNPs over the 3 570 cM of the autosomes: ~340 neighbours per SNP at --ld-wind-cm 1), so the
windows have C4's size while the files stay small (24-32 MB each).  Checked:
  * one rank, in process: >= 8 targets per chromosome (both ends, where the windows are one-sided, and the
    edges of two 32-SNP blocks mid-chromosome) against the oracle's targets mode and the exact fp64 truth, with
    conftest.TOL and exact window counts; every SNP of every chromosome by invariants;
  * two ranks (torchrun, gloo: both ranks on this box's GPU), chromosome units assigned by LPT: every output
    file byte-identical to the one-rank run's.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, assert_ld_close, max_errors, progress, record
from oracle import oracle as O

pytestmark = pytest.mark.gpu

N = 315_599
# approximate sex-averaged genetic map lengths of the 22 autosomes (cM), as bench.py's C4 workload
AUTOSOME_CM = [278, 263, 224, 214, 209, 193, 184, 169, 167, 181, 158, 174, 126, 119, 141, 134, 128, 117, 108, 108,
               63, 72]
DENSITY = 600_000 / sum(AUTOSOME_CM)  # C4 SNPs per cM
ARGS = dict(ld_wind=1.0, maf=1e-4, std_thr=1e-5)


def c4_sizes() -> list[int]:
    L = np.asarray(AUTOSOME_CM, float)
    return [int(m) for m in np.maximum(200, np.round(400 * L / L.max()))]


def targets(m: int) -> np.ndarray:
    mid = 32 * (m // 64)
    t = {0, 1, 31, 32, mid - 1, mid, mid + 31, mid + 32, m - 2, m - 1}
    return np.array(sorted(x for x in t if 0 <= x < m), np.int32)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def c4(tmp_path_factory):
    import torch
    torch.cuda.init()
    from nldsc_amd import synth
    d = tmp_path_factory.mktemp("c4")
    fam = "".join(f"F{i}\tI{i}\t0\t0\t{1 + (i & 1)}\t-9\n" for i in range(N))
    data = {}
    for c, m in enumerate(c4_sizes(), start=1):
        buf, pos = synth.device_bed(m, N, seed=500 + c, length_cm=m / DENSITY, missing=0.01)
        bed = buf.cpu().numpy().tobytes()
        del buf
        stem = d / f"chr{c}"
        stem.with_suffix(".bed").write_bytes(bed)
        bp = np.round(pos * 1e6).astype(np.int64)
        stem.with_suffix(".bim").write_text("".join(f"{c}\trs{c}_{j + 1}\t{pos[j]:.6f}\t{bp[j]}\tA\tG\n"
                                                    for j in range(m)))
        stem.with_suffix(".fam").write_text(fam)
        data[c] = (bed, pos)
    progress(f"c4 fixture: {len(data)} chromosome files written")
    return d, data


def _columns(df) -> dict:
    return dict(l2=df["L2"].to_numpy(np.float64), l2d=df["L2D"].to_numpy(np.float64),
                maf=df["MAF"].to_numpy(np.float64), residuals_std=df["RSTD"].to_numpy(np.float64),
                l2_ws=df["WSA"].to_numpy(np.int32), l2d_ws=df["WSD"].to_numpy(np.int32),
                l2d_wse=df["WSDE"].to_numpy(np.int32))


def test_c4_genome_one_rank_vs_oracle_and_truth(c4):
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    d, data = c4
    res = estimate_lds_genome(str(d / "chr@"), ARGS["ld_wind"], "cm", maf_thr=ARGS["maf"], std_thr=ARGS["std_thr"],
                              extra=True, rank=0, world=1, device=0, progress=False)
    assert sorted(res, key=int) == [str(c) for c in data]
    report = {}
    for c, (bed, pos) in data.items():
        m = len(pos)
        got = _columns(res[str(c)])
        t = targets(m)
        args = (ARGS["ld_wind"], ARGS["maf"], ARGS["std_thr"], 1.0 / m)
        exp = O.run_c(bed, m, N, *args, pos, targets=t, flags=O.NO_COPIES)
        rows = np.frombuffer(bed, np.uint8, offset=3).reshape(m, -1)
        truth = O.run_f64_targets(rows, N, *args, pos, t, bed=bed)
        sub = {k: v[t] for k, v in got.items()}
        report[c] = dict(n_snp=m, targets=t.tolist(), gpu_vs_oracle=max_errors(sub, exp),
                         gpu_vs_truth=max_errors(sub, truth))
        assert_ld_close(sub, truth, label=f"chr{c} vs fp64 truth")
        assert_ld_close(sub, exp, label=f"chr{c} vs oracle")
        for k in ("l2", "l2d"):  # exact integer Gram + fp64 epilogue
            assert np.max(np.abs(sub[k] - truth[k])) < 1e-8, (c, k)
        for k in ("l2_ws", "l2d_ws", "l2d_wse"):
            np.testing.assert_array_equal(sub[k], truth[k], err_msg=f"chr{c} {k}")
        # every SNP: C4-sized windows, finite scores, L2 >= 1 - a rounding margin of the adjusted r^2
        assert np.isfinite(got["l2"]).all() and np.isfinite(got["l2d"]).all()
        assert (got["l2_ws"] > 100).all() and got["l2_ws"].max() >= min(250, m - 1), c
        assert (got["l2d_ws"] <= got["l2_ws"]).all() and (got["l2d_wse"] <= got["l2d_ws"]).all()
        progress(f"c4 chr{c}: {m} SNPs checked")
    record("c4_genome", report)


def test_c4_genome_two_ranks_equal_one_rank(c4, tmp_path):
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    d, data = c4
    estimate_lds_genome(str(d / "chr@"), ARGS["ld_wind"], "cm", maf_thr=ARGS["maf"], std_thr=ARGS["std_thr"],
                        out=str(tmp_path / "one_@.L2"), extra=True, write_m=True, rank=0, world=1, device=0,
                        progress=False)
    env = dict(os.environ, NLDSC_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "nldsc_amd", "ld", "--bfile", str(d / "chr@"),
           "--ld-wind-cm", "1", "-maf", "1e-4", "--std-thr", "1e-5", "--extra", "--write-m",
           "--out", str(tmp_path / "two_@.L2")]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0 and "crashed" not in p.stderr, p.stderr[-3000:]
    assert "ld rank 0" in p.stderr and "ld rank 1" in p.stderr
    for c in data:
        one, two = tmp_path / f"one_{c}.L2", tmp_path / f"two_{c}.L2"
        assert two.read_bytes() == one.read_bytes(), f"chr{c}"
        assert (tmp_path / f"two_{c}.M").read_text() == (tmp_path / f"one_{c}.M").read_text()
