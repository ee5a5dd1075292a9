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
