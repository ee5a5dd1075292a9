"""Whole-genome driver (`--bfile chr@`): chromosome expansion, LPT assignment over ranks, per-chromosome
outputs identical to single-chromosome runs.  CPU tests use the oracle as the per-chromosome compute; the
GPU test uses the engine."""
import os

import numpy as np
import pandas as pd
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def genome(tmp_path_factory):
    from nldsc_amd import synth
    d = tmp_path_factory.mktemp("genome")
    sizes = {"1": 300, "2": 180, "5": 90, "22": 40}
    for i, (c, m) in enumerate(sizes.items()):
        synth.write_plink(str(d / f"chr{c}"), synth.SynthSpec(n_org=257, n_snp=m, length_cm=m / 60, seed=40 + i),
                          chrom=int(c))
    return d, sizes


def oracle_runner(bed, n_snp, n_org, w, maf, std_thr, rsq, pos, flags):
    return O.run_c(bed.tobytes(), n_snp, n_org, w, maf, std_thr, rsq, pos, threads=1), {}


def test_expand_bfile(genome):
    from nldsc_amd.ldscore.genome import expand_bfile
    d, sizes = genome
    units = expand_bfile(str(d / "chr@"))
    assert [c for c, _ in units] == ["1", "2", "5", "22"]
    with pytest.raises(Exception):
        expand_bfile(str(d / "chr1"))


@pytest.mark.parametrize("world", [1, 2, 3])
def test_genome_ranks_cover_every_chromosome_once(genome, tmp_path, world):
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    d, sizes = genome
    seen = []
    for rank in range(world):
        res = estimate_lds_genome(str(d / "chr@"), "1", "cm", maf_thr="0.01", std_thr=1e-5, out=str(tmp_path / "o@.L2"),
                                  extra=True, write_m=True, runner=oracle_runner, rank=rank, world=world)
        seen += list(res)
    assert sorted(seen) == sorted(sizes)
    for c, m in sizes.items():
        df = pd.read_csv(tmp_path / f"o{c}.L2", sep="\t")
        assert len(df) == m and (df["CHR"] == int(c)).all()
        assert (tmp_path / f"o{c}.M").exists()


def test_genome_output_equals_single_chromosome_runs(genome, tmp_path):
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    from nldsc_amd.ldscore.routine import make_output
    from nldsc_amd.ldscore.common import BIMFile
    d, sizes = genome
    res = estimate_lds_genome(str(d / "chr@"), "1", "cm", maf_thr="0.01", std_thr=1e-5, extra=True,
                              runner=oracle_runner, rank=0, world=1)
    for c, m in sizes.items():
        bim = BIMFile(str(d / f"chr{c}.bim"))
        bed = open(d / f"chr{c}.bed", "rb").read()
        r = O.run_c(bed, m, 257, 1.0, 0.01, 1e-5, 1.0 / m, bim.cm.to_numpy(np.float64), threads=1)
        exp = make_output(bim, type("R", (), {k: list(v) for k, v in r.items()}), extra=True)
        pd.testing.assert_frame_equal(res[c], exp)


@pytest.mark.gpu
def test_genome_on_gpu_matches_oracle(genome, tmp_path):
    import torch
    torch.cuda.init()
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    d, sizes = genome
    res = estimate_lds_genome(str(d / "chr@"), "1", "cm", maf_thr="0.01", std_thr=1e-5, extra=True, rank=0, world=1,
                              device=0)
    for c, m in sizes.items():
        ref = estimate_lds_genome(str(d / "chr@"), "1", "cm", maf_thr="0.01", std_thr=1e-5, extra=True,
                                  runner=oracle_runner, rank=0, world=1)[c]
        for col in ("WSA", "WSD", "MAF"):
            np.testing.assert_array_equal(res[c][col].to_numpy(), ref[col].to_numpy())
        for col in ("L2", "L2D"):
            np.testing.assert_allclose(res[c][col].to_numpy(), ref[col].to_numpy(), atol=1e-4, equal_nan=True)
