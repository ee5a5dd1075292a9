"""The host layer (nldsc_amd.ldscore.common / routine, CLI) against vectors produced by the
reference's own Python (tests/golden/reference_python.json, tests/golden/make_golden.py): the
LDScoreParams it hands to `calculate`, the TSV it writes, and its validation errors."""
import hashlib
import json
import os
import subprocess
import sys
import types

import numpy as np
import pytest

from conftest import GOLDEN, REPO

REF = json.load(open(os.path.join(GOLDEN, "reference_python.json")))


class _Recorder:
    def __init__(self, result):
        from nldsc_amd.ldscore import _ldscore
        self.real = _ldscore
        self.result = result
        self.params = None
        self.LDScoreParams = _ldscore.LDScoreParams
        self.LDScoreResult = _ldscore.LDScoreResult

    def calculate(self, params):
        self.params = params
        r = self.real.LDScoreResult()
        for k, v in self.result.items():
            setattr(r, k, v.tolist())
        return r


@pytest.mark.parametrize("sc", REF["scenarios"], ids=[s["set"] for s in REF["scenarios"]])
def test_estimate_lds_matches_reference_python(sc, tmp_path, monkeypatch):
    from nldsc_amd.ldscore import routine
    name = sc["set"]
    orc = dict(np.load(os.path.join(GOLDEN, name + ".oracle.npz")))
    rec = _Recorder(orc)
    monkeypatch.setattr(routine, "lds", rec)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / (name + ".L2")
    a = sc["args"]
    routine.estimate_lds(os.path.join(GOLDEN, name), ld_wind=a["ld_wind"], wind_metric=a["wind_metric"],
                         maf_thr=a["maf_thr"], std_thr=a["std_thr"], rsq_thr=a["rsq_thr"], out=str(out),
                         extra=a["extra"], summary=False)
    p, e = rec.params, sc["params"]
    assert os.path.basename(p.bedfile) == e["bfile_basename"]
    assert (p.n_snp, p.n_org) == (e["n_snp"], e["n_org"])
    assert (p.ld_wind, p.maf, p.std_thr, p.rsq_thr) == (e["ld_wind"], e["maf"], e["std_thr"], e["rsq_thr"])
    pos = np.asarray(p.positions, dtype=np.float64)
    assert len(pos) == e["positions_len"]
    assert hashlib.sha256(pos.tobytes()).hexdigest() == e["positions_sha256"]
    text = out.read_text()
    assert text == open(os.path.join(GOLDEN, sc["tsv_file"])).read()
    assert hashlib.sha256(text.encode()).hexdigest() == sc["tsv_sha256"]


@pytest.mark.parametrize("case", REF["errors"], ids=[f"{c['cls']}{c['args']}" for c in REF["errors"]])
def test_validation_errors_match_reference(case):
    from nldsc_amd.ldscore import common
    cls = getattr(common, case["cls"])
    if case["error"] is None:
        cls(*case["args"])
        return
    with pytest.raises(Exception) as ei:
        cls(*case["args"])
    assert type(ei.value).__name__ == case["error"]
    assert str(ei.value) == case["message"]


def test_bim_single_chromosome(tmp_path):
    from nldsc_amd.ldscore.common import BIMFile, NLDSCParameterError
    f = tmp_path / "x.bim"
    f.write_text("1\trs1\t0.1\t100\tA\tG\n2\trs2\t0.2\t200\tA\tG\n")
    with pytest.raises(NLDSCParameterError, match="one chromosome"):
        BIMFile(str(f))


def test_parse_accepts_any_of_the_three_files():
    from nldsc_amd.ldscore.common import PLINKFile
    for ext in ("", ".bed", ".bim", ".fam"):
        bed, bim, fam = PLINKFile.parse(os.path.join(GOLDEN, "n1000" + ext))
        assert bed.data.endswith("n1000.bed") and bim.n_snp == 1200 and fam.n_org == 1000


def test_m_file_values(tmp_path):
    from nldsc_amd.ldscore import routine
    from nldsc_amd.ldscore.common import BIMFile
    orc = dict(np.load(os.path.join(GOLDEN, "n1000.oracle.npz")))
    ld = types.SimpleNamespace(**{k: v.tolist() for k, v in orc.items()})
    m, md = routine.m_values(BIMFile(os.path.join(GOLDEN, "n1000.bim")), ld)
    import pandas as pd
    ref = pd.read_csv(os.path.join(GOLDEN, "n1000.ref.L2"), sep="\t")
    sc = ref.sort_values(by=["CHR", "BP"]).dropna().drop_duplicates(subset="SNP")
    assert m == len(sc) and md == int(len(sc) * (sc["WSDE"] / sc["WSA"]).mean())


def test_cli_requires_exactly_one_window():
    r = subprocess.run([sys.executable, "-m", "nldsc_amd", "ld", "--bfile", os.path.join(GOLDEN, "n1000"),
                        "-maf", "0.01"], cwd=REPO, capture_output=True, text=True, timeout=120)
    assert "Please, specify exactly one --ld-wind option" in r.stderr
    assert "The program crashed with RuntimeError" in r.stderr


def test_native_tsv_writer_is_byte_identical_to_pandas(tmp_path):
    """nldsc_format_scores (the CLI's writer) against make_output(...).to_csv(sep="\\t", float_format="%.5f")
    on awkward values: NaN, -0.0, rounding ties at the 5th decimal, huge and tiny magnitudes, inf, -1
    window sizes, string and integer chromosome columns."""
    import pandas as pd

    from nldsc_amd.ldscore.common import BIMFile
    from nldsc_amd.ldscore.routine import format_scores, make_output
    rng = np.random.default_rng(3)
    n = 5000
    for chrom in ("7", "X", "NA-ids"):
        path = tmp_path / f"t{chrom}.bim"
        with open(path, "w") as fh:
            for i in range(n):
                # pandas' default na_values read SNP ids such as 'NA' / 'NULL' as NaN (an object column with nulls)
                snp = ("NA" if i % 7 == 0 else "NULL" if i % 11 == 0 else f"rs{i}") if chrom == "NA-ids" else f"rs{i}"
                fh.write(f"{chrom if chrom != 'NA-ids' else '3'}\t{snp}\t{i * 0.001:.6f}\t{1000 + 37 * i}\tA\tG\n")
        bim = BIMFile(str(path))

        class LD:
            pass
        ld = LD()
        vals = rng.normal(0, 50, (4, n))
        special = np.array([np.nan, -0.0, 0.0, 1.000005, 2.500005, -1e-7, 1e300, -1e300, np.inf, 0.123455,
                            1234567.891234, 5e-6, -5e-6, 4.9999999e-6])
        vals[:, :len(special)] = special
        ld.l2, ld.l2d, ld.maf, ld.residuals_std = (list(v) for v in vals)
        ws = rng.integers(-1, 700, (3, n)).astype(np.int32)
        ld.l2_ws, ld.l2d_ws, ld.l2d_wse = (list(int(x) for x in w) for w in ws)
        for extra in (False, True):
            ref = make_output(bim, ld, extra=extra).to_csv(sep="\t", index=False, float_format="%.5f").encode()
            assert format_scores(bim, ld, extra=extra) == ref, (chrom, extra)


def test_native_f5_matches_python_formatting():
    """The writer's integer-arithmetic "%.5f" against Python's correctly rounded formatting on 300k values:
    random magnitudes 1e-15 .. 1e15, random bit patterns, values next to rounding boundaries."""
    import ctypes

    from nldsc_amd import _lib
    rng = np.random.default_rng(11)
    n = 100_000
    x = np.concatenate([rng.uniform(-1, 1, n) * 10.0 ** rng.integers(-15, 15, n),
                        rng.integers(0, 2**63, n, dtype=np.uint64).view(np.float64),
                        np.round(rng.uniform(-100, 100, n), 5) + rng.choice([-5e-6, 5e-6, 4.9999e-6], n)])
    x = x[~np.isnan(x)]
    zeros = np.zeros(len(x))
    prefix = b"\n".join(b"p" for _ in range(len(x)))
    out = np.empty(len(prefix) + len(x) * 900, np.uint8)
    got = _lib.lib().nldsc_format_scores(prefix, len(prefix), len(x), x.ctypes.data, zeros.ctypes.data, None, None,
                                         None, None, None, 0, out.ctypes.data, out.size)
    assert got > 0
    lines = out[:got].tobytes().decode().splitlines()
    exp = ["p\t%.5f\t0.00000" % v for v in x]
    bad = [(v, a, b) for v, a, b in zip(x, lines, exp) if a != b]
    assert not bad, bad[:5]


def test_progress_is_throttled_and_quiet():
    """a13: at most one line per interval plus the final one (the reference ticks stdout once per SNP,
    ldscalc.h:59); nothing with enabled=False / $NLDSC_QUIET; only RANK 0 unless any_rank."""
    import io

    from nldsc_amd.core.progress import Progress
    t = [0.0]
    buf = io.StringIO()
    bar = Progress(1000, "SNPs", interval=1.0, enabled=True, stream=buf, clock=lambda: t[0])
    for k in range(1, 1001):
        t[0] = k * 0.01            # 10 s in total, 1000 updates
        bar.update(k)
    bar.close()
    lines = buf.getvalue().splitlines()
    assert 9 <= len(lines) <= 12, lines
    assert lines[-1].startswith("[ld] 1,000/1,000 SNPs") and "100 SNPs/s" in lines[-1]
    assert "ETA" in lines[1]
    quiet = io.StringIO()
    q = Progress(10, enabled=False, stream=quiet)
    q.update(5, force=True)
    q.close()
    assert quiet.getvalue() == ""
    import os
    old = os.environ.get("RANK")
    os.environ["RANK"] = "3"
    try:
        r = io.StringIO()
        Progress(10, enabled=True, stream=r).close()
        assert r.getvalue() == ""
        Progress(10, enabled=True, any_rank=True, stream=r).close()
        assert r.getvalue() != ""
    finally:
        if old is None:
            os.environ.pop("RANK")
        else:
            os.environ["RANK"] = old


@pytest.mark.parametrize("text", ["a\tb\t0\t0\t1\t-9\n" * 5, "a\tb\t0\t0\t1\t-9\n" * 4 + "a\tb\t0\t0\t1\t-9",
                                  "a\tb\t0\t0\t1\t-9\n\n\na\tb\t0\t0\t1\t-9\n", "a\tb\t0\t0\t1\t-9\r\n" * 3,
                                  "a\tb\t0\t0\t1\t-9\r" * 4, "a\tb\t0\t0\t1\t-9\r\ra\tb\t0\t0\t1\t-9\n",
                                  "", "\n\n", " \r\n", "a\n  \nb\n", "\t\n", "\x0b\n"])
def test_fam_count_equals_pandas_rows(tmp_path, text):
    """FAMFile counts its individuals from the lines (a whole-genome run reads a 315 599-line .fam per chromosome):
    the same number as the rows the reference's pandas parse gives (blank and space-only lines skipped, CRLF, lone CR,
    no final newline, an empty file: 0 rows), and the table itself is still available."""
    import pandas as pd
    from nldsc_amd.ldscore.common import FAMFile
    p = tmp_path / "x.fam"
    p.write_bytes(text.encode())
    f = FAMFile(str(p))
    rows = pd.read_csv(p, sep="\t", names=FAMFile.COLUMNS)
    assert f.n_org == len(rows) and len(f.data) == len(rows) and repr(f) == f"FAMFile(n_org={len(rows)})"

