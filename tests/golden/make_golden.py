"""Generate the committed golden fixtures under tests/golden/.  Run in the build container:

    python tests/golden/make_golden.py

1. Small synthetic PLINK sets (nldsc_amd/synth.py) covering N % 4 in {0,1,2,3}, 1 % missing,
   a monomorphic SNP, a SNP with only hom-A1/het genotypes (residual std 0), an unused SNP
   (position -1, also as the last SNP), an exact window-boundary tie, and an all-missing SNP.
2. Expected `LDScoreResult` for each set from the C oracle (oracle/ldscore_oracle.c, the
   reference's fp32 structure) and from the fp64 closed-form restatement (oracle/oracle.py).
3. Reference-pinned vectors for the Python layer: the reference's own `estimate_lds`
   (nldsc/ldscore/routine.py:51-102, imported read-only from /root/reference) is run with
   a recording stand-in for its unbuilt C++ `_ldscore` module that returns the C-oracle
   result.  Saved: the LDScoreParams the reference builds (bfile basename, n_snp, n_org,
   ld_wind, maf, std_thr, rsq_thr, positions) and the TSV it writes, per scenario, plus the
   reference's validation error messages.  These pin our host layer to the reference.

Nothing from /root/reference is copied: only inputs and outputs are stored.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)

from nldsc_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

REF = "/root/reference/nldsc"

SETS = {
    # name: (spec kwargs, window metric, window value)
    "n1000": (dict(n_org=1000, n_snp=1200, length_cm=8.0, seed=11, monomorphic=[5], hom1_het_only=[17],
                   negative_pos=[100], tie_pairs=[200]), "cm", 1.0),
    "n1001": (dict(n_org=1001, n_snp=1200, length_cm=8.0, seed=12, monomorphic=[6], hom1_het_only=[18],
                   negative_pos=[101], tie_pairs=[300]), "cm", 1.0),
    "n1002": (dict(n_org=1002, n_snp=1200, length_cm=8.0, seed=13, monomorphic=[7], hom1_het_only=[19],
                   negative_pos=[102], tie_pairs=[400]), "kbp", 1000.0),
    "n1003": (dict(n_org=1003, n_snp=1200, length_cm=8.0, seed=14, monomorphic=[8], hom1_het_only=[20],
                   negative_pos=[103, 1199], tie_pairs=[500]), "kbp", 500.0),
    "allmiss": (dict(n_org=1000, n_snp=600, length_cm=4.0, seed=15, all_missing=[50]), "cm", 1.0),
    # N % 4 != 0: the reference reads one padding pair (hom A1) in the last byte, so an
    # "all-missing" SNP has one observed genotype, MAF 0 and fails the MAF filter.
    "allmiss_pad": (dict(n_org=1001, n_snp=600, length_cm=4.0, seed=16, all_missing=[50]), "cm", 1.0),
}
MAF_THR, STD_THR = 0.01, 1e-5


def window_args(metric, value, pos_cm, bp):
    if metric == "cm":
        return float(value), pos_cm.astype(np.float64)
    return float(value) * 1000.0, bp.astype(np.float64)


def make_sets():
    meta = {}
    for name, (kw, metric, wval) in SETS.items():
        spec = synth.SynthSpec(**kw)
        prefix = os.path.join(HERE, name)
        d = synth.write_plink(prefix, spec)
        rows, cm, bp = d["rows"], d["pos_cm"], d["bp"]
        w, pos = window_args(metric, wval, cm, bp)
        M, N = spec.n_snp, spec.n_org
        rsq = 1.0 / M
        bed = open(prefix + ".bed", "rb").read()
        c = O.run_c(bed, M, N, w, MAF_THR, STD_THR, rsq, pos, threads=1)
        f = O.run_f64(rows, N, w, MAF_THR, STD_THR, rsq, pos)
        np.savez_compressed(os.path.join(HERE, name + ".oracle.npz"), **c)
        np.savez_compressed(os.path.join(HERE, name + ".f64.npz"), **f)
        meta[name] = dict(n_snp=M, n_org=N, metric=metric, window=wval, ld_wind=w, maf=MAF_THR, std_thr=STD_THR,
                          rsq_thr=rsq, bed_sha256=hashlib.sha256(bed).hexdigest())
    with open(os.path.join(HERE, "sets.json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    return meta


# ---- reference-Python vectors ------------------------------------------------------------

class _Rec:
    params = None
    result = None


def _fake_ldscore_module():
    m = types.ModuleType("ldscore._ldscore")

    class LDScoreParams:
        def __init__(self, bfile=None, *, n_snp=None, n_org=None, ld_wind=None, maf=None, std_thr=None,
                     rsq_thr=None, positions=None):
            self.bedfile, self.n_snp, self.n_org, self.ld_wind = bfile, n_snp, n_org, ld_wind
            self.maf, self.std_thr, self.rsq_thr, self.positions = maf, std_thr, rsq_thr, positions

    class LDScoreResult:
        pass

    def calculate(params):
        _Rec.params = params
        r = LDScoreResult()
        for k, v in _Rec.result.items():
            setattr(r, k, [float(x) for x in v] if v.dtype.kind == "f" else [int(x) for x in v])
        return r

    m.LDScoreParams, m.LDScoreResult, m.calculate = LDScoreParams, LDScoreResult, calculate
    return m


SCENARIOS = [
    # (set, ld_wind (CLI string), wind_metric, maf (CLI string), std_thr, rsq_thr, extra)
    ("n1000", "1", "cm", "0.01", 1e-5, None, True),
    ("n1001", "1", "cm", "0.01", 1e-5, None, False),
    ("n1002", "1000", "kbp", "0.01", 1e-5, None, True),
    ("n1003", "500", "kbp", "0.01", 1e-5, "0.002", True),
    ("allmiss", "1", "cm", "0.01", 1e-5, None, True),
]

ERROR_CASES = [
    ("LDWindow", ("0", "cm")), ("LDWindow", ("101", "cm")), ("LDWindow", ("5001", "kbp")),
    ("LDWindow", ("1", "mb")), ("MAF", ("1.0",)), ("MAF", ("-0.1",)), ("ResidualsSTDThreshold", ("1",)),
    ("RSQThreshold", ("0.1",)),
]


def make_reference_vectors():
    tmp = tempfile.mkdtemp(prefix="nldsc_golden_")
    cwd = os.getcwd()
    os.chdir(tmp)  # the reference's logger creates ./nldsc.log on import
    sys.path.insert(0, REF)
    sys.modules["ldscore._ldscore"] = _fake_ldscore_module()
    try:
        import ldscore  # noqa: F401  (reference package, Python layer only)
        from ldscore import routine as ref_routine
        from ldscore import common as ref_common
        out = {"scenarios": [], "errors": []}
        for name, wind, metric, maf, std_thr, rsq, extra in SCENARIOS:
            _Rec.result = dict(np.load(os.path.join(HERE, name + ".oracle.npz")))
            tsv = os.path.join(tmp, name + ".L2")
            ref_routine.estimate_lds(os.path.join(HERE, name), ld_wind=wind, wind_metric=metric, maf_thr=maf,
                                     std_thr=std_thr, rsq_thr=rsq, out=tsv, extra=extra, summary=False)
            p = _Rec.params
            pos = np.asarray(list(p.positions), dtype=np.float64)
            text = open(tsv).read()
            with open(os.path.join(HERE, f"{name}.ref.L2"), "w") as fh:
                fh.write(text)
            out["scenarios"].append(dict(
                set=name, args=dict(ld_wind=wind, wind_metric=metric, maf_thr=maf, std_thr=std_thr, rsq_thr=rsq,
                                    extra=extra),
                params=dict(bfile_basename=os.path.basename(p.bedfile), n_snp=int(p.n_snp), n_org=int(p.n_org),
                            ld_wind=float(p.ld_wind), maf=float(p.maf), std_thr=float(p.std_thr),
                            rsq_thr=float(p.rsq_thr), positions_sha256=hashlib.sha256(pos.tobytes()).hexdigest(),
                            positions_len=int(len(pos))),
                tsv_file=f"{name}.ref.L2", tsv_sha256=hashlib.sha256(text.encode()).hexdigest()))
        for cls, args in ERROR_CASES:
            try:
                getattr(ref_common, cls)(*args)
                out["errors"].append(dict(cls=cls, args=list(args), error=None, message=None))
            except Exception as ex:  # noqa: BLE001
                out["errors"].append(dict(cls=cls, args=list(args), error=type(ex).__name__, message=str(ex)))
        with open(os.path.join(HERE, "reference_python.json"), "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
    finally:
        os.chdir(cwd)
        sys.path.remove(REF)


if __name__ == "__main__":
    O.build()
    make_sets()
    if os.path.isdir(REF):
        make_reference_vectors()
    else:
        print("reference not present: reference_python.json left as committed")
