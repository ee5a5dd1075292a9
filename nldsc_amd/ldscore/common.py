"""Input / parameter model of `nldsc ld` (the validation contract of nldsc/ldscore/common.py:10-182).

The reference's public names, validation rules and messages, written table-driven:
  LDWindow               kb -> bp x 1000; > 0; <= 5 Mbp or <= 100 cM
  PLINKFile.parse        prefix or one of the three paths -> (BEDFile, BIMFile, FAMFile)
  BIMFile / FAMFile      tab-separated tables, one chromosome per .bim; n_snp / n_org = number of lines
  MAF, ResidualsSTDThreshold, RSQThreshold: [0, 1), [0, 1), [0, 0.1)
(RSQThreshold's repr says `std_thr=`, as the reference's does.)
"""
from __future__ import annotations

import os
from pathlib import Path

import pandas as pd

from ..core.common import Data, NLDSCParameterError

__all__ = ["LDWindow", "PLINKFile", "BEDFile", "BIMFile", "FAMFile", "MAF", "ResidualsSTDThreshold",
           "RSQThreshold", "NLDSCParameterError"]

# window metric -> (largest window, how the message names it)
_WINDOW_LIMITS = {"bp": (5 * 10 ** 6, "5 Mbp"), "cm": (100, "100 cm")}


class LDWindow(Data):
    def __init__(self, ld_wind: float, metric: str = "bp"):
        scale = 1000 if metric == "kbp" else 1  # kilobases are carried as base pairs
        self._data = float(ld_wind) * scale
        self._metric = "bp" if metric == "kbp" else metric
        self._validate()

    @property
    def metric(self) -> str:
        return self._metric

    def __repr__(self) -> str:
        return f"LDWindow(ld_wind={self._data}, metric='{self._metric}')"

    def _validate(self):
        limit = _WINDOW_LIMITS.get(self._metric)
        if limit is None:
            raise NLDSCParameterError("Invalid metric")
        if self._data <= 0:
            raise NLDSCParameterError("The ld-window must be greater than 0")
        if self._data > limit[0]:
            raise NLDSCParameterError(f"The ld-window cannot be larger than {limit[1]}")


class PLINKFile(Data):
    """One file of a PLINK 1 binary set; a table file keeps its columns in `_data`."""
    EXT = ""
    COLUMNS: tuple = ()

    def __init__(self, path: str):
        self._path = str(path)
        if not os.path.exists(self._path):
            raise FileNotFoundError(f'No such file: "{self._path}"')
        if self.COLUMNS:
            self._data = pd.read_csv(self._path, sep="\t", names=self.COLUMNS)
        self._validate()

    def _validate(self):
        pass

    def __repr__(self):
        return f"{type(self).__name__}(path='{self._path}')"

    @staticmethod
    def parse(bfile: str):
        """`bfile` is a prefix or the path of one of the three files -> (BEDFile, BIMFile, FAMFile)."""
        path = Path(bfile).resolve()
        if path.suffix in (".bed", ".bim", ".fam"):
            path = path.with_suffix("")
        elif path.is_dir():
            raise NotImplementedError("")
        return tuple(kind(path.as_posix() + kind.EXT) for kind in (BEDFile, BIMFile, FAMFile))


def _column(name: str):
    return property(lambda self: self._data[name])


class BEDFile(PLINKFile):
    EXT = ".bed"

    def __init__(self, path: str):
        super().__init__(path)
        self._data = path  # the engine reads the file itself


class BIMFile(PLINKFile):
    EXT = ".bim"
    COLUMNS = ("CHR", "SNP", "CM", "BP", "A1", "A2")
    chr, snp, cm, bp = (_column(c) for c in ("CHR", "SNP", "CM", "BP"))

    def __init__(self, path: str, **kwargs):
        super().__init__(path)

    @property
    def n_snp(self) -> int:
        return len(self._data)

    def __repr__(self):
        return f"BIMFile(n_snp={self.n_snp})"

    def _validate(self):
        if self._data["CHR"].nunique(dropna=False) != 1:
            raise NLDSCParameterError("The current version of the program "
                                      "can only work with one chromosome in one file.")


class FAMFile(PLINKFile):
    """Only the number of individuals is used: it is counted from the lines (the rows pandas would parse: non-blank
    lines; a whole-genome run reads 22 copies of a 315 599-line file, ~0.15 s each through pandas), and the table is
    parsed when `data` is first asked for."""
    EXT = ".fam"
    COLUMNS = ("FID", "IID", "FATHER", "MOTHER", "SEX", "TRAIT")

    def __init__(self, path: str):
        self._path = str(path)
        if not os.path.exists(self._path):
            raise FileNotFoundError(f'No such file: "{self._path}"')
        with open(self._path, "rb") as fh:
            # \n, \r\n and lone \r all end a row for pandas' C parser, which skips lines that are empty or hold
            # only spaces (an empty file is 0 rows, as the reference's read_csv with `names` gives)
            self._n_org = sum(1 for line in fh.read().splitlines() if line.strip(b" "))
        self._table = None

    @property
    def data(self) -> pd.DataFrame:
        if self._table is None:
            self._table = pd.read_csv(self._path, sep="\t", names=self.COLUMNS)
        return self._table

    @property
    def n_org(self) -> int:
        return self._n_org

    def __repr__(self):
        return f"FAMFile(n_org={self.n_org})"


def _threshold(name: str, field: str, hi: float, message: str):
    """A validated threshold in [0, hi) whose repr is `name(field=value)`."""
    def __init__(self, value: float):
        self._data = float(value)
        self._validate()

    def _validate(self):
        if not (0 <= self._data < hi):
            raise NLDSCParameterError(message)

    return type(name, (Data,), {"__init__": __init__, "_validate": _validate,
                                "__repr__": lambda self: f"{name}({field}={self._data})",
                                "__module__": __name__})


MAF = _threshold("MAF", "maf", 1.0, "Minor allele frequency must be between 0 and 1!")
ResidualsSTDThreshold = _threshold("ResidualsSTDThreshold", "std_thr", 1.0,
                                   "standard deviation threshold must be between 0 and 1!")
RSQThreshold = _threshold("RSQThreshold", "std_thr", 0.1, "r-squared threshold must be between 0 and 0.1!")
