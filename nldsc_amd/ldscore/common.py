"""Input / parameter model of `nldsc ld` (behaviour of nldsc/ldscore/common.py:10-182).

Same classes, validation rules and messages: LDWindow (kb -> bp x 1000; > 0; <= 5 Mbp or
<= 100 cM), PLINKFile.parse, BIMFile (tab-separated, one chromosome per file), FAMFile
(N = number of lines), MAF [0, 1), ResidualsSTDThreshold [0, 1), RSQThreshold [0, 0.1).
"""
from __future__ import annotations

import os
from abc import ABC
from pathlib import Path

import pandas as pd

from ..core.common import Data, NLDSCParameterError

__all__ = ["LDWindow", "PLINKFile", "BEDFile", "BIMFile", "FAMFile", "MAF", "ResidualsSTDThreshold",
           "RSQThreshold", "NLDSCParameterError"]


class LDWindow(Data):
    def __init__(self, ld_wind: float, metric: str = "bp"):
        self._data = float(ld_wind)
        self._metric = metric
        if self._metric == "kbp":  # kilobases are carried as base pairs
            self._data *= 1000
            self._metric = "bp"
        self._validate()

    @property
    def metric(self) -> str:
        return self._metric

    def __repr__(self) -> str:
        return f"LDWindow(ld_wind={self._data}, metric='{self._metric}')"

    def _validate(self):
        if self._metric not in ("bp", "cm"):
            raise NLDSCParameterError("Invalid metric")
        if self._data <= 0:
            raise NLDSCParameterError("The ld-window must be greater than 0")
        if self._metric == "bp" and self._data > 5 * 10 ** 6:
            raise NLDSCParameterError("The ld-window cannot be larger than 5 Mbp")
        if self._metric == "cm" and self._data > 100:
            raise NLDSCParameterError("The ld-window cannot be larger than 100 cm")


class PLINKFile(Data, ABC):
    def __init__(self, path: str):
        self._path = str(path)
        if not os.path.exists(self._path):
            raise FileNotFoundError(f'No such file: "{self._path}"')

    @staticmethod
    def parse(bfile: str):
        """`bfile` is a prefix or the path of one of the three files."""
        path = Path(bfile).resolve()
        if any(path.match(ext) for ext in ("*.bed", "*.bim", "*.fam")):
            path = path.with_suffix("")
        elif path.is_dir():
            raise NotImplementedError("")
        stem = path.as_posix()
        return BEDFile(stem + ".bed"), BIMFile(stem + ".bim"), FAMFile(stem + ".fam")


class BEDFile(PLINKFile):
    def __init__(self, path: str):
        super().__init__(path)
        self._data = path

    def __repr__(self):
        return f"BEDFile(path='{self._data}')"

    def _validate(self):
        pass


class BIMFile(PLINKFile):
    COLUMNS = ("CHR", "SNP", "CM", "BP", "A1", "A2")

    def __init__(self, path: str, **kwargs):
        super().__init__(path)
        self._data = pd.read_csv(path, sep="\t", names=self.COLUMNS)
        self._validate()

    def __repr__(self):
        return f"BIMFile(n_snp={self.n_snp})"

    @property
    def chr(self) -> pd.Series:
        return self._data["CHR"]

    @property
    def snp(self) -> pd.Series:
        return self._data["SNP"]

    @property
    def cm(self) -> pd.Series:
        return self._data["CM"]

    @property
    def bp(self) -> pd.Series:
        return self._data["BP"]

    @property
    def n_snp(self) -> int:
        return len(self._data)

    def _validate(self):
        if self._data["CHR"].nunique(dropna=False) != 1:
            raise NLDSCParameterError("The current version of the program "
                                      "can only work with one chromosome in one file.")


class FAMFile(PLINKFile):
    COLUMNS = ("FID", "IID", "FATHER", "MOTHER", "SEX", "TRAIT")

    def __init__(self, path: str):
        super().__init__(path)
        self._data = pd.read_csv(path, sep="\t", names=self.COLUMNS)

    def __repr__(self):
        return f"FAMFile(n_org={self.n_org})"

    @property
    def n_org(self) -> int:
        return len(self._data)

    def _validate(self):
        pass


class _UnitInterval(Data):
    _what = ""
    _hi = 1.0

    def __init__(self, value: float):
        self._data = float(value)
        self._validate()

    def _validate(self):
        if not (0 <= self._data < self._hi):
            raise NLDSCParameterError(self._what)


class MAF(_UnitInterval):
    _what = "Minor allele frequency must be between 0 and 1!"

    def __repr__(self) -> str:
        return f"MAF(maf={self._data})"


class ResidualsSTDThreshold(_UnitInterval):
    _what = "standard deviation threshold must be between 0 and 1!"

    def __repr__(self) -> str:
        return f"ResidualsSTDThreshold(std_thr={self._data})"


class RSQThreshold(_UnitInterval):
    _what = "r-squared threshold must be between 0 and 0.1!"
    _hi = 0.1

    def __repr__(self) -> str:
        return f"RSQThreshold(std_thr={self._data})"
