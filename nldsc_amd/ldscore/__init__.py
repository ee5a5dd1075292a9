"""GPU (MI355X) drop-in for nldsc's `ldscore` package (nldsc/ldscore/__init__.py:1-2)."""
from ._ldscore import *  # noqa: F401,F403  LDScoreParams, LDScoreResult, calculate
from .routine import estimate_lds  # noqa: F401
