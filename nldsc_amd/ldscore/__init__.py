"""GPU (MI355X) drop-in for nldsc's `ldscore` package (nldsc/ldscore/__init__.py:1-2)."""
import os as _os

if int(_os.environ.get("WORLD_SIZE", "1")) > 1:
    # torchrun: torch (which bundles its own libamdhip64.so.7) must bind the process's one HIP runtime before
    # _ldscore pulls in libnldsc_amd.so; the collectives of the sharded path need torch anyway
    import torch as _torch  # noqa: F401

from ._ldscore import *  # noqa: F401,F403,E402  LDScoreParams, LDScoreResult, calculate
from .routine import estimate_lds  # noqa: F401,E402
