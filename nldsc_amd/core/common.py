"""Shared helpers of the host layer (counterpart of nldsc/core/common.py:11-43)."""
from __future__ import annotations

import functools
import time
from abc import ABC, abstractmethod
from datetime import timedelta
from typing import Any

from .logger import log


def elapsed_time(func):
    """Log the wall time of `func` as the reference's decorator does (core/common.py:11-20)."""
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        t0 = time.time()
        out = func(*args, **kwargs)
        log.info(f"Elapsed time: {timedelta(seconds=time.time() - t0)}")
        return out
    return wrapper


class NLDSCParameterError(Exception):
    """Invalid user parameter (reference: core/common.py:23)."""


class Data(ABC):
    """Validated value holder (reference: core/common.py:27-43)."""
    _data = None

    @property
    def data(self) -> Any:
        return self._data

    def __str__(self):
        return repr(self)

    @abstractmethod
    def __repr__(self):
        ...

    @abstractmethod
    def _validate(self):
        ...
