"""Throttled progress reporting (replaces the reference's per-SNP progress bar, ldscalc.h:9-11,59 +
indicators.h:4742-4756, which ticks and flushes stdout once per SNP).

One line to stderr at most every `interval` seconds (default 1 s) plus a final line: units done / total,
rate, elapsed and ETA.  Disabled with `--quiet` (or $NLDSC_QUIET=1); only the process with RANK 0 reports.
"""
from __future__ import annotations

import os
import sys
import time


class Progress:
    def __init__(self, total: float, unit: str = "SNPs", *, label: str = "ld", interval: float = 1.0,
                 enabled: bool | None = None, any_rank: bool = False, stream=None, clock=time.monotonic):
        if enabled is None:
            enabled = os.environ.get("NLDSC_QUIET", "0") in ("", "0")
        self.enabled = enabled and (any_rank or os.environ.get("RANK", "0") == "0")
        self.total, self.unit, self.label, self.interval = float(total), unit, label, float(interval)
        self.stream = stream if stream is not None else sys.stderr
        self.clock = clock
        self.t0 = clock()
        self.last = None
        self.done = 0.0
        self.lines = 0

    def _line(self, note: str) -> str:
        el = max(self.clock() - self.t0, 1e-9)
        rate = self.done / el
        s = f"[{self.label}] {self.done:,.0f}/{self.total:,.0f} {self.unit}, {rate:,.0f} {self.unit}/s, {el:.1f} s"
        if 0 < self.done < self.total and rate > 0:
            s += f", ETA {(self.total - self.done) / rate:.1f} s"
        return s + (f" ({note})" if note else "")

    def update(self, done: float, note: str = "", *, force: bool = False) -> bool:
        """Set the units done; print if `interval` has passed since the last line (or `force`)."""
        self.done = float(done)
        if not self.enabled:
            return False
        now = self.clock()
        if not force and self.last is not None and now - self.last < self.interval:
            return False
        self.last = now
        self.stream.write(self._line(note) + "\n")
        self.stream.flush()
        self.lines += 1
        return True

    def close(self, note: str = "") -> None:
        self.update(self.total if self.done < self.total else self.done, note, force=True)
