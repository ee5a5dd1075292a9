#!/usr/bin/env python3
"""Host side of a run with the results landing in ordinary numpy arrays (the engine's pinned landing buffer + host
copies) vs nldsc_host_alloc arrays (written by the GPU in place), C2 and C3, engine option debug_timing on:
    python tools/hostpath_probe.py [--runs 6]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from nldsc_amd import _lib, synth
    from nldsc_amd.engine import Engine
    for name, N, add in (("c2", 50_000, True), ("c3", 315_599, False)):
        M = 80_000
        buf, pos = synth.device_bed(M, N, seed=7, length_cm=280.0)
        e = Engine(0, options={"debug_timing": 1})
        e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
        del buf
        flags = _lib.FLAG_ADDITIVE_ONLY if add else 0
        pinned = _lib.alloc_result(M, pinned=True)[0]
        ppos = _lib.pinned_empty(M, np.float64)
        ppos[:] = pos
        for mode in ("fresh", "reused", "pinned"):
            out = None if mode == "fresh" else (_lib.alloc_result(M)[0] if mode == "reused" else pinned)
            p = ppos if mode == "pinned" else pos
            for r in range(a.runs):
                t = time.perf_counter()
                res = e.run(1.0, 1e-4, 1e-5, 1.0 / M, p, flags=flags, out=out)
                dt = time.perf_counter() - t
                tm = e.timings()
                print(f"{name} {mode} run {r}: wall {1e3 * dt:.3f} ms engine total {tm['total_ms']:.3f} band "
                      f"{tm['band_ms']:.3f} pairs {tm['pairs']:.0f}", file=sys.stderr, flush=True)
                if out is not None:
                    out = res
        e.close()


if __name__ == "__main__":
    main()
