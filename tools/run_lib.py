#!/usr/bin/env python3
"""Run the C3 workload (or C2: --n-org 50000 --additive-only) on one build of libnldsc_amd.so, one engine per process
(for per-build PMC passes and single-engine timing):
    python tools/run_lib.py [lib.so] [--runs 2] [--n-org N] [--additive-only]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=None)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--n-snp", type=int, default=80000)
    ap.add_argument("--n-org", type=int, default=315_599)
    ap.add_argument("--additive-only", action="store_true")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from nldsc_amd import synth
    from nldsc_amd import _lib
    from nldsc_amd.engine import Engine
    M, N = a.n_snp, a.n_org
    flags = _lib.FLAG_ADDITIVE_ONLY if a.additive_only else 0
    buf, pos = synth.device_bed(M, N, seed=7, length_cm=280.0 * M / 80000)
    e = Engine(0, lib_path=a.lib)
    e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    del buf
    for _ in range(a.runs):
        e.run(1.0, 1e-4, 1e-5, 1.0 / M, pos, flags=flags)
        t = e.timings()
        print(f"band {t['band_ms']:.3f} ms total {t['total_ms']:.3f} ms " +
              " ".join(f"{k} {t[k]:.3f}" for k in ("count_ms", "stats_ms", "schedule_ms", "finalize_ms")), flush=True)


if __name__ == "__main__":
    main()
