#!/usr/bin/env python3
"""Where a load's time goes: C3 rows loaded from a device .bed image several times into one engine (the bench's
oneshot load), wall clock per load; run under rocprofv3 --kernel-trace for the kernels:
    python tools/ab/load_probe.py [--loads 5]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loads", type=int, default=5)
    ap.add_argument("--libs", nargs="*", default=[], help="name=path.so builds to alternate (default: the tree's)")
    ap.add_argument("--shift", type=int, default=0,
                    help="place the image this many bytes into a fresh buffer (13: its rows start 16-byte aligned)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    M, N = 80_000, 315_599
    buf, pos = synth.device_bed(M, N, seed=7, length_cm=280.0)
    if a.shift:
        big = torch.empty(buf.numel() + 64, dtype=torch.uint8, device=buf.device)
        big[a.shift:a.shift + buf.numel()].copy_(buf)
        del buf
        buf = big[a.shift:a.shift + big.numel() - 64]
        print(f"image at base + {a.shift}: rows at {(buf.data_ptr() + 3) % 16} mod 16", file=sys.stderr)
    libs = dict(x.split("=", 1) for x in a.libs) or {"tree": None}
    engines = {name: Engine(0, lib_path=path) for name, path in libs.items()}
    times = {name: [] for name in libs}
    for k in range(a.loads):
        for name, e in engines.items():
            torch.cuda.synchronize()
            t = time.perf_counter()
            e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
            times[name].append(1e3 * (time.perf_counter() - t))
            print(f"{name} load {k}: {times[name][-1]:.3f} ms", file=sys.stderr, flush=True)
    for name, v in times.items():
        print(f"{name}: median {sorted(v[1:])[len(v[1:]) // 2]:.3f} ms over loads 1..", file=sys.stderr)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
