#!/usr/bin/env python3
"""Where a short run's wall time goes outside the engine's own total: per-step Python wall time around
Engine.run / run_device (+ timings) against the engine's total_ms and band_ms, for a tiny chromosome (fixed costs
dominate) and a 1/8 shard of C3 (one rank of the 8-GPU run).  One JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.init()
    from nldsc_amd import _lib, synth
    from nldsc_amd.distributed import halo_range, shard_ranges
    from nldsc_amd.engine import Engine
    out = {}
    cases = {"tiny": (1000, 2000, 7.0), "c3_shard_r0of8": (315_599, 80_000, 280.0)}
    for name, (N, M, L) in cases.items():
        buf, pos = synth.device_bed(M, N, seed=7, length_cm=L)
        own = None
        if name.startswith("c3_shard"):
            lo, hi = shard_ranges(pos, 1.0, 8)[0]
            a, b = halo_range(pos, 1.0, (lo, hi))
            nb = (N + 3) // 4
            buf = torch.cat([buf[:3], buf[3 + a * nb:3 + b * nb]])
            pos, M, own = pos[a:b], b - a, (lo - a, hi - a)
        e = Engine(0)
        e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
        del buf
        args = (1.0, 1e-4, 1e-5, 1.0 / 80_000)
        res = {}
        pos_p = _lib.pinned_empty(M, np.float64)
        pos_p[:] = pos
        outp = _lib.alloc_result(M, pinned=True)[0]
        w = own[1] - own[0] if own else M
        table = torch.empty((7, w), dtype=torch.float64, device="cuda:0")
        for mode in ("run_numpy", "run_pinned", "run_device"):
            walls, tot, band, tcall = [], [], [], []
            for k in range(40):
                t0 = time.perf_counter()
                if mode == "run_numpy":
                    e.run(*args, pos, own=own)
                elif mode == "run_pinned":
                    e.run(*args, pos_p, own=own, out=outp)
                else:
                    e.run_device(*args, pos, table, own=own)
                t1 = time.perf_counter()
                tm = e.timings()
                t2 = time.perf_counter()
                if k >= 5:
                    walls.append(1e3 * (t2 - t0))
                    tcall.append(1e3 * (t1 - t0))
                    tot.append(tm["total_ms"])
                    band.append(tm["band_ms"])
            res[mode] = {"wall_ms": float(np.median(walls)), "call_ms": float(np.median(tcall)),
                         "engine_total_ms": float(np.median(tot)), "band_ms": float(np.median(band)),
                         "outside_engine_ms": float(np.median(np.array(walls) - np.array(tot))),
                         "call_minus_engine_ms": float(np.median(np.array(tcall) - np.array(tot)))}
        out[name] = res
        e.close()
        print(json.dumps({name: res}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
