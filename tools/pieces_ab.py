#!/usr/bin/env python3
"""One chromosome (C3) split into P owned SNP ranges, each on its own engine (its halo slice resident,
its own streams) and run from P host threads at once: step wall time vs P = 1 (one engine), interleaved.
Checks the assembled table against the single-engine run."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pieces", default="1,2,3,4")
    ap.add_argument("--n-org", type=int, default=315_599)
    ap.add_argument("--n-snp", type=int, default=80_000)
    ap.add_argument("--length-cm", type=float, default=280.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    from nldsc_amd import synth
    from nldsc_amd.distributed import RESULT_KEYS, halo_range, shard_ranges
    from nldsc_amd.engine import Engine
    N, M, w = args.n_org, args.n_snp, 1.0
    nb = (N + 3) // 4
    buf, pos = synth.device_bed(M, N, seed=7, length_cm=args.length_cm)
    setups = {}
    for P in [int(x) for x in args.pieces.split(",")]:
        parts = []
        for lo, hi in shard_ranges(pos, w, P):
            a, b = halo_range(pos, w, (lo, hi))
            sl = torch.cat([buf[:3], buf[3 + a * nb:3 + b * nb]])
            e = Engine(0)
            e.load_bed_device(sl.data_ptr(), sl.numel(), b - a, N)
            del sl
            parts.append((e, a, b, lo, hi))
        setups[P] = (parts, ThreadPoolExecutor(max_workers=P))
    del buf
    torch.cuda.empty_cache()

    def step(P):
        parts, pool = setups[P]
        full = {k: np.empty(M, np.float64 if k in ("l2", "l2d", "maf", "residuals_std") else np.int32)
                for k in RESULT_KEYS}

        def one(x):
            e, a, b, lo, hi = x
            r = e.run(w, 1e-4, 1e-5, 1.0 / M, pos[a:b], own=(lo - a, hi - a))
            for k in RESULT_KEYS:
                full[k][lo:hi] = r[k][lo - a:hi - a]
            return e.timings()
        t = time.perf_counter()
        tims = list(pool.map(one, parts)) if P > 1 else [one(parts[0])]
        return time.perf_counter() - t, full, tims

    res = {P: [] for P in setups}
    outs = {}
    for r in range(args.rounds + 1):
        for P in setups:
            dt, full, tims = step(P)
            if r > 0:
                res[P].append((dt, tims))
            outs[P] = full
    ref = outs[min(setups)]
    summary = {}
    for P, xs in res.items():
        ms = [1e3 * dt for dt, _ in xs]
        pairs = float(ref["l2_ws"][ref["l2_ws"] > 0].sum())
        summary[P] = dict(step_ms_median=float(np.median(ms)), step_ms_min=float(min(ms)),
                          gpairs_per_s=pairs / (np.median(ms) * 1e-3) / 1e9,
                          band_ms_per_piece=[round(t["band_ms"], 3) for t in xs[-1][1]],
                          count_ms_per_piece=[round(t["count_ms"], 3) for t in xs[-1][1]],
                          items_per_piece=[t["band_items"] for t in xs[-1][1]],
                          max_abs_l2_vs_single=float(np.nanmax(np.abs(outs[P]["l2"] - ref["l2"]))),
                          ws_equal=bool(all(np.array_equal(outs[P][k], ref[k]) for k in ("l2_ws", "l2d_ws", "l2d_wse"))))
    print(json.dumps(summary, indent=1))
    if args.out:
        json.dump(dict(config=vars(args), summary=summary), open(args.out, "w"), indent=1)
    for parts, pool in setups.values():
        pool.shutdown()
        for e, *_ in parts:
            e.close()


if __name__ == "__main__":
    main()
