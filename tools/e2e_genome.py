#!/usr/bin/env python3
"""Whole-genome `nldsc ld --bfile chr@` I/O path on one GPU: K synthetic chromosome files written to disk, then
estimate_lds_genome timed in process (files in the page cache) with
  engine  - the default runner: the engine's own reader (file -> pinned slots -> pitched H2D), next file read ahead
  bytes   - a runner fed by the host-thread prefetch (np.fromfile) and load_bed_bytes (pageable H2D)
alternately, and the outputs compared.
    python tools/e2e_genome.py --chroms 4 --n-snp 20000 --out gpurun_out/e2e_genome.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chroms", type=int, default=4)
    ap.add_argument("--n-org", type=int, default=315_599)
    ap.add_argument("--n-snp", type=int, default=20_000)
    ap.add_argument("--dir", default="/tmp/nldsc_genome")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    os.makedirs(a.dir, exist_ok=True)
    N, M = a.n_org, a.n_snp
    nb = (N + 3) // 4
    for c in range(1, a.chroms + 1):
        stem = os.path.join(a.dir, f"chr{c}")
        buf, pos = synth.device_bed(M, N, seed=100 + c, length_cm=70.0)
        with open(stem + ".bed", "wb") as fh:
            fh.write(buf.cpu().numpy().tobytes())
        del buf
        bp = np.round(pos * 1e6).astype(np.int64)
        with open(stem + ".bim", "w") as fh:
            fh.writelines(f"{c}\trs{c}_{j}\t{pos[j]:.6f}\t{bp[j]}\tA\tG\n" for j in range(M))
        with open(stem + ".fam", "w") as fh:
            fh.writelines(f"f{i}\ti{i}\t0\t0\t0\t-9\n" for i in range(N))
    torch.cuda.empty_cache()
    gb = a.chroms * (3 + M * nb) / 1e9
    eng = Engine(0)

    def bytes_runner(bed, n_snp, n_org, ld_wind, maf, std_thr, rsq_thr, positions, flags):
        eng.load_bed_bytes(bed, n_snp, n_org)
        return eng.run(ld_wind, maf, std_thr, rsq_thr, positions, flags=flags), eng.timings()

    times = {"engine": [], "bytes": []}
    outs = {}
    for r in range(a.rounds):
        for name, runner in (("engine", None), ("bytes", bytes_runner)):
            t = time.perf_counter()
            res = estimate_lds_genome(os.path.join(a.dir, "chr@"), "1", "cm", maf_thr="0.0001", std_thr=1e-5,
                                      extra=True, rank=0, world=1, device=0, runner=runner)
            times[name].append(time.perf_counter() - t)
            outs[name] = res
    # counts exact; the fp64 sums are atomically accumulated, so equal up to summation order
    def close(x, y):
        ints = all(np.array_equal(x[k].to_numpy(), y[k].to_numpy()) for k in ("WSA", "WSD", "WSDE", "MAF"))
        return ints and all(np.allclose(x[k].to_numpy(), y[k].to_numpy(), rtol=1e-12, atol=1e-12, equal_nan=True)
                            for k in ("L2", "L2D", "RSTD"))
    same = all(close(outs["engine"][c], outs["bytes"][c]) for c in outs["engine"])
    doc = dict(chroms=a.chroms, n_org=N, n_snp_per_chrom=M, bed_gb=gb,
               seconds={k: [round(x, 3) for x in v] for k, v in times.items()},
               gb_per_s={k: round(gb / min(v), 2) for k, v in times.items()}, tables_agree=bool(same))
    print(json.dumps(doc))
    if a.out:
        json.dump(doc, open(a.out, "w"), indent=1)
    eng.close()


if __name__ == "__main__":
    main()
