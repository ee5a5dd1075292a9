#!/usr/bin/env python3
"""Interleaved A/B of band-kernel variants in ONE process on the C3 workload (cdna_hip_programming.md
§5.4 rule 24).  Variants are engine knobs read at engine creation (NLDSC_BAND_WPS, NLDSC_BAND_NC).

    python tools/band_ab.py [--rounds 3] [--n-snp 20000] [--variants wps1:nc2,wps2:nc2,v1=ab_libs/v1.so:wps2:nc2]

A variant is `[label=][libpath:]token:token...`; `libpath` loads another build of libnldsc_amd.so (same
ABI).  Tokens: wpsW, ncC (fp32 path), i8 (exact path), i8nc2, tile (exact path on skewed 2x2 tiles),
xcd (XCD-contiguous item order), f4 (exact path on fp4 MFMAs), f4nc2 (fp4 items of two column
blocks), roundR (R fp4 items per launch; round-1 = one launch per round of resident waves), grpS (fp4 on
4-wave workgroups of skewed 2x2 tiles, a barrier every S chunk pairs; grp0: no barriers), ringD (fp4
strips through a D-deep per-wave LDS ring filled by LDS-DMA), trR / tcC (item order: tiles of R row blocks x C
diagonal offsets; tr1 = row-major), noori (keep the file's allele coding instead of minor-homozygote-as-00), dl (diagonal items last in
every XCD run), dsplit (diagonal items in a launch of their own first).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n-org", type=int, default=315_599)
    ap.add_argument("--n-snp", type=int, default=20_000)
    ap.add_argument("--length-cm", type=float, default=70.0)
    ap.add_argument("--variants", default="wps1:nc2,wps2:nc2,wps2:nc1,wps1:nc1")
    ap.add_argument("--window", type=float, default=1.0, help="window in position units (C5: 1e6 bp)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--additive-only", action="store_true", help="additive L2 only (C2)")
    ap.add_argument("--major", action="store_true",
                    help="swap hom-A1/hom-A2 codes of every SNP (.bim A2 = the major allele, as in PLINK's usual "
                         "A1 = minor convention)")
    args = ap.parse_args()
    import torch

    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = args.n_org, args.n_snp
    buf, pos = synth.device_bed(M, N, seed=7, length_cm=args.length_cm)
    if args.major:  # 00 <-> 11 in every bit pair (het 10 and missing 01 unchanged)
        body = buf[3:]
        eq = torch.bitwise_and(torch.bitwise_not(torch.bitwise_xor(body, body >> 1)), 0x55)
        body.bitwise_xor_(torch.bitwise_or(eq, eq << 1))
    engines = {}
    for v in args.variants.split(","):
        label, spec = v.split("=", 1) if "=" in v else (v, v)
        parts = spec.split(":")
        lib = parts[0] if parts[0].endswith(".so") else None
        knobs = dict((p[:3] if p.startswith("wps") else p[:2], p[3:] if p.startswith("wps") else p[2:])
                     for p in parts if p.startswith(("wps", "nc")))
        os.environ["NLDSC_BAND_WPS"] = knobs.get("wps", "2")
        os.environ["NLDSC_BAND_NC"] = knobs.get("nc", "2")
        os.environ["NLDSC_BAND_MODE"] = ("f4" if any(x.startswith("f4") for x in parts) else
                                         "i8" if any(x.startswith("i8") or x == "tile" for x in parts) else "f32")
        os.environ["NLDSC_BAND_I8_NC"] = "2" if "i8nc2" in parts else "1"
        os.environ["NLDSC_BAND_F4_NC"] = "2" if "f4nc2" in parts else "1"
        os.environ["NLDSC_BAND_TILE"] = "1" if "tile" in parts else "0"
        os.environ["NLDSC_XCD"] = "1" if "xcd" in parts else "0"
        grp = [p[3:] for p in parts if p.startswith("grp")]
        os.environ["NLDSC_BAND_F4_GRP"] = grp[0] if grp else "-1"
        ring = [p[4:] for p in parts if p.startswith("ring")]
        os.environ["NLDSC_BAND_F4_RING"] = ring[0] if ring else "0"
        rnd = [p[5:] for p in parts if p.startswith("round")]
        os.environ["NLDSC_BAND_ROUND"] = rnd[0] if rnd else "0"
        tr = [p[2:] for p in parts if p.startswith("tr")]
        tc = [p[2:] for p in parts if p.startswith("tc")]
        os.environ["NLDSC_TILE_R"] = tr[0] if tr else "16"
        os.environ["NLDSC_TILE_C"] = tc[0] if tc else "16"
        os.environ["NLDSC_ORIENT"] = "0" if "noori" in parts else "1"
        os.environ["NLDSC_DIAG_LAST"] = "2" if "dsplit" in parts else "1" if "dl" in parts else "0"
        e = Engine(0, lib_path=lib)
        v = label
        e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
        engines[v] = e
    del buf
    torch.cuda.empty_cache()
    res = {v: [] for v in engines}
    outs = {}
    for r in range(args.rounds + 1):
        for v, e in engines.items():
            o = e.run(args.window, 1e-4, 1e-5, 1.0 / M, pos, flags=2 if args.additive_only else 0)  # _lib.FLAG_ADDITIVE_ONLY
            t = e.timings()
            if r > 0:
                res[v].append(t)
            outs[v] = o
    ref = next(iter(outs.values()))
    summary = {}
    for v, ts in res.items():
        band = [t["band_ms"] for t in ts]
        fa, fi = ts[-1]["flop_alg"], ts[-1]["flop_issued"]
        med = float(np.median(band))
        summary[v] = dict(band_ms_median=med, band_ms_min=float(min(band)),
                          total_ms_median=float(np.median([t["total_ms"] for t in ts])),
                          count_ms_median=float(np.median([t["count_ms"] for t in ts])),
                          alg_tflops=fa / med / 1e9,
                          issued_tflops=fi / med / 1e9, items=ts[-1]["band_items"],
                          alg_over_issued=fa / fi,
                          max_abs_l2_vs_first=float(np.nanmax(np.abs(outs[v]["l2"] - ref["l2"]))),
                          ws_equal=bool(np.array_equal(outs[v]["l2_ws"], ref["l2_ws"])))
    print(json.dumps(summary, indent=1))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(dict(config=vars(args), summary=summary), fh, indent=1)


if __name__ == "__main__":
    main()
