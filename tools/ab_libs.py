#!/usr/bin/env python3
"""Same-box, same-process A/B of engine builds: every build runs the same resident synthetic chromosome, the builds
interleaved run by run (so clock drift and box-to-box spread fall on all of them alike); band / total ms medians
per build and workload as one JSON line.
    python tools/ab_libs.py --libs new=nldsc_amd/libnldsc_amd.so old=ab_libs/r2base.so --workload c2 c3 --runs 8
Workloads: c2 (N 50 000, additive only), c3 (N 315 599, add+dom, 1 % missing), c3m0 (c3 without missing calls),
c5 (1000 kb windows, 288 bp per SNP, missing-free; --c5-snp SNPs), c3r0of8 (rank 0's owned range + halo of C3 over 8
GPUs, as bench.py --rehearse 0/8)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WORKLOADS = {  # name: (N, M, length_cm, window, missing, additive_only)
    "c2": (50_000, 80_000, 280.0, 1.0, 0.01, True),
    "c3": (315_599, 80_000, 280.0, 1.0, 0.01, False),
    "c3m0": (315_599, 80_000, 280.0, 1.0, 0.0, False),
    "c5": (315_599, None, None, 1.0e6, 0.0, False),
    "c3r0of8": (315_599, 80_000, 280.0, 1.0, 0.01, False),  # rank 0's shard of the 8-GPU strong-scaling run
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True,
                    help="name=path.so[,option=value...] (engine options, nldsc_engine_set_option; builds before round 5 "
                         "read NLDSC_<OPTION> environment variables when an engine is created, which is set for those)")
    ap.add_argument("--workload", nargs="+", default=["c3"], choices=sorted(WORKLOADS))
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--c5-snp", type=int, default=300_000)
    ap.add_argument("--no-check", action="store_true", help="study builds whose outputs differ (timing only)")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from nldsc_amd import _lib, synth
    from nldsc_amd.engine import Engine
    libs = dict(x.split("=", 1) for x in a.libs)
    out = {}
    for wl in a.workload:
        N, M, L, w, miss, add = WORKLOADS[wl]
        if wl == "c5":
            M, L = a.c5_snp, 288.0 * a.c5_snp
        buf, pos = synth.device_bed(M, N, seed=7, length_cm=L, missing=miss)
        if wl == "c5":
            pos = np.round(pos)
        own = None
        if wl == "c3r0of8":
            from nldsc_amd.distributed import halo_range, shard_ranges
            lo, hi = shard_ranges(pos, w, 8)[0]
            ha, hb = halo_range(pos, w, (lo, hi))
            nb = (N + 3) // 4
            buf = torch.cat([buf[:3], buf[3 + ha * nb:3 + hb * nb]])
            pos, M, own = pos[ha:hb], hb - ha, (lo - ha, hi - ha)
        flags = _lib.FLAG_ADDITIVE_ONLY if add else 0
        engines = {}
        for name, spec in libs.items():
            path, *kv = spec.split(",")
            opts = dict(x.split("=", 1) for x in kv)
            env = {"NLDSC_" + k.upper(): v for k, v in opts.items()}
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                e = Engine(0, lib_path=path)
                if hasattr(e._L, "nldsc_engine_set_option"):
                    for k, v in opts.items():
                        e.set_option(k, int(v))
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
            engines[name] = e
        del buf
        torch.cuda.empty_cache()
        stages = ("count_ms", "stats_ms", "schedule_ms", "band_ms", "finalize_ms", "total_ms")
        res = {name: {"band": [], "total": [], "kernel": None, "stages": {k: [] for k in stages}} for name in libs}
        ref = None
        dl2 = {name: 0.0 for name in libs}  # max |L2 - first build's L2| (and L2D), computed SNPs
        for r in range(a.runs + 1):
            for name, e in engines.items():
                got = e.run(w, 1e-4, 1e-5, 1.0 / (M if own is None else 80_000), pos, flags=flags, own=own)
                t = e.timings()
                res[name]["kernel"] = t.get("band_kernel")
                if r > 0:  # run 0 is the warmup
                    res[name]["band"].append(t["band_ms"])
                    res[name]["total"].append(t["total_ms"])
                    for k in stages:
                        res[name]["stages"][k].append(t[k])
                if ref is None:
                    ref = got
                elif not a.no_check:  # every build must agree on the integer outputs
                    for k in ("l2_ws", "l2d_ws"):
                        assert np.array_equal(got[k], ref[k]), (wl, name, k)
                if ref is not None and got is not ref:
                    ok = ref["l2_ws"] > 0
                    for k in ("l2", "l2d"):
                        d = np.abs(np.asarray(got[k])[ok] - np.asarray(ref[k])[ok])
                        d = d[np.isfinite(d)]
                        if d.size:
                            dl2[name] = max(dl2[name], float(d.max()))
        out[wl] = {name: {"band_ms_median": float(np.median(v["band"])), "band_ms_min": float(np.min(v["band"])),
                          "total_ms_median": float(np.median(v["total"])), "runs": len(v["band"]),
                          "band_kernel": v["kernel"], "max_abs_dl2_vs_first": dl2[name],
                          "stages_ms_median": {k: round(float(np.median(x)), 4) for k, x in v["stages"].items()}}
                   for name, v in res.items()}
        print(json.dumps({wl: out[wl]}), file=sys.stderr, flush=True)
        for e in engines.values():
            e.close()
    print(json.dumps({"ab": out, "libs": libs, "runs": a.runs}))


if __name__ == "__main__":
    main()
