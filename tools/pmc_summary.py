#!/usr/bin/env python3
"""HBM traffic and MFMA utilisation per kernel from three rocprofv3 --pmc passes of one bench command
(MI355X_MICROARCH.md §HBM: one counter group per pass, --kernel-trace only):

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir>/fetch -o f --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d <dir>/write -o w --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --kernel-trace \\
        -d <dir>/sq -o s --output-format csv -- python3 bench.py ...

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d <dir>/l2 -o l --output-format csv -- ...  (optional)
    rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --kernel-trace \
        -d <dir>/lds -o d --output-format csv -- ...  (optional)

    python tools/pmc_summary.py <dir> --workload "..." --alg-bytes band_f4_kernel=6312960000 > profiles/rNN_pmc.json

FETCH_SIZE / WRITE_SIZE are in KB; gfx950 reports half of wide streaming reads, so FETCH_SIZE is
doubled (calibrated by repack_count_kernel, whose corrected fetch equals its .bed input).  Values are
averaged over the launches of each kernel (per launch); `traffic_bytes_per_run` sums a kernel's launches of one
engine run (the band kernel goes in several launches of one round each).  MFMA busy fraction per SIMD =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); effective clock = GRBM_GUI_ACTIVE / 8 /
duration (GRBM_GUI_ACTIVE is reported summed over the 8 XCDs).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

N_SIMD = 256 * 4
N_XCD = 8  # GRBM_GUI_ACTIVE comes summed over the 8 XCDs


def read_counters(d):
    """{short kernel name: {counter: [per-dispatch values]}, '_dur': [...]} from one pass directory."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = defaultdict(lambda: defaultdict(list))
    seen = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nldsc::", "")
            key = (r["Dispatch_Id"], r["Counter_Name"])
            if key in seen:  # counters summed over XCD/SE instances already; keep one row per dispatch
                out[name][r["Counter_Name"]][seen[key]] += float(r["Counter_Value"])
                continue
            seen[key] = len(out[name][r["Counter_Name"]])
            out[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "GRBM_GUI_ACTIVE"):
                out[name]["_dur_" + r["Counter_Name"]].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return out


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--alg-bytes", action="append", default=[], help="kernel=bytes algorithmic bytes per launch")
    args = ap.parse_args()
    alg = dict((k, float(v)) for k, v in (a.split("=") for a in args.alg_bytes))
    fetch, write, sq, l2, lds = (read_counters(os.path.join(args.dir, p))
                                 for p in ("fetch", "write", "sq", "l2", "lds"))
    # engine runs in the profiled command: tail_counts_kernel runs once per run (the band may take several launches;
    # round 4's per-run finalize_kernel is finalize_out_kernel for host results since round 5)
    runs = next((len(fetch[k]["FETCH_SIZE"]) for k in ("tail_counts_kernel", "finalize_out_kernel", "finalize_kernel")
                 if fetch.get(k, {}).get("FETCH_SIZE")), None)
    kernels = {}
    for name in sorted(set(fetch) | set(write) | set(sq)):
        if name.startswith("__amd"):
            continue
        f = mean(fetch.get(name, {}).get("FETCH_SIZE", []))
        w = mean(write.get(name, {}).get("WRITE_SIZE", []))
        g = mean(sq.get(name, {}).get("GRBM_GUI_ACTIVE", []))
        busy = mean(sq.get(name, {}).get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        valu = mean(sq.get(name, {}).get("SQ_INSTS_VALU", []))
        dur = mean(sq.get(name, {}).get("_dur_GRBM_GUI_ACTIVE", []))
        k = {"fetch_size_bytes_raw": f * 1024 if f is not None else None,
             "fetch_bytes_corrected_x2": 2 * f * 1024 if f is not None else None,
             "write_bytes": w * 1024 if w is not None else None}
        k["traffic_bytes"] = (k["fetch_bytes_corrected_x2"] or 0) + (k["write_bytes"] or 0)
        n_disp = len(fetch.get(name, {}).get("FETCH_SIZE", []))
        if runs and n_disp:  # per engine run: all launches of this kernel in one run
            k["dispatches_per_run"] = n_disp / runs
            k["traffic_bytes_per_run"] = k["traffic_bytes"] * n_disp / runs
        base = name.split("<")[0]
        if base in alg:
            k["algorithmic_bytes"] = alg[base]
            k["traffic_over_algorithmic"] = k.get("traffic_bytes_per_run", k["traffic_bytes"]) / alg[base]
        k.update(duration_s_pmc_run=dur, grbm_gui_active=g, sq_valu_mfma_busy_cycles=busy, sq_insts_valu=valu)
        if g and busy is not None:
            k["mfma_busy_frac_per_simd"] = busy / (g / N_XCD * N_SIMD)
        if g and dur:
            k["effective_clock_ghz"] = g / N_XCD / dur / 1e9
        if k["traffic_bytes"] and dur:
            k["hbm_gbps"] = k["traffic_bytes"] / dur / 1e9
        hit, miss = mean(l2.get(name, {}).get("TCC_HIT_sum", [])), mean(l2.get(name, {}).get("TCC_MISS_sum", []))
        if hit is not None and miss is not None:
            k.update(l2_hit=hit, l2_miss=miss, l2_hit_rate=hit / max(hit + miss, 1.0))
        for c in ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_LDS_IDX_ACTIVE"):
            v = mean(lds.get(name, {}).get(c, []))
            if v is not None:
                k[c.lower()] = v
        if k.get("sq_lds_idx_active"):
            k["lds_bank_conflict_frac"] = k.get("sq_lds_bank_conflict", 0.0) / k["sq_lds_idx_active"]
        kernels[name] = k
    import hashlib
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nldsc_amd", "csrc", "ld_kernels.hip")
    json.dump({"workload": args.workload,
               "kernels_source_sha16": hashlib.sha256(open(src, "rb").read()).hexdigest()[:16],
               "method": "rocprofv3 --pmc <one counter group> --kernel-trace, separate passes for FETCH_SIZE, "
                         "WRITE_SIZE and SQ/GRBM; FETCH_SIZE/WRITE_SIZE in KB; FETCH_SIZE doubled per "
                         "MI355X_MICROARCH.md §HBM (gfx950 reports half of wide streaming reads; calibrated by the "
                         "repack kernel, whose corrected fetch equals its input); per-launch means",
               "kernels": kernels}, fp := __import__("sys").stdout, indent=1)
    fp.write("\n")


if __name__ == "__main__":
    main()
