#!/usr/bin/env python3
"""Benchmark of the LD-score hot path (BASELINE.json metric: SNP-pairs/s, chr1 N=315 599, 1 cM window).

One step = one full `calculate` pass (repack + statistics + window schedule + band correlation kernel
+ finalize + results to host) over a chromosome-sized synthetic .bed image already resident in HBM
(BASELINE.json configs[2]: N = 315 599, M = 80 000 over 280 cM, additive + dominance, --ld-wind-cm 1).
With N GPUs (torchrun, one process per GPU, RCCL) the ONE chromosome is position-sharded over the ranks
(strong scaling, as the BASELINE metric reads: chr1 at 1/2/4/8 GPUs): rank g keeps its owned SNP range plus
one window of halo rows resident, computes the owned SNPs (no hot-path exchange) and the score table is
gathered to rank 0 over RCCL every step.  `--weak` runs one chromosome per GPU instead.

Prints ONE JSON line on rank 0.  `roofline` is for the band correlation kernel (HIP events on the
engine's stream, averaged over the timed steps), on SURVEY.md §8(d3)'s FLOP basis; `wall_clock_from_file_s`
times the drop-in `_ldscore.calculate` from the .bed written to local disk; `cpu_baseline` times the C port of the reference's
CPU path (oracle/, fp32 sdot per pair, OpenMP over window neighbours) on the first SNPs of the same
chromosome (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "SNP-pairs/sec + wall-clock, chr1 N=315k 1cM window, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
I8_MFMA_PEAK_TOPS = 5000.0     # MI355X_MICROARCH.md: int8 MFMA = 2x the 2.5 PF dense bf16 rate
F4_MFMA_PEAK_TFLOPS = 10000.0  # MI355X_MICROARCH.md: fp4 (block-scaled f8f6f4) ~10 PF dense

# --path -> (engine flag name, MFMA peak, unit, dominant kernel, dtype)
PATHS = {
    "f4": ("FLAG_EXACT_F4", F4_MFMA_PEAK_TFLOPS, "TFLOP/s",
           "band_f4_kernel<true> (v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 operands, exact integer Gram in fp32)",
           "fp4"),
    "i8": ("FLAG_EXACT_I8", I8_MFMA_PEAK_TOPS, "TOP/s",
           "band_i8_kernel<true> (v_mfma_i32_32x32x32_i8, exact int32 Gram)", "i8"),
    "f32": ("FLAG_FP32", FP32_MFMA_PEAK_TFLOPS, "TFLOP/s", "band_kernel<true> (v_mfma_f32_32x32x2_f32)", "f32"),
}


def band_kernel_name(variant: str, dom: bool, default: str) -> str:
    """The band kernel that ran (Engine.timings()['band_kernel']) as rocprof names it, with what it issues."""
    d = "true" if dom else "false"
    # the single-block kernel: additive-only runs pair neighbouring column blocks per wave (engine option f4_nc2, default)
    single = ("band_f4_kernel<true, 2, 0, false> (one wave per 32x32 block pair)" if dom else
              "band_f4_kernel<false, 2, 0, false, 2> (one wave per 32x64 pair of column blocks)")
    names = {
        "f4_2x2": f"band_f4_t2_kernel<{d}, 4, false> (4-wave workgroups over 2x2 block pairs sharing their strips "
                  "through LDS, global_load_lds ring; v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 operands, exact integer "
                  "Gram in fp32)",
        "f4_routed": f"band_f4_t2_kernel<{d}, 4, false> for missing-free 2x2 super-items (4-wave workgroups sharing "
                     f"their strips through LDS) + {single} for the rest; v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 "
                     "operands, exact integer Gram in fp32",
        "f4_quad": f"band_f4_q_kernel<{d}, 4, false> for missing-free 4x4 super-items (4-wave workgroups, one 64x64 "
                   f"SNP tile of 2x2 block pairs per wave, strips shared through an LDS ring) + {single} for the "
                   "rest; v_mfma_scale_f32_32x32x64_f8f6f4, e2m1 operands, exact integer Gram in fp32",
        "f4": f"band_f4_kernel<{d}, 2, 0, false> (one wave per 32x32 block pair; v_mfma_scale_f32_32x32x64_f8f6f4, "
              "e2m1 operands, exact integer Gram in fp32)",
        "f4_ksplit": f"band_f4_part_kernel<{d}> + band_f4_epi_kernel (K-split; v_mfma_scale_f32_32x32x64_f8f6f4)",
        "f4_seg": f"band_f4_kernel<{d}, ., 4096, false> (segmented K loop; v_mfma_scale_f32_32x32x64_f8f6f4)",
    }
    return names.get(variant, default.replace("<true>", f"<{d}>"))


def kernel_source_sha16() -> str:
    """Fingerprint of the kernels' source (a PMC summary counts only for the kernels it was measured on)."""
    import hashlib
    with open(os.path.join(REPO, "nldsc_amd", "csrc", "ld_kernels.hip"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def pmc_traffic(kernel_key: str, n_org: int, n_snp: int, missing: float):
    """HBM-side bytes per engine run of `kernel_key` (all its launches) from the committed rocprofv3 PMC summary measured on the same
    workload AND the same kernel source (profiles/*_pmc*.json carrying `kernels_source_sha16`): (bytes, file),
    or (None, reason) when no summary matches the current kernels."""
    import glob
    # profiles/pmc_current.txt names the summary measured on the current kernels; then any other
    current = os.path.join(REPO, "profiles", "pmc_current.txt")
    first = []
    if os.path.exists(current):
        first = [os.path.join(REPO, "profiles", open(current).read().strip())]
    sha = kernel_source_sha16()
    stale = None
    for path in first + sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc*.json")), reverse=True):
        try:
            doc = json.load(open(path))
        except (OSError, ValueError):
            continue
        wl = doc.get("workload", "")
        if f"N={n_org}" not in wl or f"M={n_snp}" not in wl or f"missing={missing:g}" not in wl:
            continue
        if doc.get("kernels_source_sha16") != sha:
            stale = stale or os.path.relpath(path, REPO)
            continue
        keys = [kernel_key] if isinstance(kernel_key, str) else list(kernel_key)
        found = [k.get("traffic_bytes_per_run", k["traffic_bytes"]) for name, k in doc.get("kernels", {}).items()
                 if any(name.startswith(key + "<") or name == key for key in keys)]
        if found:  # (the routed fp4 band: both kernels' bytes per launch pair)
            return float(sum(found)), os.path.relpath(path, REPO)
    return None, (f"no PMC summary of the current kernels (source sha {sha}); newest for this workload: {stale}"
                  if stale else "no PMC summary for this workload")


def table_digest(out) -> dict:
    """A fingerprint of the gathered score table (outside the timed region): sha256 of the three window-count
    columns (exact integers) and the fp64 sums of L2 / L2D, so runs at different rank counts can be compared.
    `out`: the result dict, or the raw [7, M] table of a sharded run (RESULT_KEYS rows)."""
    import hashlib
    if isinstance(out, np.ndarray):
        from nldsc_amd.distributed import RESULT_KEYS
        out = {k: out[i] for i, k in enumerate(RESULT_KEYS)}
    h = hashlib.sha256()
    for k in ("l2_ws", "l2d_ws", "l2d_wse"):
        if k in out:
            h.update(np.ascontiguousarray(np.asarray(out[k]), dtype=np.int32).tobytes())
    d = {"counts_sha16": h.hexdigest()[:16], "n_snp": int(len(out["l2_ws"]))}
    for k in ("l2", "l2d"):
        if k in out:
            d[k + "_sum"] = float(np.nansum(np.asarray(out[k], dtype=np.float64)))
    return d


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(bed_host: bytes, n_snp, n_org, w, maf, std_thr, rsq, pos, target_s=15.0):
    """Time the C port of the reference CPU path on the first K SNPs (K sized for ~target_s), on the threads the box
    gives this job, then on one thread (~target_s / 4).  The host's load average and affinity set are recorded with
    it: the cores are shared with other jobs, which is what moves this figure between boxes of one CPU model."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)

    def rate(nth, target):
        # the cost per SNP grows while the first window fills, so K is sized from the marginal cost
        # between two prefixes grown geometrically until they take a quarter of the target
        def timed(k):
            t = time.perf_counter()
            r = O.run_c(bed_host, n_snp, n_org, w, maf, std_thr, rsq, pos, end=k, threads=nth)
            return r, time.perf_counter() - t
        k_prev, t_prev = 0, 0.0
        k = min(n_snp, 16)
        r0, t0 = timed(k)
        while t0 < target / 4 and k < n_snp:
            k_prev, t_prev = k, t0
            k = min(n_snp, 3 * k)
            r0, t0 = timed(k)
        if t0 < 0.6 * target and k < n_snp:
            marginal = max((t0 - t_prev) / max(k - k_prev, 1), 1e-6)
            k = int(min(n_snp, k + (target - t0) / marginal))
            r0, t0 = timed(k)
        ws = r0["l2_ws"][:k]
        return k, float(ws[ws > 0].sum()), t0

    load0 = os.getloadavg()
    k, pairs, t0 = rate(threads, target_s)
    k1, pairs1, t1 = rate(1, target_s / 4)
    load1 = os.getloadavg()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return dict(value=pairs / t0, unit="SNP-pairs/s", cores=threads, kind="port", cpu_model=cpu_model(),
                one_thread_value=pairs1 / t1, scaling_over_one_thread=(pairs / t0) / (pairs1 / t1),
                host_loadavg_1m_before_after=[round(load0[0], 2), round(load1[0], 2)], affinity_cpus=affinity,
                host_cpus=os.cpu_count(),
                sample=f"first {k} SNPs of the same chromosome (full sliding window from SNP 0), "
                       f"{pairs:.0f} pairs in {t0:.2f} s on {threads} threads; one thread: first {k1} SNPs, "
                       f"{pairs1:.0f} pairs in {t1:.2f} s; C port of the reference path (oracle/ldscore_oracle.c: "
                       f"fp32 sdot + per-pair vector copies, OpenMP over neighbours)")


def file_wall_clock(bed_host: bytes, n_snp, n_org, w, maf, std_thr, rsq, pos, flags) -> dict:
    """The metric's wall-clock half: the synthetic .bed written to a local file once, then the drop-in
    `_ldscore.calculate(params)` (nldsc/ldscore/_ldscore/ldscore.cpp:17-54 — file read, H2D, every kernel,
    results back as Python lists) timed from that file, first after the file's pages were dropped from the
    page cache (fsync + posix_fadvise DONTNEED: read from the device), then again with the file cached."""
    import tempfile
    from nldsc_amd.ldscore import _ldscore as lds
    d = tempfile.mkdtemp(prefix="nldsc_bench_", dir=os.environ.get("TMPDIR", "/tmp"))
    path = os.path.join(d, "chr1.bed")
    out = {}
    try:
        t = time.perf_counter()
        with open(path, "wb") as fh:
            fh.write(bed_host)
            fh.flush()
            os.fsync(fh.fileno())
        write_s = time.perf_counter() - t
        p = lds.LDScoreParams(path, n_snp=n_snp, n_org=n_org, ld_wind=w, maf=maf, std_thr=std_thr, rsq_thr=rsq,
                              positions=[float(x) for x in pos])
        p.flags = flags
        times = []
        for drop in (True, False):
            if drop:
                fd = os.open(path, os.O_RDONLY)
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                os.close(fd)
            t = time.perf_counter()
            r = lds.calculate(p)
            times.append(time.perf_counter() - t)
        ws = np.asarray(r.l2_ws)
        out["wall_clock_from_file_s"] = times[0]
        out["wall_clock_from_file"] = {
            "what": "_ldscore.calculate(LDScoreParams(bedfile, ...)) on the same chromosome, from a %.2f GB .bed on "
                    "local disk (written in %.1f s): file -> pinned slots -> pitched H2D -> kernels -> result lists"
                    % (len(bed_host) / 1e9, write_s),
            "page_cache_dropped_s": times[0], "page_cache_warm_s": times[1],
            "pairs": int(ws[ws > 0].sum()), "file_gbps_cold": len(bed_host) / times[0] / 1e9}
    except OSError as ex:
        out["wall_clock_from_file_s"] = None
        out["wall_clock_from_file"] = {"error": f"{type(ex).__name__}: {ex}"}
    finally:
        try:
            os.unlink(path)
            os.rmdir(d)
        except OSError:
            pass
    return out


def extra_records(eng, img_dev, M, N, w, args, rsq, pos, flags, res, res_arrays) -> dict:
    """After the timed region (N = 1, C3):
    fp32_path — the north star's fp32 MFMA GEMM (band_kernel, v_mfma_f32_32x32x2_f32) on the same resident rows, 3 timed
      runs after one warm-up: band time, its fraction of the 157.3 TF fp32 MFMA peak on the §8(d3) basis, and the table
      digest (its window counts must equal the default path's);
    oneshot_gpu_ms — what one `calculate(params)` costs per chromosome on the GPU beside the file read: the per-load
      kernels (the rows of a device image placed, oriented and scanned for missing calls: nldsc_engine_load_bed_device)
      and one run, wall clock around both (synchronous calls)."""
    import torch
    from nldsc_amd import _lib
    out = {}
    f32_flags = (flags & ~_lib.FLAG_EXACT_F4) | _lib.FLAG_FP32
    r = None
    eng.run(w, args.maf, args.std_thr, rsq, pos, flags=f32_flags)
    tims, t0 = [], time.perf_counter()
    for _ in range(3):
        r = eng.run(w, args.maf, args.std_thr, rsq, pos, flags=f32_flags)
        tims.append(eng.timings())
    wall = (time.perf_counter() - t0) / 3
    band = float(np.mean([t["band_ms"] for t in tims]))
    flop = tims[-1]["flop_alg"]
    dig = table_digest(r)
    ref = res_arrays  # the default path's last table (same rows, same parameters)
    ok = np.asarray(ref["l2_ws"]) > 0
    cmp = {"l2_ws_equal": bool(np.array_equal(r["l2_ws"], ref["l2_ws"])),
           "l2d_ws_equal": bool(np.array_equal(r["l2d_ws"], ref["l2d_ws"])),
           # WSDE counts r2adj > rsq_thr: pairs within fp32 rounding of the threshold may flip
           "l2d_wse_snps_differing": int(np.sum(np.asarray(r["l2d_wse"]) != np.asarray(ref["l2d_wse"]))),
           "l2_max_abs_diff": float(np.max(np.abs(np.asarray(r["l2"])[ok] - np.asarray(ref["l2"])[ok])))
           if ok.any() else 0.0}
    out["fp32_path"] = {
        "kernel": "band_kernel<true, 2> (v_mfma_f32_32x32x2_f32 on fp32 standardised values, LDS-staged lookup of the "
                  "2-bit rows)", "steps": 3, "ms_per_step": round(1e3 * wall, 3), "band_ms": round(band, 3),
        "achieved_tflops": flop / (band * 1e-3) / 1e12, "peak_tflops": FP32_MFMA_PEAK_TFLOPS,
        "frac": flop / (band * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
        "pairs_per_s": tims[-1]["pairs"] / wall, "table_digest": dig,
        "counts_equal_default_path": dig["counts_sha16"] == res["table_digest"]["counts_sha16"],
        "vs_default_path": cmp, "l2_sum_delta_vs_default": dig["l2_sum"] - res["table_digest"]["l2_sum"]}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.load_bed_device(img_dev.data_ptr(), img_dev.numel(), M, N)
    t1 = time.perf_counter()
    eng.run(w, args.maf, args.std_thr, rsq, pos, flags=flags)
    t2 = time.perf_counter()
    out["oneshot_gpu_ms"] = {"total": round(1e3 * (t2 - t0), 3), "load": round(1e3 * (t1 - t0), 3),
                             "run": round(1e3 * (t2 - t1), 3),
                             "what": "nldsc_engine_load_bed_device (rows placed in the resident layout, oriented, scanned "
                                     "for missing calls) + one run, from a .bed image already in HBM: the GPU side of "
                                     "one calculate(params) per chromosome (the file read apart)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n-org", type=int, default=315_599)
    ap.add_argument("--n-snp", type=int, default=80_000)
    ap.add_argument("--length-cm", type=float, default=280.0)
    ap.add_argument("--window-cm", type=float, default=1.0)
    ap.add_argument("--maf", type=float, default=1e-4)
    ap.add_argument("--std-thr", type=float, default=1e-5)
    ap.add_argument("--additive-only", action="store_true")
    ap.add_argument("--missing", type=float, default=None,
                    help="missing-call rate of the synthetic genotypes (default 0.01; C5: 0, imputed hard calls)")
    ap.add_argument("--path", choices=tuple(PATHS), default="f4",
                    help="correlation path: exact Gram on fp4 MFMAs (default), on int8 MFMAs, or fp32 "
                         "standardised values")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="collectives backend for N > 1 (gloo: rehearse several ranks on one GPU)")
    ap.add_argument("--workload", choices=("c3", "c4", "c5"), default="c3",
                    help="c3: one chr1-like chromosome per GPU (default, the BASELINE metric); c4: the 22-autosome "
                         "whole genome (sum M ~ 600k, BASELINE.json configs[3]) spread over the GPUs by LPT; c5: one "
                         "eighth of the imputed genome per GPU (BASELINE.json configs[4]: M ~ 10M over 2.88 Gb, "
                         "--ld-wind-kb 1000; --n-snp defaults to 1.25M per GPU)")
    ap.add_argument("--weak", action="store_true",
                    help="c3 with N > 1: one chromosome per GPU (weak scaling) instead of the default, ONE chromosome "
                         "position-sharded over the GPUs (strong scaling, what the BASELINE metric reads: chr1 at "
                         "1/2/4/8 GPUs)")
    ap.add_argument("--split", action="store_true", help=argparse.SUPPRESS)  # the default since round 2
    ap.add_argument("--rehearse", default=None, metavar="R/N",
                    help="one process on one GPU doing exactly what rank R of an N-GPU strong-scaling run does "
                         "(its owned range + halo resident, its share of the chromosome), without the gather")
    ap.add_argument("--no-file", action="store_true",
                    help="skip the wall clock from a PLINK file (rank 0, N = 1: the synthetic .bed written to "
                         "$TMPDIR, then _ldscore.calculate timed from the file)")
    ap.add_argument("--no-gather-overlap", action="store_true",
                    help="strong scaling over RCCL: gather each step's table before the next step starts (default: "
                         "on a side stream, beside the next step's compute)")
    ap.add_argument("--split-halo", action="store_true",
                    help="N > 1: compute each boundary pair once, on the rank owning the lower SNP, and send the right "
                         "halo's sums to the next rank point to point, instead of a two-sided halo on both ranks "
                         "(measured equal at C3/8, so not the default)")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the process group and run the sharded path (owned range, device table, collective "
                         "gather) even with one rank: the RCCL code of an N-GPU run rehearsed on one GPU")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the default line's extra records after the timed region (N = 1, C3): the fp32 MFMA path "
                         "(fp32_path) and the one-shot load + run GPU time (oneshot_gpu_ms)")
    ap.add_argument("--concurrent", type=int, default=3,
                    help="c4: chromosomes computed at once per GPU (host threads, one engine stream each)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option (nldsc_engine_set_option, include/nldsc_ld.h), repeatable: a study of a "
                         "non-default schedule, e.g. --option debug_timing=1")
    args = ap.parse_args()
    args.engine_options = {k: int(v) for k, v in (o.split("=", 1) for o in args.option)}

    # --gpus N without a launcher: start the N ranks here (torch.distributed.run in a child process, before
    # anything touches the GPU) and exit with their status; under a launcher, WORLD_SIZE must equal --gpus
    if not args.rehearse:
        from nldsc_amd.launch import ranks_or_spawn
        rc = ranks_or_spawn(os.path.abspath(__file__), sys.argv[1:], args.gpus, args.backend)
        if rc is not None:
            sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    if args.backend == "gloo":
        local = 0  # rehearsal: every rank shares GPU 0
    torch.cuda.set_device(local)
    use_dist = world > 1 or args.force_dist
    if use_dist and "MASTER_ADDR" not in os.environ:  # --force-dist without a launcher: a group of one
        from nldsc_amd.launch import free_port
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    if use_dist:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    coll = "cuda" if args.backend == "nccl" else "cpu"

    from nldsc_amd import _lib, synth
    from nldsc_amd.engine import Engine

    if args.workload == "c4":
        return whole_genome(args, world, rank, local, coll)
    if args.workload == "c5":  # bp positions: 2.88 Gb / 10M SNPs = 288 bp per SNP, window 1000 kb
        if args.n_snp == ap.get_default("n_snp"):
            args.n_snp = 1_250_000
        args.length_cm = 288.0 * args.n_snp
        args.window_cm = 1.0e6
        args.no_cpu = True
        if args.missing is None:
            args.missing = 0.0  # imputed genotypes (hard calls) have no missing calls
    if args.missing is None:
        args.missing = 0.01
    N, M = args.n_org, args.n_snp
    flags = (_lib.FLAG_ADDITIVE_ONLY if args.additive_only else 0) | getattr(_lib, PATHS[args.path][0])
    t = time.perf_counter()
    s_rank, s_world = rank, world
    if args.rehearse:
        if world > 1:
            raise SystemExit("--rehearse is a single-process mode")
        s_rank, s_world = (int(x) for x in args.rehearse.split("/"))
    split = (s_world > 1 or (args.force_dist and not args.rehearse)) and not args.weak
    plan = None  # split halo plan (boundary pairs once), when `split`
    overlap = False  # (strong scaling over RCCL: the gather beside the next step, below)
    buf, pos = synth.device_bed(M, N, seed=7 if split else 7 + rank, length_cm=args.length_cm,
                                missing=args.missing, device=local)
    eng = Engine(local, options=args.engine_options)
    own = (0, M)
    if split:
        # --split: ONE chromosome position-sharded over the ranks (strong scaling): rank g keeps only its
        # owned SNP range plus one window of halo rows resident and computes the owned SNPs
        from nldsc_amd.distributed import (RESULT_KEYS, exchange_halo, gather_spans, gather_table, halo_range,
                                           shard_ranges, split_plan, table_width)
        # --split-halo: rank g loads its owned range + the right halo, computes the pairs whose lower SNP it owns and
        # sends the halo's sums to rank g + 1 (one point-to-point block per step); by default a two-sided halo with
        # the boundary pairs computed by both neighbours (the same band time at C3/8, no exchange)
        plan = split_plan(pos, args.window_cm, s_world) if args.split_halo else None
        if plan is not None:
            lo, hi, b = plan[s_rank]
            a = lo
            n_recv = plan[s_rank - 1][2] - plan[s_rank - 1][1] if s_rank > 0 else 0
        else:
            lo, hi = shard_ranges(pos, args.window_cm, s_world)[s_rank]
            a, b = halo_range(pos, args.window_cm, (lo, hi))
        nb = (N + 3) // 4
        sl = torch.cat([buf[:3], buf[3 + a * nb:3 + b * nb]])
        eng.load_bed_device(sl.data_ptr(), sl.numel(), b - a, N)
        del sl
        own, own_rel, pos = (lo, hi), (lo - a, hi - a), pos[a:b]
        # the owned slice of the score table stays in HBM ([7, width] fp64 block, nldsc_engine_run_device); the
        # blocks are gathered device to device (RCCL) and only rank 0 copies the gathered table to the host
        spans = gather_spans(own, device=coll) if use_dist else [own]  # the sharding is fixed across steps
        table = torch.empty((len(RESULT_KEYS), table_width(spans)), dtype=torch.float64, device=f"cuda:{local}")
        gbuf = torch.empty(world * table.numel(), dtype=torch.float64,
                           device=table.device if coll == "cuda" else "cpu") if use_dist else None
        # RCCL: step k's table is gathered on a side stream while step k + 1 computes into the other table buffer (the
        # gather is an RCCL all-gather + rank 0's assembly and one D2H copy; every step's gather is still inside the
        # timed region: the closing synchronize waits for the last)
        overlap = use_dist and coll == "cuda" and plan is None and not args.no_gather_overlap
        if overlap:
            tables, gbufs = [table, torch.empty_like(table)], [gbuf, torch.empty_like(gbuf)]
            gstream = torch.cuda.Stream(device=table.device)
            gdone = [None, None]
        if plan is not None:
            export = torch.empty(6 * max(b - hi, 1), dtype=torch.int64, device=table.device)
            imported = torch.zeros(6 * max(n_recv, 1), dtype=torch.int64, device=table.device)
    else:
        eng.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
    if not split:
        # the run's positions and result arrays in pinned host memory (nldsc_host_alloc): the positions go up by DMA in
        # place and the GPU writes the results into the arrays themselves (include/nldsc_ld.h; ordinary numpy arrays work
        # too, through the engine's landing buffer and a host copy)
        pos_p = _lib.pinned_empty(M, np.float64)
        pos_p[:] = pos
        pos = pos_p
        out = _lib.alloc_result(M, pinned=True)[0]
    bed_host = None
    want_file = rank == 0 and not use_dist and not args.no_file and args.workload == "c3"
    if rank == 0 and not use_dist and (not args.no_cpu or want_file):
        bed_host = buf.cpu().numpy().tobytes()
    # (N = 1: the device image stays for the one-shot measurement after the timed region)
    want_extra = (rank == 0 and not use_dist and not split and not args.no_extra and args.workload == "c3"
                  and args.path == "f4")
    img_dev = buf if want_extra else None
    del buf
    torch.cuda.empty_cache()
    log(f"[rank {rank}] data ready ({(3 + M * ((N + 3) // 4)) / 1e9:.2f} GB .bed image) in "
        f"{time.perf_counter() - t:.1f} s")
    w, rsq = args.window_cm, 1.0 / M
    out = out if not split else None
    n_step = 0
    gath = []  # overlapped gathers: (step, start event, end event) on gstream, read after the timed region

    def step():
        nonlocal out, n_step
        if split and overlap:
            cur = n_step % 2
            n_step += 1
            tw = time.perf_counter()
            if gdone[cur] is not None:
                gdone[cur].synchronize()  # the gather of step k - 2 has read this table buffer
            wait_ms = 1e3 * (time.perf_counter() - tw)
            eng.run_device(w, args.maf, args.std_thr, rsq, pos, tables[cur], own=own_rel, flags=flags)
            tim = eng.timings()
            tg = time.perf_counter()
            with torch.cuda.stream(gstream):
                # the gather's own GPU time (RCCL all-gather, rank 0's assembly and D2H) between two events on gstream,
                # read after the timed region (gather_ms); the host's enqueue time apart (gather_enqueue_ms)
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(gstream)
                full = gather_table(tables[cur], spans, M, out=gbufs[cur], raw=True, slot=cur, sync=False)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(gstream)
            gdone[cur] = ev
            gath.append((n_step - 1, e0, ev))
            out = full if full is not None else out  # (rank 0: read after the closing synchronize)
            tim["gather_enqueue_ms"] = 1e3 * (time.perf_counter() - tg)
            tim["gather_wait_ms"] = wait_ms  # this step's wait for the gather of step k - 2
            return tim
        if split:  # owned slice of the one chromosome, then the table assembled on rank 0 (RCCL over xGMI)
            if plan is not None:  # (a rehearsal of one rank adds a zero block in place of its neighbour's)
                n_send = eng.run_device_split(w, args.maf, args.std_thr, rsq, pos, table, export, own=own_rel,
                                              flags=flags)
                if use_dist:
                    exchange_halo(export, n_send, imported, n_recv)
                eng.run_device_finish(imported, n_recv)
            else:
                eng.run_device(w, args.maf, args.std_thr, rsq, pos, table, own=own_rel, flags=flags)
            tim = eng.timings()
            tg = time.perf_counter()
            if use_dist:  # (RCCL: rank 0 gets the assembled table in pinned host memory, no per-step host copies)
                full = gather_table(table if coll == "cuda" else table.cpu(), spans, M, out=gbuf, raw=True)
                out = full if full is not None else out
            else:  # rehearsal of one rank: its slice to the host
                out = {"l2_ws": table[4].cpu().numpy()}
            tim["gather_ms"] = 1e3 * (time.perf_counter() - tg)
            return tim
        out = eng.run(w, args.maf, args.std_thr, rsq, pos, flags=flags, out=out)
        if world > 1:  # assemble the score tables on rank 0 (RCCL over xGMI)
            tab = torch.from_numpy(np.stack([out["l2"], out["l2d"], out["maf"], out["residuals_std"],
                                             out["l2_ws"].astype(np.float64), out["l2d_ws"].astype(np.float64),
                                             out["l2d_wse"].astype(np.float64)])).to(coll)
            gathered = [torch.empty_like(tab) for _ in range(world)]
            dist.all_gather(gathered, tab)
        return eng.timings()

    for _ in range(args.warmup):
        step()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    gath.clear()
    t0 = time.perf_counter()
    tims = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for (k, e0, e1), tim in zip(gath, tims):  # overlapped gathers: GPU time on gstream (all-gather + assembly + D2H)
        tim["gather_ms"] = float(e0.elapsed_time(e1))
    el = torch.tensor([elapsed], dtype=torch.float64, device=coll)
    pairs_step = torch.tensor([tims[-1]["pairs"]], dtype=torch.float64, device=coll)
    if use_dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(pairs_step, op=dist.ReduceOp.SUM)
    t_max = float(el.item())
    total_pairs = float(pairs_step.item()) * args.steps
    # per-rank stage times (band kernel, gather, engine total) for the scaling record
    mine = torch.tensor([float(np.mean([x["band_ms"] for x in tims])),
                         float(np.mean([x.get("gather_ms", 0.0) for x in tims])),
                         float(np.mean([x["total_ms"] for x in tims])), float(tims[-1]["pairs"]),
                         float(own[1] - own[0]), float(np.mean([x.get("gather_enqueue_ms", 0.0) for x in tims])),
                         float(np.mean([x.get("gather_wait_ms", 0.0) for x in tims]))],
                        dtype=torch.float64, device=coll)
    per_rank = [mine]
    if use_dist:
        per_rank = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)

    res = None
    if rank == 0:
        band_ms = float(np.mean([x["band_ms"] for x in tims]))
        t_band = band_ms * 1e-3
        flop = tims[-1]["flop_alg"]
        path = tims[-1]["path"]
        _, peak, unit, kname, dtype = PATHS[path]
        kname = band_kernel_name(tims[-1].get("band_kernel", path), not args.additive_only, kname)
        # roofline on SURVEY.md §8(d3)'s basis for every path: FLOP_alg = 2N(1/2 sumWSA + sumWSD) (the reference
        # formulation's multiply-adds) over the band kernel's time, against the dense MFMA peak of the dtype
        # that ran.  The exact paths issue more: 8 integer Gram entries per pair (frac_8_product_basis).
        roof = {"bound": "mfma", "achieved": flop / t_band / 1e12, "peak": peak, "unit": unit, "kernel": kname,
                "flop_alg_per_launch": flop,
                "flop_alg_definition": "SURVEY.md §8(d3): 2N(1/2 sumWSA + sumWSD) multiply-adds x2 (additive Gram "
                                       "once per unordered pair, dominance cross term per ordered pair)"}
        roof["frac"] = roof["achieved"] / peak
        if path != "f32":
            # the exact formulation's floor: 8 integer Gram entries per unordered pair for add+dom (vv, vm, mv, mm;
            # vh, mh, hv, hm) against the 3 dots FLOP_alg counts (one additive, two dominance cross terms) = 8/3; 4
            # per 1 additive-only.  Above the floor: products of 32x32 blocks that fall outside the windows
            roof.update(issued_over_alg=tims[-1]["flop_issued"] / flop if flop > 0 else None,
                        issued_over_alg_floor=(4.0 if args.additive_only else 8.0 / 3.0),
                        issued_over_alg_note="a ratio of FLOP counts, not a fraction of peak: the MFMA products the "
                                             "band kernels issued (counted per item on the GPU, skipped products "
                                             "of missing-free blocks excluded) over FLOP_alg")
        traffic, traffic_src = pmc_traffic(
            ("band_f4_t2_kernel", "band_f4_q_kernel", "band_f4_kernel", "band_f4_part_kernel",
             "band_f4_epi_kernel")  # (any super-item kernel + the single-block kernel + the K-split tail)
            if path == "f4" else kname.split("<")[0],
            N, M, args.missing)
        if split:  # (the summaries are of the whole chromosome on one GPU, not of one rank's shard)
            traffic, traffic_src = None, "no PMC summary of a sharded run (profiles' summaries: the whole chromosome)"
        roof.update(traffic=traffic, traffic_source=traffic_src,
                    algorithmic_bytes_per_launch=eng.n_snp * 4 * ((((N + 3) // 4) + 31) // 32 * 8),
                    avg_launch_ms=band_ms,
                    launch_note=("the band of one run (all its launches: %d items in launches of %d, one round of "
                                 "the wave slots each; rocprofv3 lists each launch) timed with HIP events on the "
                                 "engine stream" % (tims[-1]["band_items"], tims[-1]["band_round_items"])
                                 if tims[-1].get("band_round_items") else
                                 "one band launch per run, timed with HIP events on the engine stream"),
                    issued_per_launch=tims[-1]["flop_issued"], work_items=tims[-1]["band_items"],
                    mfma_pipe_frac=tims[-1]["flop_issued"] / t_band / 1e12 / peak)
        stages = {k: round(float(np.mean([x[k] for x in tims])), 3)
                  for k in ("count_ms", "stats_ms", "schedule_ms", "band_ms", "finalize_ms", "total_ms")}
        if split:
            stages["gather_ms"] = round(float(np.mean([x["gather_ms"] for x in tims])), 3)
        if isinstance(out, np.ndarray):  # a sharded run's raw [7, M] table (RESULT_KEYS rows)
            from nldsc_amd.distributed import RESULT_KEYS
            out = {k: out[i] for i, k in enumerate(RESULT_KEYS)}
        ws = np.asarray(out["l2_ws"])
        res = {
            "metric": METRIC,
            "value": total_pairs / t_max,
            "unit": "SNP-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_max / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if split else "weak",
            **({"rehearsal": f"rank {s_rank} of {s_world} on one GPU (no gather): its owned SNPs / time"}
               if args.rehearse else {}),
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (GPU-generated PLINK .bed, AR(1) haplotypes, %g%% missing calls; %s)"
                    % (100 * args.missing, "one chromosome split over the GPUs" if split else "one chromosome per GPU"),
            "config": {
                "workload": (("%s: chr1-like N=%d individuals, M=%d SNPs over %.0f cM, "
                              "%s, --ld-wind-cm %g, maf %g, std-thr %g, rsq 1/M" %
                              ("C2 (BASELINE.json configs[1])" if N == 50_000 and args.additive_only else
                               "C3 (BASELINE.json configs[2])" if N == 315_599 and not args.additive_only else
                               "C3-shaped variant (BASELINE.json configs[2] with N / coding changed)",
                               N, M, args.length_cm, "additive only" if args.additive_only else "additive+dominance",
                               w, args.maf, args.std_thr)) if args.workload == "c3" else
                             ("C5 slice (BASELINE.json configs[4]: imputed genome, M~10M over 2.88 Gb, --ld-wind-kb "
                              "1000, 8 GPUs): per GPU N=%d individuals, M=%d SNPs over %.0f Mb (1/8 genome at M=1.25M), "
                              "%s, window %g bp, maf %g, std-thr %g, rsq 1/M" %
                              (N, M, args.length_cm / 1e6, "additive only" if args.additive_only else
                               "additive+dominance", w, args.maf, args.std_thr))),
                **({"engine_options": args.engine_options} if args.engine_options else {}),
                "n_org": N, "n_snp": M, "mean_window": float(ws[ws > 0].mean()),
                "pairs_per_step_per_gpu": tims[-1]["pairs"],
                "parallelism": (f"one chromosome position-sharded over {world} GPUs (owned SNP ranges balanced by "
                                f"pair work, " + ("one window of right-halo rows per rank, boundary pairs computed "
                                                  "once and the halo's sums sent to the next rank point to point"
                                                  if plan is not None else "one window of halo rows per rank") +
                                f", score table gathered over {'RCCL' if coll == 'cuda' else 'gloo'}" +
                                (" on a side stream beside the next step's compute" if overlap else "") + ")"
                                if split else f"position sharding, one chromosome unit per GPU x {world}"),
            },
            "roofline": roof,
            "stages_ms": stages,
            "per_rank": [dict(rank=g, band_ms=round(float(v[0]), 3), gather_ms=round(float(v[1]), 3),
                              engine_ms=round(float(v[2]), 3), pairs=int(v[3]), owned_snps=int(v[4]),
                              **({"gather_enqueue_ms": round(float(v[5]), 3), "gather_wait_ms": round(float(v[6]), 3)}
                                 if overlap else {}))
                         for g, v in enumerate(x.cpu() for x in per_rank)],
            **({"rccl_world": dist.get_world_size(), "collectives_backend": dist.get_backend()} if use_dist else {}),
            **({"gather_note": "gather_ms: each step's score-table gather (RCCL all-gather, rank 0's assembly and its "
                               "D2H copy) timed with HIP events on the side stream it runs on, beside the next step's "
                               "compute; gather_wait_ms: the host's wait for the gather two steps back before reusing its "
                               "buffer; gather_enqueue_ms: the host time to enqueue it"} if overlap else {}),
            "cpu_baseline": None,
            "table_digest": table_digest(out),
        }
    if want_extra:
        res.update(extra_records(eng, img_dev, M, N, w, args, rsq, pos, flags, res,
                                 {k: np.array(v) for k, v in out.items()}))
        del img_dev
    if want_file:
        log("[rank 0] wall clock from a PLINK file ...")
        res.update(file_wall_clock(bed_host, M, N, w, args.maf, args.std_thr, rsq, pos, flags))
    if bed_host is not None and not args.no_cpu:
        log("[rank 0] timing the CPU baseline ...")
        res["cpu_baseline"] = cpu_baseline(bed_host, M, N, w, args.maf, args.std_thr, rsq, pos,
                                           target_s=args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    eng.close()
    if use_dist:
        dist.destroy_process_group()


# approximate sex-averaged genetic map lengths of the 22 autosomes (cM)
AUTOSOME_CM = [278, 263, 224, 214, 209, 193, 184, 169, 167, 181, 158, 174, 126, 119, 141, 134, 128, 117, 108, 108,
               63, 72]


def whole_genome(args, world, rank, local, coll):
    """C4: 22 autosomes, M_c proportional to genetic length (sum ~600k), N = 315 599, --ld-wind-cm 1.  Chromosome
    units are assigned to ranks by LPT; each rank keeps its units resident in HBM; one step = every unit of every
    rank computed; value = all ranks' pairs / max-over-ranks wall time."""
    import torch
    import torch.distributed as dist

    from nldsc_amd import _lib, synth
    from nldsc_amd.distributed import assign_units
    from nldsc_amd.engine import Engine
    N, total = args.n_org, 600_000
    L = np.array(AUTOSOME_CM, dtype=float)
    Mc = np.maximum(1000, np.round(total * L / L.sum())).astype(int)
    mine = assign_units(list(Mc * 1.0), world)[rank]
    flags = getattr(_lib, PATHS[args.path][0])
    units = []
    t = time.perf_counter()
    for u in mine:
        buf, pos = synth.device_bed(int(Mc[u]), N, seed=100 + u, length_cm=float(L[u]), device=local)
        e = Engine(local, options=args.engine_options)
        e.load_bed_device(buf.data_ptr(), buf.numel(), int(Mc[u]), N)
        del buf
        units.append((u, e, pos))
    torch.cuda.empty_cache()
    log(f"[rank {rank}] {len(units)} chromosomes resident ({int(Mc[mine].sum())} SNPs) in {time.perf_counter() - t:.1f} s")

    # chromosomes run from `--concurrent` host threads (each engine has its own streams; the ctypes
    # calls release the GIL), so one chromosome's count, schedule and band tail overlap another's band
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=max(1, args.concurrent))

    def one(unit):
        u, e, pos = unit
        e.run(args.window_cm, args.maf, args.std_thr, 1.0 / int(Mc[u]), pos, flags=flags)
        return e.timings()["pairs"]

    def step():
        if args.concurrent <= 1:
            return sum(one(x) for x in units)
        return sum(pool.map(one, units))

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pairs = sum(step() for _ in range(args.steps))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll)
    pr = torch.tensor([pairs], dtype=torch.float64, device=coll)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(pr, op=dist.ReduceOp.SUM)
    if rank == 0:
        t_max = float(el.item())
        print(json.dumps({
            "metric": METRIC, "value": float(pr.item()) / t_max, "unit": "SNP-pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": PATHS[args.path][4],
            "data": "synthetic (GPU-generated PLINK .bed per autosome)",
            "config": {"workload": "C4 (BASELINE.json configs[3]): 22 autosomes, sum M=%d (M_c proportional to cM "
                                   "length), N=%d, --ld-wind-cm %g, additive+dominance, chromosome units over GPUs "
                                   "by LPT, %d at once per GPU" % (int(Mc.sum()), N, args.window_cm, args.concurrent),
                       "whole_genome_seconds": t_max / args.steps},
        }), flush=True)
    pool.shutdown()
    for _, e, _ in units:
        e.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
