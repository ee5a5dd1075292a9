#!/usr/bin/env python3
"""Whole-genome `nldsc ld --bfile chr@` from .bed files on one GPU (BASELINE.json configs[3], the north star's
"22 autosomes, N=315k, M~600k, 1 cM in < 5 min"; the reference's per-file caller is nldsc/ldscore/routine.py:51-102).

  --autosomes   the 22 autosomes at C4 sizes: M_c proportional to each chromosome's genetic length (sum ~600 k),
                N = 315 599 (~47 GB of .bed), cM positions over the chromosome's length
  --chroms K    K equal chromosomes of --n-snp SNPs over 70 cM (the round-1 I/O study)

Files are written to --dir (a .bed of the right size already there is reused).  Afterwards, unless --keep, the tool
removes exactly the files it wrote (chrN.bed/.bim/.fam, its out/ TSVs) and --dir only if it created it and it is then
empty — never anything else found there.  Then, with every .bed's pages dropped
from the page cache (fsync + POSIX_FADV_DONTNEED) before each cold run:
  cli      - `python -m nldsc_amd ld --bfile <dir>/chr@ --ld-wind-cm 1 --out <out>/o@.L2 --extra --quiet` as a child
             process: the wall clock a user sees (interpreter start, imports, every file, every TSV)
  stages   - estimate_lds_genome in this process with a runner that times each chromosome's load (read + H2D +
             row placement) and run (every kernel + results to host); the TSV write is the rest of each chromosome
  warm     - the CLI again with the files in the page cache
and an 8-GPU projection: the measured per-chromosome times assigned to 8 ranks by LPT (the CLI's own assignment),
bounded below by the bytes over the box's measured cold read rate (8 ranks share one host's disk).
    python tools/e2e_genome.py --autosomes --out gpurun_out/e2e_genome_c4.json
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# approximate sex-averaged genetic map lengths of the 22 autosomes (cM), as bench.py's C4 workload
AUTOSOME_CM = [278, 263, 224, 214, 209, 193, 184, 169, 167, 181, 158, 174, 126, 119, 141, 134, 128, 117, 108, 108,
               63, 72]


def drop_pages(paths):
    for p in paths:
        fd = os.open(p, os.O_RDONLY)
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)


def write_set(stem, chrom, M, N, seed, length_cm, missing, created):
    """stem.bed/.bim/.fam; the .bed generated on the GPU (synth.device_bed) and streamed to disk.  Every path this
    call writes is appended to `created` (the cleanup removes those and nothing else)."""
    from nldsc_amd import synth
    nb = (N + 3) // 4
    want = 3 + M * nb
    buf, pos = synth.device_bed(M, N, seed=seed, length_cm=length_cm, missing=missing)
    if not (os.path.exists(stem + ".bed") and os.path.getsize(stem + ".bed") == want):
        created.append(stem + ".bed")
        with open(stem + ".bed", "wb") as fh:
            step = 1 << 30
            for o in range(0, want, step):  # 1 GiB pieces: bounded host memory
                fh.write(buf[o:o + step].cpu().numpy().tobytes())
    del buf
    bp = np.round(pos * 1e6).astype(np.int64)
    if not os.path.exists(stem + ".bim"):
        created.append(stem + ".bim")
    with open(stem + ".bim", "w") as fh:
        fh.writelines(f"{chrom}\trs{chrom}_{j}\t{pos[j]:.6f}\t{bp[j]}\tA\tG\n" for j in range(M))
    if not os.path.exists(stem + ".fam"):
        created.append(stem + ".fam")
        with open(stem + ".fam", "w") as fh:
            fh.writelines(f"f{i}\ti{i}\t0\t0\t0\t-9\n" for i in range(N))
    return want


def lpt(times, world):
    load = np.zeros(world)
    for t in sorted(times, reverse=True):
        load[int(np.argmin(load))] += t
    return float(load.max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--autosomes", action="store_true")
    ap.add_argument("--first", type=int, default=22, help="--autosomes: only the first K autosomes (disk space)")
    ap.add_argument("--chroms", type=int, default=4)
    ap.add_argument("--n-org", type=int, default=315_599)
    ap.add_argument("--n-snp", type=int, default=20_000)
    ap.add_argument("--missing", type=float, default=0.01)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "nldsc_genome"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--keep", action="store_true", help="keep the files afterwards")
    ap.add_argument("--fit", action="store_true", help="run the largest prefix of the chromosomes that fits the disk")
    a = ap.parse_args()
    import torch
    from nldsc_amd.engine import Engine
    from nldsc_amd.ldscore.genome import estimate_lds_genome
    made_dir = not os.path.isdir(a.dir)
    os.makedirs(a.dir, exist_ok=True)
    created = []  # files this run wrote (removed at the end unless --keep)
    N = a.n_org
    nb = (N + 3) // 4
    if a.autosomes:
        L = np.array(AUTOSOME_CM, dtype=float)
        Mc = np.maximum(1000, np.round(600_000 * L / L.sum())).astype(int)
        chroms = [(c + 1, int(Mc[c]), float(L[c])) for c in range(a.first)]
    else:
        chroms = [(c, a.n_snp, 70.0) for c in range(1, a.chroms + 1)]
    need = sum(3 + M * nb for _, M, _ in chroms)
    du = shutil.disk_usage(a.dir)
    full_bytes = need
    if a.fit:  # the largest prefix of the autosomes that fits the disk (leaving 4 GB), scaled to all of them by bytes
        while len(chroms) > 1 and need > du.free - (4 << 30):
            chroms = chroms[:-1]
            need = sum(3 + M * nb for _, M, _ in chroms)
    doc = dict(workload=("C4 (BASELINE.json configs[3]): %d autosomes, M_c proportional to cM length (sum M=%d), N=%d, "
                         "--ld-wind-cm 1, additive+dominance, %g%% missing" %
                         (len(chroms), sum(m for _, m, _ in chroms), N, 100 * a.missing)),
               bed_bytes=need, disk_free_bytes=du.free, dir=a.dir)
    print(json.dumps(doc), flush=True)
    if need > du.free - (2 << 30):
        raise SystemExit(f"not enough disk in {a.dir}: need {need / 1e9:.1f} GB, free {du.free / 1e9:.1f} GB")
    t = time.perf_counter()
    for c, M, length in chroms:
        write_set(os.path.join(a.dir, f"chr{c}"), c, M, N, 100 + c, length, a.missing, created)
        print(f"[write] chr{c} M={M} ({time.perf_counter() - t:.1f} s)", file=sys.stderr, flush=True)
    torch.cuda.empty_cache()
    doc["write_s"] = round(time.perf_counter() - t, 2)
    beds = [os.path.join(a.dir, f"chr{c}.bed") for c, _, _ in chroms]
    outdir = os.path.join(a.dir, "out")
    made_out = not os.path.isdir(outdir)
    os.makedirs(outdir, exist_ok=True)
    outs = [os.path.join(outdir, f"{s}{c}.L2") for s in ("o", "s") for c, _, _ in chroms]
    outs += [o + ".M" for o in outs]
    cli = [sys.executable, "-m", "nldsc_amd", "ld", "--bfile", os.path.join(a.dir, "chr@"), "--ld-wind-cm", "1",
           "-maf", "0.0001", "--out", os.path.join(outdir, "o@.L2"), "--extra", "--quiet"]

    def run_cli():
        t0 = time.perf_counter()
        p = subprocess.run(cli, cwd=REPO, capture_output=True, text=True)
        dt = time.perf_counter() - t0
        if p.returncode != 0 or "crashed" in p.stderr:
            raise SystemExit(p.stderr[-3000:])
        return dt

    drop_pages(beds)
    doc["cli_cold_s"] = round(run_cli(), 3)
    print(json.dumps({"cli_cold_s": doc["cli_cold_s"]}), flush=True)

    # per-stage times, in process, cold again
    eng = Engine(0)
    stages = []

    def runner(bed_path, n_snp, n_org, ld_wind, maf, std_thr, rsq_thr, positions, flags):
        t0 = time.perf_counter()
        eng.load_bed_file(bed_path, n_snp, n_org)
        t1 = time.perf_counter()
        r = eng.run(ld_wind, maf, std_thr, rsq_thr, positions, flags=flags)
        t2 = time.perf_counter()
        tim = eng.timings()
        stages.append(dict(bed=os.path.basename(bed_path), n_snp=n_snp, load_s=t1 - t0, run_s=t2 - t1,
                           gpu_ms=tim["total_ms"], band_ms=tim["band_ms"], pairs=tim["pairs"], t_in=t0, t_out=t2))
        return r, tim
    runner.wants_path = True
    drop_pages(beds)
    t0 = time.perf_counter()
    estimate_lds_genome(os.path.join(a.dir, "chr@"), "1", "cm", maf_thr="0.0001", std_thr=1e-4, extra=True,
                        out=os.path.join(outdir, "s@.L2"), rank=0, world=1, runner=runner, progress=False)
    t_end = time.perf_counter()
    total = t_end - t0
    eng.close()
    # chromosome k's TSV write (and host bookkeeping): from the end of its run to the next chromosome's load
    for k, s in enumerate(stages):
        s["write_s"] = (stages[k + 1]["t_in"] if k + 1 < len(stages) else t_end) - s["t_out"]
    for s in stages:
        del s["t_in"], s["t_out"]
    load = sum(s["load_s"] for s in stages)
    run = sum(s["run_s"] for s in stages)
    gpu = sum(s["gpu_ms"] for s in stages) / 1e3
    write = sum(s["write_s"] for s in stages)
    doc["stages_cold"] = dict(total_s=round(total, 3), load_s=round(load, 3), run_s=round(run, 3),
                              gpu_s=round(gpu, 3), band_s=round(sum(s["band_ms"] for s in stages) / 1e3, 3),
                              write_and_host_s=round(write, 3), read_gbps=round(need / load / 1e9, 2),
                              pairs=float(sum(s["pairs"] for s in stages)),
                              per_chrom=[{k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.items()}
                                         for s in stages])
    doc["cli_warm_s"] = round(run_cli(), 3)
    per = [s["load_s"] + s["run_s"] + s["write_s"] for s in stages]
    doc["projection_8gpu"] = dict(
        lpt_max_rank_s=round(lpt(per, 8), 3),
        disk_bound_s=round(load, 3),  # all bytes at the cold read rate measured here (one host disk for 8 ranks)
        note="8 ranks, chromosomes by LPT over the measured per-chromosome (load + run + write) times; the ranks "
             "share one host disk, so the cold projection is max(LPT, all bytes / the measured cold read rate)")
    doc["projection_8gpu"]["cold_s"] = max(doc["projection_8gpu"]["lpt_max_rank_s"],
                                           doc["projection_8gpu"]["disk_bound_s"])
    if need < full_bytes:  # a prefix ran: every time scaled by bytes to the whole set
        f = full_bytes / need
        doc["scaled_to_all"] = dict(factor=round(f, 4), bed_bytes=full_bytes, cli_cold_s=round(doc["cli_cold_s"] * f, 3),
                                    cli_warm_s=round(doc["cli_warm_s"] * f, 3),
                                    projection_8gpu_cold_s=round(doc["projection_8gpu"]["cold_s"] * f, 3))
    print(json.dumps(doc), flush=True)
    if a.out:
        json.dump(doc, open(a.out, "w"), indent=1)
    if not a.keep:
        cleanup(created, outs, outdir if made_out else None, a.dir if made_dir else None)


def cleanup(created, outputs, outdir, topdir):
    """Remove the files this run wrote and the directories it created, if they are then empty (never
    rmtree a directory the user passed, which may hold other data)."""
    for p in list(created) + list(outputs):
        try:
            os.unlink(p)
        except FileNotFoundError:
            pass
    for d in (outdir, topdir):
        if d is not None:
            try:
                os.rmdir(d)  # only when empty
            except OSError:
                pass


if __name__ == "__main__":
    main()
