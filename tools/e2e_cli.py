#!/usr/bin/env python3
"""End-to-end wall clock of `nldsc ld` from PLINK files (the BASELINE metric's "wall-clock" half):
writes a synthetic chromosome (GPU-generated genotypes) to disk, then times
  (1) the CLI in a fresh process:  python -m nldsc_amd ld --bfile X --ld-wind-cm 1 ... --out X.L2 --extra
  (2) in-process stages: .bim/.fam parse, _ldscore.calculate (file -> HBM -> scores), TSV formatting + write.
The .bed was just written, so it is read from the page cache (disk speed not included).
    python tools/e2e_cli.py --n-org 50000 --n-snp 80000 --dir /tmp/e2e --out gpurun_out/e2e.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-org", type=int, default=50_000)
    ap.add_argument("--n-snp", type=int, default=80_000)
    ap.add_argument("--length-cm", type=float, default=280.0)
    ap.add_argument("--dir", default="/tmp/nldsc_e2e")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from nldsc_amd import synth
    os.makedirs(a.dir, exist_ok=True)
    stem = os.path.join(a.dir, "chr1")
    t = time.perf_counter()
    buf, pos = synth.device_bed(a.n_snp, a.n_org, seed=11, length_cm=a.length_cm)
    with open(stem + ".bed", "wb") as fh:
        fh.write(buf.cpu().numpy().tobytes())
    del buf
    torch.cuda.empty_cache()
    bp = np.round(pos * 1e6).astype(np.int64)
    with open(stem + ".bim", "w") as fh:
        fh.writelines(f"1\trs{j + 1}\t{pos[j]:.6f}\t{bp[j]}\tA\tG\n" for j in range(a.n_snp))
    with open(stem + ".fam", "w") as fh:
        fh.writelines(f"F{i}\tI{i}\t0\t0\t1\t-9\n" for i in range(a.n_org))
    t_gen = time.perf_counter() - t
    bed_gb = os.path.getsize(stem + ".bed") / 1e9

    cmd = [sys.executable, "-m", "nldsc_amd", "ld", "--bfile", stem, "--ld-wind-cm", "1", "-maf", "1e-4",
           "--std-thr", "1e-5", "--out", stem + ".L2", "--extra"]
    t = time.perf_counter()
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True)
    t_cli = time.perf_counter() - t
    if r.returncode != 0 or not os.path.exists(stem + ".L2"):
        print(r.stdout[-2000:], r.stderr[-2000:], file=sys.stderr)
        raise SystemExit("CLI failed")

    # in-process stages (what the CLI does after its imports)
    from nldsc_amd.ldscore import _ldscore as lds
    from nldsc_amd.ldscore.common import BIMFile, FAMFile
    from nldsc_amd.ldscore.routine import format_scores
    t0 = time.perf_counter()
    bim, fam = BIMFile(stem + ".bim"), FAMFile(stem + ".fam")
    t1 = time.perf_counter()
    p = lds.LDScoreParams(stem + ".bed", n_snp=bim.n_snp, n_org=fam.n_org, ld_wind=1.0, maf=1e-4, std_thr=1e-5,
                          rsq_thr=1.0 / bim.n_snp, positions=np.asarray(bim.cm, dtype=np.float64).tolist())
    ld = lds.calculate(p)
    t2 = time.perf_counter()
    data = format_scores(bim, ld, extra=True)
    with open(stem + ".L2b", "wb") as fh:
        fh.write(data)
    t3 = time.perf_counter()
    same = open(stem + ".L2", "rb").read() == data
    pairs = float(np.sum([w for w in ld.l2_ws if w > 0]))
    res = dict(workload=f"chr1-like N={a.n_org} M={a.n_snp} over {a.length_cm:g} cM, --ld-wind-cm 1, add+dom, --extra",
               bed_gb=bed_gb, generate_files_s=t_gen, cli_wall_s=t_cli, parse_bim_fam_s=t1 - t0,
               calculate_s=t2 - t1, tsv_s=t3 - t2, in_process_total_s=t3 - t0, snp_pairs=pairs,
               pairs_per_s_cli_wall=pairs / t_cli, pairs_per_s_in_process=pairs / (t3 - t0),
               cli_output_equals_in_process=same,
               note="the .bed is read from the page cache right after being written (disk bandwidth excluded); "
                    "cli_wall_s includes interpreter start, torch-free imports and the summary print")
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
    for ext in (".bed", ".bim", ".fam", ".L2", ".L2b"):
        os.remove(stem + ext)


if __name__ == "__main__":
    main()
