#!/usr/bin/env python3
"""Diagnostic: are the C5 slice's rows past ~380 000 in the synthetic image, and what MAF does the engine see there."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    torch.cuda.init()
    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 315_599, int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    nb = (N + 3) // 4
    buf, pos = synth.device_bed(M, N, seed=7, length_cm=288.0 * M, missing=0.0)
    rows = buf[3:].view(M, nb)
    nz = np.concatenate([(rows[a:a + 50_000, :4096] != 0).sum(dim=1).cpu().numpy() for a in range(0, M, 50_000)])
    print(json.dumps({"rows_all_zero": int((nz == 0).sum()), "first_zero_row": int(np.argmax(nz == 0)) if (nz == 0).any() else -1}), flush=True)
    for env in ({}, {"NLDSC_ORIENT": "0"}):
        os.environ.update(env)
        e = Engine(0)
        for k in env:
            os.environ.pop(k)
        e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
        r = e.run(1.0e6, 1e-4, 1e-5, 1.0 / M, pos)
        ws, maf = r["l2_ws"], r["maf"]
        j = int(np.argmax(ws < 0)) if (ws < 0).any() else -1
        print(json.dumps({"env": env, "first_neg": j, "n_neg": int((ws < 0).sum()),
                          "maf_around": [float(x) for x in maf[max(j - 3, 0):j + 3]],
                          "maf_zero": int((maf == 0).sum()), "rstd_nan": int(np.isnan(r["residuals_std"]).sum())}), flush=True)
        e.close()


if __name__ == "__main__":
    main()
