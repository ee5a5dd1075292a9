#!/usr/bin/env python3
"""Diagnostic: computed-SNP and pair counts of the C5-shaped slice under the band-kernel variants ($NLDSC_T2 0 / 1 / 3,
$NLDSC_GPU_PLAN 0) at two slice sizes; prints one JSON line per run and whether the integer outputs agree."""
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
    N = 315_599
    for M in [int(x) for x in sys.argv[1:]] or [300_000]:
        buf, pos = synth.device_bed(M, N, seed=7, length_cm=288.0 * M, missing=0.0)
        ref = None
        for env in ({"NLDSC_T2": "3"}, {"NLDSC_T2": "0"}, {"NLDSC_T2": "1"}, {"NLDSC_GPU_PLAN": "0"}):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                e = Engine(0)
            finally:
                for k, v in old.items():
                    os.environ.pop(k) if v is None else os.environ.__setitem__(k, v)
            e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
            r = e.run(1.0e6, 1e-4, 1e-5, 1.0 / M, pos)
            t = e.timings()
            ws = r["l2_ws"]
            line = dict(M=M, env=env, pairs=float(ws[ws > 0].sum()), computed=int((ws >= 0).sum()),
                        positive=int((ws > 0).sum()), neg=int((ws < 0).sum()), band_kernel=t.get("band_kernel"),
                        band_ms=round(t["band_ms"], 2), maf_nan=int(np.isnan(r["maf"]).sum()),
                        first_neg=int(np.argmax(ws < 0)) if (ws < 0).any() else -1)
            if ref is None:
                ref = r
            else:
                line["equal_to_first"] = {k: bool(np.array_equal(r[k], ref[k], equal_nan=True)) for k in ("l2_ws", "l2d_ws", "l2")}
            print(json.dumps(line), flush=True)
            e.close()
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
