"""Images past 2^32 sixteen-byte units (> 68.7 GB of resident rows: a C5 slice is 98.6 GB): every row must be placed.
A launch with one work-item per unit wraps there (an HSA dispatch counts its grid in 32 bits) and silently left the
rows past ~379 000 of the C5 bench slice empty (MAF 0, not computed) until load_rows_kernel went grid-stride."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rows_past_2p32_units_are_loaded():
    import torch

    from nldsc_amd import synth
    from nldsc_amd.engine import Engine
    N, M = 315_599, 900_000  # 71.0 GB of rows: 4.44e9 units of 16 bytes
    nb = (N + 3) // 4
    buf, pos = synth.device_bed(M, N, seed=11, length_cm=2.0 * M / 1000.0, missing=0.01)
    tail = 96  # the last rows (three blocks) again, as a small image of their own
    small = torch.cat([buf[:3], buf[3 + (M - tail) * nb:]])
    args = (1e-4, 1e-4, 1e-5, 1.0 / M)  # a tiny window: diagonal blocks only
    with Engine(0) as e:
        e.load_bed_device(buf.data_ptr(), buf.numel(), M, N)
        del buf
        torch.cuda.empty_cache()
        big = e.run(*args, pos)
    with Engine(0) as e:
        e.load_bed_device(small.data_ptr(), small.numel(), tail, N)
        ref = e.run(*args, pos[M - tail:])
    assert (big["maf"] > 0).all() and (big["l2_ws"] >= 0).all(), (int((big["maf"] == 0).sum()),
                                                                    int(np.argmax(big["maf"] == 0)))
    np.testing.assert_array_equal(big["maf"][M - tail:], ref["maf"])
    np.testing.assert_array_equal(big["residuals_std"][M - tail:], ref["residuals_std"])
