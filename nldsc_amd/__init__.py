"""nldsc_amd — MI355X-native LD-score engine, a drop-in for bayarpark/nldsc's `ldscore` hot path.

Layout: `ldscore/` mirrors the reference's `nldsc.ldscore` (pybind11 `_ldscore` + `estimate_lds`),
`engine.py` / `_lib.py` bind the C ABI of libnldsc_amd.so (include/nldsc_ld.h), `distributed.py`
shards SNPs by position over GPUs, `synth.py` makes synthetic PLINK data.
"""
__version__ = "0.1.0"
