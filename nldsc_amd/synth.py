"""Synthetic PLINK 1 (.bed/.bim/.fam) generator for tests and benchmarks.

Model: per SNP an allele frequency p ~ U(0.02, 0.5); each
haplotype carries the second (.bim A2) allele where a latent AR(1) Gaussian
process over SNPs (rho = 0.9) falls below Phi^-1(p); genotype = number of A2
alleles on the two haplotypes; a fraction of calls is set missing; genetic
positions are cumulative exponential gaps over ``length_cm`` with
``bp = cM * 1e6``.  Packing is PLINK-correct (SNP-major, sample 4b+k in bits
2k..2k+1 of byte b, zero padding in the high bits of the last byte), which is
exactly the case where the reference's high-bits-first unpack
(``stream.h:55-66``) differs from PLINK for N % 4 != 0.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

# PLINK 2-bit codes: genotype (A2 count) -> bit pair; missing -> 01
_CODE_OF_GENO = np.array([0b00, 0b10, 0b11], dtype=np.uint8)
MISSING_CODE = 0b01


@dataclass
class SynthSpec:
    n_org: int
    n_snp: int
    length_cm: float = 72.0
    seed: int = 7
    rho: float = 0.9
    missing: float = 0.01
    # indices of forced edge-case SNPs
    monomorphic: list = field(default_factory=list)   # all hom A1 -> MAF 0, fails MAF filter
    hom1_het_only: list = field(default_factory=list)  # genotypes {0,1} only -> residual std 0
    het_hom2_only: list = field(default_factory=list)  # genotypes {1,2} only -> residual std 0
    all_missing: list = field(default_factory=list)    # every call missing -> MAF NaN
    negative_pos: list = field(default_factory=list)   # position -1 -> SNP unused
    tie_pairs: list = field(default_factory=list)      # a: put the next SNP exactly one window after a
    tie_window_cm: float = 1.0


def genotypes(spec: SynthSpec, snp_begin: int = 0, snp_end: int | None = None) -> np.ndarray:
    """int8 genotype matrix [M][N] (A2 allele counts 0/1/2, -1 = missing)."""
    rng = np.random.default_rng(spec.seed)
    from scipy.special import ndtri

    M, N = spec.n_snp, spec.n_org
    snp_end = M if snp_end is None else snp_end
    p = rng.uniform(0.02, 0.5, size=M)
    thr = ndtri(p)
    z = rng.standard_normal((2, N)).astype(np.float64)
    s = np.sqrt(1.0 - spec.rho ** 2)
    out = np.empty((snp_end - snp_begin, N), dtype=np.int8)
    for j in range(snp_end):
        if j > 0:
            z = spec.rho * z + s * rng.standard_normal((2, N))
        miss = rng.random(N) < spec.missing
        if j < snp_begin:
            continue
        g = (z[0] < thr[j]).astype(np.int8) + (z[1] < thr[j]).astype(np.int8)
        g[miss] = -1
        out[j - snp_begin] = g
    for j in spec.monomorphic:
        if snp_begin <= j < snp_end:
            out[j - snp_begin] = 0
    for j in spec.hom1_het_only:
        if snp_begin <= j < snp_end:
            r = out[j - snp_begin]
            r[r == 2] = 1
    for j in spec.het_hom2_only:
        if snp_begin <= j < snp_end:
            r = out[j - snp_begin]
            r[r == 0] = 1
    for j in spec.all_missing:
        if snp_begin <= j < snp_end:
            out[j - snp_begin] = -1
    return out


def positions_cm(spec: SynthSpec) -> np.ndarray:
    rng = np.random.default_rng(spec.seed + 1_000_003)
    gaps = rng.exponential(spec.length_cm / spec.n_snp, size=spec.n_snp)
    pos = np.cumsum(gaps)
    pos = np.round(pos, 6)
    for a in spec.tie_pairs:
        # exact boundary tie: pos_a a dyadic multiple of 1/64 cM (exact in binary64,
        # in "%.6f" text and in bp = cM * 1e6), pos_b = pos_a + window exactly.
        pa = np.ceil(pos[a] * 64.0) / 64.0
        pos[a] = pa
        pos[a + 1:] = np.maximum(pos[a + 1:], pa)
        b = int(np.searchsorted(pos, pa + spec.tie_window_cm))
        if b < spec.n_snp:
            pos[b] = pa + spec.tie_window_cm
    pos = np.maximum.accumulate(pos)
    for j in spec.negative_pos:
        pos[j] = -1.0
    return pos


def pack_bed_rows(g: np.ndarray) -> np.ndarray:
    """Pack an int8 genotype matrix [M][N] into PLINK SNP-major rows [M][ceil(N/4)]."""
    M, N = g.shape
    nb = (N + 3) // 4
    codes = np.where(g < 0, MISSING_CODE, _CODE_OF_GENO[np.clip(g, 0, 2)]).astype(np.uint8)
    pad = np.zeros((M, nb * 4), dtype=np.uint8)  # padding pairs are 00
    pad[:, :N] = codes
    pad = pad.reshape(M, nb, 4)
    return (pad[:, :, 0] | (pad[:, :, 1] << 2) | (pad[:, :, 2] << 4) | (pad[:, :, 3] << 6)).astype(np.uint8)


def bed_bytes(rows: np.ndarray) -> bytes:
    return b"\x6c\x1b\x01" + np.ascontiguousarray(rows).tobytes()


def device_bed(n_snp: int, n_org: int, *, seed: int = 7, length_cm: float = 280.0, rho: float = 0.9,
               missing: float = 0.01, device: int = 0):
    """Synthetic .bed image generated on the GPU (same model, device RNG): returns
    (torch uint8 tensor holding the whole file image, positions in cM as numpy float64)."""
    import torch
    from scipy.special import ndtri

    from .engine import synth_bed_device
    rng = np.random.default_rng(seed)
    thr = ndtri(rng.uniform(0.02, 0.5, size=n_snp)).astype(np.float32)
    pos = np.round(np.cumsum(rng.exponential(length_cm / n_snp, size=n_snp)), 6)
    nb = (n_org + 3) // 4
    buf = torch.empty(3 + nb * n_snp, dtype=torch.uint8, device=f"cuda:{device}")
    synth_bed_device(device, buf.data_ptr(), n_snp, n_org, thr, rho=rho, missing=missing, seed=seed)
    return buf, pos


def write_plink(prefix: str, spec: SynthSpec, chrom: int = 22, positions_metric: str = "cm") -> dict:
    """Write prefix.bed/.bim/.fam. Returns dict(rows=..., pos_cm=..., bp=...)."""
    g = genotypes(spec)
    rows = pack_bed_rows(g)
    cm = positions_cm(spec)
    bp = np.where(cm < 0, -1, np.round(cm * 1e6)).astype(np.int64)
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    with open(prefix + ".bed", "wb") as f:
        f.write(bed_bytes(rows))
    with open(prefix + ".bim", "w") as f:
        for j in range(spec.n_snp):
            f.write(f"{chrom}\trs{j + 1}\t{cm[j]:.6f}\t{bp[j]}\tA\tG\n")
    with open(prefix + ".fam", "w") as f:
        for i in range(spec.n_org):
            f.write(f"F{i}\tI{i}\t0\t0\t{1 + (i & 1)}\t-9\n")
    return dict(rows=rows, pos_cm=cm, bp=bp, geno=g)
