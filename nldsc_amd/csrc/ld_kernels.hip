// ld_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the LD-score engine.
//
// Pipeline for one `calculate` (reference: nldsc/ldscore/_ldscore/ldscalc.h:8-65):
//   1. count_rows_kernel    per-SNP genotype-code counts over the resident .bed rows (kept at an aligned
//                           pitch by the loaders), the reference's last-byte rule applied
//                           (stream.h:55-66).  HBM-bound byte work.
//   2. snp_stats_kernel     per-SNP MAF / filters / residual std and two 4-entry fp32 lookup tables
//                           (standardised additive value and standardised dominance residual per
//                           2-bit code), in closed form from the counts (encoder.h:91-133,
//                           tools.h:54-85).
//   3. band_kernel<NC,DOM>  the windowed correlation block: for a 32-SNP row block I and NC 32-SNP
//                           column blocks, X_I^T X_J, X_I^T R_J and R_I^T X_J over all samples with
//                           v_mfma_f32_32x32x2_f32.  Operands are decoded straight from the 2-bit
//                           rows into VGPRs through a per-wave LDS table [code][snp] -> (a, r); a
//                           fused epilogue applies r2adj (tools.h:87-92), the window / MAF / residual
//                           masks and reduces per-SNP sums (ldscalc.h:34-54).
//   4. finalize_kernel      L2 = 1 + sum, NaN / -1 for SNPs that are not computed (ldscalc.h:16-21).
//   (+) synth_bed_kernel    deterministic synthetic .bed image for benchmarks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>
#include <algorithm>
#include <type_traits>

#include "ld_kernels.h"

namespace nldsc {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------------
// 1. resident row layout + per-run count
// ------------------------------------------------------------------------------------------
// Resident layout ("block-interleaved rows").  A row is the .bed row of nb = ceil(N / 4) bytes padded to
// row_bytes = ceil(nb / 64) * 64; the rows of each 32-SNP block b are interleaved in 32-byte chunks: byte k of chunk
// t of row 32 b + i sits at (b * 32 * row_bytes) + t * 1024 + i * 32 + k (tile_off).  One chunk of a block — what a
// band wave consumes per K step pair, 32 rows x 128 samples — is then 1 KiB contiguous (eight whole 128-byte lines)
// instead of 32 pieces of 32 bytes a row pitch apart, whose lines the band kernels fetched from L2 up to four times
// (C2 band -18 %, C3 -3.5 %, C5 -6 % measured against the row-major layout: profiles/r03_ab_tiled_layout.json).
// Byte p of a row keeps the .bed byte (4 samples, first sample in bits 7:6 per the reference's unpack order — any
// fixed slot order is fine for dot products as long as every SNP uses the same one).  Bytes past the row are 01 pairs
// ("missing"), and each run rewrites the last byte from its saved original so that only the bit pairs that are
// individuals for that run's order (reference: high pairs first; PLINK: low pairs) stay and the rest read as missing
// — which contributes nothing to any dot product.  Rows past n_snp (the last block's padding) are all 0x55.
__device__ __forceinline__ size_t tile_off(int r, int b, int row_bytes) {
    return (size_t)(r >> 5) * 32 * (size_t)row_bytes + (size_t)(b >> 5) * 1024 + (size_t)(r & 31) * 32 + (b & 31);
}
// the band kernels' view: uint4 index of row r's chunk 0 (a lane's half h adds h) and the uint4 stride of chunks
constexpr int CHUNK_U4 = 64;
__device__ __forceinline__ size_t row_u4(int r, int pitch_words) {
    return (size_t)(r >> 5) * 8 * (size_t)pitch_words + (size_t)(r & 31) * 2;
}

__device__ __forceinline__ void count_codes(uint32_t word, int& c0, int& c1, int& c2) {
    const uint32_t hi = (word >> 1) & 0x55555555u, lo = word & 0x55555555u;
    c0 += __popc(~hi & ~lo & 0x55555555u);  // 00 hom A1
    c1 += __popc(hi & ~lo);                 // 10 het
    c2 += __popc(hi & lo);                  // 11 hom A2
}
__device__ __forceinline__ int count_missing(uint32_t word) {
    return __popc(~(word >> 1) & word & 0x55555555u);  // pairs 01
}

// Block sweeps of the resident layout: a workgroup of 4 waves takes 32-SNP block b; per chunk t a wave reads the
// chunk's 1 KiB with one 16-byte load per lane — lane l always lands on row l / 2 (half l % 2 of its 32 bytes), so
// per-row sums stay in the lane and meet its partner's (l ^ 1) and the other waves' at the end.  Wave w takes chunks
// t = w, w + 4, ... of [t_lo, t_hi).
struct BlockRed {
    int v[4][32][3];
};
// sums c[0..2] of lanes l and l ^ 1 (one row), then over the 4 waves: row i's totals on thread i (< 32) in out[]
__device__ __forceinline__ void block_row_sums(BlockRed& sh, const int (&c)[3], int (&out)[3]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int t[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = c[k] + __shfl_xor(c[k], 1, 64);
    if ((lane & 1) == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) sh.v[w][lane >> 1][k] = t[k];
    }
    __syncthreads();
    if (threadIdx.x < 32) {
#pragma unroll
        for (int k = 0; k < 3; ++k) out[k] = sh.v[0][threadIdx.x][k] + sh.v[1][threadIdx.x][k] + sh.v[2][threadIdx.x][k] +
                                             sh.v[3][threadIdx.x][k];
    }
}

// ---- loads: .bed rows -> the resident layout, oriented, with per-row missing flags (one pass over the rows) ----
// A load takes slices of whole 32-SNP blocks (row0 a multiple of 32; the last slice may end mid-block) of a .bed image
// (src: the slice's row r at r * nb bytes, any alignment: the file's rows follow a 3-byte magic number).  Per slice:
//   load_orient_kernel   per row: the stored orientation (flip) from the codes of its first LOAD_ORIENT_BYTES bytes
//                        (rows with more hom-A2 than hom-A1 calls there are stored 00 <-> 11 swapped, see below) and
//                        its missing-flag word cleared;
//   load_tiled_kernel    per (block, part): the block's chunks in the interleaved layout (a wave writes whole 1 KiB
//                        chunks: lane l = row l / 2, half l % 2 of its 32 bytes), swapped where flipped, the pitch
//                        padding and the padding rows of the last block 0x55, each row's (stored) last byte saved, and
//                        the row's missing calls among the individual slots of both sample orders ORed into its flags.
// Then load_flags_kernel narrows the flags to row_miss.  Any orientation gives the same results (the stats and the
// replay take flip into account); deciding it from the row's head keeps the load one pass over the rows, where the
// whole-row count it replaces needed a second pass that read and rewrote every swapped row (PLINK data, A1 minor:
// nearly all).
constexpr int LOAD_ORIENT_BYTES = 1024;

// 16 source bytes at any alignment (src + o .. + 16 within the buffer): one global_load_dwordx4 — the HSA memory model
// runs in unaligned access mode, and the compiler emits the vector load for this 1-byte-aligned type (five dword loads
// and byte shifts before: the load kernel's source reads took 5x the vector-memory instructions)
struct __attribute__((packed, aligned(1))) Bytes16 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t* __restrict__ src, size_t o) {
    const Bytes16 q = *reinterpret_cast<const Bytes16*>(src + o);
    return make_uint4(q.x, q.y, q.z, q.w);
}
// bytes [p0, p0 + 16) of a row of nb bytes (bytes past it read as `fill`), one byte at a time
__device__ __forceinline__ uint4 load16_bytes(const uint8_t* __restrict__ row, int p0, int nb, uint32_t fill) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = p0 + 4 * q + k;
            v |= (uint32_t)(p < nb ? row[p] : fill) << (8 * k);
        }
        w[q] = v;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint32_t swap_hom(uint32_t v) {  // 00 <-> 11 in every bit pair (het, missing unchanged)
    const uint32_t q = ~(v ^ (v >> 1)) & 0x55555555u;
    return v ^ (q | (q << 1));
}

// one wave per row (4 per workgroup): flip[row0 + r] and the row's missing-flag word cleared
__global__ void __launch_bounds__(256) load_orient_kernel(const uint8_t* __restrict__ src, int nb, int row0, int n_rows,
                                                          int orient, uint8_t* __restrict__ flip,
                                                          uint32_t* __restrict__ miss_flags, int* __restrict__ lcounts) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= n_rows) return;
    int c0 = 0, c1 = 0, c2 = 0;
    if (orient) {
        const int head = min(nb, LOAD_ORIENT_BYTES);
        const uint8_t* row = src + (size_t)r * nb;
        const int p0 = 16 * lane;
        if (p0 < head) {
            // (bytes past the head, or past the row, read as 0x55: missing, counted in neither class)
            const uint4 v = p0 + 16 <= head ? load16_unaligned(src, (size_t)r * nb + p0)
                                                               : load16_bytes(row, p0, head, 0x55u);
            count_codes(v.x, c0, c1, c2);
            count_codes(v.y, c0, c1, c2);
            count_codes(v.z, c0, c1, c2);
            count_codes(v.w, c0, c1, c2);
        }
        for (int o = 32; o > 0; o >>= 1) {
            c0 += __shfl_xor(c0, o, 64);
            c2 += __shfl_xor(c2, o, 64);
        }
    }
    if (lane < 3) lcounts[3 * (size_t)(row0 + r) + lane] = 0;  // (the tiled kernel's parts add into them)
    if (lane == 0) {
        flip[row0 + r] = (uint8_t)(c2 > c0);
        miss_flags[row0 + r] = 0u;
    }
}

// grid (block of the slice, part): part p of P sweeps the block's chunks [p n_ch / P, (p + 1) n_ch / P) in stages of
// LOAD_SC chunks: the workgroup reads the stage's 32 row segments (LOAD_SC x 32 bytes each) row by row — 32 threads per
// row, 512 contiguous bytes per half wave (8 threads x 128 bytes before: load_tiled 2.64 -> 2.55 ms at C3) — into
// registers one stage ahead, then through LDS, and wave w writes chunks t = t0 + w, t0 + w + 4, ... of the stage
// (lane l: row l / 2, half l % 2) as whole 1 KiB chunks (profiles/r05_ab_load_reader.json).  Reading the source 32 bytes per row and chunk
// straight into the chunk layout touched 32 rows' lines at once per wave: 4.0 TB/s of read + write at C3 (3.16 ms).
// n_snp: the image's SNPs (rows past it, in its last block: 0x55).  keep_compat / keep_strict: the last byte's bit
// pairs that are individuals in the reference's / PLINK's sample order.
constexpr int LOAD_SC = 16;  // chunks per stage (LDS: 32 rows x LOAD_SC x 32 bytes)
__global__ void __launch_bounds__(256) load_tiled_kernel(const uint8_t* __restrict__ src, int nb, int row0,
                                                         int n_rows, int n_snp, uint8_t* __restrict__ img,
                                                         int row_bytes, int P, const uint8_t* __restrict__ flip,
                                                         uint8_t* __restrict__ last, uint32_t keep_compat,
                                                         uint32_t keep_strict, uint32_t* __restrict__ miss_flags,
                                                         int* __restrict__ lcounts) {
    __shared__ uint32_t rowflags[4][32];
    __shared__ BlockRed red;
    __shared__ uint4 tile[32][2 * LOAD_SC + 1];  // (+1 unit: rows 528 bytes apart in LDS)
    const int bl = blockIdx.x / P, part = blockIdx.x % P, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = lane >> 1, h = lane & 1;
    const int r = 32 * bl + i, j = row0 + r;  // the lane's row: in the slice, in the image
    const bool real = r < n_rows && j < n_snp;
    const bool fl = real && flip[j];
    const int n_ch = row_bytes >> 5;
    const int t_lo = (int)((long long)n_ch * part / P), t_hi = (int)((long long)n_ch * (part + 1) / P);
    uint8_t* blk = img + (size_t)(row0 / 32 + bl) * 32 * (size_t)row_bytes;
    // units [0, n_fast) of 16 bytes lie inside the row: one vector load each
    const int n_fast = nb / 16;
    uint32_t mflags = 0;  // bit 0 / 1: a missing call among the reference's / PLINK's individual slots
    int cnt[3] = {0, 0, 0};  // genotype codes of the stored row in bytes [0, nb - 1) (hom A1, het, hom A2)
    // whole units before the last byte, per 16-code word with hi / lo the pairs' high / low bits: popcounts of hi,
    // hi & lo (hom A2) and hi | lo (not hom A1), and lo & ~hi (missing) ORed — the classes follow at the end
    int n_hi = 0, n_and = 0, n_or = 0, n_words = 0;
    uint32_t miss_or = 0;
    auto tally = [&](uint32_t word) {
        const uint32_t hi = (word >> 1) & 0x55555555u, lo = word & 0x55555555u;
        n_hi += __popc(hi);
        n_and += __popc(hi & lo);
        n_or += __popc(hi | lo);
        miss_or |= lo & ~hi;
    };
    auto one = [&](int t, const uint4 v_in) {
        const int u = 2 * t + h, p0 = 16 * u;
        uint4 v = v_in;
        if (fl) v = make_uint4(swap_hom(v.x), swap_hom(v.y), swap_hom(v.z), swap_hom(v.w));
        // (nontemporal: the image is written once and read by the runs, far past the caches; load_tiled 2.55 ->
        // 2.46 ms at C3, profiles/r05_ab_load_reader.json)
        typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w},
                                    reinterpret_cast<u32x4_t*>(blk + (size_t)t * 1024 + (size_t)i * 32 + 16 * h));
        if (!real) return;
        if (p0 + 16 <= nb - 1) {
            tally(v.x);
            tally(v.y);
            tally(v.z);
            tally(v.w);
            n_words += 4;
        } else if (p0 <= nb - 1) {  // the unit holding the last byte: the bytes before it, then the byte per order
            const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int p = p0 + 4 * q + k;
                    const uint32_t byte = (wd[q] >> (8 * k)) & 0xFFu;
                    if (p < nb - 1) {
                        if (count_missing(byte)) mflags |= 3u;
                        // (a byte's four pairs, counted as a word whose upper bytes are 01 pairs: missing, no class)
                        count_codes(byte | 0x55555500u, cnt[0], cnt[1], cnt[2]);
                    }
                    if (p == nb - 1) {
                        last[j] = (uint8_t)byte;
                        if (count_missing(byte & keep_compat)) mflags |= 1u;
                        if (count_missing(byte & keep_strict)) mflags |= 2u;
                    }
                }
        }
    };
    // the stage reader: thread tid takes unit tid % TPR of the stage in rows tid / TPR + RPP k of the block (a wave
    // reads 64 / TPR row segments of 16 TPR contiguous bytes per instruction)
    constexpr int TPR = 2 * LOAD_SC, RPP = 256 / TPR;
    const int uu = threadIdx.x % TPR, rr0 = threadIdx.x / TPR;
    uint4 pre[32 / RPP];  // the next stage's units, read while this stage is written (2.46 -> 2.42 ms at C3)
    auto fetch = [&](int t0) {
        const int nu = 2 * min(LOAD_SC, t_hi - t0), u = 2 * t0 + uu;
        if (uu < nu) {
#pragma unroll
            for (int k = 0; k < 32 / RPP; ++k) {
                const int rr = rr0 + RPP * k, gr = 32 * bl + rr;
                const size_t gbase = (size_t)gr * nb;
                pre[k] = gr >= n_rows ? make_uint4(0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u)
                         : u < n_fast ? load16_unaligned(src, gbase + 16 * (size_t)u)
                                      : load16_bytes(src + gbase, 16 * u, nb, 0x55u);
            }
        }
    };
    if (t_lo < t_hi) fetch(t_lo);
    for (int t0 = t_lo; t0 < t_hi; t0 += LOAD_SC) {
        const int nu = 2 * min(LOAD_SC, t_hi - t0);
        if (uu < nu) {
#pragma unroll
            for (int k = 0; k < 32 / RPP; ++k) tile[rr0 + RPP * k][uu] = pre[k];
        }
        __syncthreads();
        if (t0 + LOAD_SC < t_hi) fetch(t0 + LOAD_SC);
        for (int t = t0 + w; t < t0 + nu / 2; t += 4) one(t, tile[i][2 * (t - t0) + h]);
        __syncthreads();
    }
    cnt[0] += 16 * n_words - n_or;
    cnt[1] += n_hi - n_and;
    cnt[2] += n_and;
    if (miss_or) mflags |= 3u;
    // rows' counts of this part (block_row_sums: the lane pair, then the four waves) added into lcounts[3 j + k]
    // (integer atomics: exact in any order; a separate pass folding P per-part copies cost 0.15 ms at C3)
    {
        int tot[3];
        block_row_sums(red, cnt, tot);
        const int jj = row0 + 32 * bl + threadIdx.x;
        if (threadIdx.x < 32 && 32 * bl + (int)threadIdx.x < n_rows && jj < n_snp) {
            int* o = lcounts + (size_t)jj * 3;
            atomicAdd(o, tot[0]);
            atomicAdd(o + 1, tot[1]);
            atomicAdd(o + 2, tot[2]);
        }
    }
    // rows' flags: the lane pair, then the four waves, then one atomic per row and workgroup
    mflags |= __shfl_xor(mflags, 1, 64);
    if (h == 0) rowflags[w][i] = mflags;
    __syncthreads();
    if (threadIdx.x < 32) {
        const uint32_t f = rowflags[0][threadIdx.x] | rowflags[1][threadIdx.x] | rowflags[2][threadIdx.x] |
                           rowflags[3][threadIdx.x];
        const int jj = row0 + 32 * bl + threadIdx.x;
        if (f && 32 * bl + threadIdx.x < n_rows && jj < n_snp) atomicOr(miss_flags + jj, f);
    }
}

__global__ void load_flags_kernel(const uint32_t* __restrict__ miss_flags, int n_snp, uint8_t* __restrict__ row_miss) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_snp) row_miss[j] = (uint8_t)miss_flags[j];
}


// Halo pairs computed once across ranks (nldsc_engine_run_device_split): only pairs whose lower SNP lies in
// [pair_lo, pair_hi) — the rank's owned range — keep flag bit 3 (snp_stats_kernel sets it on every SNP); the pairs of
// a rank's owned SNPs with the right halo are computed here for both SNPs, the halo SNPs' sums exported to their
// owner (export_acc_kernel / import_acc_kernel: the fixed-point accumulators and counts add exactly).
__global__ void pair_range_kernel(uint8_t* __restrict__ sflags, int n_snp, int pair_lo, int pair_hi) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_snp && (j < pair_lo || j >= pair_hi)) sflags[j] &= (uint8_t)~8u;
}
// rows k of `out` (n = hi - lo columns): l2 / l2d fixed-point accumulators, WSA, WSD, WSDE, non-finite flags
__global__ void export_acc_kernel(const double* __restrict__ l2_acc, const double* __restrict__ l2d_acc,
                                  const int* __restrict__ ws_acc, int n_snp, int lo, int hi, long long* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, g = lo + c, n = hi - lo;
    if (g >= hi) return;
    out[c] = reinterpret_cast<const long long*>(l2_acc)[g];
    out[(size_t)n + c] = reinterpret_cast<const long long*>(l2d_acc)[g];
    for (int k = 0; k < 4; ++k) out[(size_t)(2 + k) * n + c] = ws_acc[(size_t)k * n_snp + g];
}
__global__ void import_acc_kernel(double* __restrict__ l2_acc, double* __restrict__ l2d_acc, int* __restrict__ ws_acc,
                                  int n_snp, int lo, int n, const long long* __restrict__ in) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, g = lo + c;
    if (c >= n || g >= n_snp) return;
    reinterpret_cast<long long*>(l2_acc)[g] += in[c];
    reinterpret_cast<long long*>(l2d_acc)[g] += in[(size_t)n + c];
    for (int k = 0; k < 3; ++k) ws_acc[(size_t)k * n_snp + g] += (int)in[(size_t)(2 + k) * n + c];
    ws_acc[3 * (size_t)n_snp + g] |= (int)in[5 * (size_t)n + c];
}

// per run: blk_miss[b] = block b holds a row with a missing call in this run's sample order (bit `order` of row_miss)
__global__ void block_missing_rows_kernel(const uint8_t* __restrict__ row_miss, int n_snp, int order,
                                          uint8_t* __restrict__ blk_miss) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (32 * b >= n_snp) return;
    uint8_t m = 0;
    for (int j = 32 * b; j < min(n_snp, 32 * b + 32); ++j) m |= (row_miss[j] >> order) & 1;
    blk_miss[b] = m;
}

// Per run, one thread per row: the row's non-individual slots — the last byte's bit pairs that are not individuals
// for this run's sample order, (saved byte & keep) | (pad & ~keep), and the pitch padding after it — set to this run's
// pad code: 0x55 ("missing": x = h = o = 0 for the int8 / fp32 kernels) or 0x00 for the fp4 kernel, whose
// missing-indicator plane m must be 0 there so that SNPs without missing calls have an all-zero m plane (their m
// products are skipped; its epilogue counts o = 1 - m over the n_org individual slots); and the row's genotype counts:
// the load's counts of bytes [0, nb - 1) (lcounts, P parts: load_tiled_kernel — the run's count pass over every row
// until round 4, 6.3 GB at C3, now read where the load writes the rows) plus the last byte's individual pairs, to
// counts3[3 j + k] (k = hom A1, het, hom A2; the statistics kernel's input as one part).
__global__ void __launch_bounds__(256) tail_counts_kernel(uint8_t* __restrict__ img, const uint8_t* __restrict__ last,
                                                          int n_snp, int nb, int row_bytes, uint32_t tail_keep,
                                                          uint32_t pad, const int* __restrict__ lcounts, int P,
                                                          int* __restrict__ counts3) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_snp) return;
    int c[3] = {0, 0, 0};
    for (int p = 0; p < P; ++p) {
        const int* o = lcounts + ((size_t)p * n_snp + j) * 3;
        c[0] += o[0];
        c[1] += o[1];
        c[2] += o[2];
    }
    const uint32_t lb = ((uint32_t)last[j] & tail_keep) | (pad & ~tail_keep & 0xFFu);
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // the last byte's individual pairs
        if (((tail_keep >> (2 * k)) & 3u) == 0) continue;
        const uint32_t code = (lb >> (2 * k)) & 3u;
        c[0] += code == 0;
        c[1] += code == 2;
        c[2] += code == 3;
    }
    uint8_t* rbase = img + (size_t)(j >> 5) * 32 * (size_t)row_bytes + (size_t)(j & 31) * 32;
    const int n_ch = row_bytes >> 5, tc0 = (nb - 1) >> 5;  // chunks [tc0, n_ch) hold the last byte and padding
    for (int t = tc0; t < n_ch; ++t)
        for (int h = 0; h < 2; ++h) {
            uint4* unit = reinterpret_cast<uint4*>(rbase + (size_t)t * 1024 + 16 * h);
            const uint4 v = *unit;
            uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t o = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int p = 32 * t + 16 * h + 4 * q + k;
                    const uint32_t byte = p < nb - 1 ? (wd[q] >> (8 * k)) & 0xFFu : p == nb - 1 ? lb : (pad & 0xFFu);
                    o |= byte << (8 * k);
                }
                wd[q] = o;
            }
            *unit = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        }
    counts3[3 * (size_t)j] = c[0];
    counts3[3 * (size_t)j + 1] = c[1];
    counts3[3 * (size_t)j + 2] = c[2];
}

// ------------------------------------------------------------------------------------------
// 2. per-SNP statistics -> lookup tables
// ------------------------------------------------------------------------------------------
// Closed form of SNPInMemory::decode + standardise (encoder.h:91-133, tools.h:54-85) from the
// genotype counts c0 (hom A1), c1 (het), c2 (hom A2) over the n_org individuals the reference
// reads.  Missing calls are mean-imputed by the reference, so their centred value is exactly 0.
// Moments of one coding from its genotype counts (c0 hom A1, c1 het, c2 hom A2; N = n_org slots).
struct Coding {
    double abar, dbar, beta, sd_a, rstd, da[3], r[3];
};
__device__ __forceinline__ Coding coding_moments(double c0, double c1, double c2, double N) {
    Coding m;
    const double n_obs = c0 + c1 + c2;
    m.abar = (c1 + 2.0 * c2) / n_obs;
    m.dbar = 2.0 * (c1 + c2) / n_obs;
    m.da[0] = -m.abar; m.da[1] = 1.0 - m.abar; m.da[2] = 2.0 - m.abar;
    const double dd0 = -m.dbar, dd1 = 2.0 - m.dbar, dd2 = 2.0 - m.dbar;
    const double var_a = (c0 * m.da[0] * m.da[0] + c1 * m.da[1] * m.da[1] + c2 * m.da[2] * m.da[2]) / N;
    const double cov = (c0 * m.da[0] * dd0 + c1 * m.da[1] * dd1 + c2 * m.da[2] * dd2) / N;
    m.beta = cov / var_a;  // Math::regression_residuals slope
    m.r[0] = dd0 - m.beta * m.da[0]; m.r[1] = dd1 - m.beta * m.da[1]; m.r[2] = dd2 - m.beta * m.da[2];
    const int distinct = (c0 > 0) + (c1 > 0) + (c2 > 0);
    // <= 2 observed genotypes: the dominance coding is affine in the additive one, the residual is
    // exactly constant, its std exactly 0.
    const double var_r = distinct <= 2 ? 0.0 : (c0 * m.r[0] * m.r[0] + c1 * m.r[1] * m.r[1] + c2 * m.r[2] * m.r[2]) / N;
    m.sd_a = sqrt(var_a);
    m.rstd = sqrt(var_r);
    return m;
}

// flip[j]: the resident row of SNP j stores the swapped coding (00 <-> 11, see orient_rows_kernel).
// MAF, residual std and the filters come from the file's coding (the reference's); the constants of
// the exact epilogue and the fp32 lookup table describe the stored coding the band kernels read.
// Swapping the alleles negates A and leaves R unchanged (the residual of [x >= 1] and of [x <= 1] on
// span{1, x} is the same vector), so every r^2 is the same.
// parts / P: the count kernel's per-part genotype counts, summed here into counts[4 j + k] (read by the rare-variant
// kernels after this one).  zero: a word to clear (the deferred rare-variant slot counter), no memset of its own.
__global__ void snp_stats_kernel(const int* __restrict__ parts, int P, int* __restrict__ counts, int* __restrict__ zero,
                                 const uint8_t* __restrict__ flip,
                                 const double* __restrict__ pos, int n_snp, int n_snp_pad, int n_org, double maf_thr,
                                 double std_thr, float2* __restrict__ lut, SnpConst* __restrict__ cst,
                                 uint8_t* __restrict__ sflags, double* __restrict__ maf_out,
                                 double* __restrict__ rstd_out, double* __restrict__ l2_acc,
                                 double* __restrict__ l2d_acc, int* __restrict__ ws_acc, uint8_t* __restrict__ blk_rep) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_snp_pad) return;
    if (j == 0 && zero != nullptr) *zero = 0;
    if (j < n_snp && l2_acc != nullptr) {  // the band's per-SNP accumulators and the replay's block flags start at 0
        l2_acc[j] = 0.0;
        l2d_acc[j] = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) ws_acc[(size_t)k * n_snp + j] = 0;
        if (blk_rep != nullptr && (j & 31) == 0) blk_rep[j >> 5] = 0;
    }
    float2 L[4] = {make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f), make_float2(0.f, 0.f)};
    SnpConst K = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    uint8_t fl = 0;
    double sX = 0.0, sH = 0.0, sOb = 0.0;
    if (j < n_snp) {
        int q[3] = {0, 0, 0};
        for (int p = 0; p < P; ++p) {
            const int* o = parts + ((size_t)p * n_snp + j) * 3;
            q[0] += o[0];
            q[1] += o[1];
            q[2] += o[2];
        }
        counts[4 * (size_t)j] = q[0];
        counts[4 * (size_t)j + 1] = q[1];
        counts[4 * (size_t)j + 2] = q[2];
        const double s0 = q[0], c1 = q[1], s2 = q[2];
        const bool fj = flip != nullptr && flip[j];
        const double c0 = fj ? s2 : s0, c2 = fj ? s0 : s2;  // the file's coding
        sX = c1 + 2.0 * s2;  // sums over the stored coding's indicators
        sH = c1 + s2;
        sOb = s0 + c1 + s2;
        const double qnan = __builtin_nan("");
        double maf_d = qnan, rstd_d = qnan;
        if (pos[j] >= 0.0) {  // SNPFilter::is_used (tools.h:15-23)
            const double n_obs = c0 + c1 + c2;
            const double N = (double)n_org;
            // MAF exactly as encoder.h:114-118 (fp64 mean of integers cast to fp32)
            const float add_mean = (float)((c1 + 2.0 * c2) / n_obs);
            const float f2 = add_mean / 2;
            const float maf = f2 < 0.5f ? f2 : 1 - f2;
            maf_d = (double)maf;
            if (!((double)maf <= maf_thr)) {  // encoder.h:120
                fl |= 1;  // MAF pass
                if (n_obs == 0.0) {
                    // every call missing: the reference's vectors are all NaN (MAF NaN passes the
                    // filter); they poison every window containing this SNP.
                    for (int c = 0; c < 4; ++c) L[c] = make_float2(qnan, 0.f);
                    K = SnpConst{qnan, qnan, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                } else {
                    const Coding f = coding_moments(c0, c1, c2, N);
                    rstd_d = f.rstd;
                    const bool rpass = rstd_d > std_thr;  // SNPFilter::residuals_std (tools.h:40-43)
                    if (rpass) fl |= 2;
                    const Coding m = fj ? coding_moments(s0, c1, s2, N) : f;  // the stored coding
                    const float ia = (float)(m.da[0] / m.sd_a), ib = (float)(m.da[1] / m.sd_a),
                                ic = (float)(m.da[2] / m.sd_a);
                    float ra = 0.f, rb = 0.f, rc = 0.f;
                    if (rpass) { ra = (float)(m.r[0] / m.rstd); rb = (float)(m.r[1] / m.rstd); rc = (float)(m.r[2] / m.rstd); }
                    L[0] = make_float2(ia, ra);   // stored code 00 (hom A1, or hom A2 when flipped)
                    L[1] = make_float2(0.f, 0.f); // code 01 missing (imputed -> centred 0)
                    L[2] = make_float2(ib, rb);   // code 10 het
                    L[3] = make_float2(ic, rc);   // stored code 11
                    // exact path: A = (x - mu o) / sa,  R = (2h - beta x - c o) / s   (x, h, o integer)
                    K = SnpConst{m.abar, m.sd_a, rpass ? m.dbar - m.beta * m.abar : 0.0, rpass ? m.beta : 0.0,
                                 rpass ? m.rstd : 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                }
            }
        }
        if (s0 + c1 + s2 < (double)n_org) fl |= 4;  // some individual's call is missing (m plane not all zero)
        maf_out[j] = maf_d;
        rstd_out[j] = (fl & 1) ? rstd_d : qnan;
    }
    for (int c = 0; c < 4; ++c) lut[(size_t)j * 4 + c] = L[c];
    K.X = sX; K.H = sH; K.Ob = sOb;
    K.SA = K.sa != 0.0 ? (sX - K.mu * sOb) / K.sa : 0.0;  // ~0: exactly centred
    K.SR = K.s != 0.0 ? (2.0 * sH - K.beta * sX - K.c * sOb) / K.s : 0.0;
    K.isa = K.sa != 0.0 ? 1.0 / K.sa : 0.0;  // (NaN for an all-missing SNP: its windows stay poisoned)
    K.is = K.s != 0.0 ? 1.0 / K.s : 0.0;
    cst[j] = K;
    sflags[j] = fl | 8;  // bit 3: the pairs whose lower SNP this is are computed here (pair_range_kernel clears it)
}

// ------------------------------------------------------------------------------------------
// 2b. the reference's residual of nearly degenerate SNPs, in its own fp32 arithmetic
// ------------------------------------------------------------------------------------------
// SNPs with a nearly empty genotype class (rare variants; at most REF_RESIDUAL_MIN_CLASS calls in one class) have
// a residual close to degenerate, where the reference's fp32 rounding is not small against it: at N = 315 599
// its residual std is off the exact one by up to ~1e-2 relative for SNPs with <= 7 calls in a class (the
// oracle: tests/test_oracle.py), and its residual vector carries a noise component along the additive one.
// The extreme case: a SNP whose read samples hold het and hom-A2 calls but no hom-A1 call has a constant dominance coding
// (2 for every observed call, and 2 imputed for missing ones), so its regression residual is exactly
// constant and the closed form above reports std 0.  The reference computes that residual in fp32
// (encoder.h:124-133, tools.h:54-85): slope = (x.y/n - x_mean y_mean) / (x.x/n - x_mean^2) from fp32 sums in
// two different orders (arma::mean: two interleaved accumulators; BLAS sdot: 64 lanes), so the slope is not
// exactly 0 and the residual 2 - slope x has a rounding-noise std that mostly exceeds --std-thr (all 96 of
// such SNPs at N = 50 000, std-thr 1e-5: tests/test_oracle.py) — the reference then counts the SNP in its
// neighbours' WSD and L2D with that noise vector, which is +-its additive vector.  These SNPs are rare
// variants with A1 the minor allele (PLINK's default) and only exist when every sample slot the reference
// reads is an individual (N % 4 == 0, or the strict PLINK order): for N % 4 != 0 it reads a padding
// hom-A1 call in every row.  This kernel replays that arithmetic step for step, in the sample order the
// reference reads, with the oracle's model of the third-party sums (oracle/ldscore_oracle.c: arma::mean,
// OpenBLAS 0.3.28's SkylakeX sdot, g++'s FMA contraction of `dot/n - x_mean*y_mean` and `y - slope*x`): the
// residual takes one fp32 value per genotype code, which enter the exact epilogue as R = (2h - beta x - c o) / s
// and the fp32 path's lookup table.  One wave per SNP; SNPs of any other kind return at once.
// Every operation is an explicit correctly rounded one and contraction is off: hipcc would otherwise fuse a*b+c.

// a value per 2-bit code, selected in registers (indexing a private array would go through scratch memory)
struct Vals4 {
    float v0, v1, v2, v3;
    __device__ __forceinline__ float operator()(int c) const { return c == 0 ? v0 : c == 1 ? v1 : c == 2 ? v2 : v3; }
};

// The row goes through LDS in chunks of REF_CHUNK bytes (4 REF_CHUNK samples, a multiple of 64): every lane loads
// its share of the next chunk into registers before the current one is processed, so the loads hide behind the
// sequential sums.
constexpr int REF_CHUNK = 2048;

struct RefPass {
    // per pass: up to two sdots (all lanes: lane L takes samples t = L mod 64 below n64) and two means (lanes 0-1:
    // the even / odd accumulators of the first, lanes 2-3 of the second)
    Vals4 dx, dy, du, dv, mv, mw;
    bool two_dots, two_means, means;
};

// One resident row in the block-interleaved layout (tile_off): 16-byte vector v and byte k of the row.
struct TiledRow {
    const uint8_t* base;  // the row's bytes of chunk 0
    __device__ __forceinline__ uint4 u4(int v) const {
        return *reinterpret_cast<const uint4*>(base + (size_t)(v >> 1) * 1024 + 16 * (v & 1));
    }
    __device__ __forceinline__ uint32_t byte(int k) const { return base[(size_t)(k >> 5) * 1024 + (k & 31)]; }
};

// One pass over the n samples of `row` in the reference's order; codes are read as stored (values are given per
// stored code, the file's coding folded in).  Returns the lane's sdot accumulators (x.y, u.v) and, on lanes 0-3,
// its mean accumulator.
__device__ void ref_pass(const TiledRow row, int n, int row_bytes, bool strict, const RefPass& P, uint32_t* buf,
                         float2* tab, float& acc_d, float& acc_e, float& acc_m) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    // the mean lanes read, per byte, the values of their two samples in it (tab[m][byte], m = lane: 0 / 1 the
    // even / odd samples of the first mean, 2 / 3 of the second)
    if (P.means) {
        __syncthreads();
        for (int e = lane; e < 4 * 256; e += 64) {
            const int m = e >> 8, byte = e & 255, k0 = m & 1;
            const Vals4 V = m < 2 ? P.mv : P.mw;
            const int sa = strict ? 2 * k0 : 6 - 2 * k0, sb = strict ? 2 * (k0 + 2) : 6 - 2 * (k0 + 2);
            tab[e] = make_float2(V((byte >> sa) & 3), V((byte >> sb) & 3));
        }
    }
    const int n64 = (n & -32) & ~63;
    const int n_bytes = (n + 3) >> 2;
    const int n_vec = row_bytes >> 4;  // 16-byte vectors in the row (never read past it)
    constexpr int PER = REF_CHUNK / 16 / 64;  // 16-byte vectors per lane per chunk
    uint4 nxt[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) nxt[u] = (u * 64 + lane < n_vec) ? row.u4(u * 64 + lane) : make_uint4(0, 0, 0, 0);
    const int par = lane & 1;
    const Vals4 M = lane < 2 ? P.mv : P.mw;  // the tail samples
    const bool my_mean = P.means && (lane < 2 || (P.two_means && lane < 4));
    for (int b0 = 0; b0 < n_bytes; b0 += REF_CHUNK) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PER; ++u) reinterpret_cast<uint4*>(buf)[u * 64 + lane] = nxt[u];
        __syncthreads();
        const int b1 = b0 + REF_CHUNK;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int v = (b1 >> 4) + u * 64 + lane;
            nxt[u] = (b1 < n_bytes && v < n_vec) ? row.u4(v) : make_uint4(0, 0, 0, 0);
        }
        const uint8_t* bb = reinterpret_cast<const uint8_t*>(buf);
        // sdots: sample t = 4 b0 + 64 s + lane, byte 16 s + lane / 4
        const int sh_l = strict ? 2 * (lane & 3) : 6 - 2 * (lane & 3);
        const int s_end = min(REF_CHUNK / 16, (n64 - 4 * b0 + 63 - lane) / 64);
        for (int s = 0; s < s_end; ++s) {
            const int c = (bb[16 * s + (lane >> 2)] >> sh_l) & 3;
            acc_d = __fmaf_rn(P.dx(c), P.dy(c), acc_d);
            if (P.two_dots) acc_e = __fmaf_rn(P.du(c), P.dv(c), acc_e);
        }
        // means: lane 0 / 2 the even samples, 1 / 3 the odd ones, in order
        if (my_mean) {
            const int t_end = min(4 * REF_CHUNK, n - 4 * b0);  // samples of this chunk
            const int n_full = t_end >> 4;                    // whole 16-sample words
            const uint32_t* bw = buf;
            const float2* T = tab + 256 * lane;
#pragma unroll 2
            for (int q = 0; q < n_full; ++q) {
                const uint32_t x = bw[q];
#pragma unroll
                for (int b = 0; b < 4; ++b) {  // byte b: samples 16 q + 4 b + par, then + 2
                    const float2 v = T[(x >> (8 * b)) & 0xFFu];
                    acc_m = acc_m + v.x;
                    acc_m = acc_m + v.y;
                }
            }
            for (int t = 16 * n_full + par; t < t_end; t += 2) {
                const int shift = strict ? 2 * (t & 3) : 6 - 2 * (t & 3);
                acc_m = acc_m + M((bb[t >> 2] >> shift) & 3);
            }
        }
    }
}

// the lanes' sdot accumulators -> arma::dot (oracle/ldscore_oracle.c dot_f): lanes folded (k, k + 8), one
// 32-sample FMA step if n1 % 64 = 32, summed, then the tail in double.  n <= 32: Armadillo's two FMA
// accumulators.  On every lane.
__device__ float ref_dot_finish(const TiledRow row, int n, bool strict, float acc, Vals4 X, Vals4 Y, float* sh) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    auto code = [&](int t) { return (int)((row.byte(t >> 2) >> (strict ? 2 * (t & 3) : 6 - 2 * (t & 3))) & 3); };
    __syncthreads();
    sh[lane] = acc;
    __syncthreads();
    if (lane == 0) {
        if (n <= 32) {
            float a = 0.f, b = 0.f;
            int t = 0;
            for (; t + 1 < n; t += 2) {
                const int c0 = code(t), c1 = code(t + 1);
                a = __fmaf_rn(X(c0), Y(c0), a);
                b = __fmaf_rn(X(c1), Y(c1), b);
            }
            if (t < n) { const int c0 = code(t); a = __fmaf_rn(X(c0), Y(c0), a); }
            sh[64] = a + b;
        } else {
            const int n1 = n & -32, n64 = n1 & ~63;
            float b[4][8];
            for (int q = 0; q < 4; ++q)
                for (int k = 0; k < 8; ++k) b[q][k] = sh[16 * q + k] + sh[16 * q + k + 8];
            if (n1 > n64)
                for (int q = 0; q < 4; ++q)
                    for (int k = 0; k < 8; ++k) {
                        const int c = code(n64 + 8 * q + k);
                        b[q][k] = __fmaf_rn(X(c), Y(c), b[q][k]);
                    }
            float cc[8], h[4];
            for (int k = 0; k < 8; ++k) cc[k] = ((b[0][k] + b[1][k]) + b[2][k]) + b[3][k];
            for (int k = 0; k < 4; ++k) h[k] = cc[k] + cc[k + 4];
            double d = (double)((h[0] + h[1]) + (h[2] + h[3]));
            for (int t = n1; t < n; ++t) {
                const int c = code(t);
                d = d + (double)(X(c) * Y(c));
            }
            sh[64] = (float)d;
        }
    }
    __syncthreads();
    return sh[64];
}

// lanes 0 / 1 (or 2 / 3) accumulators -> arma::mean = (a + b) / n, on every lane
__device__ float ref_mean_finish(int n, float acc, int first, float* sh) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    __syncthreads();
    if (lane < 4) sh[lane] = acc;
    __syncthreads();
    return (sh[first] + sh[first + 1]) / (float)n;
}

// the SNPs the replay handles: MAF-passing, observed, at most REF_RESIDUAL_MIN_CLASS calls in a genotype class
__device__ __forceinline__ bool replayed_snp(const int* counts, const uint8_t* flip, const uint8_t* sflags, int j) {
    if (!(sflags[j] & 1)) return false;  // MAF-failed or unused: no residual
    const int s0 = counts[4 * (size_t)j], c1 = counts[4 * (size_t)j + 1], s2 = counts[4 * (size_t)j + 2];
    (void)flip;  // the class counts do not depend on the stored orientation
    return s0 + c1 + s2 > 0 && min(s0, min(c1, s2)) <= REF_RESIDUAL_MIN_CLASS;
}

// per 32-SNP block: does it hold a replayed SNP?  Cheap and first, so that the band launch for the other items
// (KC = false) can run while reference_residual_kernel's long sequential sums run beside it.
__global__ void replay_flags_kernel(const int* __restrict__ counts, const uint8_t* __restrict__ flip,
                                    const uint8_t* __restrict__ sflags, int n_snp, uint8_t* __restrict__ blk_rep) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_snp && replayed_snp(counts, flip, sflags, j)) blk_rep[j >> 5] = 1;
}

__global__ void __launch_bounds__(64) reference_residual_kernel(const uint8_t* __restrict__ img, int row_bytes,
                                                                int n_org, int strict, const int* __restrict__ counts,
                                                                const uint8_t* __restrict__ flip, int n_snp,
                                                                double std_thr, SnpConst* __restrict__ cst,
                                                                float2* __restrict__ lut, uint8_t* __restrict__ sflags,
                                                                double* __restrict__ rstd_out) {
#pragma clang fp contract(off)
    const int j = blockIdx.x;
    if (j >= n_snp || !replayed_snp(counts, flip, sflags, j)) return;
    const int s0 = counts[4 * (size_t)j], c1 = counts[4 * (size_t)j + 1], s2 = counts[4 * (size_t)j + 2];
    const bool fj = flip != nullptr && flip[j];
    const int c0 = fj ? s2 : s0, c2 = fj ? s0 : s2;
    __shared__ uint32_t buf[REF_CHUNK / 4];
    __shared__ float2 tab[4 * 256];
    __shared__ float sh[72];
    const TiledRow row{img + tile_off(j, 0, row_bytes)};
    const bool st = strict != 0;
    const double nn = (double)n_org, n_obs = (double)(c0 + c1 + c2);
    // per STORED code (00, 01, 10, 11): the file's code is 3, 1, 2, 0 when the row is stored flipped
    auto stored = [&](float hom1, float miss, float het, float hom2) {
        return fj ? Vals4{hom2, miss, het, hom1} : Vals4{hom1, miss, het, hom2};
    };
    // decode (encoder.h:95-129): fp64 sums of integers, means cast to fp32 impute the missing calls
    const float mua = (float)(((double)c1 + 2.0 * (double)c2) / n_obs);
    const float mud = (float)(2.0 * ((double)c1 + (double)c2) / n_obs);
    const Vals4 X = stored(0.f, mua, 1.f, 2.f), Y = stored(0.f, mud, 2.f, 2.f);
    // pass 1: arma::mean of x and y, x.y and x.x (Math::regression_residuals, tools.h:54-68)
    float d1 = 0.f, e1 = 0.f, m1 = 0.f;
    ref_pass(row, n_org, row_bytes, st, RefPass{X, Y, X, X, X, Y, true, true, true}, buf, tab, d1, e1, m1);
    const float x_mean_f = ref_mean_finish(n_org, m1, 0, sh);
    const double x_mean = (double)x_mean_f, y_mean = (double)ref_mean_finish(n_org, m1, 2, sh);
    const double dxy = (double)ref_dot_finish(row, n_org, st, d1, X, Y, sh);
    const double dxx = (double)ref_dot_finish(row, n_org, st, e1, X, X, sh);
    // g++'s FMA contractions of `dot/n - x_mean*y_mean` and `y - slope * x`
    const double slope = __fma_rn(-x_mean, y_mean, dxy / nn) / __fma_rn(-x_mean, x_mean, dxx / nn);
    const float k = (float)slope;
    const Vals4 R = {__fmaf_rn(-X.v0, k, Y.v0), __fmaf_rn(-X.v1, k, Y.v1), __fmaf_rn(-X.v2, k, Y.v2),
                     __fmaf_rn(-X.v3, k, Y.v3)};
    // Math::standardise (tools.h:70-85): mean, centre, var_ = sdot * (1 / n), sqrt, divide — of the additive
    // vector (encoder.h:130-132; its mean is x_mean) and of the residual
    const Vals4 CA = {X.v0 - x_mean_f, X.v1 - x_mean_f, X.v2 - x_mean_f, X.v3 - x_mean_f};
    float d2 = 0.f, e2 = 0.f, m2 = 0.f;  // pass 2: mean of the residual, (x - x_mean).(x - x_mean)
    ref_pass(row, n_org, row_bytes, st, RefPass{CA, CA, CA, CA, R, R, false, false, true}, buf, tab, d2, e2, m2);
    const float m = ref_mean_finish(n_org, m2, 0, sh);
    const float var_a = (float)((double)ref_dot_finish(row, n_org, st, d2, CA, CA, sh) * (1.0 / nn));
    const Vals4 C = {R.v0 - m, R.v1 - m, R.v2 - m, R.v3 - m};
    float d3 = 0.f, e3 = 0.f, m3 = 0.f;  // pass 3: (r - m).(r - m)
    ref_pass(row, n_org, row_bytes, st, RefPass{C, C, C, C, C, C, false, false, false}, buf, tab, d3, e3, m3);
    const float var = (float)((double)ref_dot_finish(row, n_org, st, d3, C, C, sh) * (1.0 / nn));
    const float sd = (float)sqrt((double)var);  // = correctly rounded sqrtf (__fsqrt_rn is the native 1-ulp one)
    const float sd_a = (float)sqrt((double)var_a);
    if ((threadIdx.x & 63) != 0) return;
    rstd_out[j] = (double)sd;
    SnpConst K = cst[j];
    float2* L = lut + (size_t)j * 4;
    // stored codes 00, 10, 11 (slots 0, 2, 3 of the tables) and their call counts; missing is slot 1
    const int sc[3] = {0, 2, 3};
    const int ns[3] = {s0, c1, s2};
    // A = (x - mu o) / sa + ka: ka = the missing calls' value, then a line in x through the two stored codes
    // with the most calls (the third, with <= REF_RESIDUAL_MIN_CLASS calls, is off it by rounding noise)
    double a[3];
    const double ka = (double)(CA(1) / sd_a);
    for (int q = 0; q < 3; ++q) a[q] = (double)(CA(sc[q]) / sd_a) - ka;
    const int drop = (ns[0] <= ns[1] && ns[0] <= ns[2]) ? 0 : (ns[1] <= ns[2] ? 1 : 2);
    const double u = drop == 0 ? a[2] - a[1] : drop == 1 ? 0.5 * (a[2] - a[0]) : a[1] - a[0];  // 1 / sa
    const double w = drop == 0 ? u - a[1] : -a[0];                                               // mu / sa
    K.sa = 1.0 / u;
    K.isa = u;
    K.mu = w / u;
    K.ka = ka;
    K.SA = (K.X - K.mu * K.Ob) / K.sa;
    for (int c = 0; c < 4; ++c) L[c].x = CA(c) / sd_a;
    if (!((double)sd > std_thr)) {  // SNPFilter::residuals_std: excluded (also NaN: a constant additive coding)
        sflags[j] &= (uint8_t)~2u;
        K.c = K.beta = K.s = K.kr = K.SR = K.is = 0.0;
        for (int c = 0; c < 4; ++c) L[c].y = 0.f;
        cst[j] = K;
        return;
    }
    sflags[j] |= 2;
    // R = (2h - beta x - c o) / s + kr: exact on all four codes (the second difference 2 r10 - r00 - r11 is
    // 2 / sd before standardising, never 0)
    double r[3];
    const double kr = (double)(C(1) / sd);
    for (int q = 0; q < 3; ++q) r[q] = (double)(C(sc[q]) / sd) - kr;
    K.s = 2.0 / (2.0 * r[1] - r[0] - r[2]);
    K.is = 0.5 * (2.0 * r[1] - r[0] - r[2]);
    K.beta = -(r[2] - r[1]) * K.s;
    K.c = -r[0] * K.s;
    K.kr = kr;
    K.SR = (2.0 * K.H - K.beta * K.X - K.c * K.Ob) / K.s;
    for (int c = 0; c < 4; ++c) L[c].y = C(c) / sd;
    cst[j] = K;
}

// Exact left pointer of ChunkwiseReader (stream.h:182-197) for positions sorted over the used SNPs,
// from the flag-independent all-pass replay: A_j = the all-pass left pointer (the first used SNP in
// j's window), -1 where the reference never computes j whatever the MAF flags (unused SNP, or its
// lagging right pointer).  Then L_j = the first used MAF-passing SNP in [A_j, j), or j itself, and
// -1 for SNPs failing MAF (tests/test_plan.py checks this against the sequential replay).
__global__ void left_pointer_kernel(const int* __restrict__ A, const uint8_t* __restrict__ sflags,
                                    const double* __restrict__ pos, int n, int* __restrict__ L) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    int l = -1;
    if (A[j] >= 0 && (sflags[j] & 1)) {
        l = A[j];
        while (l < j && !((sflags[l] & 1) && pos[l] >= 0.0)) ++l;
    }
    L[j] = l;
}

// ---- band schedule on the GPU (every position >= 0 and sorted; ld_engine.cpp plan_items is the host
// reference for any positions).  With all SNPs used, ChunkwiseReader's pointers reduce to window edges
// (stream.h:142-155,182-197): the all-pass left pointer A_j = first k with pos_j - pos_k <= w, and the
// right pointer R_j = min(n - 1, max(R_{j-1} + 1, E_j)) with E_j = first k > j with pos_k - pos_j > w
// (its extend_cache advances at least one SNP per SNP), i.e. R_j = min(n - 1, j + max_{k<=j}(E_k - k)).
// Row block I needs columns up to E_{i_end} - 1 (its last row's window edge; every later SNP whose
// window reaches back into I lies before it too).  Items are emitted in tiles of PLAN_R row blocks x
// PLAN_C diagonal offsets (see order_items_tiled), each tile's items row by row.
constexpr int PLAN_R = 16, PLAN_C = 16;

// Window edges of the sorted positions: A[j] = the first k <= j with pos_j - pos_k <= w, E[j] = the first k > j with
// pos_k - pos_j > w (n: none) — the predicates of the reference's window (tools.h:41-49), as the epilogue evaluates
// them.  Launched ahead of the count kernel: beside it, these dependent loads wait on its saturated HBM (a 1/8 shard of
// C3: 55-100 us instead of ~5).  Block 0 also zeroes the schedule's counters for the kernels after it.
__global__ void __launch_bounds__(256) plan_edges_kernel(const double* __restrict__ pos, int n, double w,
                                                         int* __restrict__ A, int* __restrict__ E,
                                                         int* __restrict__ meta) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 4) meta[threadIdx.x] = 0;
    if (j >= n) return;
    const double pj = pos[j];
    int lo = j + 1, hi = n;  // first k in (j, n] with pos_k - pos_j > w (n: none)
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pos[mid] - pj > w) hi = mid; else lo = mid + 1;
    }
    E[j] = lo;
    lo = 0; hi = j;  // first k in [0, j] with pos_j - pos_k <= w
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pj - pos[mid] <= w) hi = mid; else lo = mid + 1;
    }
    A[j] = lo;
}

// The plan's single-workgroup scans and its tile kernels run with 256-thread workgroups: they share the GPU with the
// count pass, whose 256-thread workgroups refill every CU as they finish — a 1024-thread workgroup (16 waves on one
// CU) waited for a CU to drain (C3 trace: plan_scan 0.57 ms, the old one-workgroup right-pointer walk 0.3 ms).
constexpr int PLAN_WG = 256;

// exclusive scan of v over the PLAN_WG threads (op: sum or max, identity id); the total on every thread
template <bool MAX>
__device__ __forceinline__ int block_scan_excl(int v, int id, int* part, int& total) {
    const int t = threadIdx.x;
    part[t] = v;
    __syncthreads();
    for (int o = 1; o < PLAN_WG; o <<= 1) {
        const int u = t >= o ? part[t - o] : id;
        __syncthreads();
        part[t] = MAX ? max(part[t], u) : part[t] + u;
        __syncthreads();
    }
    total = part[PLAN_WG - 1];
    const int ex = t > 0 ? part[t - 1] : id;
    __syncthreads();
    return ex;
}

// one workgroup: exclusive scan in place of n values, chunked per thread (thread t: [t per, (t + 1) per)); returns the
// total (sum, or max) on every thread
template <bool MAX>
__device__ __forceinline__ int chunked_scan_excl(int* __restrict__ v, int n, int id, int* part) {
    const int t = threadIdx.x, per = (n + PLAN_WG - 1) / PLAN_WG;
    const int b = min(n, t * per), e = min(n, b + per);
    int acc = id;
    for (int k = b; k < e; ++k) acc = MAX ? max(acc, v[k]) : acc + v[k];
    int total;
    int run = block_scan_excl<MAX>(acc, id, part, total);
    for (int k = b; k < e; ++k) {
        const int c = v[k];
        v[k] = run;
        run = MAX ? max(run, c) : run + c;
    }
    return total;
}

// R_j = min(n - 1, j + running max of (E_k - k)): a max-scan in tiles of PLAN_WG SNPs — the tiles' maxima, their
// exclusive scan (one workgroup), then each tile's inclusive scan from its prefix.
__global__ void __launch_bounds__(PLAN_WG) plan_tile_max_kernel(const int* __restrict__ E, int n, int* __restrict__ tmax) {
    __shared__ int part[PLAN_WG];
    const int k = blockIdx.x * PLAN_WG + threadIdx.x;
    int total;
    (void)block_scan_excl<true>(k < n ? E[k] - k : INT_MIN, INT_MIN, part, total);
    if (threadIdx.x == 0) tmax[blockIdx.x] = total;
}
// in place: tmax[b] = max of the tiles before b (INT_MIN for the first)
__global__ void __launch_bounds__(PLAN_WG) plan_tile_scan_kernel(int* __restrict__ tmax, int ntile) {
    __shared__ int part[PLAN_WG];
    (void)chunked_scan_excl<true>(tmax, ntile, INT_MIN, part);
}
__global__ void __launch_bounds__(PLAN_WG) plan_right_kernel(const int* __restrict__ E, int n,
                                                           const int* __restrict__ tpre, int* __restrict__ R) {
    __shared__ int part[PLAN_WG];
    const int k = blockIdx.x * PLAN_WG + threadIdx.x;
    const int v = k < n ? E[k] - k : INT_MIN;
    int total;
    const int ex = block_scan_excl<true>(v, INT_MIN, part, total);
    if (k < n) R[k] = min(n - 1, k + max(max(ex, v), tpre[blockIdx.x]));
}

// per row block I: useful column offsets d = J - I, [d0, d1] (empty: d0 > d1); meta[0] = max d1 + 1,
// meta[2] = diagonal items
__global__ void plan_rows_kernel(const int* __restrict__ E, const int* __restrict__ A, int n, int nblk, int own_lo,
                                 int own_hi, int2* __restrict__ rows, int* __restrict__ meta) {
    const int I = blockIdx.x * blockDim.x + threadIdx.x;
    if (I >= nblk) return;
    int2 r = make_int2(1, 0);
    if (I >= A[own_lo] / 32 && I * 32 < own_hi) {
        const int i_end = min(n, 32 * I + 32) - 1;
        const int Jmax = min(nblk - 1, (E[i_end] - 1) / 32);
        const int ob0 = own_lo / 32, ob1 = (own_hi - 1) / 32;
        const bool own_row = I >= ob0 && I <= ob1;
        const int J0 = own_row ? I : max(I, ob0), J1 = own_row ? Jmax : min(Jmax, ob1);
        r = make_int2(J0 - I, J1 - I);
    }
    rows[I] = r;
    if (r.x <= r.y) {
        atomicMax(&meta[0], r.y + 1);
        if (r.x == 0) atomicAdd(&meta[2], 1);
    }
}

__device__ __forceinline__ int plan_n_c(const int* meta) { return (meta[0] + PLAN_C - 1) / PLAN_C; }

// per tile (T, c) of PLAN_R row blocks x PLAN_C offsets, in (T, c) order: its item count (pair: items of two
// neighbouring column blocks, (I, J, 2), the last of a row's run in a tile possibly (I, J, 1))
__global__ void plan_count_kernel(const int2* __restrict__ rows, int nblk, const int* __restrict__ meta,
                                  int* __restrict__ counts, int pair) {
    const int n_t = (nblk + PLAN_R - 1) / PLAN_R, n_c = plan_n_c(meta);
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n_t * n_c; k += gridDim.x * blockDim.x) {
        const int T = k / n_c, c = k % n_c;
        int cnt = 0;
        for (int I = T * PLAN_R; I < min(nblk, T * PLAN_R + PLAN_R); ++I) {
            const int a = max(rows[I].x, c * PLAN_C), b = min(rows[I].y, c * PLAN_C + PLAN_C - 1);
            if (a <= b) cnt += pair ? (b - a + 2) / 2 : b - a + 1;
        }
        counts[k] = cnt;
    }
}

// one workgroup: exclusive scan of the tile counts in place; meta[1] = total items
__global__ void __launch_bounds__(PLAN_WG) plan_scan_kernel(int* __restrict__ counts, int nblk, int* __restrict__ meta) {
    __shared__ int part[PLAN_WG];
    const int total = chunked_scan_excl<false>(counts, (nblk + PLAN_R - 1) / PLAN_R * plan_n_c(meta), 0, part);
    if (threadIdx.x == 0) meta[1] = total;
}

// one workgroup: exclusive scan of n counts in place; *total = their sum
__global__ void __launch_bounds__(PLAN_WG) scan_counts_kernel(int* __restrict__ counts, int n, int* __restrict__ total) {
    __shared__ int part[PLAN_WG];
    const int t = chunked_scan_excl<false>(counts, n, 0, part);
    if (threadIdx.x == 0) *total = t;
}

__global__ void plan_emit_kernel(const int2* __restrict__ rows, int nblk, const int* __restrict__ meta,
                                 const int* __restrict__ offsets, int4* __restrict__ items, int pair) {
    const int n_t = (nblk + PLAN_R - 1) / PLAN_R, n_c = plan_n_c(meta);
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n_t * n_c; k += gridDim.x * blockDim.x) {
        const int T = k / n_c, c = k % n_c;
        int o = offsets[k];
        for (int I = T * PLAN_R; I < min(nblk, T * PLAN_R + PLAN_R); ++I) {
            const int a = max(rows[I].x, c * PLAN_C), b = min(rows[I].y, c * PLAN_C + PLAN_C - 1);
            for (int d = a; d <= b; d += 1 + pair) items[o++] = make_int4(I, I + d, pair ? min(2, b - d + 1) : 1, 0);
        }
    }
}

// The whole schedule of a short slice in one workgroup (n <= PLAN_SMALL_N: a rank's shard of a chromosome): the right
// pointers (plan_tile_max / tile_scan / right), the row ranges (plan_rows), the tile counts and their scan (plan_count /
// plan_scan) and the items (plan_emit) — the same values, in one launch instead of seven on the critical path of a
// ~2.5 ms run (each a few us of work behind ~5-20 us of launch latency).  Row ranges and tile counts stay in LDS between
// the phases; `items` must hold every block pair I <= J (the count is known only here).
constexpr int PLAN_SMALL_WG = 1024;
template <bool MAX>
__device__ __forceinline__ int small_scan_excl(int v, int id, int* part, int& total) {
    const int t = threadIdx.x;
    part[t] = v;
    __syncthreads();
    for (int o = 1; o < PLAN_SMALL_WG; o <<= 1) {
        const int u = t >= o ? part[t - o] : id;
        __syncthreads();
        part[t] = MAX ? max(part[t], u) : part[t] + u;
        __syncthreads();
    }
    total = part[PLAN_SMALL_WG - 1];
    const int ex = t > 0 ? part[t - 1] : id;
    __syncthreads();
    return ex;
}
__global__ void __launch_bounds__(PLAN_SMALL_WG) plan_small_kernel(const int* __restrict__ A, const int* __restrict__ E,
                                                                   int n, int own_lo, int own_hi, int* __restrict__ R,
                                                                   int2* __restrict__ rows, int* __restrict__ counts,
                                                                   int* __restrict__ meta, int4* __restrict__ items,
                                                                   int pair) {
    constexpr int MAX_BLK = PLAN_SMALL_N / 32, MAX_TILES = ((MAX_BLK + 15) / 16) * ((MAX_BLK + 15) / 16);
    __shared__ int part[PLAN_SMALL_WG];
    __shared__ int2 srows[MAX_BLK];
    __shared__ int scnt[MAX_TILES];
    __shared__ int s_maxd, s_diag;
    const int t = threadIdx.x, nblk = (n + 31) / 32;
    if (t == 0) { s_maxd = 0; s_diag = 0; }
    {  // R_k = min(n - 1, k + max_{j <= k} (E_j - j)): a chunked max-scan
        const int per = (n + PLAN_SMALL_WG - 1) / PLAN_SMALL_WG, b = min(n, t * per), e = min(n, b + per);
        int acc = INT_MIN;
        for (int k = b; k < e; ++k) acc = max(acc, E[k] - k);
        int total;
        int run = small_scan_excl<true>(acc, INT_MIN, part, total);
        for (int k = b; k < e; ++k) {
            run = max(run, E[k] - k);
            R[k] = min(n - 1, k + run);
        }
    }
    for (int I = t; I < nblk; I += PLAN_SMALL_WG) {  // as plan_rows_kernel
        int2 r = make_int2(1, 0);
        if (I >= A[own_lo] / 32 && I * 32 < own_hi) {
            const int i_end = min(n, 32 * I + 32) - 1;
            const int Jmax = min(nblk - 1, (E[i_end] - 1) / 32);
            const int ob0 = own_lo / 32, ob1 = (own_hi - 1) / 32;
            const bool own_row = I >= ob0 && I <= ob1;
            const int J0 = own_row ? I : max(I, ob0), J1 = own_row ? Jmax : min(Jmax, ob1);
            r = make_int2(J0 - I, J1 - I);
        }
        srows[I] = r;
        rows[I] = r;
        if (r.x <= r.y) {
            atomicMax(&s_maxd, r.y + 1);
            if (r.x == 0) atomicAdd(&s_diag, 1);
        }
    }
    __syncthreads();
    const int n_t = (nblk + PLAN_R - 1) / PLAN_R, n_c = (s_maxd + PLAN_C - 1) / PLAN_C, nk = n_t * n_c;
    auto tile = [&](int k, auto&& emit) {  // the items of tile (T, c), row by row (plan_count / plan_emit)
        const int T = k / n_c, c = k % n_c;
        for (int I = T * PLAN_R; I < min(nblk, T * PLAN_R + PLAN_R); ++I) {
            const int a = max(srows[I].x, c * PLAN_C), b = min(srows[I].y, c * PLAN_C + PLAN_C - 1);
            for (int d = a; d <= b; d += 1 + pair) emit(make_int4(I, I + d, pair ? min(2, b - d + 1) : 1, 0));
        }
    };
    for (int k = t; k < nk; k += PLAN_SMALL_WG) {
        int cnt = 0;
        tile(k, [&](int4) { ++cnt; });
        scnt[k] = cnt;
    }
    __syncthreads();
    int total;
    {  // exclusive scan of the tile counts in place (LDS)
        const int per = (nk + PLAN_SMALL_WG - 1) / PLAN_SMALL_WG, b = min(nk, t * per), e = min(nk, b + per);
        int acc = 0;
        for (int k = b; k < e; ++k) acc += scnt[k];
        int run = small_scan_excl<false>(acc, 0, part, total);
        for (int k = b; k < e; ++k) {
            const int c = scnt[k];
            scnt[k] = run;
            counts[k] = run;
            run += c;
        }
    }
    __syncthreads();
    if (t == 0) {
        meta[0] = s_maxd;
        meta[1] = total;
        meta[2] = s_diag;
    }
    for (int k = t; k < nk; k += PLAN_SMALL_WG) {
        int o = scnt[k];
        tile(k, [&](int4 it) { items[o++] = it; });
    }
}

// Per-SNP sums across work items: every item adds its partial sums (fp64, per 32-SNP block) as fixed-point
// integers (2^-44 units; |partial| <= 32, a SNP's total < 2^19) with 64-bit integer atomics, so the total does not
// depend on the order in which items finish and L2 / L2D are bit-reproducible run to run (fp64 atomics are not).
// Non-finite partials (windows poisoned by an all-missing SNP) set a flag instead (nanf: bit 1 L2, bit 2 L2D).
constexpr double ACC_SCALE = 17592186044416.0;  // 2^44
__device__ __forceinline__ void acc_fixed(double* acc, int* nanf, int bit, double v) {
    if (!isfinite(v)) {
        atomicOr(nanf, bit);
        return;
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(acc), (unsigned long long)__double2ll_rn(v * ACC_SCALE));
}

// ------------------------------------------------------------------------------------------
// 3. band correlation kernel
// ------------------------------------------------------------------------------------------
// One wave per work item (I, J0, NC): row SNPs 32*I..+31, column SNPs 32*(J0+b)..+31.
// Lane l: i = l & 31 (its row SNP for the A operand and its column SNP for the B operand),
// h = l >> 5 (which half of each 32-byte chunk of the 2-bit rows it decodes).  At every MFMA
// step lane (i, h) supplies A[i][h] and B[h][j=i] for the same sample slot, so D accumulates
// sum_k A[i][k] B[k][j] over all sample slots.  fp32 partial sums are flushed into a second
// fp32 accumulator every FLUSH_IT chunks (2048 samples) to keep the K = N fp32 chain short.
constexpr int FLUSH_IT = 16;

struct SnpSlot {
    double pos;
    int L, R, fl, g;
};

__device__ __forceinline__ double r2_adjusted(double dot, double n) {
    // Math::r2_adjusted (tools.h:87-92)
    const double corr = dot * (1. / n);
    const double r2 = corr * corr;
    return 1. - (1. - r2) * (n - 1) / (n - 2);
}

// The same with the per-run constants 1 / n and (n - 1) / (n - 2) hoisted (no fp64 division per pair).
struct R2Adj {
    double inv_n, q;
    __device__ __forceinline__ explicit R2Adj(double n) : inv_n(1. / n), q((n - 1) / (n - 2)) {}
    __device__ __forceinline__ double operator()(double dot) const {
        const double corr = dot * inv_n;
        return 1. - (1. - corr * corr) * q;
    }
};

// ---- per-SNP sums of a block pair by wavefront reductions (ldscalc.h:34-47's reduction over neighbours) ----
// A 32x32 Gram tile is spread over the wave as MFMA accumulators: lane (i, h) holds column SNP i against the 16
// row SNPs rb + (r & 3) + 8 (r >> 2) + 4 h, r = 0..15.  Column sums are the lane's own 16 values plus its partner
// lane's (i, 1 - h); row sums are reduced across the 32 lanes of a half in registers (cross-lane DPP / swizzle
// moves, fixed order: bit-reproducible), with no LDS atomics and no barrier.
struct SlotSum {
    double l2, l2d;
    int cnt;  // WSA | WSD << 8 | WSDE << 16 (each <= 64 per block pair)
};
__device__ __forceinline__ SlotSum operator+(const SlotSum& a, const SlotSum& b) {
    return SlotSum{a.l2 + b.l2, a.l2d + b.l2d, a.cnt + b.cnt};
}

// v from lane (lane ^ M): M = 1, 2 quad permutes and 8 a row rotation (DPP, no LDS), 4 and 16 ds_swizzle
// (bit mode, within 32 lanes), 32 the other half of the wave (ds_bpermute)
template <int M>
__device__ __forceinline__ int xlane(int v) {
    if constexpr (M == 1) return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    else if constexpr (M == 2) return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    else if constexpr (M == 8) return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    else if constexpr (M == 4 || M == 16) return __builtin_amdgcn_ds_swizzle(v, 0x1F | (M << 10));
    else return __shfl_xor(v, M, 64);
}
template <int M>
__device__ __forceinline__ double xlane(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = xlane<M>((int)(b & 0xFFFFFFFFll)), hi = xlane<M>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int M>
__device__ __forceinline__ SlotSum xlane(const SlotSum& v) {
    return SlotSum{xlane<M>(v.l2), xlane<M>(v.l2d), xlane<M>(v.cnt)};
}

// Transposed reduction of 4 row values per lane (rows k = 0..3 of a row group) over the 32 lanes of a half: two
// halving exchanges (each lane sends the rows it gives up and keeps the others), then a butterfly over lane octets.
// Afterwards the 8 lanes i with i >> 3 == k hold row k's total.  5 cross-lane moves per quantity for 4 rows.
__device__ __forceinline__ SlotSum reduce_rows4(const SlotSum (&v)[4], int i) {
    const bool b16 = (i & 16) != 0, b8 = (i & 8) != 0;
    SlotSum k0 = b16 ? v[2] : v[0], k1 = b16 ? v[3] : v[1];
    const SlotSum s0 = b16 ? v[0] : v[2], s1 = b16 ? v[1] : v[3];
    k0 = k0 + xlane<16>(s0);
    k1 = k1 + xlane<16>(s1);
    SlotSum k = b8 ? k1 : k0;
    k = k + xlane<8>(b8 ? k0 : k1);
    k = k + xlane<4>(k);
    k = k + xlane<2>(k);
    k = k + xlane<1>(k);
    return k;
}

// One slot's sums of one work item -> the per-SNP totals (2^-44 fixed point, order-independent across items).
__device__ __forceinline__ void flush_slot(const SnpSlot& si, const SlotSum& v, int own_lo, int own_hi, int n_snp,
                                           double* l2_acc, double* l2d_acc, int* ws_acc) {
    const int g = si.g;
    if (v.cnt == 0 || g < own_lo || g >= own_hi || g >= n_snp) return;
    const int wsa = v.cnt & 0xFF, wsd = (v.cnt >> 8) & 0xFF, wse = v.cnt >> 16;
    int* nanf = &ws_acc[3 * (size_t)n_snp + g];
    if (wsa) {
        acc_fixed(&l2_acc[g], nanf, 1, v.l2);
        atomicAdd(&ws_acc[g], wsa);
    }
    if (wsd) {
        acc_fixed(&l2d_acc[g], nanf, 2, v.l2d);
        atomicAdd(&ws_acc[(size_t)n_snp + g], wsd);
        if (wse) atomicAdd(&ws_acc[2 * (size_t)n_snp + g], wse);
    }
}

constexpr int NC_MAX = 2;
constexpr int NS_MAX = 32 * (1 + NC_MAX);

struct BandLds {
    float2 tab[4 * NS_MAX];  // [code][slot], slot stride NS = 32 * (1 + NC) of the body
    SnpSlot info[NS_MAX];
};

// DIAG0: column block 0 is the row block itself (J0 == I).  Its R_I^T X_I product is the
// transpose of X_I^T R_I and is never needed, so those MFMAs are skipped.
template <int NC, bool DOM, bool DIAG0>
__device__ __forceinline__ void band_body(BandLds& sh, const int4 it, const uint32_t* __restrict__ geno,
                                          int pitch_words, int n_it, const float2* __restrict__ lut,
                                          const double* __restrict__ pos, const int* __restrict__ Lw,
                                          const int* __restrict__ Rw, const uint8_t* __restrict__ sflags, int n_snp,
                                          double ld_wind, double n_org, double rsq_thr, int own_lo, int own_hi,
                                          double* __restrict__ l2_acc, double* __restrict__ l2d_acc,
                                          int* __restrict__ ws_acc) {
    constexpr int NS = 32 * (1 + NC);  // SNP slots: 32 rows, then NC x 32 columns
    float2 (*tab)[NS] = reinterpret_cast<float2 (*)[NS]>(sh.tab);
    SnpSlot* info = sh.info;

    const int lane = threadIdx.x;
    const int i = lane & 31, h = lane >> 5;
    const int I = it.x, J0 = it.y;

    for (int s = lane; s < NS; s += 64) {
        const int g = s < 32 ? I * 32 + s : (J0 + (s - 32) / 32) * 32 + (s & 31);
        const float4 l01 = *reinterpret_cast<const float4*>(lut + (size_t)g * 4);
        const float4 l23 = *reinterpret_cast<const float4*>(lut + (size_t)g * 4 + 2);
        tab[0][s] = make_float2(l01.x, l01.y);
        tab[1][s] = make_float2(l01.z, l01.w);
        tab[2][s] = make_float2(l23.x, l23.y);
        tab[3][s] = make_float2(l23.z, l23.w);
        SnpSlot si;
        si.g = g;
        if (g < n_snp) {
            si.pos = pos[g]; si.L = Lw[g]; si.R = Rw[g]; si.fl = sflags[g];
        } else {
            si.pos = 0.0; si.L = -1; si.R = -2; si.fl = 0;
        }
        info[s] = si;
    }
    __syncthreads();

    f32x16 aa[NC], ar[NC], ra[NC], haa[NC], har[NC], hra[NC];
#pragma unroll
    for (int b = 0; b < NC; ++b) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            aa[b][r] = 0.f; haa[b][r] = 0.f;
            if (DOM) { ar[b][r] = 0.f; ra[b][r] = 0.f; har[b][r] = 0.f; hra[b][r] = 0.f; }
        }
    }

    const uint4* rowp = reinterpret_cast<const uint4*>(geno) + row_u4(I * 32 + i, pitch_words) + h;
    const uint4* colp[NC];
#pragma unroll
    for (int b = 0; b < NC; ++b) colp[b] = reinterpret_cast<const uint4*>(geno) + row_u4((J0 + b) * 32 + i, pitch_words) + h;

    const char* tabc = reinterpret_cast<const char*>(&tab[0][0]);
    const uint32_t rbase = (uint32_t)i * 8u;

    uint4 nr = rowp[0];
    uint4 nc[NC];
#pragma unroll
    for (int b = 0; b < NC; ++b) nc[b] = colp[b][0];

    for (int t0 = 0; t0 < n_it; t0 += FLUSH_IT) {
      const int t1 = min(t0 + FLUSH_IT, n_it);
      for (int t = t0; t < t1; ++t) {
        const uint4 wr4 = nr;
        uint4 wc4[NC];
#pragma unroll
        for (int b = 0; b < NC; ++b) wc4[b] = nc[b];
        if (t + 1 < n_it) {  // prefetch the next 32-byte chunk of every row
            nr = rowp[CHUNK_U4 * (t + 1)];
#pragma unroll
            for (int b = 0; b < NC; ++b) nc[b] = colp[b][CHUNK_U4 * (t + 1)];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t wr = q == 0 ? wr4.x : q == 1 ? wr4.y : q == 2 ? wr4.z : wr4.w;
            uint32_t wc[NC];
#pragma unroll
            for (int b = 0; b < NC; ++b) wc[b] = q == 0 ? wc4[b].x : q == 1 ? wc4[b].y : q == 2 ? wc4[b].z : wc4[b].w;
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const uint32_t cr = (wr >> (2 * s)) & 3u;
                const float2 vr = *reinterpret_cast<const float2*>(tabc + cr * (uint32_t)(NS * 8) + rbase);
#pragma unroll
                for (int b = 0; b < NC; ++b) {
                    const uint32_t cc = (wc[b] >> (2 * s)) & 3u;
                    const float2 vc = *reinterpret_cast<const float2*>(tabc + cc * (uint32_t)(NS * 8) +
                                                                       (uint32_t)(32 + 32 * b) * 8u + rbase);
                    aa[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr.x, vc.x, aa[b], 0, 0, 0);
                    if (DOM) {
                        ar[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr.x, vc.y, ar[b], 0, 0, 0);
                        if (!(DIAG0 && b == 0))
                            ra[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr.y, vc.x, ra[b], 0, 0, 0);
                    }
                }
            }
        }
      }
      // flush the fp32 chain of the last <= 2048 samples into the second-level sum
#pragma unroll
      for (int b = 0; b < NC; ++b) {
          haa[b] += aa[b];
          aa[b] = 0.f;
          if (DOM) { har[b] += ar[b]; hra[b] += ra[b]; ar[b] = 0.f; ra[b] = 0.f; }
      }
    }

    // ---- fused epilogue: r2adj, window / MAF / residual masks, per-SNP sums ------------------
    // (the row SNPs' sums over both column blocks, then reduced across the wave as in pair_epilogue)
    const double n_pad = 16.0 * (double)pitch_words - n_org;
    const R2Adj r2adj(n_org);
    SlotSum col[NC], mine = {0.0, 0.0, 0};
    int my_row = -1;
#pragma unroll
    for (int b = 0; b < NC; ++b) col[b] = SlotSum{0.0, 0.0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        SlotSum rowv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) rowv[k] = SlotSum{0.0, 0.0, 0};
#pragma unroll
        for (int b = 0; b < NC; ++b) {
            const int sj = 32 + 32 * b + i;
            const SnpSlot cj = info[sj];
            const bool diag = (J0 + b) == I;
            const bool pj = cj.fl & 1, rpj = (cj.fl & 2) != 0;
            const bool compj = cj.L >= 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = 4 * q + k;
                const int si = k + 8 * q + 4 * h;
                const SnpSlot ci = info[si];
                const bool pi = ci.fl & 1, rpi = (ci.fl & 2) != 0;
                const bool inwin = fabs(cj.pos - ci.pos) <= ld_wind && ci.g != cj.g;
                // j in N(i): SNP i's window scan (stream.h:142-155) covers j
                // (flag bit 3 of the pair's lower SNP: this engine computes the pair, see pair_range_kernel)
                const bool lo_ok = ((ci.g < cj.g ? ci.fl : cj.fl) & 8) != 0;
                const bool nij = lo_ok && inwin && ci.L >= 0 && cj.g >= ci.L && cj.g <= ci.R && pj;
                // i in N(j): only for off-diagonal blocks (a diagonal block holds both orders)
                const bool nji = lo_ok && !diag && inwin && compj && ci.g >= cj.L && ci.g <= cj.R && pi;
                if (nij || nji) {
                    // the n_pad non-individual slots hold code 01 (missing): remove their products (non-zero only
                    // for the replayed rare variants, whose missing calls are not centred at 0)
                    const float2 mi = tab[1][si], mj = tab[1][sj];
                    const double r2 = r2adj((double)haa[b][r] - n_pad * mi.x * mj.x);
                    if (nij) { rowv[k].l2 += r2; rowv[k].cnt += 1; }
                    if (nji) { col[b].l2 += r2; col[b].cnt += 1; }
                    if (DOM) {
                        if (nij && rpj) {  // a_i . r_j -> L2D_i (ldscalc.h:40-46)
                            const double rd = r2adj((double)har[b][r] - n_pad * mi.x * mj.y);
                            rowv[k].l2d += rd;
                            rowv[k].cnt += (1 << 8) + (rd > rsq_thr ? 1 << 16 : 0);
                        }
                        if (nji && rpi) {  // r_i . a_j -> L2D_j
                            const double rd = r2adj((double)hra[b][r] - n_pad * mi.y * mj.x);
                            col[b].l2d += rd;
                            col[b].cnt += (1 << 8) + (rd > rsq_thr ? 1 << 16 : 0);
                        }
                    }
                }
            }
        }
        const SlotSum t = reduce_rows4(rowv, i);
        if ((i & 7) == q) {
            mine = t;
            my_row = (i >> 3) + 8 * q + 4 * h;
        }
    }
    if (my_row >= 0) flush_slot(info[my_row], mine, own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
#pragma unroll
    for (int b = 0; b < NC; ++b) {
        const SlotSum c = col[b] + xlane<32>(col[b]);
        if (h == 0) flush_slot(info[32 + 32 * b + i], c, own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
    }
}

// One launch for all work items; `nc` (1 or 2 column blocks) is wave-uniform per item.
// WPS = minimum waves per SIMD the register allocation must allow (1: up to 512 VGPR+AGPR,
// 2: <= 256).
template <bool DOM, int WPS>
__global__ void __launch_bounds__(64, WPS) band_kernel(const uint32_t* __restrict__ geno, int pitch_words, int n_it,
                                                  const float2* __restrict__ lut, const int4* __restrict__ items,
                                                  const double* __restrict__ pos, const int* __restrict__ Lw,
                                                  const int* __restrict__ Rw, const uint8_t* __restrict__ sflags,
                                                  int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                                                  int own_hi, double* __restrict__ l2_acc, double* __restrict__ l2d_acc,
                                                  int* __restrict__ ws_acc) {
    __shared__ BandLds sh;
    const int4 it = items[blockIdx.x];
#define NLDSC_BODY(NC_, DIAG_)                                                                                        \
    band_body<NC_, DOM, DIAG_>(sh, it, geno, pitch_words, n_it, lut, pos, Lw, Rw, sflags, n_snp, ld_wind, n_org,     \
                               rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc)
    const bool diag = it.y == it.x;
    if (it.z == 2) { if (diag) NLDSC_BODY(2, true); else NLDSC_BODY(2, false); }
    else { if (diag) NLDSC_BODY(1, true); else NLDSC_BODY(1, false); }
#undef NLDSC_BODY
}

// ------------------------------------------------------------------------------------------
// 3b. exact-integer band kernel (int8 MFMA on genotype indicators)
// ------------------------------------------------------------------------------------------
// Per SNP and sample slot: x = additive count {0,1,2}, h = [genotype >= 1], o = [observed]; missing
// calls and padding slots are all-zero.  The reference's standardised vectors are affine in these
// (SnpConst), so every dot product it needs is an fp64 combination of 8 integer Gram entries per
// SNP pair: x.x, x.o, o.x, o.o (additive) and x.h, o.h, h.x, h.o (dominance, both directions).
// They are computed EXACTLY with v_mfma_i32_32x32x32_i8 (int32 sums, N < 2^29) — no rounding
// before the fp64 epilogue.  One wave per (row block I, column block J): lane i&31 = its SNP,
// lane>>5 = which 16-sample word of each K step it decodes.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// 16 two-bit codes of one word -> x, h, o as 16 bytes each (byte b of dword k = bit pair k of byte b;
// any fixed slot permutation is fine since A and B operands use the same one).
__device__ __forceinline__ void decode16(uint32_t w, i32x4& X, i32x4& H, i32x4& O) {
    const uint32_t hiw = (w >> 1) & 0x55555555u, low = w & 0x55555555u;
    const uint32_t xw = hiw + (hiw & low);             // 00->0, 01->0, 10->1, 11->2 (no carries)
    const uint32_t ow = (hiw | ~low) & 0x55555555u;     // 01 (missing / padding) -> 0
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        X[k] = (int)((xw >> (2 * k)) & 0x03030303u);
        H[k] = (int)((hiw >> (2 * k)) & 0x01010101u);
        O[k] = (int)((ow >> (2 * k)) & 0x01010101u);
    }
}

// The dispatcher places workgroup b on XCD b % 8, each XCD with its own L2.  xcd_slot gives every
// XCD a contiguous run of the (row-major) schedule instead, so the workgroups resident on one XCD
// work on neighbouring blocks of the band and share their strips in that XCD's L2.
__device__ __forceinline__ int xcd_slot(int b, int n) {
    const int per = n >> 3, rem = n & 7, x = b & 7;
    return x * per + min(x, rem) + (b >> 3);
}

// Which of the pair (row SNP ci, column SNP cj)'s two terms the epilogue adds: nij, j in N(i): SNP i's window scan
// (stream.h:142-155) covers j; nji, i in N(j), only off the diagonal.  The pair's lower SNP carries flag bit 3: this
// engine computes the pair (pair_range_kernel).
struct PairNeed {
    bool nij, nji;
};
__device__ __forceinline__ PairNeed pair_need(const SnpSlot& ci, const SnpSlot& cj, bool diag, double ld_wind) {
    const bool inwin = fabs(cj.pos - ci.pos) <= ld_wind && ci.g != cj.g;
    const bool lo_ok = ((ci.g < cj.g ? ci.fl : cj.fl) & 8) != 0;
    PairNeed n;
    n.nij = lo_ok && inwin && ci.L >= 0 && cj.g >= ci.L && cj.g <= ci.R && (cj.fl & 1);
    n.nji = lo_ok && !diag && inwin && cj.L >= 0 && ci.g >= cj.L && ci.g <= cj.R && (ci.fl & 1);
    return n;
}

// Epilogue of one 32x32 block pair (row slots rb.., column slots cb.. of the slot tables `info` / `cst`):
// standardised dots from the 8 integer Gram entries in fp64, r2adj, window/pointer masks, and the pair's
// per-SNP sums (ldscalc.h:33-55), reduced across the wave in registers (reduce_rows4) and added to the per-SNP
// totals (flush_slot).  diag: the pair is a diagonal block (row block == column block).  Called by every lane.
// MB: the Gram is in the missing basis {x, h, m} (fp4 path): gxo holds x.m, gox m.x, goo m.m, goh m.h,
// gho h.m, and `kslots` is the number of individual slots (n_org; the other slots are all-zero in every
// plane); o = 1 - m over the individual slots.
template <bool DOM, class Acc, bool MB = false, bool KC = false>
__device__ __forceinline__ void pair_epilogue(const SnpSlot* info, const SnpConst* cst, int rb, int cb, bool diag,
                                              int i, int h, const Acc& gxx, const Acc& gxo, const Acc& gox,
                                              const Acc& goo, const Acc& gxh, const Acc& goh, const Acc& ghx,
                                              const Acc& gho, double ld_wind, double n_org, double rsq_thr,
                                              double kslots, int own_lo, int own_hi, int n_snp,
                                              double* __restrict__ l2_acc, double* __restrict__ l2d_acc,
                                              int* __restrict__ ws_acc) {
    const R2Adj r2adj(n_org);
    const int sj = cb + i;
    const SnpSlot cj = info[sj];
    const SnpConst kj = cst[sj];
    const bool rpj = (cj.fl & 2) != 0;
    SlotSum col = {0.0, 0.0, 0}, mine = {0.0, 0.0, 0};
    int my_row = -1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // row group q: registers r = 4q + k, rows rb + k + 8q + 4h
        SlotSum rowv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = 4 * q + k;
            const int si = rb + k + 8 * q + 4 * h;
            const SnpSlot ci = info[si];
            const bool rpi = (ci.fl & 2) != 0;
            const PairNeed need = pair_need(ci, cj, diag, ld_wind);
            const bool nij = need.nij, nji = need.nji;
            SlotSum rv = {0.0, 0.0, 0};
            if (nij || nji) {
                const SnpConst ki = cst[si];
                // MB: the fp4 Gram is over v = m + 2x (the raw 2-bit code placed as an e2m1 value), h and m:
                // x.x = (v.v - v.m - m.v + m.m) / 4, x.m = (v.m - m.m) / 2, m.x = (m.v - m.m) / 2 (exact)
                const double mm = (double)goo[r];
                const double xx = MB ? 0.25 * ((double)gxx[r] - (double)gxo[r] - (double)gox[r] + mm) : (double)gxx[r];
                const double xo = MB ? ki.X - 0.5 * ((double)gxo[r] - mm) : (double)gxo[r];
                const double ox = MB ? kj.X - 0.5 * ((double)gox[r] - mm) : (double)gox[r];
                const double oo = MB ? ki.Ob + kj.Ob - kslots + mm : mm;
                // KC: the item holds a replayed rare variant (ka / kr terms; kept out of the common path, whose
                // registers are all taken)
                const double aa = (xx - kj.mu * xo - ki.mu * (ox - kj.mu * oo)) * (ki.isa * kj.isa) +
                                  (KC ? kj.ka * ki.SA + ki.ka * (kj.SA + kj.ka * n_org) : 0.0);
                const double r2 = r2adj(aa);
                if (nij) { rv.l2 = r2; rv.cnt = 1; }
                if (nji) { col.l2 += r2; col.cnt += 1; }
                if (DOM) {
                    if (nij && rpj) {  // A_i . R_j -> L2D_i (ldscalc.h:40-46)
                        const double xh = MB ? 0.5 * ((double)gxh[r] - (double)goh[r]) : (double)gxh[r];
                        const double oh = MB ? kj.H - (double)goh[r] : (double)goh[r];
                        const double ar = (2.0 * xh - kj.beta * xx - kj.c * xo -
                                           ki.mu * (2.0 * oh - kj.beta * ox - kj.c * oo)) * (ki.isa * kj.is) +
                                          (KC ? kj.kr * ki.SA + ki.ka * (kj.SR + kj.kr * n_org) : 0.0);
                        const double rd = r2adj(ar);
                        rv.l2d = rd;
                        rv.cnt += (1 << 8) + (rd > rsq_thr ? 1 << 16 : 0);
                    }
                    if (!diag && nji && rpi) {  // R_i . A_j -> L2D_j
                        const double hx = MB ? 0.5 * ((double)ghx[r] - (double)gho[r]) : (double)ghx[r];
                        const double ho = MB ? ki.H - (double)gho[r] : (double)gho[r];
                        const double ra = (2.0 * hx - ki.beta * xx - ki.c * ox -
                                           kj.mu * (2.0 * ho - ki.beta * xo - ki.c * oo)) * (ki.is * kj.isa) +
                                          (KC ? ki.kr * kj.SA + kj.ka * (ki.SR + ki.kr * n_org) : 0.0);
                        const double rd = r2adj(ra);
                        col.l2d += rd;
                        col.cnt += (1 << 8) + (rd > rsq_thr ? 1 << 16 : 0);
                    }
                }
            }
            rowv[k] = rv;
        }
        const SlotSum t = reduce_rows4(rowv, i);  // lanes i >> 3 == k: row rb + k + 8q + 4h
        if ((i & 7) == q) {
            mine = t;
            my_row = rb + (i >> 3) + 8 * q + 4 * h;
        }
    }
    col = col + xlane<32>(col);  // the partner lane (i, 1 - h) holds the other 16 rows of column i
    if (my_row >= 0) flush_slot(info[my_row], mine, own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
    if (h == 0) flush_slot(cj, col, own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
}

// Items holding a rare variant whose vectors are the reference's fp32 ones (ka / kr != 0: blk_rep[block] = 1,
// set by replay_flags_kernel) need the epilogue's ka / kr terms, which the common epilogue has no
// registers left for: they run in a second launch of the kernel instantiated with KC = true, and the KC = false
// launch skips them.  blk_rep == nullptr: no replayed SNP (KC = false only).
template <bool KC>
__device__ __forceinline__ bool skip_item(const uint8_t* blk_rep, int4 it) {
    if (!KC && blk_rep == nullptr) return false;
    const bool rep = blk_rep[it.x] | blk_rep[it.y] | (it.z == 2 && blk_rep[it.y + 1]);  // (it.z: column blocks)
    return KC ? !rep : rep;
}

struct BandI8Lds {
    SnpSlot info[NS_MAX];
    SnpConst cst[NS_MAX];
};

// NC column blocks J0 .. J0+NC-1 share the row decode; DIAG0: block 0 is the diagonal (J0 == I).
template <bool DOM, int NC, bool DIAG0, bool KC>
__device__ __forceinline__ void band_i8_body(BandI8Lds& sh, const int4 it, const uint32_t* __restrict__ geno,
                                             int pitch_words, int n_it, const SnpConst* __restrict__ cst,
                                             const double* __restrict__ pos, const int* __restrict__ Lw,
                                             const int* __restrict__ Rw, const uint8_t* __restrict__ sflags,
                                             int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                                             int own_hi, double* __restrict__ l2_acc, double* __restrict__ l2d_acc,
                                             int* __restrict__ ws_acc) {
    constexpr int NS = 32 * (1 + NC);
    const int lane = threadIdx.x;
    const int i = lane & 31, h = lane >> 5;
    const int I = it.x, J0 = it.y;
    for (int s = lane; s < NS; s += 64) {
        const int g = s < 32 ? I * 32 + s : (J0 + (s - 32) / 32) * 32 + (s & 31);
        SnpSlot si;
        si.g = g;
        if (g < n_snp) {
            si.pos = pos[g]; si.L = Lw[g]; si.R = Rw[g]; si.fl = sflags[g];
        } else {
            si.pos = 0.0; si.L = -1; si.R = -2; si.fl = 0;
        }
        sh.info[s] = si;
        sh.cst[s] = cst[g];
    }
    __syncthreads();

    // Gram accumulators: additive xx, xo, ox, oo; dominance xh, oh (row -> col), hx, ho (col -> row)
    i32x16 gxx[NC], gxo[NC], gox[NC], goo[NC], gxh[NC], goh[NC], ghx[NC], gho[NC];
#pragma unroll
    for (int b = 0; b < NC; ++b) {
        gxx[b] = gxo[b] = gox[b] = goo[b] = gxh[b] = goh[b] = ghx[b] = gho[b] = i32x16{};
    }
    const uint4* rowp = reinterpret_cast<const uint4*>(geno) + row_u4(I * 32 + i, pitch_words) + h;
    const uint4* colp[NC];
#pragma unroll
    for (int b = 0; b < NC; ++b) colp[b] = reinterpret_cast<const uint4*>(geno) + row_u4((J0 + b) * 32 + i, pitch_words) + h;
    auto word_of = [](const uint4& w, int q) { return q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w; };
    uint4 wr4 = rowp[0], wc4[NC];
#pragma unroll
    for (int b = 0; b < NC; ++b) wc4[b] = colp[b][0];
    // operands of the current K step; the next step's are decoded while these feed the MFMAs
    i32x4 Xi, Hi, Oi, Xj[NC], Hj[NC], Oj[NC];
    decode16(wr4.x, Xi, Hi, Oi);
#pragma unroll
    for (int b = 0; b < NC; ++b) decode16(wc4[b].x, Xj[b], Hj[b], Oj[b]);
    for (int t = 0; t < n_it; ++t) {
        uint4 nr = wr4, ncl[NC];
#pragma unroll
        for (int b = 0; b < NC; ++b) ncl[b] = wc4[b];
        if (t + 1 < n_it) {
            nr = rowp[CHUNK_U4 * (t + 1)];
#pragma unroll
            for (int b = 0; b < NC; ++b) ncl[b] = colp[b][CHUNK_U4 * (t + 1)];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            i32x4 Xin, Hin, Oin, Xjn[NC], Hjn[NC], Ojn[NC];
            decode16(q < 3 ? word_of(wr4, q + 1) : nr.x, Xin, Hin, Oin);
#pragma unroll
            for (int b = 0; b < NC; ++b) decode16(q < 3 ? word_of(wc4[b], q + 1) : ncl[b].x, Xjn[b], Hjn[b], Ojn[b]);
#pragma unroll
            for (int b = 0; b < NC; ++b) {
                gxx[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Xi, Xj[b], gxx[b], 0, 0, 0);
                gxo[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Xi, Oj[b], gxo[b], 0, 0, 0);
                gox[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Oi, Xj[b], gox[b], 0, 0, 0);
                goo[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Oi, Oj[b], goo[b], 0, 0, 0);
                if (DOM) {
                    gxh[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Xi, Hj[b], gxh[b], 0, 0, 0);
                    goh[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Oi, Hj[b], goh[b], 0, 0, 0);
                    if (!(DIAG0 && b == 0)) {  // on a diagonal block R_i . A_j is the transposed A_j . R_i
                        ghx[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Hi, Xj[b], ghx[b], 0, 0, 0);
                        gho[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Hi, Oj[b], gho[b], 0, 0, 0);
                    }
                }
            }
            // interleave: one MFMA, then a share of the next step's decode VALU (T19)
#pragma unroll
            for (int m = 0; m < 8 * NC; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
            }
            Xi = Xin; Hi = Hin; Oi = Oin;
#pragma unroll
            for (int b = 0; b < NC; ++b) { Xj[b] = Xjn[b]; Hj[b] = Hjn[b]; Oj[b] = Ojn[b]; }
        }
        wr4 = nr;
#pragma unroll
        for (int b = 0; b < NC; ++b) wc4[b] = ncl[b];
    }

    // ---- fused epilogue (fp64): standardised dots from the integer Gram, r2adj, masks, sums ----
#pragma unroll
    for (int b = 0; b < NC; ++b)
        pair_epilogue<DOM, i32x16, false, KC>(sh.info, sh.cst, 0, 32 + 32 * b, DIAG0 && b == 0, i, h, gxx[b], gxo[b],
                                              gox[b], goo[b], gxh[b], goh[b], ghx[b], gho[b], ld_wind, n_org, rsq_thr,
                                              0.0, own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
}

// One block pair per item (the engine plans single column blocks for the exact paths), 2 waves / SIMD.
template <bool DOM, bool KC>
__global__ void __launch_bounds__(64, 2) band_i8_kernel(const uint32_t* __restrict__ geno, int pitch_words, int n_it,
                                                      const SnpConst* __restrict__ cst, const int4* __restrict__ items,
                                                      const double* __restrict__ pos, const int* __restrict__ Lw,
                                                      const int* __restrict__ Rw, const uint8_t* __restrict__ sflags,
                                                      int n_snp, double ld_wind, double n_org, double rsq_thr,
                                                      int own_lo, int own_hi, double* __restrict__ l2_acc,
                                                      double* __restrict__ l2d_acc, int* __restrict__ ws_acc,
                                                      int xcd, const uint8_t* __restrict__ blk_rep) {
    __shared__ BandI8Lds sh;
    const int4 it = items[xcd ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x];
    if (skip_item<KC>(blk_rep, it)) return;
#define NLDSC_BODY(DIAG_)                                                                                             \
    band_i8_body<DOM, 1, DIAG_, KC>(sh, it, geno, pitch_words, n_it, cst, pos, Lw, Rw, sflags, n_snp, ld_wind, n_org,\
                                    rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc)
    if (it.y == it.x) NLDSC_BODY(true); else NLDSC_BODY(false);
#undef NLDSC_BODY
}

// ---- exact path on fp4 MFMAs: v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 operands ----
// v = m + 2x in {0, 1, 2, 4} and h, m in {0, 1} are exact e2m1 values (0000, 0010 = 1.0, 0100 = 2.0,
// 0110 = 4.0) and every product is an integer <= 16, so the fp32 accumulators hold exact integer Gram
// entries as long as they stay below 2^24: entries are <= 16N, so the engine uses this path for
// N < 2^20 (the int8 kernel above).  One K step = 64 sample slots = two 16-code words per lane (twice
// the int8 step, same 32-cycle MFMA), and the 2-bit -> 4-bit spread needs no shuffles because any fixed
// slot permutation is fine: even code pairs go to the nibbles of one dword, odd pairs to another (9
// VALU per word for v, h, m against 27 for the int8 byte spread).
// The third plane is the missing indicator m = [code 01] (missing call or padding slot) rather than
// o = 1 - m: genotypes are mostly observed, so o is mostly ones while m is mostly zeros, and an MFMA
// on mostly-zero operands draws less power (the chip holds a higher clock under this load).  The
// o-products follow exactly from per-SNP sums (pair_epilogue<.., MB = true>).
typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
constexpr int E8M0_ONE = 127;  // block scale 2^0
constexpr int E8M0_HALF = 126;  // 2^-1
// VALU instructions interleaved after each MFMA of a full 8-product K step (3, 5, 6 and alternating 4/5
// measured slower in round 1)
constexpr int F4_VPM = 4;  // (with the fenced loads, 3 / 5 measured slower / equal: profiles/r05_ab_load_fence.json)

struct F4Frag {
    i32x4 x, h, o;
};

// 16 two-bit codes (b1 b0) -> three e2m1 planes, even code pairs into the nibbles of the *0 dword, odd
// pairs into the *1 dword (any fixed slot permutation is fine: both operands use it).  The first plane is
// the code itself moved to nibble bits 2:1 — v = 0 (00 hom A1), 1.0 (01 missing), 2.0 (10 het), 4.0
// (11 hom A2) = m + 2x — which costs two VALU ops per dword instead of the three of x itself; the
// epilogue recovers the x products exactly.  WM (the block holds missing calls): h = [b1] and m = [b0 & ~b1]
// land on bit 1 (1.0), 9 VALU per word (m is one v_bitop3).  !WM (missing-free block: no m plane): h is taken
// from the two shifted words at bit 2 (2.0; the MFMAs scale such an h operand by 2^-1 through its E8M0 block
// scale, see H_SCALE), 6 VALU per word instead of 7.
template <bool WM>
__device__ __forceinline__ void decode_f4_word(uint32_t w, int& x0, int& x1, int& h0, int& h1, int& o0, int& o1) {
    constexpr uint32_t M = 0x22222222u, K6 = 0x66666666u, M4 = 0x44444444u;
    const uint32_t s1 = w << 1, s2 = w >> 1;
    x0 = (int)(s1 & K6);       // even (b1, b0) at bits (1, 0) -> (2, 1)
    x1 = (int)(s2 & K6);       // odd  (b1, b0) at bits (3, 2) -> (2, 1)
    if constexpr (WM) {
        const uint32_t w2 = w >> 2;
        h0 = (int)(w & M);
        h1 = (int)(w2 & M);
        o0 = (int)(s1 & ~w & M);   // m: code 01 -> 0010 (1.0), else 0
        o1 = (int)(s2 & ~w2 & M);
    } else {
        h0 = (int)(s1 & M4);       // b1 -> bit 2 (2.0)
        h1 = (int)(s2 & M4);
        o0 = o1 = 0;
    }
}

// decode_f4 with the two words' shifts as 64-bit shifts of (wb:wa): the bits crossing between the words land outside
// every mask (K6 and M keep nibble bits 1-2 / 1; the crossing bits are 0 of the high word and 30-31 of the low one), so
// the planes are bitwise decode_f4's, from 3 shifts per word pair instead of 6 (15 VALU instead of 18 with m planes).
// Used by the additive-only column-pair loop, where it measured C2 band -3 % (profiles/r06_ab_decode64.json); the
// add+dom single-block loop did not move and the quad kernel (register pairs moved into aligned places) slowed 6 %.
template <bool WM>
__device__ __forceinline__ F4Frag decode_f4_64(uint32_t wa, uint32_t wb) {
    constexpr uint32_t M = 0x22222222u, K6 = 0x66666666u, M4 = 0x44444444u;
    const uint64_t w = ((uint64_t)wb << 32) | wa;
    uint64_t s1, s2;  // (the compiler splits a 64-bit shift into v_alignbit + a 32-bit shift: asm keeps one instruction)
    asm("v_lshlrev_b64 %0, 1, %1" : "=v"(s1) : "v"(w));
    asm("v_lshrrev_b64 %0, 1, %1" : "=v"(s2) : "v"(w));
    const uint32_t s1a = (uint32_t)s1, s1b = (uint32_t)(s1 >> 32), s2a = (uint32_t)s2, s2b = (uint32_t)(s2 >> 32);
    F4Frag f;
    f.x = i32x4{(int)(s1a & K6), (int)(s2a & K6), (int)(s1b & K6), (int)(s2b & K6)};
    if constexpr (WM) {
        uint64_t w2;
        asm("v_lshrrev_b64 %0, 2, %1" : "=v"(w2) : "v"(w));
        const uint32_t w2a = (uint32_t)w2, w2b = (uint32_t)(w2 >> 32);
        f.h = i32x4{(int)(wa & M), (int)(w2a & M), (int)(wb & M), (int)(w2b & M)};
        f.o = i32x4{(int)(s1a & ~wa & M), (int)(s2a & ~w2a & M), (int)(s1b & ~wb & M), (int)(s2b & ~w2b & M)};
    } else {
        f.h = i32x4{(int)(s1a & M4), (int)(s2a & M4), (int)(s1b & M4), (int)(s2b & M4)};
        f.o = i32x4{0, 0, 0, 0};
    }
    return f;
}

template <bool WM>
__device__ __forceinline__ F4Frag decode_f4(uint32_t wa, uint32_t wb) {
    int x0, x1, x2, x3, h0, h1, h2, h3, o0, o1, o2, o3;
    decode_f4_word<WM>(wa, x0, x1, h0, h1, o0, o1);
    decode_f4_word<WM>(wb, x2, x3, h2, h3, o2, o3);
    F4Frag f;
    f.x = i32x4{x0, x1, x2, x3};
    f.h = i32x4{h0, h1, h2, h3};
    f.o = i32x4{o0, o1, o2, o3};
    return f;
}

// E8M0 block scale of an h operand decoded with decode_f4<WM>: h is 1.0 (WM) or 2.0 (!WM) per set slot
template <bool WM>
constexpr int H_SCALE = WM ? E8M0_ONE : E8M0_HALF;

// SA / SB: E8M0 block scales of the A / B operand (H_SCALE for an h plane)
template <int SA = E8M0_ONE, int SB = E8M0_ONE>
__device__ __forceinline__ f32x16v mfma_f4(const i32x4& a, const i32x4& b, const f32x16v& c) {
    const i32x8 A = {a[0], a[1], a[2], a[3], 0, 0, 0, 0}, B = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 4, 4, 0, SA, 0, SB);
}

// NC column blocks J0 .. J0+NC-1 share the row strip's decode; DIAG0: block 0 is the diagonal.
// tr (32 x 33 floats of LDS): on a diagonal block, m.x is the transpose of x.m, so its MFMAs are skipped and
// the epilogue reads x.m transposed through tr.
// SEG > 0 (NC == 1; rows longer than SEG chunks, N > 2^19): the K loop runs in segments of SEG chunks (128
// samples each, so a segment adds at most 16 * 128 * SEG <= 2^23 to an entry and the fp32 accumulators stay
// exact integers); after each segment the fp32 Gram is folded into int32 entries (add+dom) or its multiples
// of 2^16 move to packed 16-bit counters (additive-only), exact while every entry is <= 16N < 2^31.
// PART: K-split partial mode (small launches, see band_f4_part_kernel): run chunks [t_lo, t_hi) only and store
// the 8 fp32 Gram tiles to `part` (exact integers) instead of running the epilogue.
// the chunk loads of the K loop stay where they are written (issued two K steps before their data is decoded): left to
// itself the scheduler sank them to within ~10 MFMAs of their use, behind an s_waitcnt vmcnt(0)
#define NLDSC_LOAD_FENCE() __builtin_amdgcn_sched_barrier(0)
template <bool DOM, int NC, bool DIAG0, int SEG, bool KC, bool PART = false>
__device__ __forceinline__ void band_f4_body(BandI8Lds& sh, const int4 it, const uint32_t* __restrict__ geno,
                                             int pitch_words, int n_it, const SnpConst* __restrict__ cst,
                                             const double* __restrict__ pos, const int* __restrict__ Lw,
                                             const int* __restrict__ Rw, const uint8_t* __restrict__ sflags,
                                             int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                                             int own_hi, double* __restrict__ l2_acc, double* __restrict__ l2d_acc,
                                             int* __restrict__ ws_acc, float* tr, int t_lo = 0, int t_hi = 0,
                                             float* __restrict__ part = nullptr) {
    constexpr int NS = 32 * (1 + NC);
    const int lane = threadIdx.x & 63;
    const int i = lane & 31, h = lane >> 5;
    const int I = it.x, J0 = it.y;
    for (int s = lane; s < NS; s += 64) {
        const int g = s < 32 ? I * 32 + s : (J0 + (s - 32) / 32) * 32 + (s & 31);
        SnpSlot si;
        si.g = g;
        if (g < n_snp) {
            si.pos = pos[g]; si.L = Lw[g]; si.R = Rw[g]; si.fl = sflags[g];
        } else {
            si.pos = 0.0; si.L = -1; si.R = -2; si.fl = 0;
        }
        sh.info[s] = si;
        sh.cst[s] = cst[g];
    }
    __syncthreads();

    f32x16v gxx[NC], gxo[NC], gox[NC], goo[NC], gxh[NC], goh[NC], ghx[NC], gho[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) gxx[c] = gxo[c] = gox[c] = goo[c] = gxh[c] = goh[c] = ghx[c] = gho[c] = f32x16v{};
    const uint4* rowp = reinterpret_cast<const uint4*>(geno) + row_u4(I * 32 + i, pitch_words) + h;
    const uint4* colp[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) colp[c] = reinterpret_cast<const uint4*>(geno) + row_u4((J0 + c) * 32 + i, pitch_words) + h;
    // RM / CM: the row / column block holds missing calls.  A block without any has an all-zero m plane,
    // so the products with it are skipped (imputed hard calls: 3 of the 8 MFMAs remain).
    auto mfmas_v = [&](const F4Frag& a, const F4Frag (&b)[NC], auto RMc, auto CMc) {
        constexpr bool RM = decltype(RMc)::value, CM = decltype(CMc)::value;
        // Issue order xx, xo, xh, ox, hx, oo, oh, ho: the order alone moves the band kernel by up to 12 %
        // (decode interleave, register assignment); this one measured best of 18 orders in round 1.  On a
        // diagonal block m.x and h.x are the transposes of x.m and x.h (skipped).
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            gxx[c] = mfma_f4(a.x, b[c].x, gxx[c]);
            if (CM) gxo[c] = mfma_f4(a.x, b[c].o, gxo[c]);
            if (DOM) gxh[c] = mfma_f4<E8M0_ONE, H_SCALE<CM>>(a.x, b[c].h, gxh[c]);
            if (RM && !(DIAG0 && c == 0)) gox[c] = mfma_f4(a.o, b[c].x, gox[c]);
            if (DOM && !(DIAG0 && c == 0)) ghx[c] = mfma_f4<H_SCALE<RM>, E8M0_ONE>(a.h, b[c].x, ghx[c]);
            if (RM && CM) goo[c] = mfma_f4(a.o, b[c].o, goo[c]);
            if (DOM && RM) goh[c] = mfma_f4<E8M0_ONE, H_SCALE<CM>>(a.o, b[c].h, goh[c]);
            if (DOM && CM && !(DIAG0 && c == 0)) gho[c] = mfma_f4<H_SCALE<RM>, E8M0_ONE>(a.h, b[c].o, gho[c]);
        }
        // full 8-product steps: F4_VPM VALU after each MFMA; otherwise (additive-only items, missing-free
        // blocks) the decode is spread evenly over the MFMAs there are (additive-only C2: -6.6 % band time)
        if constexpr (RM && CM && DOM) {
#pragma unroll
            for (int m = 0; m < 8 * NC; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, NC == 1 ? F4_VPM : 4, 0);
            }
        } else {
            constexpr int n_mfma = NC * (1 + CM + RM + (RM && CM) + (DOM ? 2 + RM + CM : 0));
            constexpr int n_valu = (RM ? 9 : 6) * 2 + NC * (CM ? 9 : 6) * 2;  // the row strip decoded once
#pragma unroll
            for (int m = 0; m < n_mfma; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, (n_valu + n_mfma - 1) / n_mfma, 0);
            }
        }
    };
    // chunks [t_lo, t_hi), t_lo and t_hi even (rows are padded to 64 bytes).  Two chunk buffers: P holds
    // even chunks, Q odd ones; each is reloaded right after its last word is decoded and read again two K
    // steps later, with no register copies of loads in flight (those would force vmcnt(0)).
    // the strips' decode: with 64-bit shifts in the additive-only column-pair loop (decode_f4_64)
    auto dec = [](auto WMc, uint32_t wa, uint32_t wb) __attribute__((always_inline)) {
        constexpr bool WM = decltype(WMc)::value;
        if constexpr (NC == 2) return decode_f4_64<WM>(wa, wb);
        else return decode_f4<WM>(wa, wb);
    };
    auto kloop = [&](auto RMc, auto CMc, const int t_lo, const int t_hi) {
        const int last = t_hi - 1;
        uint4 pr = rowp[CHUNK_U4 * t_lo], qr = rowp[CHUNK_U4 * (t_lo + 1)], pc[NC], qc[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) { pc[c] = colp[c][CHUNK_U4 * t_lo]; qc[c] = colp[c][CHUNK_U4 * (t_lo + 1)]; }
        // two named fragment sets: set 1 is decoded while set 0 feeds the MFMAs and vice versa, so no
        // fragment is copied (a single rotating set costs ~12 v_mov per K step)
        F4Frag a0 = dec(RMc, pr.x, pr.y), a1, b0[NC], b1[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) b0[c] = dec(CMc, pc[c].x, pc[c].y);
        for (int t = t_lo; t < t_hi; t += 2) {
            a1 = dec(RMc, pr.z, pr.w);
#pragma unroll
            for (int c = 0; c < NC; ++c) b1[c] = dec(CMc, pc[c].z, pc[c].w);
            mfmas_v(a0, b0, RMc, CMc);  // K step 2t   (chunk t, words 0-1)
            pr = rowp[CHUNK_U4 * min(t + 2, last)];
#pragma unroll
            for (int c = 0; c < NC; ++c) pc[c] = colp[c][CHUNK_U4 * min(t + 2, last)];
            NLDSC_LOAD_FENCE();
            a0 = dec(RMc, qr.x, qr.y);
#pragma unroll
            for (int c = 0; c < NC; ++c) b0[c] = dec(CMc, qc[c].x, qc[c].y);
            mfmas_v(a1, b1, RMc, CMc);  // K step 2t+1 (chunk t, words 2-3)
            a1 = dec(RMc, qr.z, qr.w);
#pragma unroll
            for (int c = 0; c < NC; ++c) b1[c] = dec(CMc, qc[c].z, qc[c].w);
            mfmas_v(a0, b0, RMc, CMc);  // K step 2t+2 (chunk t+1, words 0-1)
            qr = rowp[CHUNK_U4 * min(t + 3, last)];
#pragma unroll
            for (int c = 0; c < NC; ++c) qc[c] = colp[c][CHUNK_U4 * min(t + 3, last)];
            NLDSC_LOAD_FENCE();
            a0 = dec(RMc, pr.x, pr.y);
#pragma unroll
            for (int c = 0; c < NC; ++c) b0[c] = dec(CMc, pc[c].x, pc[c].y);
            mfmas_v(a1, b1, RMc, CMc);  // K step 2t+3 (chunk t+1, words 2-3)
        }
    };
    // wave-uniform: does the row block / do the column blocks hold a missing call (flag bit 2)?  With PART this
    // is the only SNP state used (sh.cst and the other flag bits may be rewritten by a concurrent replay:
    // launch_reference_residuals in ld_kernels.h)
    const bool rm = __any(lane < 32 && (sh.info[lane].fl & 4));
    const bool cm = __any(32 + lane < NS && (sh.info[32 + lane].fl & 4));
    auto run = [&](const int t_lo, const int t_hi) {
        if (rm && cm) kloop(std::true_type{}, std::true_type{}, t_lo, t_hi);
        else if (rm) kloop(std::true_type{}, std::false_type{}, t_lo, t_hi);
        else if (cm) kloop(std::false_type{}, std::true_type{}, t_lo, t_hi);
        else kloop(std::false_type{}, std::false_type{}, t_lo, t_hi);
    };
    if constexpr (PART) {
        static_assert(SEG == 0 && NC == 1, "K-split: unsegmented single blocks");
        run(t_lo, t_hi);
        const f32x16v* tiles[8] = {&gxx[0], &gxo[0], &gox[0], &goo[0], &gxh[0], &goh[0], &ghx[0], &gho[0]};
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            float4* dst = reinterpret_cast<float4*>(part + t * 1024 + lane * 16);
            const f32x16v v = *tiles[t];
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        }
        return;
    } else if constexpr (SEG == 0) {
        run(0, n_it);
        if constexpr (DIAG0) {  // m.x(a, b) = x.m(b, a): lane (i, h) register r holds (row si(r), column i)
#pragma unroll
            for (int r = 0; r < 16; ++r) tr[((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + i] = gxo[0][r];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; ++r) gox[0][r] = tr[i * 33 + (r & 3) + 8 * (r >> 2) + 4 * h];
        }
#pragma unroll
        for (int c = 0; c < NC; ++c)
            pair_epilogue<DOM, f32x16v, true, KC>(sh.info, sh.cst, 0, 32 + 32 * c, DIAG0 && c == 0, i, h, gxx[c], gxo[c],
                                                  gox[c], goo[c], gxh[c], goh[c], ghx[c], gho[c], ld_wind, n_org,
                                                  rsq_thr, n_org, own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
    } else {
        static_assert(NC == 1, "segmented K loop: one column block");
        i32x16 ixx = {}, ixo = {}, iox = {}, ioo = {}, ixh = {}, ioh = {}, ihx = {}, iho = {};
        if constexpr (DOM) {
            // add+dom (1 wave / SIMD either way): the fp32 Gram is added into int32 accumulators after every
            // segment (measured 13 % faster than the packed counters below at N = 1 100 003)
            for (int t0 = 0; t0 < n_it; t0 += SEG) {
                run(t0, min(t0 + SEG, n_it));
                ixx += __builtin_convertvector(gxx[0], i32x16); ixo += __builtin_convertvector(gxo[0], i32x16);
                iox += __builtin_convertvector(gox[0], i32x16); ioo += __builtin_convertvector(goo[0], i32x16);
                ixh += __builtin_convertvector(gxh[0], i32x16); ioh += __builtin_convertvector(goh[0], i32x16);
                ihx += __builtin_convertvector(ghx[0], i32x16); iho += __builtin_convertvector(gho[0], i32x16);
                gxx[0] = gxo[0] = gox[0] = goo[0] = gxh[0] = goh[0] = ghx[0] = gho[0] = f32x16v{};
            }
        } else {
            // additive-only: after a segment every entry is < 2^16 + 2^23: its multiples of 2^16 move to a
            // 16-bit counter (entry / 2^16 <= 16N / 2^16 < 2^15 for N < 2^27) and the fp32 remainder, < 2^16,
            // stays in the accumulator (exact: both parts are integers below 2^24).  Two products share one
            // 32-bit counter register, so the fold costs 32 registers, not 64, and the kernel keeps 2 waves
            // per SIMD.
            typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
            u32x16 kxx = {}, kox = {};  // (xx | xo << 16), (ox | oo << 16)
            auto fold2 = [](f32x16v& a, f32x16v& b, u32x16& k) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float qa = floorf(a[r] * (1.0f / 65536.0f)), qb = floorf(b[r] * (1.0f / 65536.0f));
                    a[r] = fmaf(qa, -65536.0f, a[r]);
                    b[r] = fmaf(qb, -65536.0f, b[r]);
                    k[r] += (uint32_t)qa | ((uint32_t)qb << 16);
                }
            };
            for (int t0 = 0; t0 < n_it; t0 += SEG) {
                run(t0, min(t0 + SEG, n_it));
                fold2(gxx[0], gxo[0], kxx);
                fold2(gox[0], goo[0], kox);
            }
            auto whole = [](const f32x16v& a, const u32x16& k, int half) {
                i32x16 v;
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = (int)a[r] + (int)(((k[r] >> (16 * half)) & 0xffffu) << 16);
                return v;
            };
            ixx = whole(gxx[0], kxx, 0); ixo = whole(gxo[0], kxx, 1);
            iox = whole(gox[0], kox, 0); ioo = whole(goo[0], kox, 1);
        }
        if constexpr (DIAG0) {  // as above, on the int32 Gram (tr reused as 32 x 33 ints)
            int* tri = reinterpret_cast<int*>(tr);
#pragma unroll
            for (int r = 0; r < 16; ++r) tri[((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + i] = ixo[r];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; ++r) iox[r] = tri[i * 33 + (r & 3) + 8 * (r >> 2) + 4 * h];
        }
        pair_epilogue<DOM, i32x16, true, KC>(sh.info, sh.cst, 0, 32, DIAG0, i, h, ixx, ixo, iox, ioo, ixh, ioh, ihx,
                                             iho, ld_wind, n_org, rsq_thr, n_org, own_lo, own_hi, n_snp, l2_acc,
                                             l2d_acc, ws_acc);
    }
}

// Routing between the two fp4 kernels (blk_miss[b] = block b holds a missing call): a super-item whose four
// blocks are all missing-free (3 products per K step: operand-feed bound) runs in the 2 x 2 kernel, the block pairs
// of every other super-item (8 products: MFMA bound, where the single-block kernel is faster) in the single-block
// kernel.  Both kernels evaluate this predicate on the same clamped blocks, so every block pair runs exactly once.
__device__ __forceinline__ bool t2_routed(const uint8_t* blk_miss, int I2, int J2, int nblk) {
    return !(blk_miss[2 * I2] | blk_miss[min(2 * I2 + 1, nblk - 1)] | blk_miss[2 * J2] |
             blk_miss[min(2 * J2 + 1, nblk - 1)]);
}

// the 4 x 4 super-item (I4, J4) holds no missing call in its (clamped) row and column blocks
__device__ __forceinline__ bool q_routed(const uint8_t* blk_miss, int I4, int J4, int nblk) {
    uint8_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) m |= blk_miss[min(4 * I4 + k, nblk - 1)] | blk_miss[min(4 * J4 + k, nblk - 1)];
    return m == 0;
}

// Routing of the single-block items (route_shift 1: 2 x 2 super-items, t2_routed; 2: 4 x 4, q_routed): the item's
// block pair runs in the super-item kernel.
__device__ __forceinline__ bool routed_item(const uint8_t* blk_miss, int route_shift, int I, int J, int nblk) {
    return route_shift == 2 ? q_routed(blk_miss, I >> 2, J >> 2, nblk) : t2_routed(blk_miss, I >> 1, J >> 1, nblk);
}

// One block pair per item.  WPS 2, except the segmented add+dom kernel (its int32 fold registers need 1).
// NCX 2 (additive-only, unsegmented): items (I, J, 2) pair column blocks J and J + 1 in one wave (a 32 x 64 tile: the
// row strip decoded once for both), as the plan emits them with pairing; a column block the super-item routing sends
// elsewhere (blk_miss) is dropped from its item here.
template <bool DOM, int WPS, int SEG, bool KC, int NCX = 1>
__global__ void __launch_bounds__(64, WPS) band_f4_kernel(const uint32_t* __restrict__ geno, int pitch_words, int n_it,
                                                        const SnpConst* __restrict__ cst, const int4* __restrict__ items,
                                                        const double* __restrict__ pos, const int* __restrict__ Lw,
                                                        const int* __restrict__ Rw, const uint8_t* __restrict__ sflags,
                                                        int n_snp, double ld_wind, double n_org, double rsq_thr,
                                                        int own_lo, int own_hi, double* __restrict__ l2_acc,
                                                        double* __restrict__ l2d_acc, int* __restrict__ ws_acc, int xcd,
                                                        const uint8_t* __restrict__ blk_rep,
                                                        const uint8_t* __restrict__ blk_miss, int route_shift,
                                                        float* __restrict__ rep_gram, int4* __restrict__ rep_items,
                                                        int* __restrict__ rep_count) {
    __shared__ BandI8Lds sh;
    __shared__ float tr[32 * 33];
    auto item = [&](const int4 it) __attribute__((always_inline)) {  // (not a call: the body's registers stay live)
    if (skip_item<KC>(blk_rep, it)) {
        // rep_gram (unsegmented rows): an item holding a replayed rare variant runs its K loop here anyway, storing the
        // exact Gram tiles of each of its block pairs in a slot of rep_gram; band_f4_epi_kernel<DOM, true> applies the
        // epilogue (with the ka / kr terms) after the replay — so these items neither wait for the replay nor form a
        // launch of their own (one partial round of wave slots, or the whole band when most blocks hold such SNPs)
        if constexpr (!KC && SEG == 0) {
            if (rep_gram != nullptr) {
                const int nblk = (n_snp + 31) >> 5, lane = threadIdx.x & 63;
                for (int c = 0; c < (NCX == 2 ? it.z : 1); ++c) {
                    const int4 one = make_int4(it.x, it.y + c, 1, 0);
                    if (blk_miss != nullptr && routed_item(blk_miss, route_shift, one.x, one.y, nblk)) continue;
                    int slot = 0;
                    if (lane == 0) slot = atomicAdd(rep_count, 1);
                    slot = __shfl(slot, 0, 64);
                    if (lane == 0) rep_items[slot] = one;
                    __syncthreads();  // (the body rewrites the slot tables)
                    if (one.y == one.x)
                        band_f4_body<DOM, 1, true, 0, false, true>(sh, one, geno, pitch_words, n_it, cst, pos, Lw, Rw,
                                                                   sflags, n_snp, 0.0, 0.0, 0.0, 0, 0, nullptr, nullptr,
                                                                   nullptr, tr, 0, n_it, rep_gram + (size_t)slot * 8192);
                    else
                        band_f4_body<DOM, 1, false, 0, false, true>(sh, one, geno, pitch_words, n_it, cst, pos, Lw, Rw,
                                                                    sflags, n_snp, 0.0, 0.0, 0.0, 0, 0, nullptr, nullptr,
                                                                    nullptr, tr, 0, n_it, rep_gram + (size_t)slot * 8192);
                }
            }
        }
        return;
    }
#define NLDSC_BODY(NC_, DIAG_, IT_)                                                                                   \
    band_f4_body<DOM, NC_, DIAG_, SEG, KC>(sh, IT_, geno, pitch_words, n_it, cst, pos, Lw, Rw, sflags, n_snp, ld_wind, \
                                           n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc, tr)
    if constexpr (NCX == 2) {
        static_assert(!DOM && SEG == 0, "column-block pairs: additive-only, unsegmented rows");
        if (it.z == 2) {
            const int nblk = (n_snp + 31) >> 5;
            const bool r0 = blk_miss != nullptr && routed_item(blk_miss, route_shift, it.x, it.y, nblk);
            const bool r1 = blk_miss != nullptr && routed_item(blk_miss, route_shift, it.x, it.y + 1, nblk);
            if (r0 && r1) return;
            if (r0 || r1) {  // one column block left: the single-block body on it
                const int4 one = make_int4(it.x, it.y + (r0 ? 1 : 0), 1, 0);
                if (one.y == one.x) NLDSC_BODY(1, true, one); else NLDSC_BODY(1, false, one);
                return;
            }
            if (it.y == it.x) NLDSC_BODY(2, true, it); else NLDSC_BODY(2, false, it);
            return;
        }
    }
    // blk_miss: a super-item kernel runs the missing-free super-items
    if (blk_miss != nullptr && routed_item(blk_miss, route_shift, it.x, it.y, (n_snp + 31) >> 5)) return;
    if (it.y == it.x) NLDSC_BODY(1, true, it); else NLDSC_BODY(1, false, it);
#undef NLDSC_BODY
    };
    item(items[xcd ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x]);
}

// ---- 2 x 2 block-pair workgroups: the operand feed ----

// One workgroup of 4 waves per super-item (I2, J2) of the band: wave w computes the block pair
// (2 I2 + w / 2, 2 J2 + w % 2) when the plan needs it (rows[rb] = the needed column offsets of row block rb,
// plan_rows_kernel).  The four 32-SNP strips (row blocks 2 I2, 2 I2 + 1, column blocks 2 J2, 2 J2 + 1; only the
// first two on a diagonal super-item) go global -> LDS once per workgroup by global_load_lds, 1 KiB per strip and
// chunk, lane-linear in the (i, h) order the waves read them, through a ring of S two-chunk stages with S - 1
// stages in flight across the barriers (counted vmcnt, raw s_barrier): every strip byte fetched feeds two block
// pairs instead of one.  Diagonal block pairs issue all products (no transpose through LDS).
constexpr int T2_SLOTS = 128;  // LDS slot tables: 0-63 the two row blocks, 64-127 the two column blocks
template <int S>
struct T2Lds {
    uint4 stage[S][4][2][64];  // [buffer][strip][chunk of the stage][lane (i + 32 h)]
    SnpSlot info[T2_SLOTS];
    SnpConst cst[T2_SLOTS];
    // (each block pair's per-SNP sums are formed by its wave exactly as the single-block kernel forms them — the
    // same epilogue — so the fixed-point totals are bitwise that kernel's)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    // s_waitcnt encoding (gfx9): vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt[5:4] at [15:14]
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// the products of one K step for one block pair (band_f4_body's mfmas_v with one column block, no diagonal skip)
template <bool DOM, bool RM, bool CM>
__device__ __forceinline__ void f4_step(const F4Frag& a, const F4Frag& b, f32x16v& gxx, f32x16v& gxo, f32x16v& gox,
                                        f32x16v& goo, f32x16v& gxh, f32x16v& goh, f32x16v& ghx, f32x16v& gho) {
    gxx = mfma_f4(a.x, b.x, gxx);
    if (CM) gxo = mfma_f4(a.x, b.o, gxo);
    if (DOM) gxh = mfma_f4<E8M0_ONE, H_SCALE<CM>>(a.x, b.h, gxh);
    if (RM) gox = mfma_f4(a.o, b.x, gox);
    if (DOM) ghx = mfma_f4<H_SCALE<RM>, E8M0_ONE>(a.h, b.x, ghx);
    if (RM && CM) goo = mfma_f4(a.o, b.o, goo);
    if (DOM && RM) goh = mfma_f4<E8M0_ONE, H_SCALE<CM>>(a.o, b.h, goh);
    if (DOM && CM) gho = mfma_f4<H_SCALE<RM>, E8M0_ONE>(a.h, b.o, gho);
    constexpr int n_mfma = 1 + CM + RM + (RM && CM) + (DOM ? 2 + RM + CM : 0);
    constexpr int n_valu = (RM ? 18 : 12) + (CM ? 18 : 12);  // the next step's two decodes
#pragma unroll
    for (int m = 0; m < n_mfma; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, (n_valu + n_mfma - 1) / n_mfma, 0);
    }
}

template <bool DOM, int S, bool KC>
__global__ void __launch_bounds__(256, 2) band_f4_t2_kernel(
    const uint32_t* __restrict__ geno, int pitch_words, int n_it, const SnpConst* __restrict__ cst,
    const int4* __restrict__ items, const int2* __restrict__ rows, int nblk, const double* __restrict__ pos,
    const int* __restrict__ Lw, const int* __restrict__ Rw, const uint8_t* __restrict__ sflags, int n_snp,
    double ld_wind, double n_org, double rsq_thr, int own_lo, int own_hi, double* __restrict__ l2_acc,
    double* __restrict__ l2d_acc, int* __restrict__ ws_acc, int xcd, const uint8_t* __restrict__ blk_rep,
    const uint8_t* __restrict__ blk_miss) {
    static_assert(S >= 2, "ring of at least two stages");
    __shared__ T2Lds<S> sh;
    const int4 it = items[xcd ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x];
    const int I2 = it.x, J2 = it.y;
    // strip blocks (a block past the end, odd nblk, is clamped: its block pairs are not needed)
    const int b0 = 2 * I2, b1 = min(2 * I2 + 1, nblk - 1), b2 = 2 * J2, b3 = min(2 * J2 + 1, nblk - 1);
    if (KC || blk_rep != nullptr) {  // a super-item with a replayed SNP runs whole in the KC launch
        const bool rep = blk_rep[b0] | blk_rep[b1] | blk_rep[b2] | blk_rep[b3];
        if (KC ? !rep : rep) return;
    }
    if (blk_miss != nullptr && !t2_routed(blk_miss, I2, J2, nblk)) return;  // the single-block kernel's
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
    if (tid < T2_SLOTS) {
        const int blk = (tid < 64 ? 2 * I2 : 2 * J2) + ((tid >> 5) & 1);
        const int g = blk * 32 + (tid & 31);
        SnpSlot si;
        si.g = g;
        if (g < n_snp) {
            si.pos = pos[g]; si.L = Lw[g]; si.R = Rw[g]; si.fl = sflags[g];
        } else {
            si.pos = 0.0; si.L = -1; si.R = -2; si.fl = 0;
        }
        sh.info[tid] = si;
        sh.cst[tid] = blk < nblk ? cst[g] : SnpConst{};
    }
    const int rb = 2 * I2 + (w >> 1), cb = 2 * J2 + (w & 1);
    bool need = rb < nblk && cb < nblk;
    if (need) {
        const int2 r = rows[rb];
        need = cb - rb >= r.x && cb - rb <= r.y;
    }
    const bool dsup = I2 == J2;  // diagonal super-item: the column strips are the row strips
    const int sA = w >> 1, sB = dsup ? (w & 1) : 2 + (w & 1);
    const int my_blk = w == 0 ? b0 : w == 1 ? b1 : w == 2 ? b2 : b3;
    const bool loads = !(dsup && w >= 2);
    const uint4* src = reinterpret_cast<const uint4*>(geno) + row_u4(my_blk * 32 + i, pitch_words) + h;
    const int n_st = n_it >> 1;  // two-chunk stages (rows are padded to 64 bytes)
    // stage t (clamped to the last: the surplus loads of the tail rewrite the last stage's bytes into buffers no one
    // reads again) -> buffer t % S
    // (inline asm: hipcc's own LDS-DMA tracking cannot tell the ring buffers apart and would wait vmcnt(0) before
    // every stage's first ds_read; the counted waits below order them instead)
    auto issue = [&](int t) {
        const int tc = min(t, n_st - 1);
        if (loads) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const uint32_t dst = __builtin_amdgcn_readfirstlane(
                    (uint32_t)(size_t)(__attribute__((address_space(3))) void*)&sh.stage[t % S][w][c][0]);
                uint32_t keep;
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                             "s_mov_b32 m0, %0"
                             : "=&s"(keep)
                             : "v"(src + CHUNK_U4 * (2 * tc + c)), "s"(dst)
                             : "memory");
            }
        }
    };
    __syncthreads();  // slot tables written; nothing in flight yet
    const bool rm = __any(lane < 32 && (sh.info[32 * sA + lane].fl & 4));
    const bool cm = __any(lane < 32 && (sh.info[64 + 32 * (w & 1) + lane].fl & 4));
#pragma unroll
    for (int t = 0; t < S; ++t) issue(t);

    f32x16v gxx = {}, gxo = {}, gox = {}, goo = {}, gxh = {}, goh = {}, ghx = {}, gho = {};
    // Stage t is read from LDS into registers one stage ahead (during stage t - 1's MFMAs), so no ds_read latency
    // sits in front of a stage's first products.  At the barrier of iteration t every wave has stage t + 1 landed
    // and has finished reading stage t (its reads were waited for before the barrier), so buffer t % S takes stage
    // t + S right after it: S - 1 stages in flight, one in registers.
    auto read_stage = [&](int t, uint4 (&a)[2], uint4 (&b)[2]) {
        const uint4* A = &sh.stage[t % S][sA][0][0];
        const uint4* B = &sh.stage[t % S][sB][0][0];
#pragma unroll
        for (int c = 0; c < 2; ++c) { a[c] = A[c * 64 + lane]; b[c] = B[c * 64 + lane]; }
    };
    auto kloop = [&](auto RMc, auto CMc, auto ACTc) {
        constexpr bool RM = decltype(RMc)::value, CM = decltype(CMc)::value, ACT = decltype(ACTc)::value;
        uint4 ra[2], rb[2];
        wait_vmcnt<2 * (S - 1)>();  // stage 0 landed (this wave's loads)
        __builtin_amdgcn_s_barrier();  // every wave's
        asm volatile("" ::: "memory");
        if constexpr (ACT) read_stage(0, ra, rb);
        for (int t = 0; t < n_st; ++t) {
            wait_vmcnt<2 * (S - 2)>();  // this wave's loads of stage t + 1 have landed
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // its reads of stage t are in registers
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            issue(t + S);
            if constexpr (ACT) {
                uint4 na[2], nb[2];
                read_stage(t + 1, na, nb);  // past the last stage: a buffer of surplus bytes, never used
                __builtin_amdgcn_sched_barrier(0);  // issued here, ahead of the products (the scheduler sinks them)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const F4Frag a0 = decode_f4<RM>(ra[c].x, ra[c].y), f0 = decode_f4<CM>(rb[c].x, rb[c].y);
                    f4_step<DOM, RM, CM>(a0, f0, gxx, gxo, gox, goo, gxh, goh, ghx, gho);
                    const F4Frag a1 = decode_f4<RM>(ra[c].z, ra[c].w), f1 = decode_f4<CM>(rb[c].z, rb[c].w);
                    f4_step<DOM, RM, CM>(a1, f1, gxx, gxo, gox, goo, gxh, goh, ghx, gho);
                }
#pragma unroll
                for (int c = 0; c < 2; ++c) { ra[c] = na[c]; rb[c] = nb[c]; }
            }
        }
    };
    if (!need) kloop(std::false_type{}, std::false_type{}, std::false_type{});
    else if (rm && cm) kloop(std::true_type{}, std::true_type{}, std::true_type{});
    else if (rm) kloop(std::true_type{}, std::false_type{}, std::true_type{});
    else if (cm) kloop(std::false_type{}, std::true_type{}, std::true_type{});
    else kloop(std::false_type{}, std::false_type{}, std::true_type{});
    wait_vmcnt<0>();  // the tail's surplus loads
    if (!need) return;  // no barrier follows
    pair_epilogue<DOM, f32x16v, true, KC>(sh.info, sh.cst, 32 * sA, 64 + 32 * (w & 1), rb == cb, i, h, gxx, gxo, gox,
                                          goo, gxh, goh, ghx, gho, ld_wind, n_org, rsq_thr, n_org, own_lo, own_hi,
                                          n_snp, l2_acc, l2d_acc, ws_acc);
}

// ---- 4 x 4 block-pair workgroups for missing-free super-items (64 x 64 SNP tiles per wave) ----
// Measured on the 2 x 2 kernel (profiles/r03_pmc_t2_c5.json): each wave decodes two strips for the 3 products of one
// block pair per K step, ~9 VALU per MFMA, so two waves per SIMD are bound by the VALU issue port (MFMA 42 % busy).
// Here one wave per SIMD owns a 64 x 64 tile — row blocks 4 I4 + 2 (w >> 1) + {0, 1} x column blocks
// 4 J4 + 2 (w & 1) + {0, 1}, four block pairs — and decodes four strips for 12 products per K step (4 VALU per
// MFMA).  The eight strips of a super-item (four row, four column blocks; four on a diagonal super-item) go
// global -> LDS once per workgroup through the same ring of S two-chunk stages as the 2 x 2 kernel; each feeds
// four block pairs.  Only for super-items whose eight blocks hold no missing call (q_routed): the m products do
// not exist, the decode is the missing-free one.  A wave with no needed block pair issues no products; a wave
// with some computes all four and runs the epilogue of the needed ones (band edges: a few idle products).
constexpr int Q_SLOTS = 256;  // slot tables: strip s (0-3 row blocks, 4-7 column blocks) x 32 SNPs
template <int S>
struct QLds {
    uint4 stage[S][8][2][64];  // [buffer][strip][chunk of the stage][lane (i + 32 h)]
    SnpSlot info[Q_SLOTS];
    SnpConst cst[Q_SLOTS];
};

// one K step of a wave's four block pairs (a, b) of a missing-free super-item: g0 = x.x, g1 = x.h, g2 = h.x
// (2^-1-scaled h planes; additive-only: x.x alone).  (Round 3's study mode that also sent additive-only super-items
// holding missing calls here, with the four products of the missing basis, measured C2 band 2.29 -> 4.13 ms and is
// gone: profiles/r03_ab_quad_add_rejected.json.)
template <bool DOM>
__device__ __forceinline__ void q_step(const F4Frag (&A)[2], const F4Frag (&B)[2], f32x16v (&g0)[4], f32x16v (&g1)[4],
                                       f32x16v (&g2)[4]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const F4Frag& a = A[p >> 1];
        const F4Frag& b = B[p & 1];
        g0[p] = mfma_f4(a.x, b.x, g0[p]);
        if (DOM) {
            g1[p] = mfma_f4<E8M0_ONE, E8M0_HALF>(a.x, b.h, g1[p]);
            g2[p] = mfma_f4<E8M0_HALF, E8M0_ONE>(a.h, b.x, g2[p]);
        }
    }
    constexpr int n_mfma = DOM ? 12 : 4;
    constexpr int n_valu = 4 * (DOM ? 12 : 8);  // the next step's four decodes
#pragma unroll
    for (int m = 0; m < n_mfma; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, (n_valu + n_mfma - 1) / n_mfma, 0);
    }
}

template <bool DOM, int S, bool KC>
__global__ void __launch_bounds__(256, 1) band_f4_q_kernel(
    const uint32_t* __restrict__ geno, int pitch_words, int n_it, const SnpConst* __restrict__ cst,
    const int4* __restrict__ items, const int2* __restrict__ rows, int nblk, const double* __restrict__ pos,
    const int* __restrict__ Lw, const int* __restrict__ Rw, const uint8_t* __restrict__ sflags, int n_snp,
    double ld_wind, double n_org, double rsq_thr, int own_lo, int own_hi, double* __restrict__ l2_acc,
    double* __restrict__ l2d_acc, int* __restrict__ ws_acc, int xcd, const uint8_t* __restrict__ blk_rep,
    const uint8_t* __restrict__ blk_miss) {
    static_assert(S >= 2, "ring of at least two stages");
    __shared__ QLds<S> sh;
    const int4 it = items[xcd ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x];
    const int I4 = it.x, J4 = it.y;
    const bool dsup = I4 == J4;  // diagonal super-item: the column strips are the row strips
    auto strip_blk = [&](int s) { return s < 4 ? 4 * I4 + s : 4 * J4 + s - 4; };  // (may be >= nblk: no SNPs)
    if (KC || blk_rep != nullptr) {  // a super-item with a replayed SNP runs whole in the KC launch
        bool rep = false;
#pragma unroll
        for (int s = 0; s < 8; ++s) rep |= blk_rep[min(strip_blk(s), nblk - 1)] != 0;
        if (KC ? !rep : rep) return;
    }
    if (!q_routed(blk_miss, I4, J4, nblk)) return;  // the single-block kernel's
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, i = lane & 31, h = lane >> 5;
    {
        const int b = strip_blk(tid >> 5);
        const int g = b * 32 + (tid & 31);
        SnpSlot si;
        si.g = g;
        if (g < n_snp) {
            si.pos = pos[g]; si.L = Lw[g]; si.R = Rw[g]; si.fl = sflags[g];
        } else {
            si.pos = 0.0; si.L = -1; si.R = -2; si.fl = 0;
        }
        sh.info[tid] = si;
        sh.cst[tid] = b < nblk ? cst[g] : SnpConst{};
    }
    // this wave's block pairs p = 2a + b: row block 4 I4 + 2 (w >> 1) + a, column block 4 J4 + 2 (w & 1) + b
    const int rs = 2 * (w >> 1), cs = dsup ? 2 * (w & 1) : 4 + 2 * (w & 1);  // first row / column strip
    bool need[4];
    bool any = false;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int rb = strip_blk(rs + (p >> 1)), cb = 4 * J4 + 2 * (w & 1) + (p & 1);
        need[p] = rb < nblk && cb < nblk;
        if (need[p]) {
            const int2 r = rows[rb];
            need[p] = cb - rb >= r.x && cb - rb <= r.y;
        }
        any |= need[p];
    }
    // loads: wave w streams strips 2w, 2w + 1 (none for waves 2, 3 of a diagonal super-item)
    const bool loads = !(dsup && w >= 2);
    const uint4* src0 = reinterpret_cast<const uint4*>(geno) + row_u4(min(strip_blk(2 * w), nblk - 1) * 32 + i, pitch_words) + h;
    const uint4* src1 = reinterpret_cast<const uint4*>(geno) + row_u4(min(strip_blk(2 * w + 1), nblk - 1) * 32 + i, pitch_words) + h;
    const int n_st = n_it >> 1;
    auto issue = [&](int t) {
        const int tc = min(t, n_st - 1);
        if (loads) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const uint32_t dst = __builtin_amdgcn_readfirstlane(
                        (uint32_t)(size_t)(__attribute__((address_space(3))) void*)&sh.stage[t % S][2 * w + k][c][0]);
                    uint32_t keep;
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                                 "s_mov_b32 m0, %0"
                                 : "=&s"(keep)
                                 : "v"((k ? src1 : src0) + CHUNK_U4 * (2 * tc + c)), "s"(dst)
                                 : "memory");
                }
        }
    };
    __syncthreads();  // slot tables written; nothing in flight yet
#pragma unroll
    for (int t = 0; t < S; ++t) issue(t);

    f32x16v g0[4], g1[4], g2[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) g0[p] = g1[p] = g2[p] = f32x16v{};
    // as the 2 x 2 kernel's ring: stage t read into registers one stage ahead, S - 1 stages in flight
    auto read_stage = [&](int t, uint4 (&ra)[2][2], uint4 (&rb)[2][2]) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                ra[k][c] = sh.stage[t % S][rs + k][c][lane];
                rb[k][c] = sh.stage[t % S][cs + k][c][lane];
            }
    };
    // Two named fragment sets (F, G): the next K step's four strips are decoded while the current step's MFMAs issue —
    // across the stage boundary too: the next stage's first step is decoded from its registers (read from LDS a stage
    // ahead) during the current stage's last step, so after the barrier the MFMAs start at once
    auto kloop = [&](auto ACTc) {
        constexpr bool ACT = decltype(ACTc)::value;
        uint4 ra[2][2], rb[2][2];
        wait_vmcnt<4 * (S - 1)>();  // stage 0 landed (this wave's loads)
        __builtin_amdgcn_s_barrier();  // every wave's
        asm volatile("" ::: "memory");
        F4Frag FA[2], FB[2], GA[2], GB[2];
        auto dec = [&](F4Frag (&A)[2], F4Frag (&B)[2], const uint4 (&xa)[2][2], const uint4 (&xb)[2][2], int c,
                       bool hi) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                A[k] = hi ? decode_f4<false>(xa[k][c].z, xa[k][c].w) : decode_f4<false>(xa[k][c].x, xa[k][c].y);
                B[k] = hi ? decode_f4<false>(xb[k][c].z, xb[k][c].w) : decode_f4<false>(xb[k][c].x, xb[k][c].y);
            }
        };
        if constexpr (ACT) {
            read_stage(0, ra, rb);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dec(FA, FB, ra, rb, 0, false);
        }
        for (int t = 0; t < n_st; ++t) {
            wait_vmcnt<4 * (S - 2)>();  // this wave's loads of stage t + 1 have landed
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // its reads of stage t are in registers
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            issue(t + S);
            if constexpr (ACT) {
                uint4 na[2][2], nb[2][2];
                read_stage(t + 1, na, nb);  // past the last stage: a buffer of surplus bytes, never used
                __builtin_amdgcn_sched_barrier(0);
                dec(GA, GB, ra, rb, 0, true);
                q_step<DOM>(FA, FB, g0, g1, g2);  // chunk 0, words 0-1
                dec(FA, FB, ra, rb, 1, false);
                q_step<DOM>(GA, GB, g0, g1, g2);  // chunk 0, words 2-3
                dec(GA, GB, ra, rb, 1, true);
                q_step<DOM>(FA, FB, g0, g1, g2);  // chunk 1, words 0-1
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the next stage's registers
                dec(FA, FB, na, nb, 0, false);  // (the next stage's first step)
                q_step<DOM>(GA, GB, g0, g1, g2);  // chunk 1, words 2-3
#pragma unroll
                for (int k = 0; k < 2; ++k)
#pragma unroll
                    for (int c = 0; c < 2; ++c) { ra[k][c] = na[k][c]; rb[k][c] = nb[k][c]; }
            }
        }
    };
    if (!any) kloop(std::false_type{});
    else kloop(std::true_type{});
    wait_vmcnt<0>();  // the tail's surplus loads
    if (!any) return;  // no barrier follows
    const f32x16v z = {};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (!need[p]) continue;
        const int rb = strip_blk(rs + (p >> 1)), cb = 4 * J4 + 2 * (w & 1) + (p & 1);
        // (missing-free: the m products are 0, as in the single-block kernel's RM = CM = false loop)
        pair_epilogue<DOM, f32x16v, true, KC>(sh.info, sh.cst, 32 * (rs + (p >> 1)), 32 * (cs + (p & 1)), rb == cb, i,
                                              h, g0[p], z, z, z, g1[p], z, g2[p], z, ld_wind, n_org, rsq_thr, n_org,
                                              own_lo, own_hi, n_snp, l2_acc, l2d_acc, ws_acc);
    }
}

// ---- routed single-block items, compacted (order kept) ----
// With super-item routing, the single-block kernel runs only the items no super-item kernel takes.  Listing them
// apart (instead of every item returning at once when routed) sizes its launches — the round launches, the K-split
// tail — by the work it really has: missing-free data leaves it none, where round launches of all-routed items were
// thousands of empty launches.  Three passes over 1024-item chunks: per-chunk counts, their exclusive scan (one
// workgroup; meta_out = the total), the scatter.
constexpr int COMPACT_CHUNK = 256;  // (256-thread workgroups: see PLAN_WG)
__device__ __forceinline__ bool keep_item(const int4* items, int t, const uint8_t* blk_miss, int route_shift, int nblk) {
    const int4 it = items[t];
    return !routed_item(blk_miss, route_shift, it.x, it.y, nblk) ||
           (it.z == 2 && !routed_item(blk_miss, route_shift, it.x, it.y + 1, nblk));
}

__global__ void __launch_bounds__(COMPACT_CHUNK) compact_count_kernel(const int4* __restrict__ items, int n_items,
                                                             const uint8_t* __restrict__ blk_miss, int route_shift,
                                                             int nblk, int* __restrict__ chunk_counts) {
    const int t = blockIdx.x * COMPACT_CHUNK + threadIdx.x;
    const int keep = t < n_items && keep_item(items, t, blk_miss, route_shift, nblk);
    const int n = __syncthreads_count(keep);
    if (threadIdx.x == 0) chunk_counts[blockIdx.x] = n;
}

__global__ void __launch_bounds__(COMPACT_CHUNK) compact_scatter_kernel(const int4* __restrict__ items, int n_items,
                                                               const uint8_t* __restrict__ blk_miss, int route_shift,
                                                               int nblk, const int* __restrict__ chunk_offsets,
                                                               int4* __restrict__ out) {
    __shared__ int wave_base[COMPACT_CHUNK / 64];
    const int t = blockIdx.x * COMPACT_CHUNK + threadIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool keep = t < n_items && keep_item(items, t, blk_miss, route_shift, nblk);
    const unsigned long long ballot = __ballot(keep);
    const int before = __popcll(ballot & ((1ull << lane) - 1ull));
    if (lane == 0) wave_base[wv] = __popcll(ballot);
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan of the wave counts
        int run = 0;
        for (int k = 0; k < COMPACT_CHUNK / 64; ++k) {
            const int c = wave_base[k];
            wave_base[k] = run;
            run += c;
        }
    }
    __syncthreads();
    if (keep) out[chunk_offsets[blockIdx.x] + wave_base[wv] + before] = items[t];
}

// Matrix-core work the band kernels issued (32x32 block products over the whole K range), counted per work item
// exactly as each kernel decides it: kind 2 fp4 single-block items (mfmas_v: 1 + cm + rm + rm cm + dom (2 + rm +
// cm), the transposed products skipped on diagonal blocks; items the 2 x 2 kernel takes skipped when `routed`),
// kind 1 int8 items (4 + dom (2 + 2 !diag)), kind 0 fp32 items of it.z column blocks (1 + dom (2 - diag) each);
// and, when items2 != nullptr, every needed block pair of the 2 x 2 super-items (f4_step: no diagonal skip).
// rm / cm = blk_miss of the row / column block.  out[0] += products.
__global__ void issued_products_kernel(const int4* __restrict__ items, int n_items, const int4* __restrict__ items2,
                                       int n_items2, const int2* __restrict__ rows, const uint8_t* __restrict__ blk_miss,
                                       int nblk, int kind, int dom, int routed, int route_shift,
                                       unsigned long long* __restrict__ out) {
    // routed bit 0: single items the routing sends to a super-item kernel are not counted here (an uncompacted
    // list); bit 1: super-items count only when routed to their kernel
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long n = 0;
    if (t < n_items) {
        const int4 it = items[t];
        const bool diag = it.x == it.y;
        if (kind == 2) {  // (it.z == 2: additive-only column-block pairs, one product set per column block)
            for (int c = 0; c < it.z; ++c) {
                const int J = it.y + c;
                if ((routed & 1) && routed_item(blk_miss, route_shift, it.x, J, nblk)) continue;
                const int rm = blk_miss[it.x] != 0, cm = blk_miss[J] != 0, nd = it.x != J;
                n += 1 + cm + rm * nd + rm * cm + (dom ? 1 + nd + rm + cm * nd : 0);
            }
        } else if (kind == 1) {
            n = 4 + (dom ? (diag ? 2 : 4) : 0);
        } else {
            for (int b = 0; b < it.z; ++b) n += 1 + (dom ? (it.y + b == it.x ? 1 : 2) : 0);
        }
    } else if (items2 != nullptr && t < n_items + n_items2 && route_shift == 2) {
        // quad super-items (missing-free): a wave with any needed block pair issues all four pairs' products
        const int4 it = items2[t - n_items];
        if (!(routed & 2) || q_routed(blk_miss, it.x, it.y, nblk)) {
            for (int w = 0; w < 4; ++w) {
                bool any = false;
                for (int p = 0; p < 4; ++p) {
                    const int rb = 4 * it.x + 2 * (w >> 1) + (p >> 1), cb = 4 * it.y + 2 * (w & 1) + (p & 1);
                    any |= rb < nblk && cb < nblk && cb - rb >= rows[rb].x && cb - rb <= rows[rb].y;
                }
                n += any ? 4 * (dom ? 3 : 1) : 0;
            }
        }
    } else if (items2 != nullptr && t < n_items + n_items2) {
        const int4 it = items2[t - n_items];
        if (!((routed & 2) && !t2_routed(blk_miss, it.x, it.y, nblk))) {
            for (int w = 0; w < 4; ++w) {
                const int rb = 2 * it.x + (w >> 1), cb = 2 * it.y + (w & 1);
                if (rb >= nblk || cb >= nblk || cb - rb < rows[rb].x || cb - rb > rows[rb].y) continue;
                const int rm = blk_miss[rb] != 0, cm = blk_miss[cb] != 0;
                n += 1 + cm + rm + rm * cm + (dom ? 2 + rm + cm : 0);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) n += __shfl_down(n, o, 64);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(out, n);
}


// super-item rows: per row super-block I2 (row blocks 2 I2, 2 I2 + 1) the super-column offsets [d0, d1] covering both
// blocks' needed columns; meta[0] = max d1 + 1, meta[2] = diagonal super-items (plan_count / scan / emit then run on
// these rows as on the single-block ones)
// (shift 1: 2 x 2 super-items of the 2 x 2 kernel; shift 2: 4 x 4 super-items of the quad kernel)
__global__ void plan_rows2_kernel(const int2* __restrict__ rows, int nblk, int shift, int2* __restrict__ rows2,
                                  int* __restrict__ meta) {
    const int F = 1 << shift;
    const int I2 = blockIdx.x * blockDim.x + threadIdx.x, nblk2 = (nblk + F - 1) >> shift;
    if (I2 >= nblk2) return;
    int lo = INT_MAX, hi = -1;
    for (int b = F * I2; b < min(nblk, F * I2 + F); ++b) {
        const int2 r = rows[b];
        if (r.x <= r.y) { lo = min(lo, b + r.x); hi = max(hi, b + r.y); }
    }
    const int2 r2 = hi >= 0 ? make_int2((lo >> shift) - I2, (hi >> shift) - I2) : make_int2(1, 0);
    rows2[I2] = r2;
    if (r2.x <= r2.y) {
        atomicMax(&meta[0], r2.y + 1);
        if (r2.x == 0) atomicAdd(&meta[2], 1);
    }
}

// The quad kernel's super-items in tile order: row groups of QG_R super-rows, and within one the items by diagonal
// offset d, then super-row — so a run of 32 consecutive items (one XCD's share of a round launch of 256 workgroups:
// xcd_slot gives XCD x the run [32 x, 32 x + 32)) is 8 offsets of the same 4 super-rows where the band is full, and the
// 32 workgroups an XCD holds at once share 4 row and 11 column strips (4 x 4 super-strips) through its L2; in the
// 16 x 16-tile order a run straddled tile rows (2 x 16: 19 strips).  No padding: a null item would hold a wave slot of
// its round (32-item groups padded at the band edge: C5 -7.5 %).  Counted and emitted per (row group, block of QG_C
// offsets), in that order.
constexpr int QG_R = 4, QG_C = 8;
__device__ __forceinline__ int qg_n_c(const int* meta2) { return (meta2[0] + QG_C - 1) / QG_C; }
__global__ void plan_qcount_kernel(const int2* __restrict__ rows2, int nblk2, const int* __restrict__ meta2,
                                   int* __restrict__ counts) {
    const int n_r = (nblk2 + QG_R - 1) / QG_R, n_c = qg_n_c(meta2);
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n_r * n_c; k += gridDim.x * blockDim.x) {
        const int R = k / n_c, C = k % n_c;
        int n = 0;
        for (int I = R * QG_R; I < min(nblk2, R * QG_R + QG_R); ++I)
            n += max(0, min(rows2[I].y, C * QG_C + QG_C - 1) - max(rows2[I].x, C * QG_C) + 1);
        counts[k] = n;
    }
}
// one workgroup: exclusive scan of the group counts in place; meta2[1] = total items
__global__ void __launch_bounds__(PLAN_WG) plan_qscan_kernel(int* __restrict__ counts, int nblk2, int* __restrict__ meta2) {
    __shared__ int part[PLAN_WG];
    const int total = chunked_scan_excl<false>(counts, (nblk2 + QG_R - 1) / QG_R * qg_n_c(meta2), 0, part);
    if (threadIdx.x == 0) meta2[1] = total;
}
__global__ void plan_qemit_kernel(const int2* __restrict__ rows2, int nblk2, const int* __restrict__ meta2,
                                  const int* __restrict__ offsets, int4* __restrict__ items) {
    const int n_r = (nblk2 + QG_R - 1) / QG_R, n_c = qg_n_c(meta2);
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n_r * n_c; k += gridDim.x * blockDim.x) {
        const int R = k / n_c, C = k % n_c;
        int o = offsets[k];
        const int i_hi = min(nblk2, R * QG_R + QG_R);
        for (int d = C * QG_C; d < C * QG_C + QG_C; ++d)
            for (int I = R * QG_R; I < i_hi; ++I)
                if (rows2[I].x <= d && d <= rows2[I].y) items[o++] = make_int4(I, I + d, 1, 0);
    }
}

// K-split for small launches (a rank's shard of one chromosome: ~3 300 items for 2 048 wave slots leave the
// second round of items 60 % full).  Unit u = item * P + piece runs K chunks [piece n_it / P, (piece + 1) n_it / P)
// (even-aligned) and stores its 8 Gram tiles (32 KiB) to gram + u * 8192; band_f4_epi_kernel adds the P partial
// tiles of each item in piece order — integers below 2^24 (N < 2^19), so the fp32 sums are exact and equal to the
// single-pass Gram — and runs the usual epilogue.
template <bool DOM>
__global__ void __launch_bounds__(64, 2) band_f4_part_kernel(const uint32_t* __restrict__ geno, int pitch_words,
                                                           int n_it, const SnpConst* __restrict__ cst,
                                                           const int4* __restrict__ items,
                                                           const double* __restrict__ pos, const int* __restrict__ Lw,
                                                           const int* __restrict__ Rw,
                                                           const uint8_t* __restrict__ sflags, int n_snp, int P,
                                                           float* __restrict__ gram,
                                                           const uint8_t* __restrict__ blk_miss, int route_shift) {
    __shared__ BandI8Lds sh;
    __shared__ float tr[32 * 33];
    const int u = xcd_slot(blockIdx.x, gridDim.x), item = u / P, piece = u % P;
    const int4 it = items[item];
    // blk_miss: a super-item kernel runs the missing-free super-items (band_f4_epi_kernel skips the same items)
    if (blk_miss != nullptr && routed_item(blk_miss, route_shift, it.x, it.y, (n_snp + 31) >> 5)) return;
    const int t_lo = (int)(((long long)piece * n_it / P) & ~1LL);
    const int t_hi = piece == P - 1 ? n_it : (int)(((long long)(piece + 1) * n_it / P) & ~1LL);
    float* part = gram + (size_t)u * 8192;
#define NLDSC_BODY(DIAG_)                                                                                             \
    band_f4_body<DOM, 1, DIAG_, 0, false, true>(sh, it, geno, pitch_words, n_it, cst, pos, Lw, Rw, sflags, n_snp,     \
                                                0.0, 0.0, 0.0, 0, 0, nullptr, nullptr, nullptr, tr, t_lo, t_hi, part)
    if (it.y == it.x) NLDSC_BODY(true); else NLDSC_BODY(false);
#undef NLDSC_BODY
}

template <bool DOM, bool KC>
__global__ void __launch_bounds__(64, 2) band_f4_epi_kernel(const SnpConst* __restrict__ cst,
                                                          const int4* __restrict__ items,
                                                          const double* __restrict__ pos, const int* __restrict__ Lw,
                                                          const int* __restrict__ Rw,
                                                          const uint8_t* __restrict__ sflags, int n_snp,
                                                          double ld_wind, double n_org, double rsq_thr, int own_lo,
                                                          int own_hi, double* __restrict__ l2_acc,
                                                          double* __restrict__ l2d_acc, int* __restrict__ ws_acc,
                                                          const uint8_t* __restrict__ blk_rep, int P,
                                                          const float* __restrict__ gram,
                                                          const uint8_t* __restrict__ blk_miss, int route_shift,
                                                          const int* __restrict__ count = nullptr) {
    __shared__ BandI8Lds sh;
    __shared__ float tr[32 * 33];
    // count: the deferred rare-variant list of the single-block kernel (rep_items, P = 1): its first *count entries,
    // every one run (a pair item's block without a replayed SNP is listed too)
    if (count != nullptr && (int)blockIdx.x >= *count) return;
    const int4 it = items[blockIdx.x];
    if (count == nullptr && skip_item<KC>(blk_rep, it)) return;
    if (blk_miss != nullptr && routed_item(blk_miss, route_shift, it.x, it.y, (n_snp + 31) >> 5)) return;
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const int I = it.x, J = it.y;
    const bool diag = I == J;
    for (int s = lane; s < 64; s += 64) {
        const int g = s < 32 ? I * 32 + s : J * 32 + (s & 31);
        SnpSlot si;
        si.g = g;
        if (g < n_snp) {
            si.pos = pos[g]; si.L = Lw[g]; si.R = Rw[g]; si.fl = sflags[g];
        } else {
            si.pos = 0.0; si.L = -1; si.R = -2; si.fl = 0;
        }
        sh.info[s] = si;
        sh.cst[s] = cst[g];
    }
    f32x16v g8[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) g8[t] = f32x16v{};
    const float* src = gram + (size_t)blockIdx.x * P * 8192 + lane * 16;
    for (int p = 0; p < P; ++p)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const float4* q = reinterpret_cast<const float4*>(src + (size_t)p * 8192 + t * 1024);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 v = q[k];
                g8[t][4 * k] += v.x; g8[t][4 * k + 1] += v.y; g8[t][4 * k + 2] += v.z; g8[t][4 * k + 3] += v.w;
            }
        }
    __syncthreads();
    if (diag) {  // m.x(a, b) = x.m(b, a)
#pragma unroll
        for (int r = 0; r < 16; ++r) tr[((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + i] = g8[1][r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) g8[2][r] = tr[i * 33 + (r & 3) + 8 * (r >> 2) + 4 * h];
    }
    pair_epilogue<DOM, f32x16v, true, KC>(sh.info, sh.cst, 0, 32, diag, i, h, g8[0], g8[1], g8[2], g8[3], g8[4], g8[5],
                                          g8[6], g8[7], ld_wind, n_org, rsq_thr, n_org, own_lo, own_hi, n_snp, l2_acc,
                                          l2d_acc, ws_acc);
}

// ------------------------------------------------------------------------------------------
// 4. finalize
// ------------------------------------------------------------------------------------------
__global__ void finalize_kernel(const int* __restrict__ Lw, const double* __restrict__ l2_acc,
                                const double* __restrict__ l2d_acc, const int* __restrict__ ws_acc, int n_snp,
                                int own_lo, int own_hi, int dom, double* __restrict__ l2, double* __restrict__ l2d,
                                int* __restrict__ ws3) {
    const int g = own_lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= own_hi) return;
    const double qnan = __builtin_nan("");
    if (Lw[g] >= 0) {  // computed SNP (ldscalc.h:49-54)
        const int nanf = ws_acc[3 * (size_t)n_snp + g];
        const long long a = reinterpret_cast<const long long*>(l2_acc)[g];
        const long long d = reinterpret_cast<const long long*>(l2d_acc)[g];
        l2[g] = (nanf & 1) ? qnan : 1.0 + (double)a / ACC_SCALE;
        l2d[g] = dom && !(nanf & 2) ? (double)d / ACC_SCALE : qnan;
        ws3[g] = ws_acc[g];
        ws3[(size_t)n_snp + g] = dom ? ws_acc[(size_t)n_snp + g] : -1;
        ws3[2 * (size_t)n_snp + g] = dom ? ws_acc[2 * (size_t)n_snp + g] : -1;
    } else {  // not computed: initial values of ldscalc.h:16-21
        l2[g] = qnan; l2d[g] = qnan;
        ws3[g] = -1; ws3[(size_t)n_snp + g] = -1; ws3[2 * (size_t)n_snp + g] = -1;
    }
}

// finalize_kernel for host-result runs (nldsc_engine_run): the owned slice goes straight to host memory (pinned,
// device-mapped: the caller's arrays when they are nldsc_host_alloc buffers, else the engine's landing buffer) — no
// device copy, no DMA after the band — and each workgroup's sums of positive WSA / WSD to wsum (host memory, plain
// stores: a same-address atomic per workgroup serialised to ~30 us at 80 000 SNPs).
constexpr int FINALIZE_OUT_WG = 256;
__global__ void __launch_bounds__(FINALIZE_OUT_WG) finalize_out_kernel(
    const int* __restrict__ Lw, const double* __restrict__ l2_acc, const double* __restrict__ l2d_acc,
    const int* __restrict__ ws_acc, const double* __restrict__ maf_in, const double* __restrict__ rstd_in, int n_snp,
    int own_lo, int own_hi, int dom, double* __restrict__ l2, double* __restrict__ l2d, double* __restrict__ maf,
    double* __restrict__ rstd, int* __restrict__ wsa, int* __restrict__ wsd, int* __restrict__ wsde,
    unsigned long long* __restrict__ wsum) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, g = own_lo + c;
    unsigned long long sa = 0, sd = 0;
    if (g < own_hi) {
        const double qnan = __builtin_nan("");
        double a2 = qnan, d2 = qnan;
        int a = -1, d = -1, x = -1;
        if (Lw[g] >= 0) {  // computed SNP (ldscalc.h:49-54)
            const int nanf = ws_acc[3 * (size_t)n_snp + g];
            const long long la = reinterpret_cast<const long long*>(l2_acc)[g];
            const long long ld = reinterpret_cast<const long long*>(l2d_acc)[g];
            a2 = (nanf & 1) ? qnan : 1.0 + (double)la / ACC_SCALE;
            d2 = dom && !(nanf & 2) ? (double)ld / ACC_SCALE : qnan;
            a = ws_acc[g];
            d = dom ? ws_acc[(size_t)n_snp + g] : -1;
            x = dom ? ws_acc[2 * (size_t)n_snp + g] : -1;
        }
        l2[c] = a2;
        l2d[c] = d2;
        maf[c] = maf_in[g];
        rstd[c] = rstd_in[g];
        wsa[c] = a;
        wsd[c] = d;
        wsde[c] = x;
        sa = a > 0 ? (unsigned long long)a : 0ull;
        sd = d > 0 ? (unsigned long long)d : 0ull;
    }
    __shared__ unsigned long long part[2][FINALIZE_OUT_WG / 64];
    for (int o = 32; o > 0; o >>= 1) {
        sa += __shfl_down(sa, o, 64);
        sd += __shfl_down(sd, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = sa;
        part[1][threadIdx.x >> 6] = sd;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long ta = 0, td = 0;
        for (int w = 0; w < FINALIZE_OUT_WG / 64; ++w) { ta += part[0][w]; td += part[1][w]; }
        wsum[2 * blockIdx.x] = ta;
        wsum[2 * blockIdx.x + 1] = td;
    }
}

// Owned slice of the score table for the multi-GPU gather (nldsc_engine_run_device): row k of `table` = l2, l2d,
// maf, rstd, WSA, WSD, WSDE (doubles), column c = SNP own_lo + c, NaN past the slice; and the metric's pair counts
// (positive window sizes) summed per workgroup, one 64-bit atomic per workgroup and counter.
__global__ void __launch_bounds__(256) pack_table_kernel(const double* __restrict__ l2, const double* __restrict__ l2d,
                                                         const double* __restrict__ maf,
                                                         const double* __restrict__ rstd,
                                                         const int* __restrict__ ws3, int n_snp, int own_lo,
                                                         int own_hi, int width, double* __restrict__ table,
                                                         unsigned long long* __restrict__ sums) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int g = own_lo + c;
    unsigned long long sa = 0, sd = 0;
    if (c < width) {
        const double qnan = __builtin_nan("");
        const bool in = g < own_hi;
        const int a = in ? ws3[g] : -1, d = in ? ws3[(size_t)n_snp + g] : -1, x = in ? ws3[2 * (size_t)n_snp + g] : -1;
        sa = a > 0 ? (unsigned long long)a : 0ull;
        sd = d > 0 ? (unsigned long long)d : 0ull;
        if (table == nullptr) goto sum;  // (host-result runs: the pair counts only)
        table[c] = in ? l2[g] : qnan;
        table[(size_t)width + c] = in ? l2d[g] : qnan;
        table[2 * (size_t)width + c] = in ? maf[g] : qnan;
        table[3 * (size_t)width + c] = in ? rstd[g] : qnan;
        table[4 * (size_t)width + c] = in ? (double)a : qnan;
        table[5 * (size_t)width + c] = in ? (double)d : qnan;
        table[6 * (size_t)width + c] = in ? (double)x : qnan;
    }
sum:
    // one 64-bit atomic pair per workgroup (per wave, the 1 250 waves of an 80 000-SNP table serialised on the two
    // counters: 31 us of the kernel)
    __shared__ unsigned long long wsum[2][4];
    for (int o = 32; o > 0; o >>= 1) {
        sa += __shfl_down(sa, o, 64);
        sd += __shfl_down(sd, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        wsum[0][threadIdx.x >> 6] = sa;
        wsum[1][threadIdx.x >> 6] = sd;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        sa = wsum[0][0] + wsum[0][1] + wsum[0][2] + wsum[0][3];
        sd = wsum[1][0] + wsum[1][1] + wsum[1][2] + wsum[1][3];
        if (sa) atomicAdd(&sums[0], sa);
        if (sd) atomicAdd(&sums[1], sd);
    }
}

// ------------------------------------------------------------------------------------------
// synthetic .bed generator (benchmarks / full-size tests)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ float u01(uint32_t v) { return ((v >> 8) + 0.5f) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float2 normal2(uint64_t key) {
    const uint64_t r = splitmix64(key);
    const float u1 = u01((uint32_t)r), u2 = u01((uint32_t)(r >> 32));
    const float rad = sqrtf(-2.0f * __logf(u1));
    float s, c;
    __sincosf(6.283185307f * u2, &s, &c);
    return make_float2(rad * c, rad * s);
}

// Thread = one byte column (4 samples, 8 haplotypes); loops over SNPs carrying the AR(1) latent
// state.  PLINK-correct packing: sample 4b+k in bits 2k..2k+1; padding bits zero.
__global__ void __launch_bounds__(256) synth_bed_kernel(uint8_t* __restrict__ rows, int n_snp, int n_org, int nb,
                                                        const float* __restrict__ thr, float rho, float missing,
                                                        uint64_t seed) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const float sq = sqrtf(1.0f - rho * rho);
    float z[8];
    const uint64_t base = splitmix64(seed) ^ ((uint64_t)b << 20);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float2 n = normal2(base + 0xFFFFFull * 4 + k);
        z[2 * k] = n.x; z[2 * k + 1] = n.y;
    }
    for (int j = 0; j < n_snp; ++j) {
        const uint64_t key = splitmix64(base ^ ((uint64_t)j * 0x9E3779B97F4A7C15ull));
        if (j > 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float2 n = normal2(key + k);
                z[2 * k] = rho * z[2 * k] + sq * n.x;
                z[2 * k + 1] = rho * z[2 * k + 1] + sq * n.y;
            }
        }
        const float tj = thr[j];
        const uint64_t mk = splitmix64(key + 17);
        uint32_t byte = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (4 * b + k >= n_org) break;
            const int g = (z[2 * k] < tj) + (z[2 * k + 1] < tj);
            const bool miss = ((mk >> (16 * k)) & 0xFFFF) < (uint32_t)(missing * 65536.0f);
            const uint32_t code = miss ? 1u : (g == 0 ? 0u : g == 1 ? 2u : 3u);
            byte |= code << (2 * k);
        }
        rows[(size_t)j * nb + b] = (uint8_t)byte;
    }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
int load_parts(int n_snp, int row_bytes) {
    // parts per block: about 64 k workgroups over the whole image, at least 8 chunks each
    const int n_ch = row_bytes >> 5, nblk_img = (n_snp + 31) / 32;
    // (~64 k workgroups: the load of a C3 image 2.72 ms at 16 k, 2.53-2.57 ms from 48 k to 96 k, 2.65 ms at 128 k —
    // short uniform workgroups, so the count sets how much of the last wave of them idles:
    // profiles/r05_ab_load_parts.json)
    constexpr int target = 65536;
    return std::max(1, std::min(std::max(n_ch / 8, 1), (target + nblk_img - 1) / nblk_img));
}

hipError_t launch_load_slice(const uint8_t* src, int nb, int row0, int n_rows, int n_snp, uint8_t* img, int row_bytes,
                             bool orient, uint8_t* flip, uint8_t* last, uint32_t keep_compat, uint32_t keep_strict,
                             uint32_t* miss_flags, int* lcounts, hipStream_t st) {
    if (n_rows <= 0) return hipSuccess;
    if (row0 % 32 != 0 || row0 + n_rows > n_snp) return hipErrorInvalidValue;
    hipLaunchKernelGGL(load_orient_kernel, dim3((n_rows + 3) / 4), dim3(256), 0, st, src, nb, row0, n_rows,
                       orient ? 1 : 0, flip, miss_flags, lcounts);
    const int nblk = (n_rows + 31) / 32, P = load_parts(n_snp, row_bytes);
    hipLaunchKernelGGL(load_tiled_kernel, dim3(nblk * P), dim3(256), 0, st, src, nb, row0, n_rows, n_snp, img,
                       row_bytes, P, flip, last, keep_compat, keep_strict, miss_flags, lcounts);
    return hipGetLastError();
}

hipError_t launch_load_flags(const uint32_t* miss_flags, int n_snp, uint8_t* row_miss, hipStream_t st) {
    if (n_snp <= 0) return hipSuccess;
    hipLaunchKernelGGL(load_flags_kernel, dim3((n_snp + 255) / 256), dim3(256), 0, st, miss_flags, n_snp, row_miss);
    return hipGetLastError();
}

hipError_t launch_tail_counts(uint8_t* img, const uint8_t* last, int n_snp, int nb, int row_bytes, uint32_t tail_keep,
                              uint32_t pad, const int* lcounts, int P, int* counts3, hipStream_t st) {
    if (n_snp <= 0) return hipSuccess;
    hipLaunchKernelGGL(tail_counts_kernel, dim3((n_snp + 255) / 256), dim3(256), 0, st, img, last, n_snp, nb, row_bytes,
                       tail_keep, pad, lcounts, P, counts3);
    return hipGetLastError();
}

hipError_t launch_snp_stats(const int* parts, int P, int* counts, int* zero, const uint8_t* flip, const double* pos,
                            int n_snp, int n_snp_pad, int n_org, double maf_thr, double std_thr, float2* lut,
                            SnpConst* cst, uint8_t* sflags, double* maf_out, double* rstd_out, hipStream_t st,
                            double* l2_acc, double* l2d_acc, int* ws_acc, uint8_t* blk_rep) {
    const int blocks = (n_snp_pad + 255) / 256;
    hipLaunchKernelGGL(snp_stats_kernel, dim3(blocks), dim3(256), 0, st, parts, P, counts, zero, flip, pos, n_snp,
                       n_snp_pad, n_org, maf_thr, std_thr, lut, cst, sflags, maf_out, rstd_out, l2_acc, l2d_acc, ws_acc,
                       blk_rep);
    return hipGetLastError();
}

hipError_t launch_replay_flags(const int* counts, const uint8_t* flip, const uint8_t* sflags, int n_snp,
                              uint8_t* blk_rep, hipStream_t st, bool zeroed) {
    if (n_snp <= 0) return hipSuccess;
    hipError_t e = zeroed ? hipSuccess : hipMemsetAsync(blk_rep, 0, (size_t)(n_snp + 31) / 32, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(replay_flags_kernel, dim3((n_snp + 255) / 256), dim3(256), 0, st, counts, flip, sflags, n_snp,
                       blk_rep);
    return hipGetLastError();
}

hipError_t launch_reference_residuals(const uint8_t* img, int row_bytes, int n_org, bool strict, const int* counts,
                                     const uint8_t* flip, int n_snp, double std_thr, SnpConst* cst, float2* lut,
                                     uint8_t* sflags, double* rstd_out, hipStream_t st) {
    if (n_snp <= 0) return hipSuccess;
    hipLaunchKernelGGL(reference_residual_kernel, dim3(n_snp), dim3(64), 0, st, img, row_bytes, n_org, (int)strict,
                       counts, flip, n_snp, std_thr, cst, lut, sflags, rstd_out);
    return hipGetLastError();
}

hipError_t launch_pair_range(uint8_t* sflags, int n_snp, int pair_lo, int pair_hi, hipStream_t st) {
    if (n_snp <= 0) return hipSuccess;
    hipLaunchKernelGGL(pair_range_kernel, dim3((n_snp + 255) / 256), dim3(256), 0, st, sflags, n_snp, pair_lo, pair_hi);
    return hipGetLastError();
}

hipError_t launch_export_acc(const double* l2_acc, const double* l2d_acc, const int* ws_acc, int n_snp, int lo, int hi,
                             long long* out, hipStream_t st) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(export_acc_kernel, dim3((hi - lo + 255) / 256), dim3(256), 0, st, l2_acc, l2d_acc, ws_acc, n_snp,
                       lo, hi, out);
    return hipGetLastError();
}

hipError_t launch_import_acc(double* l2_acc, double* l2d_acc, int* ws_acc, int n_snp, int lo, int n, const long long* in,
                             hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(import_acc_kernel, dim3((n + 255) / 256), dim3(256), 0, st, l2_acc, l2d_acc, ws_acc, n_snp, lo, n,
                       in);
    return hipGetLastError();
}

hipError_t launch_block_missing_rows(const uint8_t* row_miss, int n_snp, int order, uint8_t* blk_miss,
                                     hipStream_t st) {
    const int nblk = (n_snp + 31) / 32;
    if (nblk <= 0) return hipSuccess;
    hipLaunchKernelGGL(block_missing_rows_kernel, dim3((nblk + 255) / 256), dim3(256), 0, st, row_miss, n_snp, order,
                       blk_miss);
    return hipGetLastError();
}

hipError_t launch_left_pointers(const int* A, const uint8_t* sflags, const double* pos, int n, int* L, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(left_pointer_kernel, dim3((n + 255) / 256), dim3(256), 0, st, A, sflags, pos, n, L);
    return hipGetLastError();
}

hipError_t launch_plan_edges(const double* pos, int n, double w, int* A, int* E, int* meta, hipStream_t st) {
    if (n <= 0) return hipMemsetAsync(meta, 0, 4 * sizeof(int), st);
    hipLaunchKernelGGL(plan_edges_kernel, dim3((n + 255) / 256), dim3(256), 0, st, pos, n, w, A, E, meta);
    return hipGetLastError();
}

hipError_t launch_plan(int n, int own_lo, int own_hi, const int* A, int* E, int* R, int2* rows, int* counts, int* meta,
                       hipStream_t st, bool pair, int4* small_items) {
    const int nblk = (n + 31) / 32;
    if (n <= 0 || own_hi <= own_lo) return hipSuccess;  // (meta zeroed by launch_plan_edges)
    if (small_items != nullptr) {
        if (n > PLAN_SMALL_N) return hipErrorInvalidValue;
        hipLaunchKernelGGL(plan_small_kernel, dim3(1), dim3(PLAN_SMALL_WG), 0, st, A, E, n, own_lo, own_hi, R, rows,
                           counts, meta, small_items, pair ? 1 : 0);
        return hipGetLastError();
    }
    const int ntile = (n + PLAN_WG - 1) / PLAN_WG;  // (E holds n + ntile ints: the tiles' maxima after the n edges)
    hipLaunchKernelGGL(plan_tile_max_kernel, dim3(ntile), dim3(PLAN_WG), 0, st, E, n, E + n);
    hipLaunchKernelGGL(plan_tile_scan_kernel, dim3(1), dim3(PLAN_WG), 0, st, E + n, ntile);
    hipLaunchKernelGGL(plan_right_kernel, dim3(ntile), dim3(PLAN_WG), 0, st, E, n, E + n, R);
    hipLaunchKernelGGL(plan_rows_kernel, dim3((nblk + 255) / 256), dim3(256), 0, st, E, A, n, nblk, own_lo, own_hi,
                       rows, meta);
    hipLaunchKernelGGL(plan_count_kernel, dim3(256), dim3(256), 0, st, rows, nblk, meta, counts, pair ? 1 : 0);
    hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(PLAN_WG), 0, st, counts, nblk, meta);
    return hipGetLastError();
}

hipError_t launch_plan_emit(int n, const int2* rows, const int* meta, const int* offsets, int4* items, hipStream_t st,
                            bool pair) {
    const int nblk = (n + 31) / 32;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(plan_emit_kernel, dim3(256), dim3(256), 0, st, rows, nblk, meta, offsets, items, pair ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_band(bool dom, int wps, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                       const float2* lut, const int4* items, const double* pos, const int* Lw, const int* Rw,
                       const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                       int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc, hipStream_t st) {
    if (n_items <= 0) return hipSuccess;
#define NLDSC_BAND(DOM_, WPS_)                                                                                       \
    hipLaunchKernelGGL((band_kernel<DOM_, WPS_>), dim3(n_items), dim3(64), 0, st, geno, pitch_words, n_it, lut, items, \
                       pos, Lw, Rw, sflags, n_snp, ld_wind, n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc)
    if (dom) { if (wps == 2) NLDSC_BAND(true, 2); else NLDSC_BAND(true, 1); }
    else { if (wps == 2) NLDSC_BAND(false, 2); else NLDSC_BAND(false, 1); }
#undef NLDSC_BAND
    return hipGetLastError();
}

hipError_t launch_band_i8(bool dom, int max_nc, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                          const SnpConst* cst, const int4* items, const double* pos, const int* Lw, const int* Rw,
                          const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                          int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc, bool xcd, const uint8_t* blk_rep,
                          int which, hipStream_t st) {
    if (n_items <= 0) return hipSuccess;
    if (max_nc != 1) return hipErrorInvalidValue;  // single block-pair items
#define NLDSC_BAND(DOM_, KC_)                                                                                       \
    hipLaunchKernelGGL((band_i8_kernel<DOM_, KC_>), dim3(n_items), dim3(64), 0, st, geno, pitch_words, n_it, cst,    \
                       items, pos, Lw, Rw, sflags, n_snp, ld_wind, n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, \
                       ws_acc, xcd ? 1 : 0, blk_rep)
    if (which & 1) { if (dom) NLDSC_BAND(true, false); else NLDSC_BAND(false, false); }
    if (blk_rep && (which & 2)) { if (dom) NLDSC_BAND(true, true); else NLDSC_BAND(false, true); }
#undef NLDSC_BAND
    return hipGetLastError();
}

int plan_super_counts(int n, int shift) {
    const int nblk2 = ((n + 31) / 32 + (1 << shift) - 1) >> shift;
    if (shift == 2) return ((nblk2 + QG_R - 1) / QG_R) * ((nblk2 + QG_C - 1) / QG_C + 1);
    const int n_t2 = (nblk2 + PLAN_R - 1) / PLAN_R;
    return n_t2 * n_t2;
}

hipError_t launch_plan_super(int n, const int2* rows, int2* rows2, int* counts2, int* meta2, int shift, hipStream_t st) {
    const int nblk = (n + 31) / 32, nblk2 = (nblk + (1 << shift) - 1) >> shift;
    hipError_t e = hipMemsetAsync(meta2, 0, 4 * sizeof(int), st);
    if (e != hipSuccess || n <= 0) return e;
    hipLaunchKernelGGL(plan_rows2_kernel, dim3((nblk2 + 255) / 256), dim3(256), 0, st, rows, nblk, shift, rows2, meta2);
    if (shift == 2) {  // the quad kernel's 32-item groups
        hipLaunchKernelGGL(plan_qcount_kernel, dim3(256), dim3(256), 0, st, rows2, nblk2, meta2, counts2);
        hipLaunchKernelGGL(plan_qscan_kernel, dim3(1), dim3(PLAN_WG), 0, st, counts2, nblk2, meta2);
    } else {
        hipLaunchKernelGGL(plan_count_kernel, dim3(256), dim3(256), 0, st, rows2, nblk2, meta2, counts2, 0);
        hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(PLAN_WG), 0, st, counts2, nblk2, meta2);
    }
    return hipGetLastError();
}


hipError_t launch_plan_emit_super(int n, const int2* rows2, const int* meta2, const int* offsets2, int4* items2,
                                  int shift, hipStream_t st) {
    const int nblk2 = ((n + 31) / 32 + (1 << shift) - 1) >> shift;
    if (n <= 0) return hipSuccess;
    if (shift == 2)
        hipLaunchKernelGGL(plan_qemit_kernel, dim3(256), dim3(256), 0, st, rows2, nblk2, meta2, offsets2, items2);
    else
        hipLaunchKernelGGL(plan_emit_kernel, dim3(256), dim3(256), 0, st, rows2, nblk2, meta2, offsets2, items2, 0);
    return hipGetLastError();
}

hipError_t launch_band_f4_t2(bool dom, int n_items2, const uint32_t* geno, int pitch_words, int n_it,
                             const SnpConst* cst, const int4* items2, const int2* rows, int nblk, const double* pos,
                             const int* Lw, const int* Rw, const uint8_t* sflags, int n_snp, double ld_wind,
                             double n_org, double rsq_thr, int own_lo, int own_hi, double* l2_acc, double* l2d_acc,
                             int* ws_acc, bool xcd, const uint8_t* blk_rep, const uint8_t* blk_miss, int which,
                             hipStream_t st) {
    if (n_items2 <= 0) return hipSuccess;
    if (n_it > F4_SEG_CHUNKS || n_it < 2 || (n_it & 1)) return hipErrorInvalidValue;
#define NLDSC_BAND(DOM_, KC_)                                                                                       \
    hipLaunchKernelGGL((band_f4_t2_kernel<DOM_, T2_STAGES, KC_>), dim3(n_items2), dim3(256), 0, st, geno,           \
                       pitch_words, n_it, cst, items2, rows, nblk, pos, Lw, Rw, sflags, n_snp, ld_wind, n_org,      \
                       rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc, xcd ? 1 : 0, blk_rep, blk_miss)
    if (which & 1) { if (dom) NLDSC_BAND(true, false); else NLDSC_BAND(false, false); }
    if (blk_rep && (which & 2)) { if (dom) NLDSC_BAND(true, true); else NLDSC_BAND(false, true); }
#undef NLDSC_BAND
    return hipGetLastError();
}

hipError_t launch_band_f4_q(bool dom, int n_items4, const uint32_t* geno, int pitch_words, int n_it,
                            const SnpConst* cst, const int4* items4, const int2* rows, int nblk, const double* pos,
                            const int* Lw, const int* Rw, const uint8_t* sflags, int n_snp, double ld_wind,
                            double n_org, double rsq_thr, int own_lo, int own_hi, double* l2_acc, double* l2d_acc,
                            int* ws_acc, bool xcd, const uint8_t* blk_rep, const uint8_t* blk_miss, int which,
                            hipStream_t st, int round_items) {
    if (n_items4 <= 0) return hipSuccess;
    if (n_it > F4_SEG_CHUNKS || n_it < 2 || (n_it & 1) || blk_miss == nullptr) return hipErrorInvalidValue;
    // round_items > 0: launches of that many super-items (one workgroup per CU each), so the workgroups on an XCD
    // start together and stream their shared strips at nearby K offsets (not the KC launch)
    int chunk = round_items > 0 ? round_items : n_items4;
#define NLDSC_BAND(DOM_, KC_)                                                                                       \
    for (int o = 0; o < n_items4; o += chunk)                                                                        \
    hipLaunchKernelGGL((band_f4_q_kernel<DOM_, Q_STAGES, KC_>), dim3(std::min(chunk, n_items4 - o)), dim3(256),     \
                       0, st, geno, pitch_words, n_it, cst, items4 + o, rows, nblk, pos, Lw, Rw, sflags, n_snp,     \
                       ld_wind, n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc, xcd ? 1 : 0, blk_rep, blk_miss)
    if (which & 1) {
        if (dom) NLDSC_BAND(true, false);
        else NLDSC_BAND(false, false);
    }
    chunk = n_items4;
    if (blk_rep && (which & 2)) {
        if (dom) NLDSC_BAND(true, true);
        else NLDSC_BAND(false, true);
    }
#undef NLDSC_BAND
    return hipGetLastError();
}

hipError_t launch_band_f4_split(bool dom, int P, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                                const SnpConst* cst, const int4* items, const double* pos, const int* Lw, const int* Rw,
                                const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr,
                                int own_lo, int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc,
                                const uint8_t* blk_rep, float* gram, int which, hipStream_t st,
                                const uint8_t* blk_miss, int route_shift) {
    if (n_items <= 0) return hipSuccess;
    if (n_it > F4_SEG_CHUNKS || P < 1 || 2 * P > n_it) return hipErrorInvalidValue;
    const dim3 grid_p((unsigned)n_items * (unsigned)P);
    if (!(which & 1)) goto kc;  // the partial tiles of every item come from the main launch
    if (dom) hipLaunchKernelGGL((band_f4_part_kernel<true>), grid_p, dim3(64), 0, st, geno, pitch_words, n_it, cst,
                                items, pos, Lw, Rw, sflags, n_snp, P, gram, blk_miss, route_shift);
    else hipLaunchKernelGGL((band_f4_part_kernel<false>), grid_p, dim3(64), 0, st, geno, pitch_words, n_it, cst,
                            items, pos, Lw, Rw, sflags, n_snp, P, gram, blk_miss, route_shift);
#define NLDSC_EPI(DOM_, KC_)                                                                                        \
    hipLaunchKernelGGL((band_f4_epi_kernel<DOM_, KC_>), dim3(n_items), dim3(64), 0, st, cst, items, pos, Lw, Rw,    \
                       sflags, n_snp, ld_wind, n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc, blk_rep, P, gram, \
                       blk_miss, route_shift, nullptr)
    if (dom) NLDSC_EPI(true, false); else NLDSC_EPI(false, false);
kc:
    if (blk_rep && (which & 2)) { if (dom) NLDSC_EPI(true, true); else NLDSC_EPI(false, true); }
#undef NLDSC_EPI
    return hipGetLastError();
}

hipError_t launch_band_f4_deferred_epi(bool dom, int max_items, const SnpConst* cst, const int4* rep_items,
                                      const int* rep_count, const float* rep_gram, const double* pos, const int* Lw,
                                      const int* Rw, const uint8_t* sflags, int n_snp, double ld_wind, double n_org,
                                      double rsq_thr, int own_lo, int own_hi, double* l2_acc, double* l2d_acc,
                                      int* ws_acc, const uint8_t* blk_rep, hipStream_t st) {
    if (max_items <= 0) return hipSuccess;
    if (dom)
        hipLaunchKernelGGL((band_f4_epi_kernel<true, true>), dim3(max_items), dim3(64), 0, st, cst, rep_items, pos, Lw,
                           Rw, sflags, n_snp, ld_wind, n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc, blk_rep,
                           1, rep_gram, nullptr, 1, rep_count);
    else
        hipLaunchKernelGGL((band_f4_epi_kernel<false, true>), dim3(max_items), dim3(64), 0, st, cst, rep_items, pos,
                           Lw, Rw, sflags, n_snp, ld_wind, n_org, rsq_thr, own_lo, own_hi, l2_acc, l2d_acc, ws_acc,
                           blk_rep, 1, rep_gram, nullptr, 1, rep_count);
    return hipGetLastError();
}

hipError_t launch_band_f4(bool dom, int max_nc, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                          const SnpConst* cst, const int4* items, const double* pos, const int* Lw, const int* Rw,
                          const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                          int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc, bool xcd, const uint8_t* blk_rep,
                          int which, hipStream_t st, const uint8_t* blk_miss, int round_items, int route_shift,
                          float* rep_gram, int4* rep_items, int* rep_count) {
    if (n_items <= 0) return hipSuccess;
    // single block-pair items, or (additive-only, unsegmented rows) column-block pairs
    if (max_nc != 1 && !(max_nc == 2 && !dom && n_it <= F4_SEG_CHUNKS)) return hipErrorInvalidValue;
    if (blk_miss != nullptr && n_it > F4_SEG_CHUNKS) return hipErrorInvalidValue;  // routing: unsegmented rows only
    // round_items > 0: the items go in launches of that many (one round of the wave slots each), see ld_engine.cpp;
    // not the KC launch (items holding a replayed rare variant: few, the others return at once)
    int chunk = round_items > 0 ? round_items : n_items;
#define NLDSC_BAND_NC(DOM_, WPS_, SEG_, KC_, NCX_)                                                                  \
    for (int o = 0; o < n_items; o += chunk)                                                                      \
    hipLaunchKernelGGL((band_f4_kernel<DOM_, WPS_, SEG_, KC_, NCX_>), dim3(std::min(chunk, n_items - o)), dim3(64), 0, \
                       st, geno, pitch_words,                                                                         \
                       n_it, cst, items + o, pos, Lw, Rw, sflags, n_snp, ld_wind, n_org, rsq_thr, own_lo, own_hi,       \
                       l2_acc, l2d_acc, ws_acc, xcd ? 1 : 0, blk_rep, blk_miss, route_shift, SEG_ ? nullptr : rep_gram, \
                       rep_items, rep_count)
#define NLDSC_BAND(DOM_, WPS_, SEG_, KC_) NLDSC_BAND_NC(DOM_, WPS_, SEG_, KC_, 1)
#define NLDSC_PICK(KC_)                                                                                              \
    if (n_it > F4_SEG_CHUNKS) { if (dom) NLDSC_BAND(true, 1, F4_SEG_CHUNKS, KC_); else NLDSC_BAND(false, 2, F4_SEG_CHUNKS, KC_); } \
    else if (dom) NLDSC_BAND(true, 2, 0, KC_);                                                                       \
    else if (max_nc == 2) NLDSC_BAND_NC(false, 2, 0, KC_, 2);                                                        \
    else NLDSC_BAND(false, 2, 0, KC_)
    // segmented kernel: the add+dom variant needs more than 256 registers (2 waves / SIMD would spill)
    if (which & 1) { NLDSC_PICK(false); }
    chunk = n_items;
    // (with rep_gram the KC items ran their K loops in the main launch: launch_band_f4_deferred_epi after the replay)
    if (blk_rep && (which & 2) && (rep_gram == nullptr || n_it > F4_SEG_CHUNKS)) { NLDSC_PICK(true); }
#undef NLDSC_PICK
#undef NLDSC_BAND
#undef NLDSC_BAND_NC
    return hipGetLastError();
}

hipError_t launch_finalize(const int* Lw, const double* l2_acc, const double* l2d_acc, const int* ws_acc, int n_snp,
                           int own_lo, int own_hi, bool dom, double* l2, double* l2d, int* ws3, hipStream_t st) {
    const int n = own_hi - own_lo;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(finalize_kernel, dim3((n + 255) / 256), dim3(256), 0, st, Lw, l2_acc, l2d_acc, ws_acc, n_snp,
                       own_lo, own_hi, dom ? 1 : 0, l2, l2d, ws3);
    return hipGetLastError();
}

int finalize_out_blocks(int n_own) { return (n_own + FINALIZE_OUT_WG - 1) / FINALIZE_OUT_WG; }

hipError_t launch_finalize_out(const int* Lw, const double* l2_acc, const double* l2d_acc, const int* ws_acc,
                               const double* maf_in, const double* rstd_in, int n_snp, int own_lo, int own_hi, bool dom,
                               double* l2, double* l2d, double* maf, double* rstd, int* wsa, int* wsd, int* wsde,
                               unsigned long long* wsum, hipStream_t st) {
    const int n = own_hi - own_lo;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(finalize_out_kernel, dim3(finalize_out_blocks(n)), dim3(FINALIZE_OUT_WG), 0, st, Lw, l2_acc,
                       l2d_acc, ws_acc, maf_in, rstd_in, n_snp, own_lo, own_hi, dom ? 1 : 0, l2, l2d, maf, rstd, wsa,
                       wsd, wsde, wsum);
    return hipGetLastError();
}

hipError_t launch_issued_products(const int4* items, int n_items, const int4* items2, int n_items2, const int2* rows,
                                 const uint8_t* blk_miss, int nblk, int kind, bool dom, int routed, int route_shift,
                                 unsigned long long* out, hipStream_t st) {
    const int n = n_items + (items2 != nullptr ? n_items2 : 0);
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(issued_products_kernel, dim3((n + 255) / 256), dim3(256), 0, st, items, n_items, items2,
                       n_items2, rows, blk_miss, nblk, kind, dom ? 1 : 0, routed, route_shift, out);
    return hipGetLastError();
}

hipError_t launch_compact_items(const int4* items, int n_items, const uint8_t* blk_miss, int route_shift, int nblk,
                                int* chunk_counts, int* total, int4* out, hipStream_t st) {
    const int n_chunks = (n_items + COMPACT_CHUNK - 1) / COMPACT_CHUNK;
    if (n_items <= 0) return hipMemsetAsync(total, 0, sizeof(int), st);
    hipLaunchKernelGGL(compact_count_kernel, dim3(n_chunks), dim3(COMPACT_CHUNK), 0, st, items, n_items, blk_miss,
                       route_shift, nblk, chunk_counts);
    hipLaunchKernelGGL(scan_counts_kernel, dim3(1), dim3(PLAN_WG), 0, st, chunk_counts, n_chunks, total);
    hipLaunchKernelGGL(compact_scatter_kernel, dim3(n_chunks), dim3(COMPACT_CHUNK), 0, st, items, n_items, blk_miss,
                       route_shift, nblk, chunk_counts, out);
    return hipGetLastError();
}

hipError_t launch_pack_table(const double* l2, const double* l2d, const double* maf, const double* rstd, const int* ws3,
                             int n_snp, int own_lo, int own_hi, int width, double* table, unsigned long long* sums,
                             hipStream_t st) {
    if (width <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_table_kernel, dim3((width + 255) / 256), dim3(256), 0, st, l2, l2d, maf, rstd, ws3, n_snp,
                       own_lo, own_hi, width, table, sums);
    return hipGetLastError();
}

hipError_t launch_synth_bed(uint8_t* rows, int n_snp, int n_org, int nb, const float* thr, float rho, float missing,
                            uint64_t seed, hipStream_t st) {
    hipLaunchKernelGGL(synth_bed_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, rows, n_snp, n_org, nb, thr, rho,
                       missing, seed);
    return hipGetLastError();
}

}  // namespace nldsc
