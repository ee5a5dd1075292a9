// Internal launcher declarations for ld_kernels.hip (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nldsc {

// Per-SNP constants of the exact-integer path: with x = additive count, h = [genotype >= 1],
// o = [observed] (all 0 for missing calls and padding), the reference's standardised vectors are
// A = (x - mu o) / sa + ka and R = (2h - beta x - c o) / s + kr over the individuals.  ka = kr = 0 except for
// rare variants whose vectors are replayed in the reference's fp32 arithmetic (reference_residual_kernel:
// the fp32 mean of a nearly constant vector does not centre it, and missing calls take the value of the
// fp32 mean, not 0).
// X, H, Ob: sums of x, h, o over the SNP's sample slots (the fp4 path's Gram uses the missing
// indicator m = 1 - o over all slots, so o-products are recovered as X - x.m, Ob_i + Ob_j - K + m.m, ...);
// SA, SR: sums of (x - mu o) / sa and (2h - beta x - c o) / s over the individuals (for the ka / kr terms).
// isa, is: 1 / sa and 1 / s (0 where sa / s are 0), so the pair epilogue multiplies instead of dividing.
struct SnpConst {
    double mu, sa, c, beta, s;
    double X, H, Ob;
    double ka, kr, SA, SR;
    double isa, is;
};

// A load, one slice of whole 32-SNP blocks at a time (row0 % 32 == 0; only the image's last slice may end mid-block):
// rows [row0, row0 + n_rows) of a .bed image (row r of nb bytes at src + r * nb, any alignment) into the resident
// layout (block-interleaved, ld_kernels.hip tile_off) — pitch padding 0x55, the last block's rows past n_snp all 0x55 —
// each stored in the orientation flip[j] chosen from its head (orient: rows with more hom-A2 than hom-A1 calls there
// stored 00 <-> 11 swapped; !orient: as in the file), its stored last byte saved to last[j], its missing calls
// among the individual slots of the reference's (bit 0) / PLINK's (bit 1) sample order ORed into miss_flags[j]
// (keep_*: the last byte's individual bit pairs per order), and the genotype counts of its stored bytes [0, nb - 1)
// (hom A1, het, hom A2) added over the load_parts(n_snp, row_bytes) parts of the row into lcounts[3 j + k] (cleared by
// the slice's orientation pass; integer atomics).  After every slice: launch_load_flags -> row_miss.
int load_parts(int n_snp, int row_bytes);
hipError_t launch_load_slice(const uint8_t* src, int nb, int row0, int n_rows, int n_snp, uint8_t* img, int row_bytes,
                             bool orient, uint8_t* flip, uint8_t* last, uint32_t keep_compat, uint32_t keep_strict,
                             uint32_t* miss_flags, int* lcounts, hipStream_t st);
hipError_t launch_load_flags(const uint32_t* miss_flags, int n_snp, uint8_t* row_miss, hipStream_t st);
// per run: set each row's non-individual slots (last byte outside tail_keep, pitch padding) to `pad` (0x55 missing,
// or 0x00 for the fp4 kernel) and its genotype counts — the load's lcounts (P parts; the loaders keep 1) plus the last byte's individual
// pairs — to counts3[3 j + k] (one thread per row; no pass over the rows)
hipError_t launch_tail_counts(uint8_t* img, const uint8_t* last, int n_snp, int nb, int row_bytes, uint32_t tail_keep,
                              uint32_t pad, const int* lcounts, int P, int* counts3, hipStream_t st);
// parts / P: genotype counts in P parts ([P][n_snp][3]: launch_tail_counts gives one), summed into counts[4 j + k]
// (n_snp * 4 ints; the rare-variant kernels read them); zero: one int cleared on the way (nullptr: none).  flip:
// per-SNP stored-orientation flags (nullptr: none flipped)
hipError_t launch_snp_stats(const int* parts, int P, int* counts, int* zero, const uint8_t* flip, const double* pos,
                            int n_snp, int n_snp_pad, int n_org, double maf_thr, double std_thr, float2* lut,
                            SnpConst* cst, uint8_t* sflags, double* maf_out, double* rstd_out, hipStream_t st,
                            double* l2_acc = nullptr, double* l2d_acc = nullptr, int* ws_acc = nullptr,
                            uint8_t* blk_rep = nullptr);
// (l2_acc, l2d_acc, ws_acc [4][n_snp] and blk_rep, when given: zeroed for the band and the replay flags)
// SNPs with at most REF_RESIDUAL_MIN_CLASS calls in one genotype class (rare variants: residual nearly degenerate):
// residual std, residual-pass flag bit 2, exact constants and fp32 table of the reference's fp32 residual,
// replayed in its arithmetic (ld_kernels.hip reference_residual_kernel)
constexpr int REF_RESIDUAL_MIN_CLASS = 16;
// blk_rep[block] = 1 for blocks holding such SNPs (cheap; first), then the replay itself (long, few waves).
// Concurrency invariant: the replay runs on the plan stream beside the main stream's band launches and rewrites
// sflags[j] bit 1 (residual pass; a plain byte read-modify-write) and cst[j] / lut[j] of replayed SNPs j only.
// Until ev_replay, main-stream readers may touch sflags bits 0 and 2 (left_pointer_kernel, the host flag copy)
// and never bit 1, cst or lut of a replayed SNP: the non-KC band launches (single-block, 2 x 2, quad, K-split
// epilogue) drop the items / super-items that hold a block with blk_rep set (skip_item); the K-split partial
// kernel runs every item but uses flag bit 2 alone (the missing-block test; band_f4_body with PART); the KC
// launches, the K-split epilogue of KC items and finalize wait on ev_replay.
hipError_t launch_replay_flags(const int* counts, const uint8_t* flip, const uint8_t* sflags, int n_snp,
                              uint8_t* blk_rep, hipStream_t st, bool zeroed = false);  // zeroed: by launch_snp_stats
hipError_t launch_reference_residuals(const uint8_t* img, int row_bytes, int n_org, bool strict, const int* counts,
                                     const uint8_t* flip, int n_snp, double std_thr, SnpConst* cst, float2* lut,
                                     uint8_t* sflags, double* rstd_out, hipStream_t st);
// halo pairs once across ranks: clear flag bit 3 (the pair's lower SNP: computed here) outside [pair_lo, pair_hi);
// the accumulator rows of SNPs [lo, hi) out to a [6][hi - lo] int64 block, and such a block added into SNPs [lo, lo + n)
hipError_t launch_pair_range(uint8_t* sflags, int n_snp, int pair_lo, int pair_hi, hipStream_t st);
hipError_t launch_export_acc(const double* l2_acc, const double* l2d_acc, const int* ws_acc, int n_snp, int lo, int hi,
                             long long* out, hipStream_t st);
hipError_t launch_import_acc(double* l2_acc, double* l2d_acc, int* ws_acc, int n_snp, int lo, int n, const long long* in,
                             hipStream_t st);
// per run (fp4): blk_miss[b] from row_miss (order 0 reference, 1 PLINK) — equal to the sflags-bit-2 predicate of the
// band kernels, known without the count kernel
hipError_t launch_block_missing_rows(const uint8_t* row_miss, int n_snp, int order, uint8_t* blk_miss,
                                     hipStream_t st);
// exact left pointers L from the all-pass replay's A and the device MAF flags (sorted positions)
hipError_t launch_left_pointers(const int* A, const uint8_t* sflags, const double* pos, int n, int* L, hipStream_t st);
// the schedule's window edges of sorted positions (all-pass left pointers A, window ends E) and meta[0..3] = 0
hipError_t launch_plan_edges(const double* pos, int n, double w, int* A, int* E, int* meta, hipStream_t st);
// band schedule on the GPU for non-negative sorted positions, from launch_plan_edges' A and E (capacity
// n + ceil(n / 256): the right-pointer scan's tile maxima follow the n edges),
// right pointers R, per-row-block offset ranges `rows` (nblk), tile item offsets `counts` (capacity
// ceil(nblk/16) * ceil(nblk/16)); meta[1] = items, meta[2] = diagonal items (read after the stream
// reaches it), then plan_emit writes the items (16 row blocks x 16 offsets tile order).  pair: items of two
// neighbouring column blocks (I, J, 2) (the additive-only fp4 kernel's 32 x 64 tiles; a row's odd last one (I, J, 1))
// small_items (n <= PLAN_SMALL_N): the whole plan in one workgroup, the items emitted too (capacity: every block pair
// I <= J, plan_small_items); launch_plan_emit is then not called
constexpr int PLAN_SMALL_N = 32768;
inline size_t plan_small_items(int n) {
    const size_t nblk = (size_t)(n + 31) / 32;
    return nblk * (nblk + 1) / 2;
}
hipError_t launch_plan(int n, int own_lo, int own_hi, const int* A, int* E, int* R, int2* rows, int* counts, int* meta,
                       hipStream_t st, bool pair = false, int4* small_items = nullptr);
hipError_t launch_plan_emit(int n, const int2* rows, const int* meta, const int* offsets, int4* items, hipStream_t st,
                            bool pair = false);
hipError_t launch_band(bool dom, int wps, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                       const float2* lut, const int4* items, const double* pos, const int* Lw, const int* Rw,
                       const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                       int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc, hipStream_t st);
hipError_t launch_band_i8(bool dom, int max_nc, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                          const SnpConst* cst, const int4* items, const double* pos, const int* Lw, const int* Rw,
                          const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                          int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc, bool xcd, const uint8_t* blk_rep,
                          int which, hipStream_t st);
// K-loop chunks (128 samples each) per fp32 accumulation segment of the fp4 path: rows longer than this
// (N > 2^19) run the segmented kernel, which folds the fp32 Gram into int32 after every segment
constexpr int F4_SEG_CHUNKS = 4096;
// exact path on fp4 MFMAs (N < 2^27), items (I, J0, 1, 0) (max_nc 1), or for additive-only unsegmented rows also
// (I, J0, 2, 0) column-block pairs (max_nc 2; blk_miss then drops routed column blocks per block).  blk_rep (or nullptr): per 32-SNP
// block, 1 if a SNP carries replayed fp32 vectors (ka / kr != 0): its items run in a second launch (the exact
// kernels' KC instantiation).  which: 1 the main launch (items of other blocks), 2 the KC launch, 3 both
hipError_t launch_band_f4(bool dom, int max_nc, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                          const SnpConst* cst, const int4* items, const double* pos, const int* Lw, const int* Rw,
                          const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr, int own_lo,
                          int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc, bool xcd, const uint8_t* blk_rep,
                          int which, hipStream_t st, const uint8_t* blk_miss = nullptr, int round_items = 0,
                          int route_shift = 1, float* rep_gram = nullptr, int4* rep_items = nullptr, int* rep_count = nullptr);
// rep_gram (unsegmented rows): the items holding a replayed rare variant run their K loops in the main launch and store
// each block pair's exact Gram tiles (rep_gram slot = atomicAdd(rep_count), 8192 floats; rep_items[slot] = the block
// pair); after the replay, launch_band_f4_deferred_epi runs their epilogues (max_items >= the slots used) in place of
// the KC launch
hipError_t launch_band_f4_deferred_epi(bool dom, int max_items, const SnpConst* cst, const int4* rep_items,
                                      const int* rep_count, const float* rep_gram, const double* pos, const int* Lw,
                                      const int* Rw, const uint8_t* sflags, int n_snp, double ld_wind, double n_org,
                                      double rsq_thr, int own_lo, int own_hi, double* l2_acc, double* l2d_acc,
                                      int* ws_acc, const uint8_t* blk_rep, hipStream_t st);
// the same with the K loop split in P pieces (small launches: better filled wave slots): partial Gram tiles to
// `gram` (n_items * P * 8192 floats), then an epilogue kernel (unsegmented rows, n_it <= F4_SEG_CHUNKS)
hipError_t launch_band_f4_split(bool dom, int P, int n_items, const uint32_t* geno, int pitch_words, int n_it,
                                const SnpConst* cst, const int4* items, const double* pos, const int* Lw, const int* Rw,
                                const uint8_t* sflags, int n_snp, double ld_wind, double n_org, double rsq_thr,
                                int own_lo, int own_hi, double* l2_acc, double* l2d_acc, int* ws_acc,
                                const uint8_t* blk_rep, float* gram, int which, hipStream_t st,
                                const uint8_t* blk_miss = nullptr, int route_shift = 1);
// 2 x 2 block-pair workgroups (unsegmented rows, gpu plan): super-items (I2, J2, 1, 0) over row / column
// super-blocks of two 32-SNP blocks, planned from the single-block rows (launch_plan) by launch_plan_super (meta2
// as meta; counts2 capacity ceil(nblk2/16)^2) and launch_plan_emit_super; the kernel reads `rows` (nblk) to skip the
// block pairs the single-block plan does not hold
constexpr int T2_STAGES = 4;  // LDS ring stages (2 chunks each) of band_f4_t2_kernel
// shift 1: 2 x 2 super-items (16 x 16 tiles); shift 2: the quad kernel's 4 x 4 super-items in row groups of 4
// super-rows, each group's items by diagonal offset then super-row (plan_qemit_kernel), NOT padded: a group's item
// count varies and the list is dense (null padding to 32-item groups held wave slots: r05_ab_quad_groups.json), so
// nothing may assume 32-aligned groups; counts2 capacity: plan_super_counts(n, shift)
int plan_super_counts(int n, int shift);
hipError_t launch_plan_super(int n, const int2* rows, int2* rows2, int* counts2, int* meta2, int shift, hipStream_t st);
hipError_t launch_plan_emit_super(int n, const int2* rows2, const int* meta2, const int* offsets2, int4* items2,
                                  int shift, hipStream_t st);
hipError_t launch_band_f4_t2(bool dom, int n_items2, const uint32_t* geno, int pitch_words, int n_it,
                             const SnpConst* cst, const int4* items2, const int2* rows, int nblk, const double* pos,
                             const int* Lw, const int* Rw, const uint8_t* sflags, int n_snp, double ld_wind,
                             double n_org, double rsq_thr, int own_lo, int own_hi, double* l2_acc, double* l2d_acc,
                             int* ws_acc, bool xcd, const uint8_t* blk_rep, const uint8_t* blk_miss, int which,
                             hipStream_t st);
// 4 x 4 block-pair workgroups (the quad kernel: one wave per SIMD, 64 x 64 SNP tiles) for the missing-free 4 x 4
// super-items (I4, J4, 1, 0) of launch_plan_super(shift 2); blk_miss required (route_shift 2 for the other kernels).
constexpr int Q_STAGES = 4;
hipError_t launch_band_f4_q(bool dom, int n_items4, const uint32_t* geno, int pitch_words, int n_it,
                            const SnpConst* cst, const int4* items4, const int2* rows, int nblk, const double* pos,
                            const int* Lw, const int* Rw, const uint8_t* sflags, int n_snp, double ld_wind,
                            double n_org, double rsq_thr, int own_lo, int own_hi, double* l2_acc, double* l2d_acc,
                            int* ws_acc, bool xcd, const uint8_t* blk_rep, const uint8_t* blk_miss, int which,
                            hipStream_t st, int round_items = 0);
// blk_miss[b] = block b holds a missing call (launch_block_missing_rows).  Passed to the fp4 kernels (unsegmented rows)
// it routes the super-items: missing-free ones to a super-item kernel (operand-feed bound at 3 products per K step,
// where sharing the strips pays), the block pairs of the others to the single-block kernel (MFMA bound at 8 products)
hipError_t launch_finalize(const int* Lw, const double* l2_acc, const double* l2d_acc, const int* ws_acc, int n_snp,
                           int own_lo, int own_hi, bool dom, double* l2, double* l2d, int* ws3, hipStream_t st);
// Results of a host-result run straight to host memory (zero-copy: device-accessible pinned pointers, index 0 = SNP
// own_lo): the finalized l2, l2d, the MAF and RSTD (from maf_in / rstd_in), WSA, WSD, WSDE of the owned slice; and per
// workgroup of finalize_out_blocks(n) the sums of positive WSA / WSD to wsum[2 b], wsum[2 b + 1] (the metric's pair
// counts; the host adds them)
int finalize_out_blocks(int n_own);
hipError_t launch_finalize_out(const int* Lw, const double* l2_acc, const double* l2d_acc, const int* ws_acc,
                               const double* maf_in, const double* rstd_in, int n_snp, int own_lo, int own_hi, bool dom,
                               double* l2, double* l2d, double* maf, double* rstd, int* wsa, int* wsd, int* wsde,
                               unsigned long long* wsum, hipStream_t st);
// the matrix-core products the band kernels issued (one per 32x32 block product over all K), counted per work item
// as each kernel decides them: kind 2 fp4 single-block items (+ the super-items when items2 != nullptr; `routed`
// bit 0: skip single items routed to a super-item kernel, bit 1: count only routed super-items), 1 int8, 0 fp32
// (items of it.z column blocks);
// blk_miss may be nullptr for kinds 0 and 1.  out[0] += the count (zeroed before)
hipError_t launch_issued_products(const int4* items, int n_items, const int4* items2, int n_items2, const int2* rows,
                                 const uint8_t* blk_miss, int nblk, int kind, bool dom, int routed, int route_shift,
                                 unsigned long long* out, hipStream_t st);
// the single-block items no super-item kernel takes (routing of 2^route_shift-block super-items), in their order, to
// `out`; *total = their count (device); chunk_counts: ceil(n_items / 256) ints of scratch
hipError_t launch_compact_items(const int4* items, int n_items, const uint8_t* blk_miss, int route_shift, int nblk,
                                int* chunk_counts, int* total, int4* out, hipStream_t st);
// the owned slice [own_lo, own_hi) of the finalized results as a [7][width] fp64 table in device memory (columns
// past the slice NaN) + sums[0] += sum of positive WSA, sums[1] += sum of positive WSD over the slice (zeroed before)
hipError_t launch_pack_table(const double* l2, const double* l2d, const double* maf, const double* rstd, const int* ws3,
                             int n_snp, int own_lo, int own_hi, int width, double* table, unsigned long long* sums,
                             hipStream_t st);
hipError_t launch_synth_bed(uint8_t* rows, int n_snp, int n_org, int nb, const float* thr, float rho, float missing,
                            uint64_t seed, hipStream_t st);

}  // namespace nldsc
