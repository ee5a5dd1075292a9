/*
 * nldsc_ld.h — C ABI of the MI355X-native LD-score engine (libnldsc_amd.so).
 *
 * Drop-in boundary for bayarpark/nldsc's `_ldscore` extension:
 *   - nldsc_ld_params  replaces  struct LDScoreParams   nldsc/ldscore/_ldscore/data.h:33-65
 *   - nldsc_ld_result  replaces  struct LDScoreResult   nldsc/ldscore/_ldscore/data.h:21-31
 *   - nldsc_ld_calculate replaces LDScoreResult calculate(LDScoreParams&)
 *                                                       nldsc/ldscore/_ldscore/ldscalc.h:8
 *     as bound by m.def("calculate", &calculate)        nldsc/ldscore/_ldscore/ldscore.cpp:53
 * The pybind11 module `_ldscore` (nldsc_amd/csrc/ldscore_py.cpp) wraps exactly
 * these entry points with the reference's Python signatures.
 *
 * The engine entry points below are the lower-level API used for device-resident
 * inputs, repeated runs (benchmarks) and position sharding across GPUs.
 *
 * Plain C types only: pointers, sizes, ints and doubles.  All output arrays are
 * caller-allocated with n_snp elements.  Every function returns NLDSC_OK (0) or
 * a negative NLDSC_E_* code; when `err` is non-NULL a NUL-terminated message is
 * written into it (at most errlen bytes).
 */
#ifndef NLDSC_LD_H
#define NLDSC_LD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NLDSC_OK 0
#define NLDSC_E_BAD_MAGIC (-1) /* "Invalid PLINK magic number..." (stream.h:88-102) -> ValueError */
#define NLDSC_E_IO (-2)        /* cannot open / read the .bed file */
#define NLDSC_E_SIZE (-3)      /* .bed shorter than 3 + n_snp * ceil(n_org / 4) bytes */
#define NLDSC_E_ARG (-4)       /* invalid argument (sizes, NULL pointers, ranges) */
#define NLDSC_E_HIP (-5)       /* HIP runtime error */
#define NLDSC_E_OOM (-6)       /* device or host allocation failed */
#define NLDSC_E_NODEV (-7)     /* no HIP device visible: there is no CPU fallback */

/* flags */
#define NLDSC_FLAG_STRICT_PLINK_ORDER 1u /* use PLINK sample order in the last .bed byte (reference
                                            keeps the high n_org%4 bit pairs, stream.h:55-66) */
#define NLDSC_FLAG_ADDITIVE_ONLY 2u      /* skip the dominance terms: l2d = NaN, l2d_ws = l2d_wse = -1 */
#define NLDSC_FLAG_EXACT_I8 4u           /* correlations from exact integer Gram products (int8 MFMA) */
#define NLDSC_FLAG_FP32 8u               /* correlations from fp32 standardised values (fp32 MFMA) */
#define NLDSC_FLAG_EXACT_F4 16u          /* exact integer Gram products on fp4 MFMAs (n_org < 2^27, segmented
                                            above 2^19; larger cohorts fall back to EXACT_I8) */
#define NLDSC_FLAG_EXACT_RARE 32u        /* rare variants (<= 16 calls in one genotype class): exact standardised
                                            vectors instead of the default, the reference's fp32 ones replayed
                                            step for step (encoder.h:124-133, tools.h:54-85) — its rounding is
                                            not small against a nearly constant vector: the fp32 mean does not
                                            centre it, and a residual without hom-A1 calls is exactly constant
                                            (std 0) but rounding noise in the reference, often above --std-thr */
/* None of EXACT_F4, EXACT_I8, FP32: the engine default, EXACT_F4 (engine option "band_mode" overrides it). */

typedef struct nldsc_ld_params {
    const char* bedfile;      /* LDScoreParams::bedfile   (data.h:34) */
    int32_t n_snp;            /* LDScoreParams::n_snp     (data.h:36) */
    int32_t n_org;            /* LDScoreParams::n_org     (data.h:37) */
    double ld_wind;           /* LDScoreParams::ld_wind   (data.h:39), same unit as positions */
    const double* positions;  /* LDScoreParams::positions (data.h:40), n_snp values; < 0 = unused */
    double maf;               /* LDScoreParams::maf       (data.h:42) */
    double std_thr;           /* LDScoreParams::std_thr   (data.h:43) */
    double rsq_thr;           /* LDScoreParams::rsq_thr   (data.h:44) */
    uint32_t flags;           /* NLDSC_FLAG_* */
    int32_t device;           /* HIP device ordinal; -1 = the calling thread's current device */
} nldsc_ld_params;

typedef struct nldsc_ld_result { /* LDScoreResult (data.h:21-31); n_snp elements each */
    double* l2;              /* additive LD score; NaN for unused / MAF-failed SNPs */
    double* l2d;             /* dominance LD score; NaN likewise */
    double* maf;             /* MAF of every decoded SNP; NaN for unused SNPs */
    double* residuals_std;   /* std of the dominance residual; NaN unless the SNP passed MAF */
    int32_t* l2_ws;          /* window size (additive), -1 when not computed */
    int32_t* l2d_ws;         /* neighbours with residual std > std_thr, -1 when not computed */
    int32_t* l2d_wse;        /* ... of which r2adj > rsq_thr, -1 when not computed */
} nldsc_ld_result;

/* One-shot call: read `p->bedfile`, compute on the GPU, fill `r`. */
int nldsc_ld_calculate(const nldsc_ld_params* p, nldsc_ld_result* r, char* err, size_t errlen);

/* Library / device information. */
const char* nldsc_version(void);
int nldsc_device_count(void);

/* ---- engine API ------------------------------------------------------------------------ */
typedef struct nldsc_engine nldsc_engine;

int nldsc_engine_create(int32_t device, nldsc_engine** out, char* err, size_t errlen);
void nldsc_engine_destroy(nldsc_engine* e);

/* Engine options (no reference counterpart: the schedule and kernel choice of this engine; every setting gives the
 * same results, which the GPU tests compare).  Read at each run (orient: at each load); NLDSC_E_ARG for an unknown
 * name or a value out of range.  Defaults in brackets.
 *   band_mode    default correlation path when a run's flags name none: 0 fp32, 1 exact int8, [2] exact fp4
 *   gpu_plan     [1] band schedule on the GPU for sorted non-negative positions; 0 the host replay always
 *   plan_fused   [1] that schedule in one launch (items included) for slices of <= 32768 SNPs; 0 the kernel chain
 *   orient       [1] store rows minor-homozygote-as-00 at load (the exact kernels' operands mostly zero)
 *   ksplit       [1] K-split small launches (a rank's shard of one chromosome)
 *   t2           super-item kernels for missing-free blocks: 0 none, 1 2x2 routed, 2 2x2 for all, [3] 4x4 quad
 *   band_rounds  [1] single-block fp4 band in launches of one round of wave slots; 0 one launch
 *   f4_nc2       [1] additive-only fp4 items of two column blocks; 0 single block pairs
 *   q_rounds     [1] quad super-items in launches of one workgroup per CU; 0 one launch
 *   defer_rep    [1] K loops of items holding a replayed rare variant in the main launch; 0 a later KC launch
 *   debug_timing [0] per-run stage timings on stderr */
int nldsc_engine_set_option(nldsc_engine* e, const char* name, int64_t value, char* err, size_t errlen);

/* Page-locked host memory mapped into every device's address space (hipHostMalloc), NULL on failure; free with
 * nldsc_host_free (which ignores pointers it did not hand out).  A host-result run whose seven result arrays (owned
 * slices) all lie in such buffers is written by the GPU directly — no landing buffer, no host copies — and positions
 * there are uploaded by DMA in place. */
void* nldsc_host_alloc(size_t bytes);
void nldsc_host_free(void* p);

/* Make a .bed image resident on the engine's device.  `bed` is the complete file content
 * (3 magic bytes + n_snp rows of ceil(n_org/4) bytes), in host memory (_host) or in device
 * memory of the engine's device (_device, e.g. a torch tensor's data pointer; copied).
 * The rows are stored at a 64-byte-aligned pitch (pitched copies; padding read as missing), the
 * layout every run reads in place. */
int nldsc_engine_load_bed_file(nldsc_engine* e, const char* path, int32_t n_snp, int32_t n_org,
                               char* err, size_t errlen);
int nldsc_engine_load_bed_host(nldsc_engine* e, const uint8_t* bed, size_t len, int32_t n_snp,
                               int32_t n_org, char* err, size_t errlen);
int nldsc_engine_load_bed_device(nldsc_engine* e, const void* bed, size_t len, int32_t n_snp,
                                 int32_t n_org, char* err, size_t errlen);

/* Compute LD scores for the SNPs with index in [own_begin, own_end) (position sharding:
 * each GPU owns a contiguous SNP range and recomputes the pairs it shares with its
 * neighbours' ranges, so no partial sums cross GPUs).  Entries of `r` outside the owned
 * range are left untouched.  p->bedfile is ignored (the loaded image is used).  `r`'s arrays
 * may be ordinary host memory or nldsc_host_alloc buffers (written by the GPU in place). */
int nldsc_engine_run(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end,
                     nldsc_ld_result* r, char* err, size_t errlen);

/* nldsc_engine_run with the owned slice of the result left in device memory (the multi-GPU gather of
 * SURVEY.md §8 e1 then runs device to device over RCCL, without a host round trip): `table_dev`, device memory
 * of the engine's device holding 7 * width doubles with width >= own_end - own_begin, receives row k =
 * l2, l2d, maf, residuals_std, l2_ws, l2d_ws, l2d_wse (LDScoreResult, data.h:21-31; window sizes as doubles),
 * column c = SNP own_begin + c, columns past the owned range NaN.  Returns once the table is written (the
 * engine stream is synchronised), so any stream may read it. */
int nldsc_engine_run_device(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end,
                            double* table_dev, int32_t width, char* err, size_t errlen);

/* nldsc_engine_run_device in two calls, computing each pair that straddles two ranks' owned ranges once (multi-GPU
 * strong scaling; no reference counterpart: the reference is single-process, ldscalc.h:34-35).  The loaded slice
 * holds the owned SNPs [own_begin, own_end) and the right halo [own_end, n_snp) (one window, no left halo).
 * _split computes the pairs whose lower SNP is owned, accumulates the per-SNP sums of every SNP of the slice, and
 * writes the right halo's accumulators (exact fixed-point sums and counts) to `export_dev`: device memory of
 * 6 * export_cap int64 (row-major [6][export_n], export_n = n_snp - own_end <= export_cap), synchronised on return.
 * The caller sends that block to the rank owning those SNPs (whose slice starts at them) and passes the block
 * received from the left neighbour to _finish, which adds it to the first import_n owned SNPs (import_n <=
 * own_end - own_begin; 0 for the first rank), finalizes and writes `table_dev` as nldsc_engine_run_device does.  Counts,
 * MAF and residual std equal those of nldsc_engine_run_device with the left halo loaded; L2 / L2D to the last bits
 * (the exchanged sums are exact integers; each work item's fp64 partial sums follow the slice's block grid). */
int nldsc_engine_run_device_split(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end,
                                  double* table_dev, int32_t width, int64_t* export_dev, int32_t export_cap,
                                  int32_t* export_n, char* err, size_t errlen);
int nldsc_engine_run_device_finish(nldsc_engine* e, const int64_t* import_dev, int32_t import_n, char* err,
                                   size_t errlen);

/* Per-stage device timings (milliseconds, HIP events on the engine stream) of the last run:
 * [0] genotype count, [1] per-SNP statistics, [2] window replay + schedule (host time; overlaps [0]),
 * [3] band correlation kernel (all launches), [4] finalize, [5] total.
 * Also: algorithmic FLOPs (2N(1/2 sum WSA + sum WSD)), FLOPs issued to the matrix cores by the
 * band kernels (counted on the GPU per work item as each kernel decides them: the products of missing-free blocks
 * and the transposed products of diagonal blocks that are skipped are not counted; padded sample slots are), SNP
 * pairs (sum WSA) of the last run, and the band kernel's work-item count. */
int nldsc_engine_timings(const nldsc_engine* e, double* ms6, double* flop_alg, double* flop_issued,
                         double* pairs, int32_t* n_band_items);
/* Path of the last run: 2 = exact Gram on fp4 MFMAs, 1 = exact Gram on int8 MFMAs, 0 = fp32;
 * *ops_alg_i8 = algorithmic ops of the exact formulation, 2N (2 sum WSA + 2 sum WSD). */
int nldsc_engine_path(const nldsc_engine* e, int32_t* exact_i8, double* ops_alg_i8);
/* K-split factor of the last run's fp4 band kernel: the number of K pieces each work item was split into
 * (1 = single pass; > 1 for launches too small to fill the GPU, e.g. one rank's shard of a chromosome). */
int nldsc_engine_ksplit(const nldsc_engine* e);
/* Band launch rounds of the last run: the number of work items per launch of the single-block fp4 band kernel when
 * its items went in launches of one round of the GPU's wave slots each (so the items of a launch stay at nearby K
 * offsets and share their strips through L2), 0 when they went in one launch. */
int nldsc_engine_band_round_items(const nldsc_engine* e);
/* K-split factor of the last run's partial last round when its band went in round launches (1: not split). */
int nldsc_engine_band_tail_ksplit(const nldsc_engine* e);
/* Band kernel of the last run: NLDSC_BAND_F32 (fp32 MFMA GEMM), NLDSC_BAND_I8, NLDSC_BAND_F4 (one wave per
 * 32x32 block pair), NLDSC_BAND_F4_SEG (rows above 2^19 samples), NLDSC_BAND_F4_KSPLIT, NLDSC_BAND_F4_2X2
 * (4-wave workgroups over 2x2 block pairs sharing their strips through LDS), NLDSC_BAND_F4_ROUTED (missing-free
 * 2x2 super-items in the 2x2 workgroups, the rest in the single-block kernel), NLDSC_BAND_F4_QUAD (the default for
 * sorted non-negative positions: missing-free 4x4 super-items in the quad workgroups, the rest in the single-block
 * kernel).  All exact paths give bitwise the same results. */
#define NLDSC_BAND_F32 0
#define NLDSC_BAND_I8 1
#define NLDSC_BAND_F4 2
#define NLDSC_BAND_F4_SEG 3
#define NLDSC_BAND_F4_KSPLIT 4
#define NLDSC_BAND_F4_2X2 5
#define NLDSC_BAND_F4_ROUTED 6
#define NLDSC_BAND_F4_QUAD 7 /* option t2 = 3: missing-free 4x4 super-items in the quad workgroups (64x64 tiles per
                                wave), the rest in the single-block kernel */
int nldsc_engine_band_kernel(const nldsc_engine* e);
/* Where the last host-result run (nldsc_engine_run) wrote its owned slice: 1 straight into the caller's arrays (all
 * seven in nldsc_host_alloc buffers, zero copy), 0 through the engine's landing buffer and host copies, -1 no host
 * result written (device-table runs, empty owned ranges). */
int nldsc_engine_result_direct(const nldsc_engine* e);

/* Load SNP rows [snp_begin, snp_end) of a .bed file of n_snp_file SNPs as the engine's image
 * (snp_end - snp_begin SNPs; the run then takes the positions of that slice).  Position sharding
 * (SURVEY.md §8 e1): each GPU reads only its owned range plus the window halo around it.
 * Same magic / size checks and messages as nldsc_engine_load_bed_file. */
int nldsc_engine_load_bed_file_range(nldsc_engine* e, const char* path, int32_t n_snp_file, int32_t n_org,
                                     int32_t snp_begin, int32_t snp_end, char* err, size_t errlen);

/* Host-only plan of the band kernel (no GPU needed; the engine calls the same code):
 * replays the reference's sliding-window pointers (stream.h:131-155,182-197) from positions and
 * MAF-pass flags (flags[j] bit 0) into L/R (n_snp each; L = -1 for SNPs the reference does not
 * compute) and lists the work items (I, J0, nc, 0) covering every needed 32x32 block pair for the
 * owned range (max_nc 1 or 2; any other value is an argument error).  Returns the item count; when it
 * exceeds `cap` (or items == NULL) nothing is written to `items` and the count is returned; < 0 on bad
 * arguments. */
int nldsc_plan_band(const double* positions, const uint8_t* flags, int32_t n_snp, double ld_wind, int32_t own_begin,
                    int32_t own_end, int32_t max_nc, int32_t* L, int32_t* R, int32_t* items, int32_t cap);

/* The score table as the reference writes it (make_output + DataFrame.to_csv(sep="\t", index=False,
 * float_format="%.5f"), nldsc/ldscore/routine.py:94-101), without the header line: row i = prefix line i
 * (the caller's "CHR\tSNP\tBP" text, lines separated by '\n'), then L2, L2D [, MAF, WSA, WSD, WSDE,
 * RSTD when extra]; floats "%.5f", NaN as an empty field.  Host-only, no GPU.  Returns the bytes
 * written to `out`, or NLDSC_E_OOM when `cap` is too small, NLDSC_E_ARG on bad arguments. */
int64_t nldsc_format_scores(const char* prefix, int64_t prefix_len, int32_t n, const double* l2, const double* l2d,
                            const double* maf, const int32_t* l2_ws, const int32_t* l2d_ws, const int32_t* l2d_wse,
                            const double* rstd, int32_t extra, char* out, int64_t cap);

/* Deterministic synthetic PLINK .bed on the device (benchmarks / full-size tests):
 * writes the complete file image (magic + rows) to `bed_dev` (len >= 3 + n_snp*ceil(n_org/4)).
 * Model as nldsc_amd/synth.py: latent AR(1) haplotypes, thr[j] = Phi^-1(p_j), `missing` rate. */
int nldsc_synth_bed_device(int32_t device, void* bed_dev, int32_t n_snp, int32_t n_org,
                           const float* thr_host, float rho, float missing, uint64_t seed,
                           char* err, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* NLDSC_LD_H */
