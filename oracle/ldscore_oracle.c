/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load or call this library, and only as the checker / CPU baseline.  The
 * product path (nldsc_amd, libnldsc_amd.so) never links or calls it.
 *
 * Clean-room CPU restatement of bayarpark/nldsc `_ldscore.calculate`
 * (nldsc/ldscore/_ldscore/ldscalc.h:8-65) and everything it calls, following
 * the reference's structure: serial 2-bit unpack + per-SNP fp32 decode and
 * standardisation, a sliding window cache over SNP index, and an OpenMP
 * reduction of one fp32 dot product per (SNP, neighbour) pair.
 *
 * PARITY STATUS: the reference C++ needs Armadillo + BLAS/LAPACK, which are
 * absent from this image, so it is unbuildable here; the
 * reference ships no tests, fixtures or golden vectors.  The hot-path
 * numerics of this oracle are therefore "parity unpinned" against the
 * reference binary; they are pinned against an independent fp64
 * closed-form restatement (oracle/oracle.py) and the committed fixtures in
 * tests/golden/.
 *
 * Third-party arithmetic restated (not vendored): Armadillo `arma::mean`
 * (fp32, two accumulators) and `arma::dot` -> BLAS `sdot` for n > 32
 * (modelled as OpenBLAS 0.3.28's SkylakeX kernel, dot_f below: 4 x 16 FMA
 * accumulators folded, a 32-step, horizontal adds, the tail added in double —
 * bit-identical to the sdot of the OpenBLAS scipy ships in this image,
 * tests/test_oracle.py); neither has a pinned version in the reference
 * (CMakeLists.txt:22-27).
 */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_OK 0
#define ORC_BAD_MAGIC -1
#define ORC_SIZE -2
#define ORC_OOM -3
#define ORC_ARG -4

/* flags */
#define ORC_F64_DOT 1u      /* accumulate pair dot products in double instead of sdot-like fp32 */
#define ORC_NO_COPIES 2u    /* skip the per-pair vector copies the reference makes (ldscalc.h:38,41) */
#define ORC_STRICT_ORDER 4u /* PLINK sample order for the last byte instead of the reference's */

/* BEDBinaryEncoding (encoder.h:11-16): codes are bit pairs shifted << 6 */
enum { HOM_FST = 0, MISS = 64, HET = 128, HOM_SND = 192 };

static inline float additive(uint8_t v) { /* encoder.h:32-34, encoding<0,1,2> */
    switch (v) {
    case HOM_FST: return 0.f;
    case MISS: return NAN;
    case HET: return 1.f;
    default: return 2.f;
    }
}
static inline float dominant(uint8_t v) { /* encoder.h:36-38, encoding<0,2,2> */
    switch (v) {
    case HOM_FST: return 0.f;
    case MISS: return NAN;
    default: return 2.f;
    }
}

/* arma::mean for fvec: fp32 accumulation in two interleaved accumulators */
static float mean_f(const float* x, int n) {
    float a = 0.f, b = 0.f;
    int i = 0;
    for (; i + 1 < n; i += 2) { a += x[i]; b += x[i + 1]; }
    if (i < n) a += x[i];
    return (a + b) / (float)n;
}

/* arma::dot for fvec (op_dot::direct_dot): its own two-accumulator loop up to 32 elements, BLAS sdot above.
 * The sdot is OpenBLAS's x86-64 SkylakeX kernel as shipped with scipy (OpenBLAS 0.3.28, DYNAMIC_ARCH, one
 * thread), restated from its observable arithmetic and pinned bit for bit against that library by
 * tests/test_oracle.py::test_dot_matches_openblas_sdot: n1 = n & -32 elements go through 4 x 16 fp32 FMA
 * accumulators (64 elements per step), folded to 4 x 8 (lane k + lane k+8), one more 4 x 8 FMA step for the
 * last 32 when n1 % 64 = 32, the four summed left to right, 128-bit halves added and two horizontal adds;
 * the remaining n - n1 products (fp32) are added to that sum in double and the result is rounded to float. */
static float sdot_kernel(const float* x, const float* y, int n1) {
    __m256 a[8]; /* accumulator q = lanes 0-7 in a[2q], lanes 8-15 in a[2q+1] */
    for (int k = 0; k < 8; ++k) a[k] = _mm256_setzero_ps();
    int i = 0;
    for (; i + 64 <= n1; i += 64)
        for (int k = 0; k < 8; ++k) a[k] = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 8 * k), _mm256_loadu_ps(y + i + 8 * k), a[k]);
    __m256 b[4];
    for (int q = 0; q < 4; ++q) b[q] = _mm256_add_ps(a[2 * q], a[2 * q + 1]);
    for (; i < n1; i += 32)
        for (int q = 0; q < 4; ++q) b[q] = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 8 * q), _mm256_loadu_ps(y + i + 8 * q), b[q]);
    float c[8];
    _mm256_storeu_ps(c, _mm256_add_ps(_mm256_add_ps(_mm256_add_ps(b[0], b[1]), b[2]), b[3]));
    float h[4];
    for (int k = 0; k < 4; ++k) h[k] = c[k] + c[k + 4];
    return (h[0] + h[1]) + (h[2] + h[3]);
}

static float dot_f(const float* x, const float* y, int n) {
    if (n <= 32) { /* op_dot::direct_dot_arma; g++ contracts `val += A[i] * B[i]` into an FMA (see below) */
        float a = 0.f, b = 0.f;
        int i = 0;
        for (; i + 1 < n; i += 2) { a = fmaf(x[i], y[i], a); b = fmaf(x[i + 1], y[i + 1], b); }
        if (i < n) a = fmaf(x[i], y[i], a);
        return a + b;
    }
    const int n1 = n & -32;
    double dot = (double)sdot_kernel(x, y, n1);
    for (int i = n1; i < n; ++i) {
        const float p = x[i] * y[i];
        dot += (double)p;
    }
    return (float)dot;
}

/* exported for the pinning test only */
float oracle_sdot(const float* x, const float* y, int n) { return dot_f(x, y, n); }
float oracle_mean(const float* x, int n) { return mean_f(x, n); }

static double dot_d(const float* x, const float* y, int n) {
    double a = 0, b = 0, c = 0, d = 0;
    int i = 0;
    for (; i + 4 <= n; i += 4) {
        a += (double)x[i] * y[i]; b += (double)x[i + 1] * y[i + 1];
        c += (double)x[i + 2] * y[i + 2]; d += (double)x[i + 3] * y[i + 3];
    }
    for (; i < n; ++i) a += (double)x[i] * y[i];
    return (a + b) + (c + d);
}

/* Math::r2_adjusted (tools.h:87-92) */
static inline double r2_adjusted(const float* a, const float* b, int n, unsigned flags) {
    double nn = (double)n;
    double corr = ((flags & ORC_F64_DOT) ? dot_d(a, b, n) : (double)dot_f(a, b, n)) * (1. / nn);
    double r2 = corr * corr;
    return 1. - (1. - r2) * (nn - 1) / (nn - 2);
}

/* BedStreamReader::read (stream.h:43-69): bit pairs of each byte high first;
 * in the last byte only the first n_org % 4 (high) pairs when n_org % 4 != 0.
 * ORC_STRICT_ORDER instead emits PLINK order (low pair = first sample). */
static void unpack_row(const uint8_t* row, int n_org, int nb, uint8_t* out, unsigned flags) {
    int r = n_org % 4;
    for (int j = 0; j < nb; ++j) {
        int pairs = (j == nb - 1 && r != 0) ? r : 4;
        uint8_t b = row[j];
        if (flags & ORC_STRICT_ORDER) {
            for (int i = 0; i < pairs; ++i) out[4 * j + i] = (uint8_t)(((b >> (2 * i)) & 3) << 6);
        } else {
            for (int i = 0; i < pairs; ++i) { out[4 * j + i] = b & 192; b = (uint8_t)((b & 63) << 2); }
        }
    }
}

typedef struct {
    float* add;   /* standardised additive vector */
    float* res;   /* standardised dominance residual */
    float maf;
    float rstd;
    int use;
} snp_t;

/* SNPInMemory ctor + decode (encoder.h:54-60, 91-133), Math::regression_residuals
 * (tools.h:54-68) and Math::standardise/var_ (tools.h:70-85).  Returns -1 on OOM. */
static int decode_snp(const uint8_t* codes, int n, double maf_thr, snp_t* s) {
    s->add = s->res = NULL;
    s->maf = NAN; s->rstd = NAN; s->use = 0;
    float* add = (float*)malloc(sizeof(float) * (size_t)n);
    float* nadd = (float*)malloc(sizeof(float) * (size_t)n);
    if (!add || !nadd) { free(add); free(nadd); return -1; }
    double add_sum = 0, nadd_sum = 0;
    int n_obs = 0;
    for (int i = 0; i < n; ++i) {
        uint8_t v = codes[i];
        float a = additive(v), d = dominant(v);
        if (v != MISS) { add_sum += a; nadd_sum += d; ++n_obs; }
        add[i] = a; nadd[i] = d;
    }
    float add_mean = (float)(add_sum / n_obs);
    float nadd_mean = (float)(nadd_sum / n_obs);
    float f2 = add_mean / 2;
    s->maf = f2 < 0.5f ? f2 : 1 - f2;
    if ((double)s->maf <= maf_thr) { free(add); free(nadd); return 0; }
    for (int i = 0; i < n; ++i)
        if (isnan(add[i])) { add[i] = add_mean; nadd[i] = nadd_mean; }
    /* regression_residuals(x = add, y = nadd) */
    double x_mean = mean_f(add, n), y_mean = mean_f(nadd, n);
    double nn = (double)n;
    /* The reference is C++ built with -O3 -march=native (CMakeLists.txt:14,24): g++ contracts a*b +- c into an
     * FMA by default in C++ (-ffp-contract=fast; only ISO C turns it off), so `dot/n - x_mean*y_mean` and
     * `y - slope * x` (tools.h:64-66) are fused multiply-adds on FMA hardware.  This file is C11, where nothing
     * is contracted implicitly: the fusions are written out. */
    double slope = fma(-x_mean, y_mean, (double)dot_f(add, nadd, n) / nn) /
                   fma(-x_mean, x_mean, (double)dot_f(add, add, n) / nn);
    float k = (float)slope; /* Armadillo converts the scalar to the element type */
    for (int i = 0; i < n; ++i) nadd[i] = fmaf(-add[i], k, nadd[i]);
    /* standardise(add) then standardise(residuals) */
    for (int v = 0; v < 2; ++v) {
        float* vec = v ? nadd : add;
        float m = mean_f(vec, n);
        for (int i = 0; i < n; ++i) vec[i] -= m; /* var_ works on a copy; same values */
        float var = (float)((double)dot_f(vec, vec, n) * (1. / nn));
        float sd = sqrtf(var);
        for (int i = 0; i < n; ++i) vec[i] /= sd;
        if (v) s->rstd = sd;
    }
    s->add = add; s->res = nadd; s->use = 1;
    return 0;
}

static void release(snp_t* s) { /* SNPInMemory::release (encoder.h:82-88) */
    free(s->add); free(s->res);
    s->add = s->res = NULL;
    s->use = 0;
}

/* SNPFilter (tools.h:5-50) */
typedef struct { const double* pos; int n_snp; double w; } filt_t;
static inline int is_used(const filt_t* f, int i) { return 0 <= i && i < f->n_snp && f->pos[i] >= 0; }
static inline int in_window(const filt_t* f, int a, int b) {
    return is_used(f, a) && is_used(f, b) && fabs(f->pos[b] - f->pos[a]) <= f->w;
}

int oracle_check_bed(size_t bed_len, const uint8_t* bed, int n_snp, int n_org) {
    if (bed_len < 3 || bed[0] != 0x6c || bed[1] != 0x1b || bed[2] != 0x01) return ORC_BAD_MAGIC;
    size_t nb = (size_t)(n_org / 4 + (n_org % 4 > 0));
    if (bed_len < 3 + nb * (size_t)n_snp) return ORC_SIZE;
    return ORC_OK;
}

/*
 * calculate() (ldscalc.h:8-65) with ChunkwiseReader (stream.h:106-198).
 * Outputs (length n_snp) are written for SNP indices in [out_begin, out_end);
 * the sliding window still runs from SNP 0 so that the window state is the
 * reference's.  With out_begin = 0, out_end = n_snp this is the full call.
 * `mafs()`/`residual_stds()` (stream.h:165-179) are reported for every SNP in
 * range: MAF for decoded SNPs, residual std for MAF-passing ones, NaN
 * otherwise.
 */
int oracle_ld_calculate(size_t bed_len, const uint8_t* bed, int n_snp, int n_org, double ld_wind,
                        double maf_thr, double std_thr, double rsq_thr, const double* pos,
                        int out_begin, int out_end, unsigned flags, int n_threads,
                        double* l2, double* l2d, double* maf, double* rstd,
                        int32_t* l2_ws, int32_t* l2d_ws, int32_t* l2d_wse) {
    int rc = oracle_check_bed(bed_len, bed, n_snp, n_org);
    if (rc) return rc;
    if (n_snp <= 0 || n_org <= 2 || out_begin < 0 || out_end > n_snp || out_begin > out_end) return ORC_ARG;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    const int nb = n_org / 4 + (n_org % 4 > 0);
    const uint8_t* rows = bed + 3;
    filt_t f = {pos, n_snp, ld_wind};

    for (int i = out_begin; i < out_end; ++i) {
        l2[i] = NAN; l2d[i] = NAN; maf[i] = NAN; rstd[i] = NAN;
        l2_ws[i] = -1; l2d_ws[i] = -1; l2d_wse[i] = -1;
    }
    snp_t* cache = (snp_t*)calloc((size_t)n_snp, sizeof(snp_t));
    uint8_t* codes = (uint8_t*)malloc((size_t)nb * 4);
    int* idx = (int*)malloc(sizeof(int) * (size_t)n_snp);
    float* tmp = NULL;
    if (!cache || !codes || !idx) { rc = ORC_OOM; goto done; }
    for (int i = 0; i < n_snp; ++i) { cache[i].maf = NAN; cache[i].rstd = NAN; }
    int decoded_upto = -1;   /* highest index emplaced into the cache */
    int left = 0, right = -1, cur = -1;

    for (int j = 0; j < out_end; ++j) {
        if (!is_used(&f, j)) { ++cur; continue; }            /* pass_chunk (stream.h:157-159) */
        ++cur;                                                /* initialize_next_chunk (stream.h:131-136) */
        do {                                                  /* extend_cache (stream.h:182-197) */
            if (right + 1 >= n_snp) break;
            ++right;
            if (is_used(&f, right)) {
                unpack_row(rows + (size_t)right * nb, n_org, nb, codes, flags);
                if (decode_snp(codes, n_org, maf_thr, &cache[right])) { rc = ORC_OOM; goto done; }
            }
            decoded_upto = right;
        } while (in_window(&f, cur, right));
        if (!(cur <= decoded_upto && cache[cur].use)) continue;   /* SNP failed MAF: NaN / -1 */
        /* chunk_indices (stream.h:142-155): neighbours + left-edge eviction */
        int n_idx = 0;
        for (int i = left; i <= right; ++i) {
            if (cache[i].use && in_window(&f, cur, i)) {
                if (i != cur) idx[n_idx++] = i;
            } else if (left == i && left < cur) {
                release(&cache[left]);
                ++left;
            }
        }
        if (j < out_begin || j >= out_end) continue;
        /* hot loop (ldscalc.h:34-47) */
        const float* y = cache[cur].add;
        double add = 1.0, dom = 0.0;
        int passed = 0, effective = 0;
        const int copies = !(flags & ORC_NO_COPIES);
        #pragma omp parallel for schedule(static) reduction(+:dom, add, passed, effective)
        for (int t = 0; t < n_idx; ++t) {
            const snp_t* s = &cache[idx[t]];
            float* cp = NULL;
            const float* av = s->add;
            if (copies) { /* snp.add() returns a copy of N floats (encoder.h:70-72) */
                cp = (float*)malloc(sizeof(float) * (size_t)n_org);
                memcpy(cp, s->add, sizeof(float) * (size_t)n_org);
                av = cp;
            }
            add += r2_adjusted(y, av, n_org, flags);
            if ((double)s->rstd > std_thr) {
                const float* rv = s->res;
                if (copies) { memcpy(cp, s->res, sizeof(float) * (size_t)n_org); rv = cp; }
                double rsq = r2_adjusted(y, rv, n_org, flags);
                dom += rsq;
                effective += rsq > rsq_thr;
            } else {
                passed += 1;
            }
            free(cp);
        }
        l2[j] = add; l2d[j] = dom;
        l2_ws[j] = n_idx; l2d_ws[j] = n_idx - passed; l2d_wse[j] = effective;
    }
    for (int i = out_begin; i < out_end; ++i) {
        if (i <= decoded_upto && is_used(&f, i)) {
            maf[i] = cache[i].maf;
            rstd[i] = cache[i].rstd; /* NaN unless the SNP passed MAF (release keeps it) */
        }
    }
done:
    if (cache) for (int i = 0; i < n_snp; ++i) { free(cache[i].add); free(cache[i].res); }
    free(cache); free(codes); free(idx); free(tmp);
    return rc;
}

/* MAF exactly as decode() computes it (encoder.h:95-118), from code counts only:
 * the sums are integers, so this is bit-identical to the full decode. */
static float maf_from_row(const uint8_t* row, int n_org, int nb, uint8_t* codes, unsigned flags) {
    unpack_row(row, n_org, nb, codes, flags);
    long cnt[4] = {0, 0, 0, 0};
    for (int i = 0; i < n_org; ++i) cnt[codes[i] >> 6]++;
    long n_obs = cnt[0] + cnt[2] + cnt[3];
    double add_sum = (double)cnt[2] + 2.0 * (double)cnt[3];
    float add_mean = (float)(add_sum / (double)n_obs);
    float f2 = add_mean / 2;
    return f2 < 0.5f ? f2 : 1 - f2;
}

/*
 * Spot-check mode for large inputs: the same outputs as oracle_ld_calculate for
 * the SNP indices in `targets` (strictly increasing), written at positions
 * 0..n_targets-1 of the output arrays.  The window state the reference builds by
 * streaming (left/right pointers, stream.h:142-155,182-197) is replayed from
 * positions and MAF-pass flags alone, and only the SNPs inside the targets'
 * windows are decoded.  tests/ check it against the full mode.
 */
int oracle_ld_targets(size_t bed_len, const uint8_t* bed, int n_snp, int n_org, double ld_wind,
                      double maf_thr, double std_thr, double rsq_thr, const double* pos,
                      const int32_t* targets, int n_targets, unsigned flags, int n_threads,
                      double* l2, double* l2d, double* maf, double* rstd,
                      int32_t* l2_ws, int32_t* l2d_ws, int32_t* l2d_wse) {
    int rc = oracle_check_bed(bed_len, bed, n_snp, n_org);
    if (rc) return rc;
    if (n_snp <= 0 || n_org <= 2 || n_targets < 0) return ORC_ARG;
    for (int t = 1; t < n_targets; ++t) if (targets[t] <= targets[t - 1]) return ORC_ARG;
    for (int t = 0; t < n_targets; ++t) if (targets[t] < 0 || targets[t] >= n_snp) return ORC_ARG;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    const int nb = n_org / 4 + (n_org % 4 > 0);
    const uint8_t* rows = bed + 3;
    filt_t f = {pos, n_snp, ld_wind};
    uint8_t* pass = (uint8_t*)calloc((size_t)n_snp, 1);
    float* mafs = (float*)malloc(sizeof(float) * (size_t)n_snp);
    int32_t* L = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_snp);
    int32_t* R = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_snp);
    snp_t* cache = (snp_t*)calloc((size_t)n_snp, sizeof(snp_t));
    int* idx = (int*)malloc(sizeof(int) * (size_t)n_snp);
    if (!pass || !mafs || !L || !R || !cache || !idx) { rc = ORC_OOM; goto done; }

    #pragma omp parallel
    {
        uint8_t* codes = (uint8_t*)malloc((size_t)nb * 4);
        #pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < n_snp; ++i) {
            mafs[i] = NAN;
            if (is_used(&f, i) && codes) {
                mafs[i] = maf_from_row(rows + (size_t)i * nb, n_org, nb, codes, flags);
                pass[i] = !((double)mafs[i] <= maf_thr);
            }
        }
        free(codes);
    }
    /* replay ChunkwiseReader's pointers */
    int left = 0, right = -1;
    for (int j = 0; j < n_snp; ++j) {
        L[j] = -1; R[j] = -2;
        if (!is_used(&f, j)) continue;
        do {
            if (right + 1 >= n_snp) break;
            ++right;
        } while (in_window(&f, j, right));
        if (!(j <= right && pass[j])) continue;
        while (left < j && !(pass[left] && in_window(&f, j, left))) ++left;
        L[j] = left; R[j] = right;
    }
    int lo = 0; /* cache holds decoded SNPs with index >= lo */
    for (int t = 0; t < n_targets; ++t) {
        int j = targets[t];
        l2[t] = NAN; l2d[t] = NAN; l2_ws[t] = -1; l2d_ws[t] = -1; l2d_wse[t] = -1;
        maf[t] = mafs[j]; rstd[t] = NAN;
        if (!is_used(&f, j) || !pass[j] || L[j] < 0) continue;
        for (; lo < L[j]; ++lo) release(&cache[lo]);
        int n_idx = 0;
        for (int i = L[j]; i <= R[j]; ++i)
            if (i != j && pass[i] && in_window(&f, j, i)) idx[n_idx++] = i;
        idx[n_idx] = j;
        int fail = 0;
        #pragma omp parallel reduction(|:fail)
        {
            uint8_t* codes = (uint8_t*)malloc((size_t)nb * 4);
            if (!codes) fail = 1;
            #pragma omp for schedule(dynamic, 1)
            for (int q = 0; q <= n_idx; ++q) {
                int i = idx[q];
                if (codes && !cache[i].use) {
                    unpack_row(rows + (size_t)i * nb, n_org, nb, codes, flags);
                    if (decode_snp(codes, n_org, maf_thr, &cache[i])) fail = 1;
                }
            }
            free(codes);
        }
        if (fail) { rc = ORC_OOM; goto done; }
        rstd[t] = cache[j].rstd;
        if (!cache[j].use) continue;  /* all-missing MAF NaN still decodes with use = 1 */
        const float* y = cache[j].add;
        double add = 1.0, dom = 0.0;
        int passed = 0, effective = 0;
        #pragma omp parallel for schedule(static) reduction(+:dom, add, passed, effective)
        for (int q = 0; q < n_idx; ++q) {
            const snp_t* s = &cache[idx[q]];
            add += r2_adjusted(y, s->add, n_org, flags);
            if ((double)s->rstd > std_thr) {
                double rsq = r2_adjusted(y, s->res, n_org, flags);
                dom += rsq;
                effective += rsq > rsq_thr;
            } else {
                passed += 1;
            }
        }
        l2[t] = add; l2d[t] = dom;
        l2_ws[t] = n_idx; l2d_ws[t] = n_idx - passed; l2d_wse[t] = effective;
    }
done:
    if (cache) for (int i = 0; i < n_snp; ++i) { free(cache[i].add); free(cache[i].res); }
    free(cache); free(idx); free(pass); free(mafs); free(L); free(R);
    return rc;
}

/*
 * Exact-arithmetic helpers for the fp64 truth (oracle.py run_f64_targets): integer genotype-code
 * counts per SNP and 4x4 code contingency tables of SNP pairs, over the samples the reference reads
 * (stream.h:43-69, same last-byte rule as unpack_row).  Counting only — no floating point.
 */
int oracle_code_counts(size_t bed_len, const uint8_t* bed, int n_snp, int n_org, unsigned flags,
                       int n_threads, int64_t* counts /* [n_snp][4] */) {
    int rc = oracle_check_bed(bed_len, bed, n_snp, n_org);
    if (rc) return rc;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    const int nb = n_org / 4 + (n_org % 4 > 0);
    int fail = 0;
    #pragma omp parallel reduction(|:fail)
    {
        uint8_t* codes = (uint8_t*)malloc((size_t)nb * 4);
        if (!codes) fail = 1;
        #pragma omp for schedule(dynamic, 16)
        for (int i = 0; i < n_snp; ++i) {
            if (!codes) continue;
            unpack_row(bed + 3 + (size_t)i * nb, n_org, nb, codes, flags);
            int64_t c[4] = {0, 0, 0, 0};
            for (int s = 0; s < n_org; ++s) c[codes[s] >> 6]++;
            for (int g = 0; g < 4; ++g) counts[4 * (size_t)i + g] = c[g];
        }
        free(codes);
    }
    return fail ? ORC_OOM : ORC_OK;
}

int oracle_code_tables(size_t bed_len, const uint8_t* bed, int n_snp, int n_org, unsigned flags,
                       int n_threads, int j, const int32_t* ks, int n_k, int64_t* tables /* [n_k][4][4] */) {
    int rc = oracle_check_bed(bed_len, bed, n_snp, n_org);
    if (rc) return rc;
    if (j < 0 || j >= n_snp) return ORC_ARG;
    for (int q = 0; q < n_k; ++q) if (ks[q] < 0 || ks[q] >= n_snp) return ORC_ARG;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    const int nb = n_org / 4 + (n_org % 4 > 0);
    uint8_t* cj = (uint8_t*)malloc((size_t)nb * 4);
    if (!cj) return ORC_OOM;
    unpack_row(bed + 3 + (size_t)j * nb, n_org, nb, cj, flags);
    for (int s = 0; s < n_org; ++s) cj[s] = (uint8_t)((cj[s] >> 6) << 2); /* row code g -> 4g */
    int fail = 0;
    #pragma omp parallel reduction(|:fail)
    {
        uint8_t* ck = (uint8_t*)malloc((size_t)nb * 4);
        if (!ck) fail = 1;
        #pragma omp for schedule(dynamic, 4)
        for (int q = 0; q < n_k; ++q) {
            if (!ck) continue;
            unpack_row(bed + 3 + (size_t)ks[q] * nb, n_org, nb, ck, flags);
            int64_t c[16] = {0};
            for (int s = 0; s < n_org; ++s) c[cj[s] | (ck[s] >> 6)]++;
            memcpy(tables + 16 * (size_t)q, c, sizeof c);
        }
        free(ck);
    }
    free(cj);
    return fail ? ORC_OOM : ORC_OK;
}
