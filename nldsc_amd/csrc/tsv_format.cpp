// tsv_format.cpp — the score table as the reference writes it (nldsc/ldscore/routine.py:94-101:
// make_output(...).to_csv(out, sep="\t", index=False, float_format="%.5f")), formatted natively.
// pandas formats each float with the printf-style "%.5f" (a correctly rounded conversion, as glibc's
// snprintf), writes NaN as an empty field and integers in decimal; the row prefix (CHR, SNP, BP) comes
// formatted from the caller, so its text is whatever pandas would print for the parsed .bim columns.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/nldsc_ld.h"

namespace {

constexpr int F5_MAX = 400;  // "%.5f" of -DBL_MAX: sign + 309 digits + '.' + 5 digits (+ NUL)

// "%.5f" of x, byte-identical to printf: |x| < 9e13 in exact integer arithmetic (x = m 2^ex, m < 2^53;
// round(x 1e5) half-to-even on the exact binary value, as glibc does), anything else via snprintf
inline char* put_f5(char* p, double x) {
    if (std::isnan(x)) return p;  // pandas na_rep ''
    const double ax = std::fabs(x);
    if (!(ax < 9.0e13)) return p + std::snprintf(p, F5_MAX, "%.5f", x);
    int e = 0;
    const double f = std::frexp(ax, &e);  // ax = f 2^e, f in [0.5, 1) (or 0)
    const uint64_t m = (uint64_t)std::ldexp(f, 53);
    const int ex = e - 53;  // ax = m 2^ex exactly
    const unsigned __int128 v = (unsigned __int128)m * 100000u;
    uint64_t q;
    if (ex >= 0) {
        q = (uint64_t)(v << ex);  // ax < 9e13: ax 1e5 < 2^63
    } else if (ex < -120) {
        q = 0;  // v < 2^70, so ax 1e5 < 2^-50: rounds to 0, never a tie
    } else {
        unsigned __int128 qq = v >> (-ex);
        const unsigned __int128 r = v - (qq << (-ex)), half = (unsigned __int128)1 << (-ex - 1);
        if (r > half || (r == half && (qq & 1))) ++qq;
        q = (uint64_t)qq;
    }
    if (std::signbit(x)) *p++ = '-';
    uint64_t ip = q / 100000u;
    const uint32_t fp = (uint32_t)(q % 100000u);
    char tmp[24];
    int k = 0;
    do {
        tmp[k++] = (char)('0' + ip % 10u);
        ip /= 10u;
    } while (ip);
    while (k) *p++ = tmp[--k];
    *p++ = '.';
    p[0] = (char)('0' + fp / 10000u);
    p[1] = (char)('0' + fp / 1000u % 10u);
    p[2] = (char)('0' + fp / 100u % 10u);
    p[3] = (char)('0' + fp / 10u % 10u);
    p[4] = (char)('0' + fp % 10u);
    return p + 5;
}

inline char* put_i(char* p, int32_t v) { return p + std::snprintf(p, 16, "%d", v); }

}  // namespace

extern "C" int64_t nldsc_format_scores(const char* prefix, int64_t prefix_len, int32_t n, const double* l2,
                                       const double* l2d, const double* maf, const int32_t* l2_ws,
                                       const int32_t* l2d_ws, const int32_t* l2d_wse, const double* rstd,
                                       int32_t extra, char* out, int64_t cap) {
    if (!prefix || !l2 || !l2d || !out || n < 0 || (extra && (!maf || !l2_ws || !l2d_ws || !l2d_wse || !rstd)))
        return NLDSC_E_ARG;
    // worst case per row besides the prefix: 7 numbers of < F5_MAX chars + separators
    char* p = out;
    const char* q = prefix;
    const char* const qend = prefix + prefix_len;
    for (int32_t i = 0; i < n; ++i) {
        const char* eol = static_cast<const char*>(std::memchr(q, '\n', (size_t)(qend - q)));
        const size_t len = (size_t)((eol ? eol : qend) - q);
        if (!eol && i + 1 < n) return NLDSC_E_ARG;  // fewer prefix lines than rows
        if ((int64_t)(p - out) + (int64_t)len + 7 * F5_MAX + 16 > cap) return NLDSC_E_OOM;
        std::memcpy(p, q, len);
        p += len;
        q = eol ? eol + 1 : qend;
        *p++ = '\t';
        p = put_f5(p, l2[i]);
        *p++ = '\t';
        p = put_f5(p, l2d[i]);
        if (extra) {
            *p++ = '\t';
            p = put_f5(p, maf[i]);
            *p++ = '\t';
            p = put_i(p, l2_ws[i]);
            *p++ = '\t';
            p = put_i(p, l2d_ws[i]);
            *p++ = '\t';
            p = put_i(p, l2d_wse[i]);
            *p++ = '\t';
            p = put_f5(p, rstd[i]);
        }
        *p++ = '\n';
    }
    return (int64_t)(p - out);
}
