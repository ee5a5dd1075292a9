// CPU sanitizer driver for the engine's host code (built by `make -C nldsc_amd/csrc sanitize` with
// -fsanitize=address,undefined; run by tests/test_sanitize.py).  No GPU, no HIP.
//  * nldsc_plan_band (band_plan.cpp): window replay and band schedule on random inputs — sorted, tied,
//    negative, NaN and unsorted positions, MAF failures, empty and partial owned ranges, windows from 0 to
//    everything — checked against a brute-force restatement of the reference's ChunkwiseReader pointers
//    (stream.h:131-155,182-197): every needed 32-SNP block pair covered exactly once, every item in range.
//  * nldsc_format_scores (tsv_format.cpp): "%.5f" fields, NaN as '', against snprintf on random, tie,
//    tiny, huge and non-finite values.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/nldsc_ld.h"
#include "../../nldsc_amd/csrc/band_plan.h"

static int fails = 0;
#define CHECK(c, ...)                                            \
    do {                                                         \
        if (!(c)) {                                              \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                   \
            std::fprintf(stderr, "\n");                          \
            if (++fails > 20) std::exit(1);                      \
        }                                                        \
    } while (0)

// brute-force ChunkwiseReader pointers (same semantics, written independently of band_plan.cpp)
static void naive_replay(const std::vector<double>& pos, const std::vector<uint8_t>& pass, double w,
                         std::vector<int>& L, std::vector<int>& R) {
    const int n = (int)pos.size();
    auto used = [&](int i) { return i >= 0 && i < n && pos[i] >= 0; };
    auto inwin = [&](int a, int b) { return used(a) && used(b) && std::fabs(pos[b] - pos[a]) <= w; };
    L.assign(n, -1);
    R.assign(n, -2);
    int left = 0, right = -1;
    for (int j = 0; j < n; ++j) {
        if (!used(j)) continue;
        for (;;) {
            if (right + 1 >= n) break;
            ++right;
            if (!inwin(j, right)) break;
        }
        if (!(j <= right && pass[j])) continue;
        while (left < j && !(pass[left] && inwin(j, left))) ++left;
        L[j] = left;
        R[j] = right;
    }
}

static void check_plan(std::mt19937_64& rng, int iter) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const int n = 1 + (int)(rng() % (iter % 5 == 0 ? 3000 : 300));
    std::vector<double> pos(n);
    double x = 0;
    const double gap = 0.01 + U(rng);
    for (int j = 0; j < n; ++j) {
        x += (U(rng) < 0.1) ? 0.0 : gap * U(rng);  // ~10 % duplicates
        pos[j] = std::round(x * 64.0) / 64.0;       // dyadic: exact window ties
    }
    const int kind = iter % 6;
    if (kind == 1) for (int k = 0; k < 1 + n / 50; ++k) pos[rng() % n] = -1.0;
    if (kind == 2) pos[rng() % n] = std::nan("");
    if (kind == 3) for (int k = 0; k < 1 + n / 20; ++k) std::swap(pos[rng() % n], pos[rng() % n]);
    std::vector<uint8_t> pass(n);
    const double fail_rate = (iter % 3) * 0.2;
    for (auto& p : pass) p = U(rng) >= fail_rate;
    const double ws[] = {0.0, 0.25, 1.0, 3.0, 1e9};
    const double w = ws[rng() % 5] * gap * 4;
    int ob = (int)(rng() % (n + 1)), oe = (int)(rng() % (n + 1));
    if (ob > oe) std::swap(ob, oe);
    if (iter % 4 == 0) { ob = 0; oe = n; }
    const int max_nc = 1 + (int)(rng() % 2);

    std::vector<int32_t> L(n), R(n);
    const int k = nldsc_plan_band(pos.data(), pass.data(), n, w, ob, oe, max_nc, L.data(), R.data(), nullptr, 0);
    CHECK(k >= 0, "plan count %d", k);
    std::vector<int32_t> items(4 * (size_t)std::max(k, 1));
    const int k2 = nldsc_plan_band(pos.data(), pass.data(), n, w, ob, oe, max_nc, L.data(), R.data(), items.data(), k);
    CHECK(k2 == k, "plan %d vs %d", k2, k);
    std::vector<int> NL, NR;
    naive_replay(pos, pass, w, NL, NR);
    for (int j = 0; j < n; ++j) CHECK(L[j] == NL[j] && R[j] == NR[j], "pointers of %d: (%d,%d) vs (%d,%d)", j, L[j], R[j], NL[j], NR[j]);
    const int nblk = (n + 31) / 32;
    std::set<std::pair<int, int>> cover;
    for (int q = 0; q < k; ++q) {
        const int I = items[4 * q], J = items[4 * q + 1], z = items[4 * q + 2];
        CHECK(I >= 0 && I <= J && (z == 1 || (z == 2 && max_nc == 2)) && J + z <= nblk, "item (%d,%d,%d)", I, J, z);
        for (int c = 0; c < z; ++c) CHECK(cover.insert({I, J + c}).second, "block pair (%d,%d) twice", I, J + c);
    }
    auto used = [&](int i) { return pos[i] >= 0; };
    for (int j = 0; j < n; ++j) {
        if (NL[j] < 0) continue;
        for (int i = NL[j]; i <= NR[j] && i < n; ++i) {
            if (i == j || !pass[i] || !used(i) || !(std::fabs(pos[i] - pos[j]) <= w)) continue;
            const bool owned = (j >= ob && j < oe) || (i >= ob && i < oe && NL[i] >= 0);
            if (!(j >= ob && j < oe)) continue;  // the pair contributes to owned j
            (void)owned;
            const int a = std::min(i, j) / 32, b = std::max(i, j) / 32;
            CHECK(cover.count({a, b}), "pair (%d,%d) of owned %d not covered (blocks %d,%d; n=%d w=%g own=[%d,%d))",
                  i, j, j, a, b, n, w, ob, oe);
        }
    }
}

static std::string f5(double v) {
    if (std::isnan(v)) return "";
    char b[512];
    std::snprintf(b, sizeof b, "%.5f", v);
    return b;
}

static void check_tsv(std::mt19937_64& rng, int iter) {
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const int n = 1 + (int)(rng() % 200);
    std::vector<double> c[5];
    std::vector<int32_t> ic[3];
    const double specials[] = {0.0, -0.0, 0.000005, 0.000015, 0.000025, 2.5e-6, 1e-300, -1e-300, 5e-324,
                               123456789.123455, 9.0e13, 8.9999999999e13, 1e300, -1e300, HUGE_VAL, -HUGE_VAL,
                               std::nan(""), 0.5, 1.0, 99999.999995, 1.000005, 2.675e-5};
    for (auto& v : c) {
        v.resize(n);
        for (auto& x : v) {
            const int m = (int)(rng() % 4);
            x = m == 0 ? specials[rng() % (sizeof specials / sizeof specials[0])]
              : m == 1 ? U(rng) * std::pow(10.0, (double)(rng() % 30) - 15.0)
              : m == 2 ? std::round(U(rng) * 1e7) / 1e5 + 5e-6 * (rng() % 2) : U(rng) * 1000.0;
        }
    }
    for (auto& v : ic) {
        v.resize(n);
        for (auto& x : v) x = (int32_t)(rng() % 100000) - 1;
    }
    const int extra = iter % 2;
    std::string prefix, expect;
    for (int i = 0; i < n; ++i) {
        const std::string p = std::to_string(1 + i % 22) + "\trs" + std::to_string(i) + "\t" + std::to_string(1000 * i);
        prefix += p + (i + 1 < n ? "\n" : "");
        expect += p + "\t" + f5(c[0][i]) + "\t" + f5(c[1][i]);
        if (extra)
            expect += "\t" + f5(c[2][i]) + "\t" + std::to_string(ic[0][i]) + "\t" + std::to_string(ic[1][i]) + "\t" +
                      std::to_string(ic[2][i]) + "\t" + f5(c[3][i]);
        expect += "\n";
    }
    std::vector<char> out(prefix.size() + (size_t)n * (16 + 7 * 400) + 1);
    const int64_t got = nldsc_format_scores(prefix.data(), (int64_t)prefix.size(), n, c[0].data(), c[1].data(),
                                            c[2].data(), ic[0].data(), ic[1].data(), ic[2].data(), c[3].data(), extra,
                                            out.data(), (int64_t)out.size());
    CHECK(got == (int64_t)expect.size() && std::memcmp(out.data(), expect.data(), expect.size()) == 0,
          "tsv mismatch (n=%d extra=%d, %lld vs %zu bytes)", n, extra, (long long)got, expect.size());
    // too small a buffer must fail cleanly, not overflow
    const int64_t small = nldsc_format_scores(prefix.data(), (int64_t)prefix.size(), n, c[0].data(), c[1].data(),
                                              c[2].data(), ic[0].data(), ic[1].data(), ic[2].data(), c[3].data(), extra,
                                              out.data(), 8);
    CHECK(small < 0, "undersized buffer accepted (%lld)", (long long)small);
}

// the GPU schedule's condition in one pass: equal to "sorted among the non-negative ones and all non-negative"
static void check_sorted(std::mt19937_64& rng, int iter) {
    const int M = (int)(rng() % 200);
    std::vector<double> P(M);
    double x = 0;
    for (int j = 0; j < M; ++j) {
        x += (double)(rng() % 3);
        const int kind = (int)(rng() % 60);
        P[j] = kind == 0 ? -1.0 : kind == 1 ? std::nan("") : kind == 2 ? x - 2.5 : x;
    }
    bool all_nonneg = true;
    for (double v : P) all_nonneg &= v >= 0.0;
    const bool expect = all_nonneg && nldsc::positions_sorted(P.data(), M);
    CHECK(nldsc::positions_nonneg_sorted(P.data(), M) == expect, "positions_nonneg_sorted (M=%d, iter %d)", M, iter);
}

int main() {
    std::mt19937_64 rng(2024);
    for (int it = 0; it < 600; ++it) check_plan(rng, it);
    for (int it = 0; it < 2000; ++it) check_sorted(rng, it);
    // argument checks of the C ABI
    double p1[2] = {0, 1};
    uint8_t f1[2] = {1, 1};
    int32_t l1[2], r1[2];
    CHECK(nldsc_plan_band(p1, f1, 2, 1.0, 1, 0, 1, l1, r1, nullptr, 0) < 0, "bad own range accepted");
    CHECK(nldsc_plan_band(p1, f1, 2, 1.0, 0, 2, 3, l1, r1, nullptr, 0) < 0, "bad max_nc accepted");
    for (int it = 0; it < 400; ++it) check_tsv(rng, it);
    if (fails) {
        std::fprintf(stderr, "%d failures\n", fails);
        return 1;
    }
    std::printf("plan_tsv_check OK (600 plans, 2000 position checks, 400 tables)\n");
    return 0;
}
