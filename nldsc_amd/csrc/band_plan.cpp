// band_plan.cpp — host-side window replay and band schedule of the engine (no HIP: also built with
// g++ -fsanitize=address,undefined for the CPU sanitizer run, tests/native/plan_tsv_check.cpp).
#include "band_plan.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/nldsc_ld.h"

namespace nldsc {

// Replay of ChunkwiseReader's pointers (stream.h:131-155,182-197) from positions and MAF-pass
// flags.  For every SNP j the reference computes, N(j) = { i in [L_j, R_j] : pass_i,
// |pos_i - pos_j| <= w, i != j }; L_j = -1 marks a SNP it does not compute (unused, MAF-failed).
void replay_windows(const double* pos, const uint8_t* flags, int n, double w, int* L, int* R) {
    auto used = [&](int i) { return 0 <= i && i < n && pos[i] >= 0; };
    auto inwin = [&](int a, int b) { return used(a) && used(b) && std::fabs(pos[b] - pos[a]) <= w; };
    int left = 0, right = -1;
    for (int j = 0; j < n; ++j) {
        L[j] = -1;
        R[j] = -2;
        if (!used(j)) continue;                       // pass_chunk
        do {                                          // extend_cache
            if (right + 1 >= n) break;
            ++right;
        } while (inwin(j, right));
        if (!(j <= right && (flags[j] & 1))) continue;  // initialize_next_chunk() == false
        // chunk_indices: evict failing SNPs at the left edge
        while (left < j && !((flags[left] & 1) && inwin(j, left))) ++left;
        L[j] = left;
        R[j] = right;
    }
}

// Positions non-decreasing over the used SNPs (pos >= 0)?
// every position >= 0 (no NaN) and non-decreasing: one branch-free pass (the GPU schedule's condition)
bool positions_nonneg_sorted(const double* pos, int M) {
    int bad = M > 0 && !(pos[0] >= 0.0);
    for (int j = 1; j < M; ++j) bad |= !(pos[j] >= 0.0) | (pos[j] < pos[j - 1]);
    return !bad;
}

bool positions_sorted(const double* pos, int M) {
    double last = -1.0;
    for (int j = 0; j < M; ++j)
        if (pos[j] >= 0) {
            if (pos[j] < last) return false;
            last = pos[j];
        }
    return true;
}

// Tile schedule of the band kernel.  A block pair (I <= J) is needed when it holds a pair (i < j)
// with j in N(i) or i in N(j) and one of i, j is owned.  Rows need columns up to the last
// in-window neighbour: R_i is the reference's (loose) cache bound — its extend_cache advances at
// least one SNP per SNP, so R_i drifts past the window — so for sorted positions the bound is
// tightened to the last index with pos <= pos_i + w (the kernel still masks with the exact
// predicate).  Columns j need rows down to L_j (exact).
void plan_items(const double* pos, const uint8_t* flags, int M, double w, const int* L, const int* R, int own_begin,
                int own_end, int max_nc, std::vector<PlanItem>& out) {
    constexpr int B = 32;
    const int nblk = (M + B - 1) / B;
    std::vector<int> blk_pass(nblk, 0), blk_own(nblk, 0);
    for (int j = 0; j < M; ++j) {
        if (flags[j] & 1) blk_pass[j / B] = 1;
        if (j >= own_begin && j < own_end) blk_own[j / B] = 1;
    }
    // sorted (non-decreasing over used SNPs)?  then the window's right edge is a binary search
    std::vector<int> used_idx;
    used_idx.reserve(M);
    bool sorted = true;
    for (int j = 0; j < M; ++j)
        if (pos[j] >= 0) {
            if (!used_idx.empty() && pos[j] < pos[used_idx.back()]) sorted = false;
            used_idx.push_back(j);
        }
    // sorted: last used index with pos <= pos_i + w (ties inclusive, tools.h:41-49) by a two-pointer sweep
    std::vector<int> hi_of;
    if (sorted) {
        hi_of.assign(M, -1);
        size_t k = 0;
        for (size_t u = 0; u < used_idx.size(); ++u) {
            const double lim = pos[used_idx[u]] + w;
            if (k < u) k = u;
            while (k + 1 < used_idx.size() && pos[used_idx[k + 1]] <= lim) ++k;
            hi_of[used_idx[u]] = used_idx[k];
        }
    }
    auto row_bound = [&](int i) { return sorted ? std::min(R[i], hi_of[i]) : R[i]; };
    std::vector<int> comp;
    comp.reserve(M);
    for (int j = 0; j < M; ++j) if (L[j] >= 0) comp.push_back(j);
    int lo_row = own_begin;  // first row an owned SNP needs: min L_j over owned computed j
    for (int j : comp) if (j >= own_begin && j < own_end) lo_row = std::min(lo_row, L[j]);
    size_t cp = 0;
    int run_rmax = -1;  // largest computed j with L_j <= current row (L non-decreasing over computed)
    out.clear();
    std::vector<PlanItem> ones;
    for (int I = std::max(0, lo_row / B); I < nblk && I * B < own_end; ++I) {
        const int i_end = std::min(M, (I + 1) * B) - 1;
        int jmax = -1;
        for (int i = I * B; i <= i_end; ++i) if (L[i] >= 0) jmax = std::max(jmax, row_bound(i));
        while (cp < comp.size() && L[comp[cp]] <= i_end) { run_rmax = comp[cp]; ++cp; }
        jmax = std::max(jmax, run_rmax);
        if (!blk_pass[I] || jmax < I * B) continue;
        const int Jmax = std::min(nblk - 1, jmax / B);
        auto useful = [&](int JJ) { return blk_pass[JJ] && (blk_own[I] || blk_own[JJ]); };
        int J = I;
        while (J <= Jmax) {
            if (!useful(J)) { ++J; continue; }
            if (max_nc == 2 && J + 1 <= Jmax && useful(J + 1)) {
                out.push_back(PlanItem{I, J, 2, 0});
                J += 2;
            } else {
                ones.push_back(PlanItem{I, J, 1, 0});
                J += 1;
            }
        }
    }
    out.insert(out.end(), ones.begin(), ones.end());
}

// Reorder single-block-pair items (row-major by I, then J) into tiles of R row blocks x C diagonal
// offsets d = J - I: tile (I / R, d / C), then I, then J.  The launch hands each XCD a contiguous
// run of the list, so the waves resident on one XCD at a time work on about R row strips and R + C
// column strips, each reused ~R or ~C times from that XCD's L2.  Row-major order (R = 1) is as good
// for narrow bands (C3: d <= 10) and poor for wide ones (C5: d <= ~220, a column strip is read by
// ~2 resident waves): 16 x 16 tiles cut the C5 band kernel by 8.5 % (profiles/r01_ab_tiles_c5.json).
void order_items_tiled(std::vector<PlanItem>& items, int nblk, int R, int C, std::vector<PlanItem>& scratch) {
    if (R <= 1 || items.empty()) return;
    std::vector<int> first(nblk + 1, 0);  // items of row block I: [first[I], first[I+1])
    int dmax = 0;
    for (const PlanItem& it : items) {
        ++first[it.x + 1];
        dmax = std::max(dmax, it.y - it.x);
    }
    if (dmax < 2 * C) return;  // narrow band: row-major is as good (C3, profiles/r01_ab_tiles_c3.json)
    for (int I = 0; I < nblk; ++I) first[I + 1] += first[I];
    std::vector<int> cur(first.begin(), first.end() - 1);  // next unread item of each row block
    scratch.clear();
    scratch.reserve(items.size());
    for (int t0 = 0; t0 < nblk; t0 += R)
        for (int c0 = 0; c0 <= dmax; c0 += C)
            for (int I = t0; I < std::min(nblk, t0 + R); ++I)
                for (int& k = cur[I]; k < first[I + 1] && items[k].y - I < c0 + C; ++k) scratch.push_back(items[k]);
    items.swap(scratch);
}

}  // namespace nldsc

extern "C" {

int nldsc_plan_band(const double* positions, const uint8_t* flags, int32_t n_snp, double ld_wind, int32_t own_begin,
                    int32_t own_end, int32_t max_nc, int32_t* L, int32_t* R, int32_t* items, int32_t cap) {
    if (!positions || !flags || !L || !R || n_snp <= 0 || own_begin < 0 || own_end > n_snp || own_begin > own_end ||
        (max_nc != 1 && max_nc != 2))
        return NLDSC_E_ARG;
    nldsc::replay_windows(positions, flags, n_snp, ld_wind, L, R);
    std::vector<nldsc::PlanItem> it;
    nldsc::plan_items(positions, flags, n_snp, ld_wind, L, R, own_begin, own_end, max_nc, it);
    if ((int64_t)it.size() > (int64_t)cap || !items) return (int)std::min<size_t>(it.size(), INT32_MAX);
    for (size_t k = 0; k < it.size(); ++k) {
        items[4 * k] = it[k].x; items[4 * k + 1] = it[k].y; items[4 * k + 2] = it[k].z; items[4 * k + 3] = 0;
    }
    return (int)it.size();
}

}  // extern "C"
