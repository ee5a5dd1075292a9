// ld_engine.cpp — host side of libnldsc_amd.so: the C ABI declared in include/nldsc_ld.h.
//
// One engine = one HIP device + one stream + device buffers that persist across runs.
// A run (nldsc_engine_run) is the whole hot path of bayarpark/nldsc's `calculate`
// (nldsc/ldscore/_ldscore/ldscalc.h:8-65) over a .bed image already resident in HBM:
//   count (resident rows, kept at an aligned pitch by the loaders) -> per-SNP statistics ->
//   window replay + tile schedule (host, O(M), overlapping the count) ->
//   band correlation kernels -> finalize -> results to host.
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "../../include/nldsc_ld.h"
#include "band_plan.h"
#include "ld_kernels.h"

#define NLDSC_VERSION "0.1.0"

namespace {

constexpr int BLK = 32;             // SNPs per MFMA block
constexpr int CHUNK_BYTES = 32;     // one K-loop chunk of a 2-bit row (16 B per lane half)
constexpr int kLoadThreads = 8;     // .bed file loads: reader threads (pread + H2D + placement per slice)
constexpr int kCopyThreads = 3;     // host result copies: helper threads beside the calling one
// resident row pitch: an even number of 32-byte chunks (the fp4 K loop takes two per iteration)
constexpr int ROW_ALIGN_BYTES = 64;
// item order of the single-block-pair schedule: tiles of TILE_R row blocks x TILE_C diagonal offsets
constexpr int TILE_R = 16, TILE_C = 16;

// resident layout of a .bed image: rows of ceil(N/4) bytes padded to row_bytes, n_rows = M rounded up to 32, the rows of
// each 32-SNP block interleaved in 32-byte chunks (ld_kernels.hip tile_off)
int row_pitch(int32_t n_org) {
    const int nb = n_org / 4 + (n_org % 4 > 0);
    return (nb + ROW_ALIGN_BYTES - 1) / ROW_ALIGN_BYTES * ROW_ALIGN_BYTES;
}
int padded_rows(int32_t n_snp) { return (n_snp + BLK - 1) / BLK * BLK; }

// Message of BedStreamReader::check_plink_magic_number (stream.h:88-102), verbatim.
const char* kBadMagic =
    "Invalid PLINK magic number in BED file.The file is incorrect, or it was created using an incompatible "
    "version of PLINK.";

int set_err(char* err, size_t errlen, int code, const char* fmt, ...) {
    if (err && errlen) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(err, errlen, fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return set_err(err, errlen, NLDSC_E_HIP, "HIP error %s at %s:%d (%s)", hipGetErrorString(e_), \
                           __FILE__, __LINE__, #expr);                                                \
    } while (0)

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(want, 1) * sizeof(T));
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// page-locked host buffer (async H2D copies out of it do not block the calling thread)
struct HostPinned {
    uint8_t* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc((void**)&p, std::max<size_t>(want, 1));
        if (e == hipSuccess) n = want;
        return e;
    }
    ~HostPinned() {
        if (p) (void)hipHostFree(p);
    }
};

// Host work of a run split over the calling thread and kCopyThreads helpers, which sleep on a condition variable
// between runs: the copies of its results (pinned landing buffer -> the caller's arrays, 3.5 MB at M = 80 000: ~0.33 ms
// on one core; below kMinParallel bytes the caller copies alone, a wake-up costs more) and of its positions, and the
// schedule's window edges.
class CopyPool {
  public:
    struct Seg {
        void* dst;
        const void* src;
        size_t n;
    };
    static constexpr size_t kMinParallel = 256 << 10;
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void copy(const Seg* segs, int nseg) {
        size_t total = 0;
        for (int k = 0; k < nseg; ++k) total += segs[k].n;
        if (total < kMinParallel) {
            for (int k = 0; k < nseg; ++k) std::memcpy(segs[k].dst, segs[k].src, segs[k].n);
            return;
        }
        // part p: bytes [total * p / parts, total * (p + 1) / parts) of the segments laid end to end
        parallel([&](int p, int parts) {
            const size_t lo = total * p / parts, hi = total * (p + 1) / parts;
            size_t base = 0;
            for (int k = 0; k < nseg && base < hi; base += segs[k].n, ++k) {
                const size_t a = std::max(lo, base), b = std::min(hi, base + segs[k].n);
                if (a < b)
                    std::memcpy(static_cast<uint8_t*>(segs[k].dst) + (a - base),
                                static_cast<const uint8_t*>(segs[k].src) + (a - base), b - a);
            }
        });
    }
    // f(part, parts) for part = 0 .. parts - 1 (parts = kCopyThreads + 1), part 0 on the calling thread.  Helper
    // threads start on first use; if the system refuses a thread, every part runs on the calling thread from then on
    // (a std::system_error must not cross the C ABI: ADVICE r04)
    void parallel(const std::function<void(int, int)>& f) {
        if (th_.empty() && !serial_) {
            try {
                for (int t = 0; t < kCopyThreads; ++t) th_.emplace_back([this, t] { loop(t + 1); });
            } catch (const std::exception&) {
                {
                    std::lock_guard<std::mutex> lk(mu_);
                    stop_ = true;
                }
                cv_.notify_all();
                for (auto& t : th_) t.join();
                th_.clear();
                stop_ = false;
                serial_ = true;
            }
        }
        if (serial_) {
            for (int p = 0; p <= kCopyThreads; ++p) f(p, kCopyThreads + 1);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            pending_ = kCopyThreads;
            ++gen_;
        }
        cv_.notify_all();
        f(0, kCopyThreads + 1);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

  private:
    void loop(int idx) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const std::function<void(int, int)>* f = job_;
            lk.unlock();
            (*f)(idx, kCopyThreads + 1);
            lk.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int, int)>* job_ = nullptr;
    int pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    bool serial_ = false;
};

// Spin on a pinned word the GPU writes (a blocking event wait wakes the thread tens of microseconds late: the host waits
// on the critical path of short runs), with a CPU pause per poll, for at most ~1 ms — then the caller's blocking event
// wait takes over (a stalled plan no longer burns 2 s of a core that loaders and RCCL proxies share).
bool spin_until_nonneg(volatile const int* w) {
    const auto t0 = std::chrono::steady_clock::now();
    while (*w < 0) {
        _mm_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(1000)) return false;
    }
    return true;
}

// Pinned host buffers handed out by nldsc_host_alloc: a run whose result arrays (or positions) lie inside one is
// written (read) by the GPU directly, without the engine's own landing buffer and host copies.
std::mutex g_host_mu;
std::map<uintptr_t, size_t> g_host_bufs;  // start -> bytes

// device pointer of [p, p + bytes) when it lies inside one nldsc_host_alloc buffer, else nullptr
void* registered_device_ptr(const void* p, size_t bytes) {
    if (!p) return nullptr;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    uintptr_t base = 0;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto it = g_host_bufs.upper_bound(a);
        if (it == g_host_bufs.begin()) return nullptr;
        --it;
        if (a + bytes > it->first + it->second) return nullptr;
        base = it->first;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(base), 0) != hipSuccess || !d) return nullptr;
    return static_cast<uint8_t*>(d) + (a - base);
}

}  // namespace

struct nldsc_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t plan_stream = nullptr;  // the GPU schedule runs here, beside the count kernel
    hipEvent_t ev_pos = nullptr;        // positions uploaded and their window edges searched (the schedule's input)
    hipEvent_t ev[6] = {};
    hipEvent_t ev_dbg[2] = {};  // option debug_timing: after the super-item launch, before the single-block launches
    bool debug_timing = false;
    hipEvent_t ev_plan = nullptr;  // GPU plan counters landed in h_meta
    hipEvent_t ev_stats = nullptr;   // SNP constants and replay flags written (the replay's inputs)
    hipEvent_t ev_replay = nullptr;  // replayed constants written (the KC launch and finalize wait on it)
    // side stream: the rare-variant replay beside the band (ev_replay), then the issued-product count (ev_issued)
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_issued = nullptr;
    // resident .bed image
    DevBuf<uint8_t> bed;      // resident rows, block-interleaved (ld_kernels.hip tile_off)
    DevBuf<uint8_t> stage_dev;  // loads: rows of the .bed layout on their way into `bed` (released after the load)
    DevBuf<uint8_t> lastb;  // each row's original last byte (the per-run count kernel masks a copy of it)
    DevBuf<uint8_t> flip;   // per SNP: resident row stores the swapped (00 <-> 11) coding
    DevBuf<uint8_t> row_miss;  // per SNP: bit 0 / 1 = a missing call among the reference's / PLINK's individual slots
    DevBuf<uint32_t> miss_flags;  // (the load kernels' per-row word of the same flags)
    DevBuf<int> lcounts;          // per row: genotype counts of its stored bytes [0, nb - 1), load_parts parts
    bool orient = true;     // store rows minor-homozygote-as-00 at load (option "orient" 0: file coding)
    bool oriented = false;  // the resident image was oriented
    int32_t n_snp = 0, n_org = 0;
    // work buffers

    DevBuf<int> counts, cparts, Lw, Rw, Aw, ws_acc;  // (cparts: the count kernel's per-part counts)
    // the per-SNP results, one allocation: L2, L2D, MAF, RSTD (fp64) then WSA, WSD, WSDE (int32), each M long, so the
    // owned slices come back in two strided copies (one when a run owns every SNP)
    DevBuf<double> res;
    template <class T>
    struct View {
        T* p = nullptr;
    };
    View<double> l2, l2d, maf, rstd;
    View<int> ws3;
    DevBuf<float2> lut;
    DevBuf<nldsc::SnpConst> cst;
    DevBuf<uint8_t> sflags;
    DevBuf<uint8_t> blk_rep;  // per 32-SNP block: holds a rare variant with replayed fp32 vectors (KC items)
    DevBuf<float> gram;       // K-split partial Gram tiles
    // rare-variant items of the single-block fp4 kernel, deferred: their Gram tiles (8192 floats per block pair), the
    // block pairs, the slot counter (launch_band_f4 rep_gram; option "defer_rep" 0: the separate KC launch instead)
    DevBuf<float> rep_gram;
    DevBuf<int4> rep_items;
    DevBuf<int> rep_count;
    bool defer_rep = true;
    // a split run between its two calls (nldsc_engine_run_device_split / _finish)
    bool split_pending = false;
    int32_t split_M = 0, split_N = 0, split_row_bytes = 0, split_width = 0;
    std::pair<int32_t, int32_t> split_own{0, 0};
    bool split_dom = true;
    double* split_table = nullptr;
    double split_ms1 = 0.0;  // the first call's host time
    bool ksplit_ok = true;    // option "ksplit" 0 disables the K-split
    static constexpr int round_min = 1;  // round launches from this many rounds of single-block items on
    // deferred rare-variant Gram tiles: at most this many block-pair slots (32 KiB each: 2 GiB)
    size_t rep_gram_max_slots = (size_t)1 << 16;
    int last_ksplit = 1;
    int last_round_items = 0;
    int last_direct = -1;  // nldsc_engine_result_direct
    int last_tail_ksplit = 1;
    // fp4 band kernels on the GPU plan (option "t2"): 3 (default) missing-free 4 x 4 super-items in the quad
    // workgroups (64 x 64 tiles per wave), the rest in the single-block kernel (C5 slice band -25 % against 1, the
    // others unchanged: profiles/r03_ab_t2_quad.json); 1 the same with missing-free 2 x 2 super-items in the 2 x 2
    // block-pair workgroups; 2 everything in the 2 x 2 workgroups; 0 single-block only
    int t2_mode = 3;
    // additive-only fp4 band in 32 x 64 tiles (column-block pair items, the row strip decoded once for two column
    // blocks; option "f4_nc2" 0 turns it off): C2 band 2.85 -> 2.78 ms, one engine per process (r03_c2_nc2.json)
    bool f4_nc2 = true;
    // single-block fp4 band in launches of one round of wave slots (option "band_rounds" 0: one launch)
    bool band_rounds = true;
    DevBuf<uint8_t> blk_miss;
    // quad super-items in launches of one workgroup per CU when there are at least 16 such rounds (option "q_rounds" 0:
    // one launch): the workgroups on an XCD then stream their shared strips at nearby K offsets; C5 slice band
    // 351 -> 333 ms, C3 missing-free (6 rounds, below the threshold) 12.34 -> 12.51 ms (profiles/r03_ab_q_rounds.json)
    bool q_rounds = true;
    int last_band_kernel = NLDSC_BAND_F4;
    // 32-SNP blocks without a missing call among the individual slots of sample order o (row_miss, at load): the
    // super-item kernels take only missing-free blocks, so with none the run skips their plan, routing and launches
    int free_blocks[2] = {0, 0};
    DevBuf<double> pos, l2_acc, l2d_acc;
    DevBuf<int4> items;
    // host scratch
    std::vector<uint8_t> h_flags, h_all_pass;
    std::vector<int> h_L, h_R;
    std::vector<nldsc::PlanItem> h_items, h_scratch;
    HostPinned h_stage;  // pinned upload staging of the plan (L, R, items)
    HostPinned h_meta;   // GPU plan counters (items, diagonal items)
    HostPinned h_pos;    // pinned copy of the positions (the upload does not stall this thread)
    HostPinned h_res;    // pinned landing buffer of host-result runs (the GPU writes it, then host copies out)
    CopyPool copies;     // the host copies out of h_res, split over threads
    // [0..1] device-table runs: sums of the positive WSA / WSD over the owned slice; [2] MFMA products issued
    DevBuf<unsigned long long> sums;
    HostPinned h_sums;
    DevBuf<int> plan_counts, plan_meta, plan_counts2;
    DevBuf<int2> plan_rows, plan_rows2;
    DevBuf<int4> items2;  // super-items of the 2 x 2 / quad kernel
    DevBuf<int4> items_u;  // routed runs: the single-block items no super-item kernel takes (compacted)
    DevBuf<int> compact_tmp;
    HostPinned h_route;    // their count
    hipEvent_t ev_route = nullptr;
    bool gpu_plan = true;  // band schedule on the GPU for non-negative sorted positions (option "gpu_plan" 0: host)
    // slices of at most PLAN_SMALL_N SNPs (a rank's shard): the GPU schedule in one fused launch, items included
    // (option "plan_fused" 0: the kernel chain of long slices)
    bool plan_fused = true;
    // timings of the last run
    double ms[6] = {0, 0, 0, 0, 0, 0};
    double flop_alg = 0, flop_issued = 0, pairs = 0, ops_alg_i8 = 0;
    int32_t n_band_items = 0;
    int last_path = 0;     // path of the last run: 0 fp32, 1 exact int8, 2 exact fp4
    int band_mode = 2;     // default correlation path (option "band_mode" 0 fp32, 1 int8, 2 fp4): exact fp4
                           // (int8 from N = 2^27)
    int n_cu = 256;

    ~nldsc_engine() {
        (void)hipSetDevice(device);
        bed.release(); stage_dev.release(); lastb.release(); flip.release(); row_miss.release(); miss_flags.release();
        lcounts.release();
        counts.release(); Lw.release(); Rw.release(); Aw.release(); ws_acc.release();
        res.release(); lut.release(); cst.release(); sflags.release(); pos.release();
        l2_acc.release(); l2d_acc.release(); items.release(); gram.release();
        rep_gram.release(); rep_items.release(); rep_count.release();
        for (auto& e : ev) if (e) (void)hipEventDestroy(e);
        for (auto& e : ev_dbg) if (e) (void)hipEventDestroy(e);
        if (ev_plan) (void)hipEventDestroy(ev_plan);
        plan_counts.release(); plan_meta.release(); plan_rows.release();
        plan_counts2.release(); plan_rows2.release(); items2.release(); blk_miss.release(); sums.release();
        cparts.release();
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        if (ev_issued) (void)hipEventDestroy(ev_issued);
        if (stream) (void)hipStreamDestroy(stream);
        if (plan_stream) (void)hipStreamDestroy(plan_stream);
        if (ev_pos) (void)hipEventDestroy(ev_pos);
        if (ev_stats) (void)hipEventDestroy(ev_stats);
        if (ev_replay) (void)hipEventDestroy(ev_replay);
        if (ev_route) (void)hipEventDestroy(ev_route);
        items_u.release(); compact_tmp.release();
    }
};

namespace {

int check_dims(int32_t n_snp, int32_t n_org, char* err, size_t errlen) {
    if (n_snp <= 0) return set_err(err, errlen, NLDSC_E_ARG, "n_snp must be positive (got %d)", n_snp);
    if (n_org <= 0) return set_err(err, errlen, NLDSC_E_ARG, "n_org must be positive (got %d)", n_org);
    return NLDSC_OK;
}

size_t bed_bytes_needed(int32_t n_snp, int32_t n_org) {
    const size_t nb = (size_t)(n_org / 4 + (n_org % 4 > 0));
    return 3 + nb * (size_t)n_snp;
}

int check_magic(const uint8_t* m, size_t len, int32_t n_snp, int32_t n_org, char* err, size_t errlen) {
    if (len < 3 || m[0] != 0x6c || m[1] != 0x1b || m[2] != 0x01)
        return set_err(err, errlen, NLDSC_E_BAD_MAGIC, "%s", kBadMagic);
    if (len < bed_bytes_needed(n_snp, n_org))
        return set_err(err, errlen, NLDSC_E_SIZE,
                       "BED file too short: %zu bytes, expected at least %zu for %d SNPs x %d individuals", len,
                       bed_bytes_needed(n_snp, n_org), n_snp, n_org);
    return NLDSC_OK;
}

int use_device(int32_t device, int* resolved, char* err, size_t errlen) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return set_err(err, errlen, NLDSC_E_NODEV, "no HIP device visible (nldsc_amd has no CPU fallback)");
    int d = device;
    if (d < 0) HIPCHK(hipGetDevice(&d));
    if (d >= n) return set_err(err, errlen, NLDSC_E_ARG, "device %d out of range (%d visible)", d, n);
    HIPCHK(hipSetDevice(d));
    *resolved = d;
    return NLDSC_OK;
}

// device buffers of a resident image of n_snp rows (all rows, pitch padding, saved last bytes, per-row flags)
hipError_t alloc_image(nldsc_engine* e, int32_t n_snp, int32_t n_org) {
    e->n_snp = e->n_org = 0;  // no valid image until finish_image
    e->oriented = e->orient;  // (the load's slices all use the orientation rule in force when it starts)
    hipError_t he = e->bed.ensure((size_t)padded_rows(n_snp) * (size_t)row_pitch(n_org));
    if (he == hipSuccess) he = e->lastb.ensure((size_t)n_snp);
    if (he == hipSuccess) he = e->flip.ensure((size_t)n_snp);
    if (he == hipSuccess) he = e->row_miss.ensure((size_t)n_snp);
    if (he == hipSuccess) he = e->miss_flags.ensure((size_t)n_snp);
    if (he == hipSuccess)
        he = e->lcounts.ensure((size_t)n_snp * 3);
    return he;
}

// Rows [row0, row0 + n_rows) (whole 32-SNP blocks but for the image's last) of n_snp from a .bed slice in device memory
// into the resident layout, oriented, last bytes saved, missing flags of both sample orders (the last byte keeps its
// high / low N % 4 pairs) — one pass over the slice (ld_kernels.h launch_load_slice)
hipError_t load_slice(nldsc_engine* e, const uint8_t* src, int32_t row0, int32_t n_rows, int32_t n_snp, int32_t n_org,
                      hipStream_t st) {
    const int nb = n_org / 4 + (n_org % 4 > 0), rem = n_org % 4;
    const uint32_t keep_compat = rem ? (0xFFu << (8 - 2 * rem)) & 0xFFu : 0xFFu;
    const uint32_t keep_strict = rem ? (1u << (2 * rem)) - 1u : 0xFFu;
    return nldsc::launch_load_slice(src, nb, row0, n_rows, n_snp, e->bed.p, row_pitch(n_org), e->oriented, e->flip.p,
                                    e->lastb.p, keep_compat, keep_strict, e->miss_flags.p, e->lcounts.p, st);
}

// after every slice is in: per-row missing flags, the missing-free block counts, and mark the image valid
hipError_t finish_image(nldsc_engine* e, int32_t n_snp, int32_t n_org) {
    hipError_t he = nldsc::launch_load_flags(e->miss_flags.p, n_snp, e->row_miss.p, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he == hipSuccess) {  // missing-free blocks per sample order
        std::vector<uint8_t> rm((size_t)n_snp);
        he = hipMemcpy(rm.data(), e->row_miss.p, (size_t)n_snp, hipMemcpyDeviceToHost);
        e->free_blocks[0] = e->free_blocks[1] = 0;
        for (int32_t b = 0; he == hipSuccess && b < (n_snp + 31) / 32; ++b) {
            uint8_t m = 0;
            for (int32_t j = 32 * b; j < std::min(n_snp, 32 * b + 32); ++j) m |= rm[(size_t)j];
            for (int o = 0; o < 2; ++o) e->free_blocks[o] += ((m >> o) & 1) ? 0 : 1;
        }
    }
    if (he == hipSuccess) {
        e->n_snp = n_snp;
        e->n_org = n_org;
    }
    return he;
}

}  // namespace

extern "C" {

const char* nldsc_version(void) { return NLDSC_VERSION; }

int nldsc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// The environment knobs of rounds 1-4 ($NLDSC_T2, $NLDSC_BAND_MODE, ...) became engine options
// (nldsc_engine_set_option) in round 5; a process that still sets one is told once, on stderr, which option replaces
// it instead of silently running the defaults.
static void warn_legacy_env_once() {
    static std::once_flag once;
    std::call_once(once, [] {
        static const char* const legacy[][2] = {
            {"NLDSC_BAND_MODE", "band_mode"}, {"NLDSC_GPU_PLAN", "gpu_plan"},   {"NLDSC_ORIENT", "orient"},
            {"NLDSC_KSPLIT", "ksplit"},       {"NLDSC_T2", "t2"},               {"NLDSC_BAND_ROUNDS", "band_rounds"},
            {"NLDSC_F4_NC2", "f4_nc2"},       {"NLDSC_Q_ROUNDS", "q_rounds"},   {"NLDSC_DEFER_REP", "defer_rep"},
            {"NLDSC_DEBUG_TIMING", "debug_timing"}, {"NLDSC_QUAD_ADD", nullptr}, {"NLDSC_REPLAY_OVERLAP", nullptr}};
        for (const auto& kv : legacy)
            if (std::getenv(kv[0]))
                std::fprintf(stderr, "nldsc_amd: $%s is no longer read; %s%s%s\n", kv[0],
                             kv[1] ? "use the engine option \"" : "the study mode it selected was removed",
                             kv[1] ? kv[1] : "", kv[1] ? "\" (nldsc_engine_set_option / Engine(options=...))" : "");
    });
}

int nldsc_engine_create(int32_t device, nldsc_engine** out, char* err, size_t errlen) {
    warn_legacy_env_once();
    if (!out) return set_err(err, errlen, NLDSC_E_ARG, "out is NULL");
    *out = nullptr;
    int d = 0;
    int rc = use_device(device, &d, err, errlen);
    if (rc) return rc;
    nldsc_engine* e = new (std::nothrow) nldsc_engine();
    if (!e) return set_err(err, errlen, NLDSC_E_OOM, "out of host memory");
    e->device = d;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && prop.multiProcessorCount > 0)
            e->n_cu = prop.multiProcessorCount;
    }
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&e->plan_stream, hipStreamNonBlocking);
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_issued, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_pos, hipEventDisableTiming);
    for (auto& ev : e->ev)
        if (he == hipSuccess) he = hipEventCreate(&ev);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_plan, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_stats, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_replay, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e->ev_route, hipEventDisableTiming);
    for (auto& ev : e->ev_dbg)
        if (he == hipSuccess) he = hipEventCreate(&ev);
    if (he != hipSuccess) {
        delete e;
        return set_err(err, errlen, NLDSC_E_HIP, "HIP error %s creating stream/events", hipGetErrorString(he));
    }
    *out = e;
    return NLDSC_OK;
}

void nldsc_engine_destroy(nldsc_engine* e) { delete e; }

int nldsc_engine_set_option(nldsc_engine* e, const char* name, int64_t value, char* err, size_t errlen) {
    if (!e || !name) return set_err(err, errlen, NLDSC_E_ARG, "NULL engine or option name");
    struct Opt {
        const char* name;
        int64_t lo, hi;
        std::function<void(int64_t)> set;
    };
    const Opt opts[] = {
        {"band_mode", 0, 2, [&](int64_t v) { e->band_mode = (int)v; }},
        {"gpu_plan", 0, 1, [&](int64_t v) { e->gpu_plan = v != 0; }},
        {"plan_fused", 0, 1, [&](int64_t v) { e->plan_fused = v != 0; }},
        {"orient", 0, 1, [&](int64_t v) { e->orient = v != 0; }},
        {"ksplit", 0, 1, [&](int64_t v) { e->ksplit_ok = v != 0; }},
        {"t2", 0, 3, [&](int64_t v) { e->t2_mode = (int)v; }},
        {"band_rounds", 0, 1, [&](int64_t v) { e->band_rounds = v != 0; }},
        {"f4_nc2", 0, 1, [&](int64_t v) { e->f4_nc2 = v != 0; }},
        {"q_rounds", 0, 1, [&](int64_t v) { e->q_rounds = v != 0; }},
        {"defer_rep", 0, 1, [&](int64_t v) { e->defer_rep = v != 0; }},
        {"debug_timing", 0, 1, [&](int64_t v) { e->debug_timing = v != 0; }},
    };
    for (const Opt& o : opts)
        if (std::strcmp(o.name, name) == 0) {
            if (value < o.lo || value > o.hi)
                return set_err(err, errlen, NLDSC_E_ARG, "option %s: value %lld outside [%lld, %lld]", name,
                               (long long)value, (long long)o.lo, (long long)o.hi);
            o.set(value);
            return NLDSC_OK;
        }
    return set_err(err, errlen, NLDSC_E_ARG, "unknown engine option \"%s\"", name);
}

void* nldsc_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_bufs[reinterpret_cast<uintptr_t>(p)] = bytes;
    return p;
}

void nldsc_host_free(void* p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto it = g_host_bufs.find(reinterpret_cast<uintptr_t>(p));
        if (it == g_host_bufs.end()) return;  // not ours
        g_host_bufs.erase(it);
    }
    (void)hipHostFree(p);
}

int nldsc_engine_load_bed_host(nldsc_engine* e, const uint8_t* bed, size_t len, int32_t n_snp, int32_t n_org,
                               char* err, size_t errlen) {
    if (!e || !bed) return set_err(err, errlen, NLDSC_E_ARG, "NULL engine or buffer");
    int rc = check_dims(n_snp, n_org, err, errlen);
    if (rc) return rc;
    rc = check_magic(bed, len, n_snp, n_org, err, errlen);
    if (rc) return rc;
    HIPCHK(hipSetDevice(e->device));
    const size_t nb = (size_t)(n_org / 4 + (n_org % 4 > 0));
    HIPCHK(alloc_image(e, n_snp, n_org));
    // rows go up in slices of ~64 MiB of whole 32-SNP blocks into a device staging buffer, then into the resident
    // layout (load_slice); the stream orders each slice's kernels before the next copy over the same staging bytes
    const size_t rows_per = std::max<size_t>(32, (size_t(64) << 20) / nb / 32 * 32);
    HIPCHK(e->stage_dev.ensure(std::min(rows_per, (size_t)n_snp) * nb + 16));
    for (size_t r0 = 0; r0 < (size_t)n_snp; r0 += rows_per) {
        const size_t nr = std::min(rows_per, (size_t)n_snp - r0);
        HIPCHK(hipMemcpyAsync(e->stage_dev.p, bed + 3 + r0 * nb, nr * nb, hipMemcpyHostToDevice, e->stream));
        HIPCHK(load_slice(e, e->stage_dev.p, (int)r0, (int)nr, n_snp, n_org, e->stream));
    }
    HIPCHK(finish_image(e, n_snp, n_org));
    e->stage_dev.release();
    return NLDSC_OK;
}

int nldsc_engine_load_bed_device(nldsc_engine* e, const void* bed, size_t len, int32_t n_snp, int32_t n_org,
                                 char* err, size_t errlen) {
    if (!e || !bed) return set_err(err, errlen, NLDSC_E_ARG, "NULL engine or buffer");
    int rc = check_dims(n_snp, n_org, err, errlen);
    if (rc) return rc;
    const size_t need = bed_bytes_needed(n_snp, n_org);
    if (len < 3) return set_err(err, errlen, NLDSC_E_BAD_MAGIC, "%s", kBadMagic);
    HIPCHK(hipSetDevice(e->device));
    uint8_t magic[3];
    HIPCHK(hipMemcpy(magic, bed, 3, hipMemcpyDeviceToHost));
    if (magic[0] != 0x6c || magic[1] != 0x1b || magic[2] != 0x01)
        return set_err(err, errlen, NLDSC_E_BAD_MAGIC, "%s", kBadMagic);
    if (len < need)
        return set_err(err, errlen, NLDSC_E_SIZE, "BED image too short: %zu bytes, expected at least %zu", len, need);
    HIPCHK(alloc_image(e, n_snp, n_org));
    HIPCHK(load_slice(e, static_cast<const uint8_t*>(bed) + 3, 0, n_snp, n_snp, n_org, e->stream));
    HIPCHK(finish_image(e, n_snp, n_org));
    return NLDSC_OK;
}

int nldsc_engine_load_bed_file_range(nldsc_engine* e, const char* path, int32_t n_snp_file, int32_t n_org,
                                     int32_t snp_begin, int32_t snp_end, char* err, size_t errlen) {
    if (!e || !path) return set_err(err, errlen, NLDSC_E_ARG, "NULL engine or path");
    int rc = check_dims(n_snp_file, n_org, err, errlen);
    if (rc) return rc;
    if (snp_begin < 0 || snp_end > n_snp_file || snp_begin >= snp_end)
        return set_err(err, errlen, NLDSC_E_ARG, "SNP range [%d, %d) outside [0, %d) or empty", snp_begin, snp_end,
                       n_snp_file);
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        // the reference's ifstream fails silently and then rejects the (unread) magic number
        return set_err(err, errlen, NLDSC_E_BAD_MAGIC, "%s", kBadMagic);
    }
    uint8_t magic[3] = {0, 0, 0};
    const size_t got = std::fread(magic, 1, 3, f);
    if (got < 3 || magic[0] != 0x6c || magic[1] != 0x1b || magic[2] != 0x01) {
        std::fclose(f);
        return set_err(err, errlen, NLDSC_E_BAD_MAGIC, "%s", kBadMagic);
    }
    const size_t nb = (size_t)(n_org / 4 + (n_org % 4 > 0));
    const size_t first = 3 + nb * (size_t)snp_begin, bytes = nb * (size_t)(snp_end - snp_begin);
    const size_t need = first + bytes;  // file bytes the slice needs (the whole file for [0, n_snp_file))
    auto too_short = [&](size_t have) {
        std::fclose(f);
        return set_err(err, errlen, NLDSC_E_SIZE,
                       "BED file too short: %zu bytes, expected at least %zu for %d SNPs x %d individuals", have,
                       need, snp_end, n_org);
    };
    if (fseeko(f, 0, SEEK_END) != 0) return too_short(3);
    const off_t fsize = ftello(f);
    if (fsize < 0 || (size_t)fsize < need) return too_short(fsize < 0 ? 0 : (size_t)fsize);
    HIPCHK(hipSetDevice(e->device));
    const int32_t n_snp = snp_end - snp_begin;
    {
        const hipError_t ha = alloc_image(e, n_snp, n_org);
        if (ha != hipSuccess) {
            std::fclose(f);
            return set_err(err, errlen, NLDSC_E_HIP, "HIP error %s allocating the image", hipGetErrorString(ha));
        }
    }
    // Rows stream through T reader threads, each with its own pinned slot (~32 MiB of whole rows), device staging slot
    // and stream: thread t reads slices t, t + T, ... with pread (several reads in flight: the page cache copies and
    // the device's queue run in parallel, where one fread loop held the load to one core's memcpy rate), then queues
    // the slice's H2D copy and the kernels that place its rows (load_slice), and waits for both before it reuses the
    // slot.  Slices are independent (each names its rows), so their order does not matter.
    const int fd = fileno(f);
    // (slices of whole 32-SNP blocks: load_slice)
    const size_t rows_per = std::max<size_t>(32, (size_t(32) << 20) / nb / 32 * 32), CH = rows_per * nb;
    const size_t n_slices = (bytes + CH - 1) / CH;
    const int T = (int)std::max<size_t>(1, std::min<size_t>(n_slices, (size_t)kLoadThreads));
    uint8_t* stage = nullptr;
    if (hipHostMalloc((void**)&stage, (size_t)T * CH) != hipSuccess) {
        std::fclose(f);
        return set_err(err, errlen, NLDSC_E_OOM, "cannot allocate pinned staging buffer");
    }
    hipError_t he = e->stage_dev.ensure((size_t)T * CH + 16);
    std::vector<hipStream_t> streams(T, nullptr);
    std::vector<hipEvent_t> done(T, nullptr);
    for (int t = 0; t < T && he == hipSuccess; ++t) {
        he = hipStreamCreateWithFlags(&streams[t], hipStreamNonBlocking);
        if (he == hipSuccess) he = hipEventCreateWithFlags(&done[t], hipEventDisableTiming);
    }
    std::atomic<bool> stop{false};
    std::atomic<size_t> short_at{SIZE_MAX};
    std::vector<hipError_t> terr(T, hipSuccess);
    const int dev = e->device;
    uint8_t* const dstage = e->stage_dev.p;
    auto reader = [&](int t) {
        hipError_t r = hipSetDevice(dev);
        uint8_t* buf = stage + (size_t)t * CH;
        uint8_t* dslot = dstage + (size_t)t * CH;
        bool pending = false;
        for (size_t k = (size_t)t; r == hipSuccess && k < n_slices && !stop.load(); k += (size_t)T) {
            const size_t off = k * CH, n = std::min(CH, bytes - off);
            if (pending) r = hipEventSynchronize(done[t]);
            if (r != hipSuccess) break;
            size_t got = 0;
            while (got < n) {
                const ssize_t q = pread(fd, buf + got, n - got, (off_t)(first + off + got));
                if (q < 0 && errno == EINTR) continue;
                if (q <= 0) break;
                got += (size_t)q;
            }
            if (got != n) {
                size_t cur = short_at.load();
                while (first + off + got < cur && !short_at.compare_exchange_weak(cur, first + off + got)) {
                }
                stop.store(true);
                break;
            }
            r = hipMemcpyAsync(dslot, buf, n, hipMemcpyHostToDevice, streams[t]);
            if (r == hipSuccess)
                r = load_slice(e, dslot, (int)(off / nb), (int)(n / nb), n_snp, n_org, streams[t]);
            if (r == hipSuccess) r = hipEventRecord(done[t], streams[t]);
            pending = true;
        }
        if (r == hipSuccess && streams[t]) r = hipStreamSynchronize(streams[t]);
        if (r != hipSuccess) stop.store(true);
        terr[t] = r;
    };
    if (he == hipSuccess) {
        std::vector<std::thread> pool;
        for (int t = 1; t < T; ++t) pool.emplace_back(reader, t);
        reader(0);
        for (auto& th : pool) th.join();
        for (hipError_t r : terr)
            if (he == hipSuccess && r != hipSuccess) he = r;
    }
    for (int t = 0; t < T; ++t) {
        if (streams[t]) (void)hipStreamDestroy(streams[t]);
        if (done[t]) (void)hipEventDestroy(done[t]);
    }
    (void)hipHostFree(stage);
    e->stage_dev.release();
    if (short_at.load() != SIZE_MAX) return too_short(short_at.load());
    std::fclose(f);
    if (he != hipSuccess) return set_err(err, errlen, NLDSC_E_HIP, "HIP error %s loading BED", hipGetErrorString(he));
    HIPCHK(finish_image(e, n_snp, n_org));
    return NLDSC_OK;
}

int nldsc_engine_load_bed_file(nldsc_engine* e, const char* path, int32_t n_snp, int32_t n_org, char* err,
                               size_t errlen) {
    if (!e || !path) return set_err(err, errlen, NLDSC_E_ARG, "NULL engine or path");
    int rc = check_dims(n_snp, n_org, err, errlen);
    if (rc) return rc;
    return nldsc_engine_load_bed_file_range(e, path, n_snp, n_org, 0, n_snp, err, errlen);
}

}  // extern "C"

namespace {

// The hot path of one run.  Results go to the host arrays of `r`, or (table_dev != nullptr) stay in device memory
// as the owned slice of the score table (nldsc_engine_run_device).
// Split runs (nldsc_engine_run_device_split, export_n != nullptr): only the pairs whose lower SNP is owned are computed,
// the per-SNP sums of every SNP of the slice accumulate, the right halo's [own_end, M) go out to export_dev and the run
// stops before finalize; nldsc_engine_run_device_finish adds the left neighbour's export and finishes.
int run_impl(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end, nldsc_ld_result* r,
             double* table_dev, int32_t width, char* err, size_t errlen, long long* export_dev = nullptr,
             int32_t export_cap = 0, int32_t* export_n = nullptr) {
    const bool split = export_n != nullptr;
    if (!e || !p || (!r && !table_dev)) return set_err(err, errlen, NLDSC_E_ARG, "NULL argument");
    // any run overwrites the accumulators a pending split run left for run_device_finish
    e->split_pending = false;
    if (!e->bed.p) return set_err(err, errlen, NLDSC_E_ARG, "no BED image loaded");
    if (p->n_snp != e->n_snp || p->n_org != e->n_org)
        return set_err(err, errlen, NLDSC_E_ARG, "params (%d SNPs x %d) do not match the loaded BED (%d x %d)",
                       p->n_snp, p->n_org, e->n_snp, e->n_org);
    if (!p->positions) return set_err(err, errlen, NLDSC_E_ARG, "positions is NULL");
    if (!table_dev && (!r->l2 || !r->l2d || !r->maf || !r->residuals_std || !r->l2_ws || !r->l2d_ws || !r->l2d_wse))
        return set_err(err, errlen, NLDSC_E_ARG, "a result array is NULL");
    const int M = p->n_snp, N = p->n_org;
    if (own_begin < 0 || own_end > M || own_begin > own_end)
        return set_err(err, errlen, NLDSC_E_ARG, "owned range [%d, %d) outside [0, %d)", own_begin, own_end, M);
    if (table_dev && (width <= 0 || width < own_end - own_begin))
        return set_err(err, errlen, NLDSC_E_ARG, "table width %d below the owned range's %d SNPs", width,
                       own_end - own_begin);
    if (split && (!table_dev || (export_cap > 0 && !export_dev)))
        return set_err(err, errlen, NLDSC_E_ARG, "split runs write a device table and need an export buffer");
    if (split && own_begin == own_end) return set_err(err, errlen, NLDSC_E_ARG, "split runs need an owned SNP");
    if (split && export_cap < p->n_snp - own_end)
        return set_err(err, errlen, NLDSC_E_ARG, "export capacity %d below the %d halo SNPs", export_cap,
                       p->n_snp - own_end);
    if (own_begin == own_end) {  // nothing owned: no kernel runs and no output is written (an empty GPU plan
        // would leave the left pointers unfilled); a device table is all NaN
        for (int k = 0; k < 6; ++k) e->ms[k] = 0.0;
        e->pairs = e->flop_alg = e->ops_alg_i8 = e->flop_issued = 0.0;
        e->n_band_items = 0;
        e->last_ksplit = 1;
        e->last_tail_ksplit = 1;
        e->last_round_items = 0;
        e->last_direct = -1;
        e->last_band_kernel = NLDSC_BAND_F4;
        if (table_dev) {
            HIPCHK(hipSetDevice(e->device));
            HIPCHK(e->sums.ensure(3));
            HIPCHK(hipMemsetAsync(e->sums.p, 0, 3 * sizeof(unsigned long long), e->stream));
            HIPCHK(nldsc::launch_pack_table(e->l2.p, e->l2d.p, e->maf.p, e->rstd.p, e->ws3.p, M, own_begin, own_end,
                                            width, table_dev, e->sums.p, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
        }
        return NLDSC_OK;
    }
    HIPCHK(hipSetDevice(e->device));
    // Host-result runs (nldsc_engine_run): where the owned slice lands.  `out_h` are host pointers (DMA targets),
    // `out_d` their device-mapped views (finalize_out_kernel writes them over the host link, no DMA after the band):
    // the caller's arrays themselves when they lie in nldsc_host_alloc buffers (`direct`), else the engine's pinned
    // landing buffer h_res, copied out by the host.  h_res also takes finalize's per-workgroup pair-count sums.
    const bool host_out = table_dev == nullptr;
    const int n_own = own_end - own_begin;
    const size_t b8 = sizeof(double) * (size_t)n_own, b4 = sizeof(int32_t) * (size_t)n_own;
    struct Out {
        double *l2, *l2d, *maf, *rstd;
        int32_t *wsa, *wsd, *wsde;
    } out_h = {}, out_d = {};
    bool direct = false;
    unsigned long long* wsum_h = nullptr;
    unsigned long long* wsum_d = nullptr;
    const int n_wsum = nldsc::finalize_out_blocks(n_own);
    e->last_direct = -1;
    if (host_out) {
        const size_t o = (size_t)own_begin, wsum_off = (4 * b8 + 3 * b4 + 7) / 8 * 8;
        HIPCHK(e->h_res.ensure(wsum_off + 2 * sizeof(unsigned long long) * (size_t)n_wsum));
        uint8_t* dres = nullptr;
        HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dres), e->h_res.p, 0));
        wsum_h = reinterpret_cast<unsigned long long*>(e->h_res.p + wsum_off);
        wsum_d = reinterpret_cast<unsigned long long*>(dres + wsum_off);
        const Out callers = {r->l2 + o, r->l2d + o, r->maf + o, r->residuals_std + o, r->l2_ws + o, r->l2d_ws + o,
                             r->l2d_wse + o};
        Out reg = {};
        reg.l2 = static_cast<double*>(registered_device_ptr(callers.l2, b8));
        reg.l2d = static_cast<double*>(registered_device_ptr(callers.l2d, b8));
        reg.maf = static_cast<double*>(registered_device_ptr(callers.maf, b8));
        reg.rstd = static_cast<double*>(registered_device_ptr(callers.rstd, b8));
        reg.wsa = static_cast<int32_t*>(registered_device_ptr(callers.wsa, b4));
        reg.wsd = static_cast<int32_t*>(registered_device_ptr(callers.wsd, b4));
        reg.wsde = static_cast<int32_t*>(registered_device_ptr(callers.wsde, b4));
        direct = reg.l2 && reg.l2d && reg.maf && reg.rstd && reg.wsa && reg.wsd && reg.wsde;
        e->last_direct = direct ? 1 : 0;
        if (direct) {
            out_h = callers;
            out_d = reg;
        } else {
            auto at = [&](uint8_t* base, size_t off) { return base + off; };
            out_h = {reinterpret_cast<double*>(at(e->h_res.p, 0)), reinterpret_cast<double*>(at(e->h_res.p, b8)),
                     reinterpret_cast<double*>(at(e->h_res.p, 2 * b8)), reinterpret_cast<double*>(at(e->h_res.p, 3 * b8)),
                     reinterpret_cast<int32_t*>(at(e->h_res.p, 4 * b8)),
                     reinterpret_cast<int32_t*>(at(e->h_res.p, 4 * b8 + b4)),
                     reinterpret_cast<int32_t*>(at(e->h_res.p, 4 * b8 + 2 * b4))};
            out_d = {reinterpret_cast<double*>(at(dres, 0)), reinterpret_cast<double*>(at(dres, b8)),
                     reinterpret_cast<double*>(at(dres, 2 * b8)), reinterpret_cast<double*>(at(dres, 3 * b8)),
                     reinterpret_cast<int32_t*>(at(dres, 4 * b8)), reinterpret_cast<int32_t*>(at(dres, 4 * b8 + b4)),
                     reinterpret_cast<int32_t*>(at(dres, 4 * b8 + 2 * b4))};
        }
    }
    const bool dom = !(p->flags & NLDSC_FLAG_ADDITIVE_ONLY);
    const bool strict = (p->flags & NLDSC_FLAG_STRICT_PLINK_ORDER) != 0;
    int path = (p->flags & NLDSC_FLAG_EXACT_F4) ? 2 : (p->flags & NLDSC_FLAG_EXACT_I8) ? 1
             : (p->flags & NLDSC_FLAG_FP32) ? 0 : e->band_mode;
    // fp4 Gram entries are <= 16N: the segmented fp4 kernel keeps them exact in int32 up to N < 2^27
    if (path == 2 && N >= (1 << 27)) path = 1;
    const bool use_i8 = path != 0, use_f4 = path == 2;
    // rows longer than one fp32-exact segment: the segmented kernel (single blocks, register strips)
    // fp32 items pair a row block with up to 2 column blocks (2 waves / SIMD); the exact paths take one
    const int max_nc = use_i8 ? 1 : 2;
    HIPCHK(hipSetDevice(e->device));
    hipStream_t st = e->stream;

    const int nb = N / 4 + (N % 4 > 0);
    const int row_bytes = row_pitch(N);
    const int pitch_words = row_bytes / 4;
    const int n_it = row_bytes / CHUNK_BYTES;
    const int nblk = (M + BLK - 1) / BLK;
    const int Mpad = nblk * BLK;
    // last .bed byte: bit pairs that are individuals for the reference (high pairs first,
    // stream.h:55-66) or for PLINK (low pairs first) — the rest are recoded as missing (-> 0)
    const int rem = N % 4;
    uint32_t tail_keep = 0xFFu;
    if (rem) tail_keep = strict ? (uint32_t)((1u << (2 * rem)) - 1u) : (uint32_t)(0xFFu << (8 - 2 * rem)) & 0xFFu;

    // the band kernels read the resident rows (Mpad rows at row_bytes pitch) in place
    const uint32_t* geno = reinterpret_cast<const uint32_t*>(e->bed.p);
    HIPCHK(e->counts.ensure((size_t)M * 4));
    HIPCHK(e->cparts.ensure((size_t)M * 3));
    HIPCHK(e->rep_count.ensure(1));  // (zeroed by the statistics kernel)
    HIPCHK(e->lut.ensure((size_t)Mpad * 4));
    HIPCHK(e->cst.ensure((size_t)Mpad));
    HIPCHK(e->sflags.ensure((size_t)Mpad));
    HIPCHK(e->blk_rep.ensure((size_t)nblk));
    HIPCHK(e->pos.ensure((size_t)M));
    HIPCHK(e->res.ensure(4 * (size_t)M + (3 * (size_t)M + 1) / 2));
    e->l2.p = e->res.p;
    e->l2d.p = e->l2.p + M;
    e->maf.p = e->l2d.p + M;
    e->rstd.p = e->maf.p + M;
    e->ws3.p = reinterpret_cast<int*>(e->rstd.p + M);
    HIPCHK(e->Lw.ensure((size_t)M));
    HIPCHK(e->Rw.ensure((size_t)M));
    HIPCHK(e->l2_acc.ensure((size_t)M));
    HIPCHK(e->l2d_acc.ensure((size_t)M));
    HIPCHK(e->ws_acc.ensure((size_t)M * 4));  // WSA, WSD, WSDE, non-finite flags

    // band schedule: on the GPU when every position is >= 0 and sorted (the kernels run ahead of the
    // count and the host only waits for two counters), else the host replay of the reference's pointers
    const bool nonneg_sorted = nldsc::positions_nonneg_sorted(p->positions, M);
    const bool sorted = nonneg_sorted || nldsc::positions_sorted(p->positions, M);
    const bool gpu_plan = e->gpu_plan && nonneg_sorted && max_nc == 1;
    // the 2 x 2 block-pair workgroups: fp4, unsegmented rows, GPU plan, and no K-split (choose_ksplit below); with
    // super-item routing (t2 modes 1 and 3) only when a missing-free block exists in this run's sample order (routing
    // takes none otherwise: C3 / C2 synthetic data, 1 % missing — the super plan, the compaction and two empty quad
    // launches cost ~50 us per run)
    const int order = strict ? 1 : 0;  // bit of row_miss: the individual slots of this run's sample order
    const bool t2_cand = e->t2_mode > 0 && gpu_plan && use_f4 && n_it <= nldsc::F4_SEG_CHUNKS && n_it >= 2 &&
                         (e->t2_mode == 2 || e->free_blocks[order] > 0);
    // additive-only fp4 items of two column blocks (GPU plan, unsegmented rows; no K-split: its partial kernel takes
    // single block pairs)
    const bool nc2 = e->f4_nc2 && gpu_plan && use_f4 && !dom && n_it <= nldsc::F4_SEG_CHUNKS;
    const bool routed = e->t2_mode == 1 || e->t2_mode == 3;
    const bool quad = e->t2_mode == 3;
    const int route_shift = quad ? 2 : 1;  // super-items of 2^route_shift blocks a side
    // K-split (f4, unsegmented rows) when the items fill the wave slots (2 per SIMD) in few, partly empty
    // rounds — a rank's shard of one chromosome — and splitting the K loop in P pieces fills them better
    // Model: a round of items takes ~0.67 us per K chunk (C3: 2 466 chunks, 1.65 ms per round, 12.7 rounds in
    // 20.9 ms); the split adds ~64 KiB of partial-tile traffic per piece at ~3 TB/s effective (measured: a 1/8
    // shard of C3, 3 300 items, band 3.35 -> 3.01 ms; a 1/2 shard, 13 000 items, P = 5 made it 7.5 % slower).
    auto choose_ksplit = [&](int n_items) {
        int ksplit = 1;
        if (use_f4 && !nc2 && n_items > 0 && n_it <= nldsc::F4_SEG_CHUNKS && e->ksplit_ok) {
            const double slots = 8.0 * (double)e->n_cu, t_round = 0.67e-6 * n_it;
            auto cost = [&](int P) {
                return std::ceil((double)n_items * P / slots) / P * t_round +
                       (P > 1 ? n_items * P * 65536.0 / 3e12 : 0.0);
            };
            double best = cost(1);
            for (int P = 2; P <= 8 && 2 * P <= n_it; ++P)
                if (cost(P) < 0.97 * best && (size_t)n_items * P * 32768 <= ((size_t)3 << 30)) {
                    best = cost(P);
                    ksplit = P;
                }
        }
        return ksplit;
    };
    int ksplit = 1;
    bool use_t2 = false;
    int n_items2 = 0;
    const bool fused_plan = gpu_plan && e->plan_fused && M <= nldsc::PLAN_SMALL_N;
    if (gpu_plan) {
        const size_t n_t = (size_t)(nblk + 15) / 16;
        // window edges A | E, then the right-pointer scan's tile maxima
        HIPCHK(e->Aw.ensure(2 * (size_t)M + (M + 255) / 256));
        HIPCHK(e->plan_rows.ensure((size_t)nblk));
        HIPCHK(e->plan_counts.ensure(n_t * n_t));
        HIPCHK(e->plan_meta.ensure(8));  // [0, 4) single-block plan, [4, 8) super-item plan
        HIPCHK(e->h_meta.ensure(8 * sizeof(int)));
        if (fused_plan) HIPCHK(e->items.ensure(nldsc::plan_small_items(M)));  // (emitted with the plan)
        if (t2_cand) {
            const size_t nblk2 = (size_t)(nblk + 1) / 2, n_t2 = (nblk2 + 15) / 16;
            HIPCHK(e->plan_rows2.ensure(nblk2));
            HIPCHK(e->plan_counts2.ensure(std::max<size_t>(n_t2 * n_t2, (size_t)nldsc::plan_super_counts(M, route_shift))));
        }
    }

    auto t_start = std::chrono::steady_clock::now();
    // The positions go up and the schedule's window edges are searched first (~0.02 ms: beside the count kernel, whose
    // streaming saturates HBM, those dependent loads took 0.05-0.1 ms on the critical path of short runs); then the
    // count kernel, with the rest of the schedule beside it on the plan stream.
    const size_t b_pos = sizeof(double) * (size_t)M;
    if (registered_device_ptr(p->positions, b_pos)) {  // (pinned: the DMA reads them in place)
        HIPCHK(hipMemcpyAsync(e->pos.p, p->positions, b_pos, hipMemcpyHostToDevice, st));
    } else {
        HIPCHK(e->h_pos.ensure(b_pos));
        const CopyPool::Seg seg = {e->h_pos.p, p->positions, b_pos};
        e->copies.copy(&seg, 1);
        HIPCHK(hipMemcpyAsync(e->pos.p, e->h_pos.p, b_pos, hipMemcpyHostToDevice, st));
    }
    if (gpu_plan) HIPCHK(nldsc::launch_plan_edges(e->pos.p, M, p->ld_wind, e->Aw.p, e->Aw.p + M, e->plan_meta.p, st));
    HIPCHK(hipEventRecord(e->ev_pos, st));
    // non-individual slots read as missing (0x55) for the int8 / fp32 kernels, as 00 (all fp4 planes zero) for fp4;
    // the genotype counts: the load's (every byte before the last) plus this run's last byte
    const uint32_t pad = use_f4 ? 0x00u : 0x55u;
    HIPCHK(hipEventRecord(e->ev[0], st));  // (count_ms: the tail kernel alone; the host total covers the above)
    HIPCHK(nldsc::launch_tail_counts(e->bed.p, e->lastb.p, M, nb, row_bytes, tail_keep, pad, e->lcounts.p,
                                     1, e->cparts.p, st));  // (the load's parts add into one: load_tiled_kernel)
    HIPCHK(hipEventRecord(e->ev[1], st));
    if (gpu_plan) {
        HIPCHK(hipStreamWaitEvent(e->plan_stream, e->ev_pos, 0));
        HIPCHK(nldsc::launch_plan(M, own_begin, own_end, e->Aw.p, e->Aw.p + M, e->Rw.p, e->plan_rows.p,
                                  e->plan_counts.p, e->plan_meta.p, e->plan_stream, nc2,
                                  fused_plan ? e->items.p : nullptr));
        if (t2_cand)
            HIPCHK(nldsc::launch_plan_super(M, e->plan_rows.p, e->plan_rows2.p, e->plan_counts2.p, e->plan_meta.p + 4,
                                            route_shift,
                                            e->plan_stream));
        for (int k = 0; k < 8; ++k) reinterpret_cast<volatile int*>(e->h_meta.p)[k] = -1;  // (counts land >= 0)
        HIPCHK(hipMemcpyAsync(e->h_meta.p, e->plan_meta.p, 8 * sizeof(int), hipMemcpyDeviceToHost, e->plan_stream));
        HIPCHK(hipEventRecord(e->ev_plan, e->plan_stream));
    }
    HIPCHK(nldsc::launch_snp_stats(e->cparts.p, 1, e->counts.p, e->rep_count.p,
                                   e->oriented ? e->flip.p : nullptr, e->pos.p, M, Mpad, N, p->maf, p->std_thr,
                                   e->lut.p, e->cst.p, e->sflags.p, e->maf.p, e->rstd.p, st, e->l2_acc.p, e->l2d_acc.p,
                                   e->ws_acc.p, e->blk_rep.p));
    // split runs: the pairs whose lower SNP is owned (flag bit 3), before the replay may touch the flags (ev_stats)
    if (split) HIPCHK(nldsc::launch_pair_range(e->sflags.p, M, own_begin, own_end, st));
    // rare variants: the reference's fp32 residual replayed (its sums assume N < 2^23); the flags per block here,
    // the replay itself after the schedule (below)
    const bool replay = N < (1 << 23) && !(p->flags & NLDSC_FLAG_EXACT_RARE);
    // Invariant of the overlap: the replay rewrites, for replayed SNPs only, sflags bit 1 (residual pass; a byte
    // read-modify-write), cst and lut.  What runs beside it on the main stream reads sflags bits 0 (MAF pass:
    // left_pointer_kernel, the host flag copy) and 2 (missing calls: the band kernels' rm / cm), which the
    // replay never changes, and never reads a replayed SNP's cst / lut before ev_replay: the items
    // of blocks holding one are skipped (skip_item) until the KC launch, and the K-split part kernel, which runs
    // them, stores Gram tiles without reading constants.  No other kernel writes sflags after snp_stats_kernel.
    if (replay) {
        HIPCHK(nldsc::launch_replay_flags(e->counts.p, e->oriented ? e->flip.p : nullptr, e->sflags.p, M,
                                          e->blk_rep.p, st, true));
        HIPCHK(hipEventRecord(e->ev_stats, st));
    }
    HIPCHK(hipEventRecord(e->ev[2], st));
    // What needs no schedule goes out before the host waits for it (C2 / a rank's shard: the count ends first, and
    // the host's enqueue after that wait is on the critical path): the left pointers (the window edges came before the
    // count), the blocks' missing flags (from the load) and the rare-variant replay — a few long sequential sums, on
    // the side stream beside the band launch for the items without a replayed SNP; only the KC launch and finalize
    // wait for it (ev_replay).  (Its sums assume N < 2^23.)
    hipStream_t cs = e->copy_stream, ps = e->plan_stream;
    if (gpu_plan) HIPCHK(nldsc::launch_left_pointers(e->Aw.p, e->sflags.p, e->pos.p, M, e->Lw.p, st));
    if (use_f4) {  // per 32-SNP block: holds a missing call (the kernels' m-product predicate: routing, issued count)
        HIPCHK(e->blk_miss.ensure((size_t)nblk));
        HIPCHK(nldsc::launch_block_missing_rows(e->row_miss.p, M, order, e->blk_miss.p, gpu_plan ? ps : st));
    }
    if (replay) {
        HIPCHK(hipStreamWaitEvent(cs, e->ev_stats, 0));
        HIPCHK(nldsc::launch_reference_residuals(e->bed.p, row_bytes, N, strict, e->counts.p,
                                                 e->oriented ? e->flip.p : nullptr, M, p->std_thr, e->cst.p, e->lut.p,
                                                 e->sflags.p, e->rstd.p, cs));
        HIPCHK(hipEventRecord(e->ev_replay, cs));
    }

    // ---- window replay + schedule ----
    auto t_host0 = std::chrono::steady_clock::now();
    int n_items = 0;
    bool compact = false;
    if (gpu_plan) {
        {  // the count kernel is running meanwhile; the host polls the pinned counters (a blocking event wait wakes
           // the thread tens of microseconds late: the schedule is on the critical path of short runs — a 1/8 shard,
           // C2 — whose count ends first), then the event confirms the whole copy
            (void)spin_until_nonneg(reinterpret_cast<volatile const int*>(e->h_meta.p) + 1);
            HIPCHK(hipEventSynchronize(e->ev_plan));
        }
        const int* meta = reinterpret_cast<const int*>(e->h_meta.p);
        n_items = meta[1];
        ksplit = choose_ksplit(n_items);
        // long rows: bands of at least round_min rounds of wave slots go in round launches (the last, partial round
        // K-split), not K-split whole — a 1/8 shard of C3 (1.6 rounds) band 2.70-2.76 -> 2.61-2.64 ms, a 1/4 shard
        // (3.2 rounds) 5.21-5.26 -> 4.87-4.89 ms (profiles/r03_ab_round_min.txt; was from 4 rounds on)
        // — in the single-block kernel, as the K-split it replaces: a shard's few super-items leave most CUs of the
        // 4 x 4 kernel idle (a missing-free 1/8 shard of C3: 2.88 ms with it, 1.93-1.99 K-split whole)
        bool rounds_forced = false;
        if (e->band_rounds && use_f4 && n_it >= 1024 && n_it <= nldsc::F4_SEG_CHUNKS &&
            n_items >= e->round_min * 8 * e->n_cu) {
            rounds_forced = ksplit > 1;
            ksplit = 1;
        }
        use_t2 = t2_cand && ksplit == 1 && n_items > 0 && !rounds_forced;
        // The work lists go out on the plan stream, beside the count kernel: the items, the super-items and, with
        // super-item routing (blk_miss, above), the list of the items the single-block kernel keeps, compacted in order,
        // so its launches (round launches, the K-split tail) are sized by its own work — its length reaches the host
        // before the band.  The main stream waits for them.
        if (use_t2) {
            n_items2 = meta[5];
            HIPCHK(e->items2.ensure(std::max<size_t>((size_t)n_items2, 1)));
            HIPCHK(nldsc::launch_plan_emit_super(M, e->plan_rows2.p, e->plan_meta.p + 4, e->plan_counts2.p,
                                                 e->items2.p, route_shift, ps));
        }
        if (!use_t2 || routed) {
            HIPCHK(e->items.ensure(std::max<size_t>((size_t)n_items, 1)));  // (fused: already holds them)
            if (n_items > 0 && !fused_plan)
                HIPCHK(nldsc::launch_plan_emit(M, e->plan_rows.p, e->plan_meta.p, e->plan_counts.p, e->items.p, ps,
                                               nc2));
        }
        compact = use_t2 && routed && n_items > 0;
        if (compact) {
            const size_t n_chunks = ((size_t)n_items + 255) / 256;  // (ld_kernels.hip COMPACT_CHUNK)
            HIPCHK(e->items_u.ensure((size_t)n_items));
            HIPCHK(e->compact_tmp.ensure(n_chunks + 1));
            HIPCHK(e->h_route.ensure(sizeof(int)));
            *reinterpret_cast<volatile int*>(e->h_route.p) = -1;  // (the copy below lands the count, >= 0)
            HIPCHK(nldsc::launch_compact_items(e->items.p, n_items, e->blk_miss.p, route_shift,
                                               nblk, e->compact_tmp.p,
                                               e->compact_tmp.p + n_chunks, e->items_u.p, ps));
            HIPCHK(hipMemcpyAsync(e->h_route.p, e->compact_tmp.p + n_chunks, sizeof(int), hipMemcpyDeviceToHost, ps));
        }
        HIPCHK(hipEventRecord(e->ev_route, ps));
        HIPCHK(hipStreamWaitEvent(st, e->ev_route, 0));  // the band reads the schedule and the lists
    } else {
    e->h_L.resize(M);
    e->h_R.resize(M);
    if (sorted) {
        // Sorted positions: nothing waits for the GPU.  The right pointers and the all-pass left
        // pointers do not depend on the MAF flags, and SNPs failing MAF only shrink the set of needed
        // block pairs (their L_j grow, their rows and columns drop), so the all-pass schedule is a
        // superset of the exact one; it is planned here while the GPU counts, and the exact left
        // pointers come from the device flags (left_pointer_kernel).  The kernels mask every pair
        // with the exact pointers.
        e->h_all_pass.assign(M, 1);
        nldsc::replay_windows(p->positions, e->h_all_pass.data(), M, p->ld_wind, e->h_L.data(), e->h_R.data());
        nldsc::plan_items(p->positions, e->h_all_pass.data(), M, p->ld_wind, e->h_L.data(), e->h_R.data(), own_begin,
                   own_end, max_nc, e->h_items);
    } else {
        // unsorted positions: the reference's sequential pointer semantics need the MAF flags first
        e->h_flags.resize(Mpad);
        HIPCHK(hipMemcpyAsync(e->h_flags.data(), e->sflags.p, Mpad, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        nldsc::replay_windows(p->positions, e->h_flags.data(), M, p->ld_wind, e->h_L.data(), e->h_R.data());
        nldsc::plan_items(p->positions, e->h_flags.data(), M, p->ld_wind, e->h_L.data(), e->h_R.data(), own_begin, own_end,
                   max_nc, e->h_items);
    }
    // the band kernel reads rows [32 I, 32 (J0 + nc)) of geno / lut: check before launching
    if (pitch_words % 8 != 0 || n_it * 8 != pitch_words)
        return set_err(err, errlen, NLDSC_E_ARG, "internal: bad row pitch %d", pitch_words);
    for (const nldsc::PlanItem& it : e->h_items)
        if (it.x < 0 || it.y < it.x || (it.z != 1 && it.z != 2) || it.y + it.z > nblk)
            return set_err(err, errlen, NLDSC_E_ARG, "internal: bad work item (%d, %d, %d) for %d blocks", it.x,
                           it.y, it.z, nblk);
    if (max_nc == 1) nldsc::order_items_tiled(e->h_items, nblk, TILE_R, TILE_C, e->h_scratch);
    HIPCHK(e->items.ensure(std::max<size_t>(e->h_items.size(), 1)));
    // the plan goes up through pinned staging: a copy from pageable memory would block this thread
    // until the stream drains (the count kernel), pinned copies are queued and return at once
    const size_t bL = sizeof(int) * (size_t)M, bI = sizeof(nldsc::PlanItem) * e->h_items.size();
    HIPCHK(e->h_stage.ensure(2 * bL + bI));
    std::memcpy(e->h_stage.p, e->h_L.data(), bL);
    std::memcpy(e->h_stage.p + bL, e->h_R.data(), bL);
    if (bI) std::memcpy(e->h_stage.p + 2 * bL, e->h_items.data(), bI);
    if (sorted) {
        HIPCHK(e->Aw.ensure((size_t)M));
        HIPCHK(hipMemcpyAsync(e->Aw.p, e->h_stage.p, bL, hipMemcpyHostToDevice, st));
        HIPCHK(nldsc::launch_left_pointers(e->Aw.p, e->sflags.p, e->pos.p, M, e->Lw.p, st));
    } else {
        HIPCHK(hipMemcpyAsync(e->Lw.p, e->h_stage.p, bL, hipMemcpyHostToDevice, st));
    }
    HIPCHK(hipMemcpyAsync(e->Rw.p, e->h_stage.p + bL, bL, hipMemcpyHostToDevice, st));
    if (bI) HIPCHK(hipMemcpyAsync(e->items.p, e->h_stage.p + 2 * bL, bI, hipMemcpyHostToDevice, st));
    n_items = (int)e->h_items.size();
    ksplit = choose_ksplit(n_items);
    }
    // (l2_acc, l2d_acc and ws_acc were zeroed by snp_stats_kernel)
    auto t_host1 = std::chrono::steady_clock::now();

    HIPCHK(hipEventRecord(e->ev[3], st));
    e->n_band_items = n_items;
    e->last_ksplit = ksplit;
    e->last_band_kernel = use_t2 ? (quad ? NLDSC_BAND_F4_QUAD : routed ? NLDSC_BAND_F4_ROUTED : NLDSC_BAND_F4_2X2) : !use_f4 ? (use_i8 ? NLDSC_BAND_I8 : NLDSC_BAND_F32)
                        : ksplit > 1 ? NLDSC_BAND_F4_KSPLIT : n_it > nldsc::F4_SEG_CHUNKS ? NLDSC_BAND_F4_SEG
                        : NLDSC_BAND_F4;
    if (ksplit > 1) HIPCHK(e->gram.ensure((size_t)n_items * ksplit * 8192));
    const int slots = 8 * e->n_cu;
    // which = 1: the launch for the items without a replayed SNP (beside the replay), 2: the KC launch after it
    const uint8_t* blk_rep = replay ? e->blk_rep.p : nullptr;
    int n_single = n_items;            // single-block items (compacted when routed)
    const int4* single = e->items.p;
    int round_items = 0, tail_p = 1, n_full = 0;
    // Unsegmented single-block fp4 items go in launches of one round of the wave slots each (2 per SIMD): the items
    // of a launch start together and, all of equal length, stay at nearby K offsets, so the waves on one XCD that
    // share a strip (the plan's 16 x 16 tiles) read it from that XCD's L2.  In one launch of all items the waves
    // drift apart and most strip bytes come from beyond L2 again (C3: 68 -> 14 GB per band, the clock 1.90 -> 2.02
    // GHz; band -2 to -4 % after the launch tails).  From one round of items on (round_min), only for long rows: the
    // waves of a round also reach their epilogues together, which then no longer overlap another wave's products —
    // at N = 50 000 (strips of 0.4 MB, L2-resident anyway; epilogue ~1/3 of an item) round launches made the band
    // 2.8 -> 5.1 ms.  The last, partial round leaves wave slots idle for a whole item length (C3: 1 458 items in
    // 2 048 slots); those items are K-split instead when the cost model finds it cheaper (C3: P = 7, 5 rounds of 1/7
    // of an item).
    // rare-variant items of the single-block fp4 kernel run their K loops in the main launch (Gram tiles kept), their
    // epilogues after the replay (launch_band_f4 rep_gram): unsegmented rows, no K-split of the whole band (whose
    // partial kernel already runs every item)
    bool defer = replay && e->defer_rep && use_f4 && ksplit == 1 && n_it <= nldsc::F4_SEG_CHUNKS;
    auto size_single = [&]() -> hipError_t {
        round_items = use_f4 && ksplit == 1 && e->band_rounds && n_it <= nldsc::F4_SEG_CHUNKS &&
                      n_it >= 1024 && n_single >= e->round_min * slots ? slots : 0;
        const int tail = round_items > 0 ? n_single % round_items : 0;
        tail_p = tail > 0 ? choose_ksplit(tail) : 1;
        n_full = tail_p > 1 ? n_single - tail : n_single;
        e->last_round_items = round_items;
        e->last_tail_ksplit = tail_p;
        // slots for every block pair of the main launch (an upper bound: which items hold a replayed SNP is known on
        // the device only); past REP_GRAM_MAX_SLOTS (32 KiB each) the KC launch after the replay runs those items
        // instead (a wide band of data with missing calls, where nearly every item stays in this kernel: ADVICE r03)
        if (defer && (size_t)n_full * (nc2 ? 2 : 1) > e->rep_gram_max_slots) defer = false;
        if (defer && n_full > 0) {
            const size_t slots = (size_t)n_full * (nc2 ? 2 : 1);
            hipError_t r = e->rep_gram.ensure(slots * 8192);
            if (r == hipSuccess) r = e->rep_items.ensure(slots);
            if (r != hipSuccess) return r;
        }
        return tail_p > 1 ? e->gram.ensure((size_t)tail * tail_p * 8192) : hipSuccess;
    };
    // per-SNP sums accumulate for the owned SNPs, or (split runs) for every SNP from own_begin on (the right halo's to
    // be exported)
    const int flush_hi = split ? M : own_end;
    auto launch_super = [&](int which) -> hipError_t {
        if (quad)
            return nldsc::launch_band_f4_q(dom, n_items2, geno, pitch_words, n_it, e->cst.p, e->items2.p,
                                           e->plan_rows.p, nblk, e->pos.p, e->Lw.p, e->Rw.p, e->sflags.p, M,
                                           p->ld_wind, (double)N, p->rsq_thr, own_begin, flush_hi, e->l2_acc.p,
                                           e->l2d_acc.p, e->ws_acc.p, true, blk_rep, e->blk_miss.p, which, st,
                                           e->q_rounds && n_items2 >= 16 * e->n_cu ? e->n_cu : 0);
        return nldsc::launch_band_f4_t2(
            dom, n_items2, geno, pitch_words, n_it, e->cst.p, e->items2.p, e->plan_rows.p, nblk, e->pos.p, e->Lw.p,
            e->Rw.p, e->sflags.p, M, p->ld_wind, (double)N, p->rsq_thr, own_begin, flush_hi, e->l2_acc.p, e->l2d_acc.p,
            e->ws_acc.p, true, blk_rep, routed ? e->blk_miss.p : nullptr, which, st);
    };
    // (column-block pair items: the compaction keeps an item while one of its blocks is unrouted, the kernel drops
    // the other)
    const uint8_t* single_miss =
        use_t2 && routed && (!compact || nc2) ? e->blk_miss.p : nullptr;
    auto launch_single = [&](int which) -> hipError_t {
        if (use_f4 && ksplit > 1)
            return nldsc::launch_band_f4_split(dom, ksplit, n_single, geno, pitch_words, n_it, e->cst.p, single,
                                               e->pos.p, e->Lw.p, e->Rw.p, e->sflags.p, M, p->ld_wind, (double)N,
                                               p->rsq_thr, own_begin, flush_hi, e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p,
                                               blk_rep, e->gram.p, which, st);
        if (use_f4) {
            const bool dfr = defer && n_full > 0;
            hipError_t r = nldsc::launch_band_f4(dom, nc2 ? 2 : 1, n_full, geno, pitch_words, n_it, e->cst.p, single,
                                                 e->pos.p, e->Lw.p, e->Rw.p, e->sflags.p, M, p->ld_wind, (double)N,
                                                 p->rsq_thr, own_begin, flush_hi, e->l2_acc.p, e->l2d_acc.p,
                                                 e->ws_acc.p, true, blk_rep, which, st, single_miss, round_items,
                                                 route_shift,
                                                 dfr ? e->rep_gram.p : nullptr, dfr ? e->rep_items.p : nullptr,
                                                 dfr ? e->rep_count.p : nullptr);
            if (r == hipSuccess && dfr && (which & 2))  // after the replay: the deferred items' epilogues
                r = nldsc::launch_band_f4_deferred_epi(dom, n_full * (nc2 ? 2 : 1), e->cst.p, e->rep_items.p,
                                                       e->rep_count.p, e->rep_gram.p, e->pos.p, e->Lw.p, e->Rw.p,
                                                       e->sflags.p, M, p->ld_wind, (double)N, p->rsq_thr, own_begin,
                                                       flush_hi, e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, blk_rep, st);
            if (r != hipSuccess || n_full == n_single) return r;
            return nldsc::launch_band_f4_split(dom, tail_p, n_single - n_full, geno, pitch_words, n_it, e->cst.p,
                                               single + n_full, e->pos.p, e->Lw.p, e->Rw.p, e->sflags.p, M,
                                               p->ld_wind, (double)N, p->rsq_thr, own_begin, flush_hi, e->l2_acc.p,
                                               e->l2d_acc.p, e->ws_acc.p, blk_rep, e->gram.p, which, st, single_miss,
                                               route_shift);
        }
        return nldsc::launch_band_i8(dom, max_nc, n_single, geno, pitch_words, n_it, e->cst.p, single, e->pos.p,
                                     e->Lw.p, e->Rw.p, e->sflags.p, M, p->ld_wind, (double)N, p->rsq_thr, own_begin,
                                     flush_hi, e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, true, blk_rep, which, st);
    };
    const bool run_single = !use_t2 || routed;  // (option t2 = 2: every block pair in the 2 x 2 workgroups)
    if (n_items > 0 && (use_f4 || use_i8)) {
        if (use_t2) HIPCHK(launch_super(1));
        if (e->debug_timing) HIPCHK(hipEventRecord(e->ev_dbg[0], st));
        const auto t_wait0 = std::chrono::steady_clock::now();
        if (compact) {  // the super-item kernel is queued: the host waits for the compacted count meanwhile
            // (polling the pinned word the copy lands in: a blocking event wait wakes the thread tens of
            // microseconds late, time the GPU would idle when the super-item kernel has nothing to do)
            volatile int* cnt = reinterpret_cast<volatile int*>(e->h_route.p);
            (void)spin_until_nonneg(cnt);
            HIPCHK(hipEventSynchronize(e->ev_route));  // (returns at once when the count has landed)
            n_single = *cnt;
            single = e->items_u.p;
        } else if (use_t2 && routed) {
            single = e->items.p;  // (no compaction: every item listed, the routed ones return at once)
        }
        HIPCHK(size_single());
        const auto t_wait1 = std::chrono::steady_clock::now();
        if (e->debug_timing) HIPCHK(hipEventRecord(e->ev_dbg[1], st));
        if (run_single) HIPCHK(launch_single(1));
        if (e->debug_timing) {
            HIPCHK(hipStreamSynchronize(st));
            float a = 0, b = 0;
            HIPCHK(hipEventElapsedTime(&a, e->ev[3], e->ev_dbg[0]));
            HIPCHK(hipEventElapsedTime(&b, e->ev_dbg[0], e->ev_dbg[1]));
            std::fprintf(stderr, "[nldsc debug] super %.3f ms, gap to single %.3f ms, host wait %.3f ms, n_single %d/%d\n",
                         a, b, std::chrono::duration<double, std::milli>(t_wait1 - t_wait0).count(), n_single, n_items);
        }
        if (replay) {
            HIPCHK(hipStreamWaitEvent(st, e->ev_replay, 0));
            if (use_t2) HIPCHK(launch_super(2));
            if (run_single) HIPCHK(launch_single(2));
        }
    } else {
        HIPCHK(size_single());
        if (replay) HIPCHK(hipStreamWaitEvent(st, e->ev_replay, 0));  // the fp32 path reads the replayed tables
    }
    if (n_items > 0 && !use_f4 && !use_i8) {
        HIPCHK(nldsc::launch_band(dom, 2, n_items, geno, pitch_words, n_it,
                                      e->lut.p, e->items.p, e->pos.p, e->Lw.p, e->Rw.p, e->sflags.p, M, p->ld_wind,
                                      (double)N, p->rsq_thr, own_begin, flush_hi, e->l2_acc.p, e->l2d_acc.p,
                                      e->ws_acc.p, st));
    }
    e->last_path = path;
    HIPCHK(hipEventRecord(e->ev[4], st));
    // matrix-core products the band kernels issued, counted on the GPU per work item as each kernel decides them
    // (missing-free blocks skip the m products, diagonal blocks the transposed ones, routed items run in the 2 x 2
    // kernel): sums[2], counted beside the band on the copy stream (after the work lists: ev[3]) and landed in
    // h_sums[2] (ev_issued); sums[0..1] are the device-table run's pair counts
    HIPCHK(e->sums.ensure(3));
    HIPCHK(e->h_sums.ensure(3 * sizeof(unsigned long long)));
    HIPCHK(hipStreamWaitEvent(cs, e->ev[3], 0));
    HIPCHK(hipMemsetAsync(e->sums.p + 2, 0, sizeof(unsigned long long), cs));
    HIPCHK(nldsc::launch_issued_products(single, run_single ? n_single : 0, use_t2 ? e->items2.p : nullptr,
                                         n_items2, gpu_plan ? e->plan_rows.p : nullptr,
                                         use_f4 ? e->blk_miss.p : nullptr, nblk, path, dom,
                                         (use_t2 && routed ? 2 : 0) | (single_miss != nullptr ? 1 : 0), route_shift,
                                         e->sums.p + 2, cs));
    HIPCHK(hipMemcpyAsync(e->h_sums.p + 2 * sizeof(unsigned long long), e->sums.p + 2, sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, cs));
    HIPCHK(hipEventRecord(e->ev_issued, cs));
    if (split) {  // the right halo's sums out; finalize waits for the left neighbour's (run_device_finish)
        HIPCHK(nldsc::launch_export_acc(e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, M, own_end, M, export_dev, st));
        HIPCHK(hipStreamSynchronize(st));
        *export_n = M - own_end;
        float f = 0;
        HIPCHK(hipEventElapsedTime(&f, e->ev[0], e->ev[1])); e->ms[0] = f;
        HIPCHK(hipEventElapsedTime(&f, e->ev[1], e->ev[2])); e->ms[1] = f;
        e->ms[2] = std::chrono::duration<double, std::milli>(t_host1 - t_host0).count();
        HIPCHK(hipEventElapsedTime(&f, e->ev[3], e->ev[4])); e->ms[3] = f;
        e->split_ms1 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        e->split_pending = true;
        e->split_M = M;
        e->split_N = N;
        e->split_dom = dom;
        e->split_own = {own_begin, own_end};
        e->split_row_bytes = row_bytes;
        e->split_table = table_dev;
        e->split_width = width;
        return NLDSC_OK;
    }
    double sw = 0, sd = 0;
    if (table_dev) {
        // the owned slice stays on the device (the caller gathers it device to device); only the pair counts of
        // the metric come back
        HIPCHK(nldsc::launch_finalize(e->Lw.p, e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, M, own_begin, own_end, dom,
                                      e->l2.p, e->l2d.p, e->ws3.p, st));
        HIPCHK(hipEventRecord(e->ev[5], st));
        HIPCHK(hipMemsetAsync(e->sums.p, 0, 2 * sizeof(unsigned long long), st));
        HIPCHK(nldsc::launch_pack_table(e->l2.p, e->l2d.p, e->maf.p, e->rstd.p, e->ws3.p, M, own_begin, own_end, width,
                                        table_dev, e->sums.p, st));
        HIPCHK(hipMemcpyAsync(e->h_sums.p, e->sums.p, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const unsigned long long* s = reinterpret_cast<const unsigned long long*>(e->h_sums.p);
        sw = (double)s[0];
        sd = dom ? (double)s[1] : 0.0;
    } else {
        // Host results: finalize writes the owned slice's seven columns straight into host memory (out_d) with its
        // per-workgroup pair-count sums — no pack kernel, no copy engine (the runtime moves device-to-pinned copies
        // with blit kernels: a 0.6 MB RSTD copy beside the C2 band took ~1 ms of its CU slots); without `direct`, the
        // host copies them from the landing buffer to the caller's arrays.
        HIPCHK(nldsc::launch_finalize_out(e->Lw.p, e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, e->maf.p, e->rstd.p, M,
                                          own_begin, own_end, dom, out_d.l2, out_d.l2d, out_d.maf, out_d.rstd,
                                          out_d.wsa, out_d.wsd, out_d.wsde, wsum_d, st));
        HIPCHK(hipEventRecord(e->ev[5], st));
        const size_t o = own_begin;
        using clk = std::chrono::steady_clock;
        clk::time_point tq[5];
        tq[2] = clk::now();
        HIPCHK(hipStreamSynchronize(st));
        tq[3] = clk::now();
        if (!direct) {
            const CopyPool::Seg segs[7] = {{r->l2 + o, out_h.l2, b8},           {r->l2d + o, out_h.l2d, b8},
                                           {r->maf + o, out_h.maf, b8},         {r->residuals_std + o, out_h.rstd, b8},
                                           {r->l2_ws + o, out_h.wsa, b4},       {r->l2d_ws + o, out_h.wsd, b4},
                                           {r->l2d_wse + o, out_h.wsde, b4}};
            e->copies.copy(segs, 7);
        }
        unsigned long long ta = 0, td = 0;
        for (int b = 0; b < n_wsum; ++b) {
            ta += wsum_h[2 * b];
            td += wsum_h[2 * b + 1];
        }
        sw = (double)ta;
        sd = dom ? (double)td : 0.0;
        tq[4] = clk::now();
        if (e->debug_timing) {
            auto ms = [&](int a, int b) { return std::chrono::duration<double, std::milli>(tq[b] - tq[a]).count(); };
            std::fprintf(stderr, "[nldsc debug] host results (%s): band wait %.3f, copies and sums %.3f ms\n",
                         direct ? "direct" : "landing buffer", ms(2, 3), ms(3, 4));
        }
    }
    {
        const auto t0 = std::chrono::steady_clock::now();
        HIPCHK(hipEventSynchronize(e->ev_issued));
        if (e->debug_timing)
            std::fprintf(stderr, "[nldsc debug] issued-count wait %.3f ms\n",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    auto t_end = std::chrono::steady_clock::now();

    float f = 0;
    HIPCHK(hipEventElapsedTime(&f, e->ev[0], e->ev[1])); e->ms[0] = f;
    HIPCHK(hipEventElapsedTime(&f, e->ev[1], e->ev[2])); e->ms[1] = f;
    e->ms[2] = std::chrono::duration<double, std::milli>(t_host1 - t_host0).count();
    HIPCHK(hipEventElapsedTime(&f, e->ev[3], e->ev[4])); e->ms[3] = f;
    HIPCHK(hipEventElapsedTime(&f, e->ev[4], e->ev[5])); e->ms[4] = f;
    e->ms[5] = std::chrono::duration<double, std::milli>(t_end - t_start).count();
    if (e->debug_timing) {  // where a run's wall time goes: GPU stages, the gap before the band, host tail
        float g23 = 0, g05 = 0;
        HIPCHK(hipEventElapsedTime(&g23, e->ev[2], e->ev[3]));
        HIPCHK(hipEventElapsedTime(&g05, e->ev[0], e->ev[5]));
        std::fprintf(stderr, "[nldsc debug] count %.3f stats %.3f gap-to-band %.3f band %.3f finalize %.3f | GPU span %.3f, "
                     "host total %.3f (host wait for the plan %.3f)\n", e->ms[0], e->ms[1], g23, e->ms[3], e->ms[4], g05,
                     e->ms[5], e->ms[2]);
    }
    e->flop_issued = (double)reinterpret_cast<const unsigned long long*>(e->h_sums.p)[2] * 2.0 * BLK * BLK *
                     (double)row_bytes * 4.0;
    e->pairs = sw;
    // BASELINE.md metric: FLOP_alg = 2N(1/2 sum WSA + sum WSD); additive-only 2N * 1/2 sum WSA
    e->flop_alg = 2.0 * (double)N * (0.5 * sw + sd);
    // exact formulation: 4 integer dot products per unordered additive pair (xx, xo, ox, oo) and
    // 2 per ordered dominance pair (xh, oh): 2N (4 * 1/2 sum WSA + 2 sum WSD) int8 ops
    e->ops_alg_i8 = 2.0 * (double)N * (2.0 * sw + 2.0 * sd);
    return NLDSC_OK;
}

}  // namespace

extern "C" {

int nldsc_engine_run(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end,
                     nldsc_ld_result* r, char* err, size_t errlen) {
    if (!r) return set_err(err, errlen, NLDSC_E_ARG, "NULL argument");
    return run_impl(e, p, own_begin, own_end, r, nullptr, 0, err, errlen);
}

int nldsc_engine_run_device(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end,
                            double* table_dev, int32_t width, char* err, size_t errlen) {
    if (!table_dev) return set_err(err, errlen, NLDSC_E_ARG, "NULL table");
    return run_impl(e, p, own_begin, own_end, nullptr, table_dev, width, err, errlen);
}

int nldsc_engine_run_device_split(nldsc_engine* e, const nldsc_ld_params* p, int32_t own_begin, int32_t own_end,
                                  double* table_dev, int32_t width, int64_t* export_dev, int32_t export_cap,
                                  int32_t* export_n, char* err, size_t errlen) {
    if (!table_dev || !export_n) return set_err(err, errlen, NLDSC_E_ARG, "NULL table or export count");
    return run_impl(e, p, own_begin, own_end, nullptr, table_dev, width, err, errlen,
                    reinterpret_cast<long long*>(export_dev), export_cap, export_n);
}

int nldsc_engine_run_device_finish(nldsc_engine* e, const int64_t* import_dev, int32_t import_n, char* err,
                                   size_t errlen) {
    if (!e) return set_err(err, errlen, NLDSC_E_ARG, "NULL engine");
    if (!e->split_pending) return set_err(err, errlen, NLDSC_E_ARG, "no split run to finish");
    const int32_t M = e->split_M, lo = e->split_own.first, hi = e->split_own.second;
    if (import_n < 0 || import_n > hi - lo || (import_n > 0 && !import_dev))
        return set_err(err, errlen, NLDSC_E_ARG, "import of %d SNPs into an owned range of %d", import_n, hi - lo);
    e->split_pending = false;
    HIPCHK(hipSetDevice(e->device));
    hipStream_t st = e->stream;
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHK(nldsc::launch_import_acc(e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, M, lo, import_n,
                                    reinterpret_cast<const long long*>(import_dev), st));
    HIPCHK(hipEventRecord(e->ev[4], st));
    HIPCHK(nldsc::launch_finalize(e->Lw.p, e->l2_acc.p, e->l2d_acc.p, e->ws_acc.p, M, lo, hi, e->split_dom, e->l2.p,
                                  e->l2d.p, e->ws3.p, st));
    HIPCHK(hipEventRecord(e->ev[5], st));
    HIPCHK(hipMemsetAsync(e->sums.p, 0, 2 * sizeof(unsigned long long), st));
    HIPCHK(nldsc::launch_pack_table(e->l2.p, e->l2d.p, e->maf.p, e->rstd.p, e->ws3.p, M, lo, hi, e->split_width,
                                    e->split_table, e->sums.p, st));
    HIPCHK(hipMemcpyAsync(e->h_sums.p, e->sums.p, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipEventSynchronize(e->ev_issued));  // (h_sums[2]: the first call's issued-product count)
    const unsigned long long* s = reinterpret_cast<const unsigned long long*>(e->h_sums.p);
    const double sw = (double)s[0], sd = e->split_dom ? (double)s[1] : 0.0, N = (double)e->split_N;
    float f = 0;
    HIPCHK(hipEventElapsedTime(&f, e->ev[4], e->ev[5])); e->ms[4] = f;
    const auto t1 = std::chrono::steady_clock::now();
    // (total: both calls' host time, without the exchange between them)
    e->ms[5] = e->split_ms1 + std::chrono::duration<double, std::milli>(t1 - t0).count();
    e->flop_issued = (double)s[2] * 2.0 * BLK * BLK * (double)e->split_row_bytes * 4.0;
    e->pairs = sw;
    e->flop_alg = 2.0 * N * (0.5 * sw + sd);
    e->ops_alg_i8 = 2.0 * N * (2.0 * sw + 2.0 * sd);
    return NLDSC_OK;
}

int nldsc_engine_timings(const nldsc_engine* e, double* ms6, double* flop_alg, double* flop_issued,
                         double* pairs, int32_t* n_band_items) {
    if (!e) return NLDSC_E_ARG;
    if (ms6) for (int k = 0; k < 6; ++k) ms6[k] = e->ms[k];
    if (flop_alg) *flop_alg = e->flop_alg;
    if (flop_issued) *flop_issued = e->flop_issued;
    if (pairs) *pairs = e->pairs;
    if (n_band_items) *n_band_items = e->n_band_items;
    return NLDSC_OK;
}

int nldsc_engine_path(const nldsc_engine* e, int32_t* exact_i8, double* ops_alg_i8) {
    if (!e) return NLDSC_E_ARG;
    if (exact_i8) *exact_i8 = e->last_path;
    if (ops_alg_i8) *ops_alg_i8 = e->ops_alg_i8;
    return NLDSC_OK;
}

int nldsc_engine_ksplit(const nldsc_engine* e) { return e ? e->last_ksplit : NLDSC_E_ARG; }
int nldsc_engine_band_round_items(const nldsc_engine* e) { return e ? e->last_round_items : NLDSC_E_ARG; }
int nldsc_engine_band_tail_ksplit(const nldsc_engine* e) { return e ? e->last_tail_ksplit : NLDSC_E_ARG; }
int nldsc_engine_band_kernel(const nldsc_engine* e) { return e ? e->last_band_kernel : NLDSC_E_ARG; }

int nldsc_engine_result_direct(const nldsc_engine* e) { return e ? e->last_direct : NLDSC_E_ARG; }

int nldsc_ld_calculate(const nldsc_ld_params* p, nldsc_ld_result* r, char* err, size_t errlen) {
    if (!p || !r || !p->bedfile) return set_err(err, errlen, NLDSC_E_ARG, "NULL argument");
    nldsc_engine* e = nullptr;
    int rc = nldsc_engine_create(p->device, &e, err, errlen);
    if (rc) return rc;
    rc = nldsc_engine_load_bed_file(e, p->bedfile, p->n_snp, p->n_org, err, errlen);
    if (!rc) rc = nldsc_engine_run(e, p, 0, p->n_snp, r, err, errlen);
    nldsc_engine_destroy(e);
    return rc;
}

int nldsc_synth_bed_device(int32_t device, void* bed_dev, int32_t n_snp, int32_t n_org, const float* thr_host,
                           float rho, float missing, uint64_t seed, char* err, size_t errlen) {
    if (!bed_dev || !thr_host) return set_err(err, errlen, NLDSC_E_ARG, "NULL argument");
    int rc = check_dims(n_snp, n_org, err, errlen);
    if (rc) return rc;
    int d = 0;
    rc = use_device(device, &d, err, errlen);
    if (rc) return rc;
    const int nb = n_org / 4 + (n_org % 4 > 0);
    float* thr = nullptr;
    HIPCHK(hipMalloc(&thr, sizeof(float) * n_snp));
    hipError_t he = hipMemcpy(thr, thr_host, sizeof(float) * n_snp, hipMemcpyHostToDevice);
    const uint8_t magic[3] = {0x6c, 0x1b, 0x01};
    if (he == hipSuccess) he = hipMemcpy(bed_dev, magic, 3, hipMemcpyHostToDevice);
    if (he == hipSuccess)
        he = nldsc::launch_synth_bed((uint8_t*)bed_dev + 3, n_snp, n_org, nb, thr, rho, missing, seed, nullptr);
    if (he == hipSuccess) he = hipDeviceSynchronize();
    (void)hipFree(thr);
    if (he != hipSuccess) return set_err(err, errlen, NLDSC_E_HIP, "HIP error %s in synth", hipGetErrorString(he));
    return NLDSC_OK;
}

}  // extern "C"
