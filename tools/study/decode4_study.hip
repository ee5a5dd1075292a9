// Study (not product code): would a resident layout of 4-bit pre-spread codes (the v plane at nibble bits 2:1 as
// today, the missing indicator at bit 0) feed the 8-product fp4 loop better than the 2-bit codes decoded in
// registers?  Per K step and operand a lane needs 32 codes: 2 words of 2-bit codes (9 VALU each: 18) or 4 dwords of
// 4-bit codes (x = w & 0x66666666, h = w & 0x44444444 with E8M0 scale 2^-1, m = w & 0x11111111 with scale 2^1: 12).
// Same MFMA work (8 products of 32x32x64 per K step), 2 waves per SIMD on every CU, genotype-like operands (1 %
// missing); operands in registers (an empty asm keeps the compiler from hoisting the decode) or loaded from a strip
// pair that stays in L2 (the 4-bit strip twice the bytes).  Interleave as the band kernel: VPM VALU per MFMA.
//   hipcc --offload-arch=gfx950 -O3 -o decode4_study tools/study/decode4_study.hip && ./decode4_study [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int SA, int SB>
__device__ __forceinline__ f32x16 m32(const i32x4& a, const i32x4& b, const f32x16& c) {
    const i32x8 A = {a[0], a[1], a[2], a[3], 0, 0, 0, 0}, B = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 4, 4, 0, SA, 0, SB);
}
struct Fr { i32x4 v, h, m; };

__device__ __forceinline__ void dec2(uint32_t w, int& x0, int& x1, int& h0, int& h1, int& o0, int& o1) {
    constexpr uint32_t M = 0x22222222u, K6 = 0x66666666u;
    const uint32_t s1 = w << 1, s2 = w >> 1, w2 = w >> 2;
    x0 = (int)(s1 & K6); x1 = (int)(s2 & K6); h0 = (int)(w & M); h1 = (int)(w2 & M);
    o0 = (int)(s1 & ~w & M); o1 = (int)(s2 & ~w2 & M);
}
__device__ __forceinline__ Fr decode2(uint32_t wa, uint32_t wb) {
    int x0, x1, x2, x3, h0, h1, h2, h3, o0, o1, o2, o3;
    dec2(wa, x0, x1, h0, h1, o0, o1); dec2(wb, x2, x3, h2, h3, o2, o3);
    Fr f; f.v = i32x4{x0, x1, x2, x3}; f.h = i32x4{h0, h1, h2, h3}; f.m = i32x4{o0, o1, o2, o3};
    return f;
}
__device__ __forceinline__ Fr decode4(const uint4 q) {
    Fr f;
    f.v = i32x4{(int)(q.x & 0x66666666u), (int)(q.y & 0x66666666u), (int)(q.z & 0x66666666u), (int)(q.w & 0x66666666u)};
    f.h = i32x4{(int)(q.x & 0x44444444u), (int)(q.y & 0x44444444u), (int)(q.z & 0x44444444u), (int)(q.w & 0x44444444u)};
    f.m = i32x4{(int)(q.x & 0x11111111u), (int)(q.y & 0x11111111u), (int)(q.z & 0x11111111u), (int)(q.w & 0x11111111u)};
    return f;
}
// 8 products, h at 1.0 (2-bit decode) or 2.0 with scale 2^-1 and m at 0.5 with scale 2^1 (4-bit)
template <bool F4>
__device__ __forceinline__ void step(const Fr& a, const Fr& b, f32x16 (&g)[8]) {
    constexpr int H = F4 ? 126 : 127, MS = F4 ? 128 : 127;
    g[0] = m32<127, 127>(a.v, b.v, g[0]); g[1] = m32<127, MS>(a.v, b.m, g[1]); g[2] = m32<127, H>(a.v, b.h, g[2]);
    g[3] = m32<MS, 127>(a.m, b.v, g[3]); g[4] = m32<H, 127>(a.h, b.v, g[4]); g[5] = m32<MS, MS>(a.m, b.m, g[5]);
    g[6] = m32<MS, H>(a.m, b.h, g[6]); g[7] = m32<H, MS>(a.h, b.m, g[7]);
}
template <int VPM>
__device__ __forceinline__ void interleave() {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
    }
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t gcode(uint32_t seed) {  // genotype-like 2-bit code
    const uint32_t r = hash32(seed) & 1023u;
    return r < 10 ? 1u : r < 430 ? 2u : r < 520 ? 3u : 0u;
}
__host__ __device__ __forceinline__ uint32_t nib4(uint32_t code) {  // v at bits 2:1, m at bit 0
    return (code << 1) | (code == 1 ? 1u : 0u);
}

// MODE 0: 2-bit codes in registers; 1: 4-bit words in registers; 2: 2-bit from the L2 strip; 3: 4-bit from L2.
// One iteration = 2 K steps.
template <int MODE>
__global__ void __launch_bounds__(64, 2) kloop(float* out, const uint4* strip, int iters, int units) {
    constexpr bool F4 = MODE & 1;
    const int lane = threadIdx.x;
    const uint32_t base = (blockIdx.x * 64 + lane) * 64;
    f32x16 g[8];
    for (int p = 0; p < 8; ++p) g[p] = f32x16{};
    if constexpr (MODE < 2) {
        uint4 r[4];  // F4: [a0, a1, b0, b1] of 32 codes each; else r[0] = a (64 codes), r[1] = b
        for (int q = 0; q < 4; ++q) {
            uint32_t w[4];
            for (int d = 0; d < 4; ++d) {
                uint32_t x = 0;
                if (F4) for (int k = 0; k < 8; ++k) x |= nib4(gcode(base + q * 32 + d * 8 + k)) << (4 * k);
                else for (int k = 0; k < 16; ++k) x |= gcode(base + q * 64 + d * 16 + k) << (2 * k);
                w[d] = x;
            }
            r[q] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(r[q].x), "+v"(r[q].y), "+v"(r[q].z), "+v"(r[q].w));
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                Fr a, b;
                if constexpr (F4) { a = decode4(r[s]); b = decode4(r[2 + s]); }
                else { a = s ? decode2(r[0].z, r[0].w) : decode2(r[0].x, r[0].y);
                       b = s ? decode2(r[1].z, r[1].w) : decode2(r[1].x, r[1].y); }
                step<F4>(a, b, g);
                interleave<F4 ? 3 : 4>();
            }
        }
    } else {
        // strip pair: 2-bit: one uint4 per lane and operand per 2 K steps; 4-bit: two
        constexpr int PER = F4 ? 2 : 1;
        int off = lane;
        uint4 pa[PER], pb[PER], qa[PER], qb[PER];
        for (int k = 0; k < PER; ++k) { pa[k] = strip[off + 64 * k]; pb[k] = strip[units + off + 64 * k]; }
        off += 64 * PER;
        for (int k = 0; k < PER; ++k) { qa[k] = strip[off + 64 * k]; qb[k] = strip[units + off + 64 * k]; }
        off += 64 * PER;
        for (int it = 0; it < iters; ++it) {
            uint4 ca[PER], cb[PER];
#pragma unroll
            for (int k = 0; k < PER; ++k) { ca[k] = pa[k]; cb[k] = pb[k]; pa[k] = qa[k]; pb[k] = qb[k]; }
            if (off + 64 * PER > units) off = lane;
#pragma unroll
            for (int k = 0; k < PER; ++k) { qa[k] = strip[off + 64 * k]; qb[k] = strip[units + off + 64 * k]; }
            off += 64 * PER;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                Fr a, b;
                if constexpr (F4) { a = decode4(ca[s]); b = decode4(cb[s]); }
                else { a = s ? decode2(ca[0].z, ca[0].w) : decode2(ca[0].x, ca[0].y);
                       b = s ? decode2(cb[0].z, cb[0].w) : decode2(cb[0].x, cb[0].y); }
                step<F4>(a, b, g);
                interleave<F4 ? 3 : 4>();
            }
        }
    }
    float acc = 0.f;
    for (int p = 0; p < 8; ++p)
        for (int r = 0; r < 16; ++r) acc += g[p][r];
    out[blockIdx.x * 64 + lane] = acc;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    const int grid = 256 * 8;  // 2 waves per SIMD on every CU
    float* out;
    hipMalloc(&out, grid * 64 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const double flop = (double)grid * iters * 16 * 2.0 * 32 * 32 * 64;
    // a C3-like strip pair: 2 x 32 rows x 315 599 samples; 2-bit: 2 x 78 912 x 32 B; the 4-bit strip twice that
    const int units2 = 78912 * 32 / 16;  // uint4 per 2-bit strip
    uint4 *s2, *s4;
    hipMalloc(&s2, (size_t)2 * units2 * sizeof(uint4));
    hipMalloc(&s4, (size_t)4 * units2 * sizeof(uint4));
    {
        uint32_t* h2 = (uint32_t*)malloc((size_t)2 * units2 * 16);
        uint32_t* h4 = (uint32_t*)malloc((size_t)4 * units2 * 16);
        for (size_t k = 0; k < (size_t)2 * units2 * 4; ++k) {
            uint32_t w = 0, lo = 0, hi = 0;
            for (int j = 0; j < 16; ++j) {
                const uint32_t r = (uint32_t)((k * 16 + j) * 2654435761u) >> 22;
                const uint32_t c = r < 10 ? 1u : r < 430 ? 2u : r < 520 ? 3u : 0u;
                w |= c << (2 * j);
                if (j < 8) lo |= nib4(c) << (4 * j); else hi |= nib4(c) << (4 * (j - 8));
            }
            h2[k] = w; h4[2 * k] = lo; h4[2 * k + 1] = hi;
        }
        hipMemcpy(s2, h2, (size_t)2 * units2 * 16, hipMemcpyHostToDevice);
        hipMemcpy(s4, h4, (size_t)4 * units2 * 16, hipMemcpyHostToDevice);
        free(h2); free(h4);
    }
    const char* names[4] = {"2-bit codes in registers (18 VALU per K step and operand)",
                            "4-bit words in registers (12 VALU per K step and operand)",
                            "2-bit codes from an L2 strip pair", "4-bit words from an L2 strip pair (2x bytes)"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 4; ++mode) {
            for (int w = 0; w < 6; ++w) {
                if (w == 3) hipEventRecord(e0);
                switch (mode) {
                    case 0: kloop<0><<<grid, 64>>>(out, s2, iters, units2); break;
                    case 1: kloop<1><<<grid, 64>>>(out, s4, iters, 2 * units2); break;
                    case 2: kloop<2><<<grid, 64>>>(out, s2, iters, units2); break;
                    default: kloop<3><<<grid, 64>>>(out, s4, iters, 2 * units2); break;
                }
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 3;
            printf("{\"mode\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n", names[mode], rep, ms,
                   flop / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return hipGetLastError() != hipSuccess;
}
