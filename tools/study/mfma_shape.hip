// Study (not product code): does the chip hold a higher clock on v_mfma_scale_f32_16x16x128_f8f6f4 than on
// the 32x32x64 form for the band kernel's fp4 operands?  Both loops issue the same 8 Gram products per 32x32
// output tile per wave on genotype-like planes (v = m + 2x, h, m; A1 allele frequency ~0.3, 1 % missing),
// same FLOPs per iteration, operands held in registers (no memory traffic), 2 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_shape tools/study/mfma_shape.hip && ./mfma_shape [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
// 8 nibbles of one plane for lane/step/word (genotype-like): returns v, h, m dwords
__device__ __forceinline__ void planes(uint32_t seed, int zero, uint32_t& v, uint32_t& h, uint32_t& m) {
    v = h = m = 0;
    if (zero) return;
    for (int k = 0; k < 8; ++k) {
        const uint32_t r = hash32(seed * 8 + k) & 1023u;
        uint32_t code = r < 10 ? 1u : r < 10 + 420 ? 2u : r < 10 + 420 + 90 ? 3u : 0u;  // miss, het, homA2, homA1
        v |= (code << 1) << (4 * k);
        h |= (code >= 2 ? 2u : 0u) << (4 * k);
        m |= (code == 1 ? 2u : 0u) << (4 * k);
    }
}

struct Fr { i32x4 v, h, m; };
__device__ __forceinline__ Fr mk(uint32_t seed, int zero) {
    Fr f;
    for (int q = 0; q < 4; ++q) {
        uint32_t a, b, c;
        planes(seed * 4 + q, zero, a, b, c);
        f.v[q] = (int)a; f.h[q] = (int)b; f.m[q] = (int)c;
    }
    return f;
}

__device__ __forceinline__ f32x16 m32(const i32x4& a, const i32x4& b, const f32x16& c) {
    const i32x8 A = {a[0], a[1], a[2], a[3], 0, 0, 0, 0}, B = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 4, 4, 0, 127, 0, 127);
}
__device__ __forceinline__ f32x4 m16(const i32x4& a, const i32x4& b, const f32x4& c) {
    const i32x8 A = {a[0], a[1], a[2], a[3], 0, 0, 0, 0}, B = {b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 4, 4, 0, 127, 0, 127);
}

// 4 K steps of 64 per iteration: 32 MFMAs 32x32x64
__global__ void __launch_bounds__(64, 2) k32(float* out, int iters, int zero) {
    const int lane = threadIdx.x;
    const uint32_t base = (blockIdx.x * 64 + lane) * 16;
    Fr a[4], b[4];
    for (int s = 0; s < 4; ++s) { a[s] = mk(base + 2 * s, zero); b[s] = mk(base + 2 * s + 1, zero); }
    f32x16 g[8];
    for (int p = 0; p < 8; ++p) g[p] = f32x16{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            g[0] = m32(a[s].v, b[s].v, g[0]);
            g[1] = m32(a[s].v, b[s].m, g[1]);
            g[2] = m32(a[s].v, b[s].h, g[2]);
            g[3] = m32(a[s].m, b[s].v, g[3]);
            g[4] = m32(a[s].h, b[s].v, g[4]);
            g[5] = m32(a[s].m, b[s].m, g[5]);
            g[6] = m32(a[s].m, b[s].h, g[6]);
            g[7] = m32(a[s].h, b[s].m, g[7]);
        }
    }
    float acc = 0.f;
    for (int p = 0; p < 8; ++p)
        for (int r = 0; r < 16; ++r) acc += g[p][r];
    out[blockIdx.x * 64 + lane] = acc;
}

// 2 K steps of 128 per iteration, 4 16x16 subtiles of the 32x32 tile: 64 MFMAs 16x16x128 (same FLOPs)
__global__ void __launch_bounds__(64, 2) k16(float* out, int iters, int zero) {
    const int lane = threadIdx.x;
    const uint32_t base = (blockIdx.x * 64 + lane) * 16;
    Fr a[2][2], b[2][2];
    for (int s = 0; s < 2; ++s)
        for (int q = 0; q < 2; ++q) { a[s][q] = mk(base + 4 * s + 2 * q, zero); b[s][q] = mk(base + 4 * s + 2 * q + 1, zero); }
    f32x4 g[4][8];
    for (int t = 0; t < 4; ++t)
        for (int p = 0; p < 8; ++p) g[t][p] = f32x4{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const Fr& A = a[s][t >> 1];
                const Fr& B = b[s][t & 1];
                g[t][0] = m16(A.v, B.v, g[t][0]);
                g[t][1] = m16(A.v, B.m, g[t][1]);
                g[t][2] = m16(A.v, B.h, g[t][2]);
                g[t][3] = m16(A.m, B.v, g[t][3]);
                g[t][4] = m16(A.h, B.v, g[t][4]);
                g[t][5] = m16(A.m, B.m, g[t][5]);
                g[t][6] = m16(A.m, B.h, g[t][6]);
                g[t][7] = m16(A.h, B.m, g[t][7]);
            }
        }
    }
    float acc = 0.f;
    for (int t = 0; t < 4; ++t)
        for (int p = 0; p < 8; ++p)
            for (int r = 0; r < 4; ++r) acc += g[t][p][r];
    out[blockIdx.x * 64 + lane] = acc;
}


// decode as the band kernel does: 16 two-bit codes -> v (= code << 1), h, m nibble planes
__device__ __forceinline__ void dec(uint32_t w, int& x0, int& x1, int& h0, int& h1, int& o0, int& o1) {
    constexpr uint32_t M = 0x22222222u, K6 = 0x66666666u;
    const uint32_t s1 = w << 1, s2 = w >> 1, w2 = w >> 2;
    x0 = (int)(s1 & K6); x1 = (int)(s2 & K6); h0 = (int)(w & M); h1 = (int)(w2 & M);
    o0 = (int)(s1 & ~w & M); o1 = (int)(s2 & ~w2 & M);
}
__device__ __forceinline__ Fr decf(uint32_t wa, uint32_t wb) {
    int x0, x1, x2, x3, h0, h1, h2, h3, o0, o1, o2, o3;
    dec(wa, x0, x1, h0, h1, o0, o1); dec(wb, x2, x3, h2, h3, o2, o3);
    Fr f; f.v = i32x4{x0, x1, x2, x3}; f.h = i32x4{h0, h1, h2, h3}; f.m = i32x4{o0, o1, o2, o3};
    return f;
}
__device__ __forceinline__ uint32_t codes(uint32_t seed) {  // 16 genotype-like 2-bit codes
    uint32_t w = 0;
    for (int k = 0; k < 16; ++k) {
        const uint32_t r = hash32(seed * 16 + k) & 1023u;
        w |= (r < 10 ? 1u : r < 430 ? 2u : r < 520 ? 3u : 0u) << (2 * k);
    }
    return w;
}
// MODE 1: operands decoded every K step from code words held in registers (rotated per iteration);
// MODE 2: code words loaded every K step from a 2.5 MB strip pair (L2-resident, all waves share it)
template <int MODE>
__global__ void __launch_bounds__(64, 2) k32d(float* out, const uint4* strip, int iters, int words) {
    const int lane = threadIdx.x;
    const uint32_t base = (blockIdx.x * 64 + lane) * 16;
    uint4 ra = make_uint4(codes(base), codes(base + 1), codes(base + 2), codes(base + 3));
    uint4 rb = make_uint4(codes(base + 4), codes(base + 5), codes(base + 6), codes(base + 7));
    f32x16 g[8];
    for (int p = 0; p < 8; ++p) g[p] = f32x16{};
    int off = lane;
    uint4 pa = ra, pb = rb, qa = ra, qb = rb;
    for (int it = 0; it < iters; ++it) {
        if (MODE == 2) {  // two iterations of prefetch distance
            ra = pa; rb = pb; pa = qa; pb = qb;
            qa = strip[off]; qb = strip[off + words];
            off += 64; if (off >= words) off = lane;
        } else {
            ra.x = __builtin_amdgcn_alignbit(ra.x, ra.y, 2); ra.y = __builtin_amdgcn_alignbit(ra.y, ra.z, 2);
            ra.z = __builtin_amdgcn_alignbit(ra.z, ra.w, 2); ra.w = __builtin_amdgcn_alignbit(ra.w, ra.x, 2);
            rb.x = __builtin_amdgcn_alignbit(rb.x, rb.y, 2); rb.y = __builtin_amdgcn_alignbit(rb.y, rb.z, 2);
            rb.z = __builtin_amdgcn_alignbit(rb.z, rb.w, 2); rb.w = __builtin_amdgcn_alignbit(rb.w, rb.x, 2);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const Fr a = s ? decf(ra.z, ra.w) : decf(ra.x, ra.y), b = s ? decf(rb.z, rb.w) : decf(rb.x, rb.y);
            g[0] = m32(a.v, b.v, g[0]); g[1] = m32(a.v, b.m, g[1]); g[2] = m32(a.v, b.h, g[2]);
            g[3] = m32(a.m, b.v, g[3]); g[4] = m32(a.h, b.v, g[4]); g[5] = m32(a.m, b.m, g[5]);
            g[6] = m32(a.m, b.h, g[6]); g[7] = m32(a.h, b.m, g[7]);
        }
    }
    float acc = 0.f;
    for (int p = 0; p < 8; ++p)
        for (int r = 0; r < 16; ++r) acc += g[p][r];
    out[blockIdx.x * 64 + lane] = acc;
}

// 64 x 32 tile per wave at 1 wave per SIMD: two row fragments share one column fragment's decode (3 decodes per
// 16 products instead of 2 per 8), operands decoded every K step from code words in registers
__global__ void __launch_bounds__(64, 1) k64d(float* out, int iters) {
    const int lane = threadIdx.x;
    const uint32_t base = (blockIdx.x * 64 + lane) * 16;
    uint4 ra = make_uint4(codes(base), codes(base + 1), codes(base + 2), codes(base + 3));
    uint4 rc = make_uint4(codes(base + 8), codes(base + 9), codes(base + 10), codes(base + 11));
    uint4 rb = make_uint4(codes(base + 4), codes(base + 5), codes(base + 6), codes(base + 7));
    f32x16 g[2][8];
    for (int q = 0; q < 2; ++q)
        for (int p = 0; p < 8; ++p) g[q][p] = f32x16{};
    for (int it = 0; it < iters; ++it) {
        ra.x = __builtin_amdgcn_alignbit(ra.x, ra.y, 2); ra.y = __builtin_amdgcn_alignbit(ra.y, ra.z, 2);
        ra.z = __builtin_amdgcn_alignbit(ra.z, ra.w, 2); ra.w = __builtin_amdgcn_alignbit(ra.w, ra.x, 2);
        rc.x = __builtin_amdgcn_alignbit(rc.x, rc.y, 2); rc.y = __builtin_amdgcn_alignbit(rc.y, rc.z, 2);
        rc.z = __builtin_amdgcn_alignbit(rc.z, rc.w, 2); rc.w = __builtin_amdgcn_alignbit(rc.w, rc.x, 2);
        rb.x = __builtin_amdgcn_alignbit(rb.x, rb.y, 2); rb.y = __builtin_amdgcn_alignbit(rb.y, rb.z, 2);
        rb.z = __builtin_amdgcn_alignbit(rb.z, rb.w, 2); rb.w = __builtin_amdgcn_alignbit(rb.w, rb.x, 2);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const Fr b = s ? decf(rb.z, rb.w) : decf(rb.x, rb.y);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint4& r = q ? rc : ra;
                const Fr a = s ? decf(r.z, r.w) : decf(r.x, r.y);
                g[q][0] = m32(a.v, b.v, g[q][0]); g[q][1] = m32(a.v, b.m, g[q][1]); g[q][2] = m32(a.v, b.h, g[q][2]);
                g[q][3] = m32(a.m, b.v, g[q][3]); g[q][4] = m32(a.h, b.v, g[q][4]); g[q][5] = m32(a.m, b.m, g[q][5]);
                g[q][6] = m32(a.m, b.h, g[q][6]); g[q][7] = m32(a.h, b.m, g[q][7]);
            }
        }
    }
    float acc = 0.f;
    for (int q = 0; q < 2; ++q)
        for (int p = 0; p < 8; ++p)
            for (int r = 0; r < 16; ++r) acc += g[q][p][r];
    out[blockIdx.x * 64 + lane] = acc;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const int grid = 256 * 8;  // 2 waves per SIMD on every CU
    float* out;
    hipMalloc(&out, grid * 64 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const double flop = (double)grid * iters * 32 * 2.0 * 32 * 32 * 64;
    for (int zero = 0; zero < 2; ++zero) {
        for (int rep = 0; rep < 2; ++rep) {
            for (int shape = 0; shape < 2; ++shape) {
                // warm the clock with back-to-back launches, time the last 3
                for (int w = 0; w < 6; ++w) {
                    if (w == 3) hipEventRecord(e0);
                    if (shape == 0) k32<<<grid, 64>>>(out, iters, zero);
                    else k16<<<grid, 64>>>(out, iters, zero);
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                ms /= 3;
                printf("{\"shape\": \"%s\", \"data\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n",
                       shape == 0 ? "32x32x64" : "16x16x128", zero ? "zero" : "genotype", rep, ms,
                       flop / (ms * 1e-3) / 1e12);
                fflush(stdout);
            }
        }
    }
    // decode-fed and load-fed loops: 2 K steps per iteration, so twice the iterations for the same FLOPs
    const int words = 2 * 78912 / 16 * 32;  // two 32-row strips of a C3 row (uint4 units per strip pair / 2)
    uint4* strip;
    hipMalloc(&strip, (size_t)2 * words * sizeof(uint4));
    hipLaunchKernelGGL(k32d<1>, dim3(1), dim3(64), 0, 0, out, strip, 0, words);  // load the module
    {
        uint32_t* h = (uint32_t*)malloc((size_t)2 * words * sizeof(uint4));
        for (size_t k = 0; k < (size_t)8 * words; ++k) {
            uint32_t w = 0;
            for (int j = 0; j < 16; ++j) {
                uint32_t r = (uint32_t)((k * 16 + j) * 2654435761u) >> 22;
                w |= (r < 10 ? 1u : r < 430 ? 2u : r < 520 ? 3u : 0u) << (2 * j);
            }
            h[k] = w;
        }
        hipMemcpy(strip, h, (size_t)2 * words * sizeof(uint4), hipMemcpyHostToDevice);
        free(h);
    }
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 1; mode <= 2; ++mode) {
            for (int w = 0; w < 6; ++w) {
                if (w == 3) hipEventRecord(e0);
                if (mode == 1) k32d<1><<<grid, 64>>>(out, strip, 2 * iters, words);
                else k32d<2><<<grid, 64>>>(out, strip, 2 * iters, words);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 3;
            printf("{\"shape\": \"32x32x64\", \"data\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n",
                   mode == 1 ? "decoded in registers" : "decoded from L2 loads", rep, ms, flop / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    for (int rep = 0; rep < 2; ++rep) {  // 64 x 32 tiles: half the waves (1 per SIMD), same FLOPs per launch
        for (int w = 0; w < 6; ++w) {
            if (w == 3) hipEventRecord(e0);
            k64d<<<grid / 2, 64>>>(out, 2 * iters);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 3;
        printf("{\"shape\": \"32x32x64, 64x32 tile per wave\", \"data\": \"decoded in registers\", \"rep\": %d, "
               "\"ms\": %.3f, \"tflops\": %.1f}\n", rep, ms, flop / (ms * 1e-3) / 1e12);
        fflush(stdout);
    }
    return hipGetLastError() != hipSuccess;
}
