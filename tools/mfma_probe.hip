// Probe for an MFMA Barrett reduction on gfx950 (standalone; not part of the library).
//  1. lane layout of v_mfma_i32_32x32x32_i8 (A, B, C) with exact integer data;
//  2. v_permlane32_swap semantics;
//  3. issue overlap: a wave stream of v_mad_u64_u32 with and without interleaved i8 MFMAs.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// A[32][32], B[32][32] (i8, row-major); the hypothesised map: lane l, r = l & 31, h = l >> 5 holds
// A[r][16h + j] and B[16h + j][r] in byte j of its 16-byte fragment; C: col = l & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 h.
__global__ void k_layout(const int8_t* A, const int8_t* B, int* C) {
    int l = threadIdx.x, r = l & 31, h = l >> 5;
    union { v4i v; int8_t b[16]; } a, b;
    for (int j = 0; j < 16; ++j) { a.b[j] = A[r * 32 + 16 * h + j]; b.b[j] = B[(16 * h + j) * 32 + r]; }
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, b.v, c, 0, 0, 0);
    for (int g = 0; g < 16; ++g) {
        int row = (g & 3) + 8 * (g >> 2) + 4 * h;
        C[row * 32 + r] = c[g];
    }
}

__global__ void k_swap(int* out) {
    int l = threadIdx.x;
    int x = 1000 + l, y = 2000 + l;
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    out[2 * l] = r[0];
    out[2 * l + 1] = r[1];
}

// overlap: each lane runs NM v_mad_u64_u32 in 4 independent chains per iteration; mode 1 adds NF MFMAs
// per iteration (two independent accumulators), mode 2 only the MFMAs.
template <int MODE>
__global__ void __launch_bounds__(512) k_overlap(uint64_t* out, int iters, uint32_t seed) {
    uint32_t a = seed + threadIdx.x, b = seed * 3 + 1;
    uint64_t c0 = a, c1 = b, c2 = a ^ b, c3 = a + b;
    v4i fa = {int(a), int(b), int(a ^ 7), int(b ^ 9)};
    v4i fb = {int(b), int(a), int(a + 7), int(b + 9)};
    v16i acc0 = {0}, acc1 = {0};
    const int wave = threadIdx.x >> 6;
    for (int it = 0; it < iters; ++it) {
        if (MODE == 3) {          // waves 0-3: MADs only, waves 4-7 (same SIMDs): MFMAs only
            if (wave < 4) {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t"
                                 "v_mad_u64_u32 %1, vcc, %4, %5, %1\n\t"
                                 "v_mad_u64_u32 %2, vcc, %4, %5, %2\n\t"
                                 "v_mad_u64_u32 %3, vcc, %4, %5, %3"
                                 : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b) : "vcc");
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb, fa, acc1, 0, 0, 0);
                }
            }
        } else if (MODE == 4 || MODE == 5) {   // plain 32-bit VALU (xor/add), alone (4) or with MFMAs (5)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                uint32_t x0 = uint32_t(c0), x1 = uint32_t(c1), x2 = uint32_t(c2), x3 = uint32_t(c3);
                asm volatile("v_xad_u32 %0, %4, %5, %0\n\tv_xad_u32 %1, %4, %5, %1\n\t"
                             "v_xad_u32 %2, %4, %5, %2\n\tv_xad_u32 %3, %4, %5, %3\n\t"
                             "v_xad_u32 %0, %5, %4, %0\n\tv_xad_u32 %1, %5, %4, %1\n\t"
                             "v_xad_u32 %2, %5, %4, %2\n\tv_xad_u32 %3, %5, %4, %3"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(a), "v"(b));
                c0 = x0; c1 = x1; c2 = x2; c3 = x3;
                if (MODE == 5 && (k & 3) == 0) acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc0, 0, 0, 0);
                if (MODE == 5 && (k & 3) == 2) acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb, fa, acc1, 0, 0, 0);
            }
        } else if (MODE != 2) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t"
                             "v_mad_u64_u32 %1, vcc, %4, %5, %1\n\t"
                             "v_mad_u64_u32 %2, vcc, %4, %5, %2\n\t"
                             "v_mad_u64_u32 %3, vcc, %4, %5, %3"
                             : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b) : "vcc");
                if (MODE == 1 && (k & 3) == 0) {
                    acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc0, 0, 0, 0);
                }
                if (MODE == 1 && (k & 3) == 2) {
                    acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb, fa, acc1, 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb, fa, acc1, 0, 0, 0);
            }
        }
    }
    uint64_t s = c0 + c1 + c2 + c3;
    for (int g = 0; g < 16; ++g) s += uint32_t(acc0[g]) + uint32_t(acc1[g]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    // 1. layout
    std::vector<int8_t> A(1024), B(1024);
    srand(7);
    for (int i = 0; i < 1024; ++i) { A[i] = int8_t(rand() % 256 - 128); B[i] = int8_t(rand() % 256 - 128); }
    int8_t *dA, *dB; int* dC;
    CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dC, 4096));
    CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    k_layout<<<1, 64>>>(dA, dB, dC);
    std::vector<int> C(1024);
    CK(hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int s = 0;
            for (int k = 0; k < 32; ++k) s += int(A[i * 32 + k]) * int(B[k * 32 + j]);
            bad += s != C[i * 32 + j];
        }
    printf("{\"probe\": \"layout_i8_32x32x32\", \"mismatches\": %d}\n", bad);
    // 2. permlane32_swap
    int* dS; CK(hipMalloc(&dS, 512));
    k_swap<<<1, 64>>>(dS);
    std::vector<int> S(128);
    CK(hipMemcpy(S.data(), dS, 512, hipMemcpyDeviceToHost));
    printf("{\"probe\": \"permlane32_swap\", \"lane0\": [%d, %d], \"lane31\": [%d, %d], \"lane32\": [%d, %d], \"lane63\": [%d, %d]}\n",
           S[0], S[1], S[62], S[63], S[64], S[65], S[126], S[127]);
    // 3. overlap: 2 waves per SIMD: 256 CUs x 2 blocks of 256 threads
    const int blocks = 256, iters = 4000;    // 512 threads: 2 waves per SIMD
    uint64_t* dO; CK(hipMalloc(&dO, size_t(blocks) * 512 * 8));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 6; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0));
            if (mode == 0) k_overlap<0><<<blocks, 512>>>(dO, iters, 5);
            if (mode == 1) k_overlap<1><<<blocks, 512>>>(dO, iters, 5);
            if (mode == 2) k_overlap<2><<<blocks, 512>>>(dO, iters, 5);
            if (mode == 3) k_overlap<3><<<blocks, 512>>>(dO, iters, 5);
            if (mode == 4) k_overlap<4><<<blocks, 512>>>(dO, iters, 5);
            if (mode == 5) k_overlap<5><<<blocks, 512>>>(dO, iters, 5);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            // per-wave work: modes 0/1: 64 MADs per iteration, 1/2: 8 MFMAs; 3: half the waves each
            double w = double(blocks) * 8 * iters;
            double mads = (mode == 0 || mode == 1) ? w * 64 * 64 : mode == 3 ? w / 2 * 64 * 64 : (mode >= 4 ? w * 128 * 64 : 0);
            double mfma = (mode == 1 || mode == 2 || mode == 5) ? w * 8 : mode == 3 ? w / 2 * 16 : 0;
            if (rep) printf("{\"probe\": \"overlap\", \"mode\": %d, \"ms\": %.3f, \"TMAD_per_s\": %.2f, \"mfma_per_s_per_simd\": %.3e}\n",
                            mode, ms, mads / ms / 1e9, mfma / ms * 1e3 / 1024);
        }
    }
    return 0;
}
