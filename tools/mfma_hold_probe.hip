// How much VALU issue a v_mfma_i32_32x32x32_i8 costs, in the instruction mix of fthe_padic_m37
// (64-bit v_mad_u64_u32 multiply-adds beside i8 MFMAs).
//   one wave per SIMD: loop { MFMA; N x v_mad_u64_u32 (4 independent chains) } -> cycles per MFMA gap
//   two waves per SIMD (512-thread workgroup, wave w and w + 4 share a SIMD): waves 0-3 run M multiply-adds,
//   waves 4-7 run K back-to-back MFMAs (or the same multiply-adds, or nothing) -> the VALU waves' cycles
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_hold_probe.hip -o tools/bin/mfma_hold_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define STR_(x) #x
#define STR(x) STR_(x)
#define MAD4 "v_mad_u64_u32 %[m0], vcc, %[x], %[y], %[m0]\n v_mad_u64_u32 %[m1], vcc, %[x], %[y], %[m1]\n" \
             "v_mad_u64_u32 %[m2], vcc, %[x], %[y], %[m2]\n v_mad_u64_u32 %[m3], vcc, %[x], %[y], %[m3]\n"

template <int N4>
__global__ __launch_bounds__(256) void one_wave(unsigned long long *out, int iters, int seed) {
    v4i a = {seed, seed + 1, seed + 2, (int)threadIdx.x}, b = a;
    v16i c0 = {}, c1 = {};
    unsigned long long m0 = threadIdx.x, m1 = 1, m2 = 2, m3 = 3;
    unsigned x = seed, y = threadIdx.x;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
        asm volatile("v_mfma_i32_32x32x32_i8 %[c0], %[a], %[b], %[c0]\n"
                     ".rept %[n]\n" MAD4 ".endr\n"
                     "v_mfma_i32_32x32x32_i8 %[c1], %[a], %[b], %[c1]\n"
                     ".rept %[n]\n" MAD4 ".endr\n"
                     : [c0] "+v"(c0), [c1] "+v"(c1), [m0] "+v"(m0), [m1] "+v"(m1), [m2] "+v"(m2), [m3] "+v"(m3)
                     : [a] "v"(a), [b] "v"(b), [x] "v"(x), [y] "v"(y), [n] "i"(N4) : "vcc");
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    unsigned long long t1 = __builtin_readcyclecounter();
    int s = 0;
    for (int k = 0; k < 16; k++) s += c0[k] + c1[k];
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    if (s == 0x12345 && m0 + m1 + m2 + m3 == 7) out[0] = 0;     // keep the results live
}

// mode 0: partner idle; 1: partner back-to-back MFMAs; 2: partner the same multiply-adds
__global__ __launch_bounds__(512) void two_waves(unsigned long long *out, int iters, int mode, int seed) {
    const int half = threadIdx.x >> 8;
    v4i a = {seed, seed + 1, seed + 2, (int)threadIdx.x}, b = a;
    v16i c0 = {}, c1 = {};
    unsigned long long m0 = threadIdx.x, m1 = 1, m2 = 2, m3 = 3;
    unsigned x = seed, y = threadIdx.x;
    unsigned long long t0 = __builtin_readcyclecounter();
    if (half == 0 || mode == 2) {
        for (int i = 0; i < iters; i++)
            asm volatile(".rept 4\n" MAD4 ".endr\n"
                         : [m0] "+v"(m0), [m1] "+v"(m1), [m2] "+v"(m2), [m3] "+v"(m3)
                         : [x] "v"(x), [y] "v"(y) : "vcc");
    } else if (mode == 1) {
        for (int i = 0; i < iters; i++)
            asm volatile("v_mfma_i32_32x32x32_i8 %[c0], %[a], %[b], %[c0]\n"
                         "v_mfma_i32_32x32x32_i8 %[c1], %[a], %[b], %[c1]\n"
                         : [c0] "+v"(c0), [c1] "+v"(c1) : [a] "v"(a), [b] "v"(b));
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    unsigned long long t1 = __builtin_readcyclecounter();
    int s = 0;
    for (int k = 0; k < 16; k++) s += c0[k] + c1[k];
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
    if (s == 0x12345 && m0 + m1 + m2 + m3 == 7) out[0] = 0;
}


// one wave per SIMD: MFMA + 6 fillers of one kind (independent of the MFMA) per gap
#define FILL6(ins) ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n"
#define FILLER_KERNEL(NAME, INS)                                                                         \
__global__ __launch_bounds__(256) void NAME(unsigned long long *out, int iters, int seed) {              \
    v4i a = {seed, seed + 1, seed + 2, (int)threadIdx.x}, b = a;                                          \
    v16i c0 = {}, c1 = {};                                                                               \
    unsigned long long m0 = threadIdx.x, m1 = 1;                                                        \
    unsigned x = seed, y = threadIdx.x, p = 5, q = 7;                                                    \
    unsigned long long t0 = __builtin_readcyclecounter();                                              \
    for (int i = 0; i < iters; i++) {                                                                     \
        asm volatile("v_mfma_i32_32x32x32_i8 %[c0], %[a], %[b], %[c0]\n" FILL6(INS)                      \
                     "v_mfma_i32_32x32x32_i8 %[c1], %[a], %[b], %[c1]\n" FILL6(INS)                      \
                     "v_mfma_i32_32x32x32_i8 %[c0], %[a], %[b], %[c0]\n" FILL6(INS)                      \
                     "v_mfma_i32_32x32x32_i8 %[c1], %[a], %[b], %[c1]\n" FILL6(INS)                      \
                     : [c0] "+v"(c0), [c1] "+v"(c1), [m0] "+v"(m0), [m1] "+v"(m1), [p] "+v"(p), [q] "+v"(q) \
                     : [a] "v"(a), [b] "v"(b), [x] "v"(x), [y] "v"(y) : "vcc");                           \
    }                                                                                                     \
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");                                            \
    unsigned long long t1 = __builtin_readcyclecounter();                                              \
    int s = 0;                                                                                           \
    for (int k = 0; k < 16; k++) s += c0[k] + c1[k];                                                     \
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                       \
    if (s == 0x12345 && m0 + m1 + p + q == 7) out[0] = 0;                                                \
}
FILLER_KERNEL(f_mad_u64, "v_mad_u64_u32 %[m0], vcc, %[x], %[y], %[m0]")
FILLER_KERNEL(f_mad_i64, "v_mad_i64_i32 %[m0], vcc, %[x], %[y], %[m0]")
FILLER_KERNEL(f_lshl_add_u64, "v_lshl_add_u64 %[m0], %[m0], 0, %[m1]")
FILLER_KERNEL(f_lshr_b64, "v_lshrrev_b64 %[m0], 28, %[m1]")
FILLER_KERNEL(f_add_u32, "v_add_u32_e32 %[p], %[x], %[p]")
FILLER_KERNEL(f_lshl_or, "v_lshl_or_b32 %[p], %[q], 8, %[p]")
FILLER_KERNEL(f_xor, "v_xor_b32_e32 %[p], 0x80808080, %[p]")
FILLER_KERNEL(f_permlane, "v_permlane32_swap_b32_e32 %[p], %[q]")
FILLER_KERNEL(f_mul_lo, "v_mul_lo_u32 %[p], %[x], %[p]")

// one wave per SIMD: 64 v_mad_u64_u32 per iteration on K independent accumulator chains
template <int K>
__global__ __launch_bounds__(256) void chains(unsigned long long *out, int iters, int seed) {
    unsigned long long m[8] = {threadIdx.x, 1, 2, 3, 4, 5, 6, 7};
    unsigned x = seed, y = threadIdx.x;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 64; j++)
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(m[j % K]) : "v"(x), "v"(y) : "vcc");
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    unsigned long long s = 0;
    for (int k = 0; k < 8; k++) s += m[k];
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    if (s == 7) out[0] = 0;
}


// one wave per SIMD: MFMA + 6 fillers per gap, dependent (one register) or independent (six registers)
#define IND6(a, b, c, d, e, f) a "\n" b "\n" c "\n" d "\n" e "\n" f "\n"
#define DEP_KERNEL(NAME, FILL)                                                                           \
__global__ __launch_bounds__(256) void NAME(unsigned long long *out, int iters, int seed) {              \
    v4i a = {seed, seed + 1, seed + 2, (int)threadIdx.x}, b = a;                                          \
    v16i c0 = {}, c1 = {};                                                                               \
    unsigned long long m0 = threadIdx.x, m1 = 1, m2 = 2, m3 = 3, m4 = 4, m5 = 5;                        \
    unsigned x = seed * 3 + 1, y = threadIdx.x ^ 5;     /* not the MFMA operands */                                                                  \
    unsigned long long t0 = __builtin_readcyclecounter();                                              \
    for (int i = 0; i < iters; i++) {                                                                     \
        asm volatile("v_mfma_i32_32x32x32_i8 %[c0], %[a], %[b], %[c0]\n" FILL                           \
                     "v_mfma_i32_32x32x32_i8 %[c1], %[a], %[b], %[c1]\n" FILL                           \
                     "v_mfma_i32_32x32x32_i8 %[c0], %[a], %[b], %[c0]\n" FILL                           \
                     "v_mfma_i32_32x32x32_i8 %[c1], %[a], %[b], %[c1]\n" FILL                           \
                     : [c0] "+v"(c0), [c1] "+v"(c1), [m0] "+v"(m0), [m1] "+v"(m1), [m2] "+v"(m2),        \
                       [m3] "+v"(m3), [m4] "+v"(m4), [m5] "+v"(m5)                                       \
                     : [a] "v"(a), [b] "v"(b), [x] "v"(x), [y] "v"(y) : "vcc");                           \
    }                                                                                                     \
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");                                            \
    unsigned long long t1 = __builtin_readcyclecounter();                                              \
    int s = 0;                                                                                           \
    for (int k = 0; k < 16; k++) s += c0[k] + c1[k];                                                     \
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                       \
    if (s == 0x12345 && m0 + m1 + m2 + m3 + m4 + m5 == 7) out[0] = 0;                                    \
}
#define MADR(r) "v_mad_u64_u32 %[" #r "], vcc, %[x], %[y], %[" #r "]"
DEP_KERNEL(d_mad6_dep, IND6(MADR(m0), MADR(m0), MADR(m0), MADR(m0), MADR(m0), MADR(m0)))
DEP_KERNEL(d_mad6_ind, IND6(MADR(m0), MADR(m1), MADR(m2), MADR(m3), MADR(m4), MADR(m5)))
DEP_KERNEL(d_mad6_two, IND6(MADR(m0), MADR(m1), MADR(m0), MADR(m1), MADR(m0), MADR(m1)))
DEP_KERNEL(d_mad12_dep, IND6(MADR(m0), MADR(m0), MADR(m0), MADR(m0), MADR(m0), MADR(m0))
                        IND6(MADR(m0), MADR(m0), MADR(m0), MADR(m0), MADR(m0), MADR(m0)))
DEP_KERNEL(d_mad12_two, IND6(MADR(m0), MADR(m1), MADR(m0), MADR(m1), MADR(m0), MADR(m1))
                        IND6(MADR(m0), MADR(m1), MADR(m0), MADR(m1), MADR(m0), MADR(m1)))
DEP_KERNEL(d_mad12_ind, IND6(MADR(m0), MADR(m1), MADR(m2), MADR(m3), MADR(m4), MADR(m5))
                        IND6(MADR(m0), MADR(m1), MADR(m2), MADR(m3), MADR(m4), MADR(m5)))

static double mean_cycles(const std::vector<unsigned long long> &v, int stride, int lo, int hi) {
    double s = 0; int n = 0;
    for (size_t i = 0; i < v.size(); i++) if ((int)(i % stride) >= lo && (int)(i % stride) < hi) { s += (double)v[i]; n++; }
    return s / n;
}

int main() {
    const int nb = 256, iters = 4096;
    unsigned long long *d;
    if (hipMalloc(&d, nb * 8 * sizeof(unsigned long long)) != hipSuccess) return 1;
    std::vector<unsigned long long> h(nb * 8);
    auto run1 = [&](auto kern, int n4) {
        // 96 KB of dynamic LDS: one workgroup (4 waves, one per SIMD) per CU
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters, 3);
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters, 3);
        if (hipMemcpy(h.data(), d, nb * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) exit(1);
        std::vector<unsigned long long> v(h.begin(), h.begin() + nb * 4);
        printf("{\"test\": \"one_wave\", \"mads_per_mfma\": %d, \"cycles_per_mfma_gap\": %.2f}\n", 4 * n4,
               mean_cycles(v, 4, 0, 4) / (2.0 * iters));
    };
    run1(one_wave<0>, 0); run1(one_wave<1>, 1); run1(one_wave<2>, 2); run1(one_wave<3>, 3);
    run1(one_wave<4>, 4); run1(one_wave<6>, 6); run1(one_wave<8>, 8);
    for (int mode = 0; mode < 3; mode++) {
        hipLaunchKernelGGL(two_waves, dim3(nb), dim3(512), 96 * 1024, 0, d, iters, mode, 3);
        hipLaunchKernelGGL(two_waves, dim3(nb), dim3(512), 96 * 1024, 0, d, iters, mode, 3);
        if (hipMemcpy(h.data(), d, nb * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("{\"test\": \"two_waves\", \"partner\": \"%s\", \"valu_wave_cycles_per_mad\": %.3f, "
               "\"partner_cycles_per_iter\": %.2f}\n", mode == 0 ? "idle" : mode == 1 ? "mfma x2" : "same mads",
               mean_cycles(h, 8, 0, 4) / (16.0 * iters), mean_cycles(h, 8, 4, 8) / iters);
    }
    auto runf = [&](auto kern, const char *name) {
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters / 2, 3);
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters / 2, 3);
        if (hipMemcpy(h.data(), d, nb * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) exit(1);
        std::vector<unsigned long long> v(h.begin(), h.begin() + nb * 4);
        printf("{\"test\": \"filler\", \"kind\": \"%s\", \"per_gap\": 6, \"cycles_per_mfma_gap\": %.2f}\n", name,
               mean_cycles(v, 4, 0, 4) / (4.0 * (iters / 2)));
    };
    runf(f_mad_u64, "v_mad_u64_u32"); runf(f_mad_i64, "v_mad_i64_i32"); runf(f_lshl_add_u64, "v_lshl_add_u64");
    runf(f_lshr_b64, "v_lshrrev_b64"); runf(f_add_u32, "v_add_u32"); runf(f_lshl_or, "v_lshl_or_b32");
    runf(f_xor, "v_xor_b32"); runf(f_permlane, "v_permlane32_swap"); runf(f_mul_lo, "v_mul_lo_u32");
    auto runc = [&](auto kern, int k) {
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters / 4, 3);
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters / 4, 3);
        if (hipMemcpy(h.data(), d, nb * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) exit(1);
        std::vector<unsigned long long> v(h.begin(), h.begin() + nb * 4);
        printf("{\"test\": \"chains\", \"chains\": %d, \"cycles_per_mad\": %.3f}\n", k,
               mean_cycles(v, 4, 0, 4) / (64.0 * (iters / 4)));
    };
    runc(chains<1>, 1); runc(chains<2>, 2); runc(chains<3>, 3); runc(chains<4>, 4); runc(chains<8>, 8);
    auto rund = [&](auto kern, const char *name) {
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters / 2, 3);
        hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 96 * 1024, 0, d, iters / 2, 3);
        if (hipMemcpy(h.data(), d, nb * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) exit(1);
        std::vector<unsigned long long> v(h.begin(), h.begin() + nb * 4);
        printf("{\"test\": \"chain_shape\", \"kind\": \"%s\", \"cycles_per_mfma_gap\": %.2f}\n", name,
               mean_cycles(v, 4, 0, 4) / (4.0 * (iters / 2)));
    };
    rund(d_mad6_dep, "6 mads, one chain"); rund(d_mad6_two, "6 mads, two chains"); rund(d_mad6_ind, "6 mads, six chains");
    rund(d_mad12_dep, "12 mads, one chain"); rund(d_mad12_two, "12 mads, two chains"); rund(d_mad12_ind, "12 mads, six chains");
    return 0;
}
