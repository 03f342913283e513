// Probe of v_mfma_i32_16x16x64_i8 on gfx950 (standalone; not part of the library): which (row, k) byte of
// A and (k, column) byte of B each lane's 16-byte fragment carries, and which (row, column) each of the
// four int32 results is, with exact integer data.  Two K maps are tried:
//   map 0: lane l, r = l & 15, h = l >> 4 holds A[r][16h + j], B[16h + j][r] in byte j;
//   map 1: byte j < 8 holds k = 8h + j, byte j >= 8 holds k = 32 + 8h + (j - 8).
// C (both): column = l & 15, row = 4h + g for result register g.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma16_probe tools/mfma16_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __host__ inline int kmap(int map, int h, int j) { return map == 0 ? 16 * h + j : (j < 8 ? 8 * h + j : 32 + 8 * h + j - 8); }

__global__ void k_layout(const int8_t *A, const int8_t *B, int *C, int map) {
    int l = threadIdx.x, r = l & 15, h = l >> 4;
    union { v4i v; int8_t b[16]; } a, b;
    for (int j = 0; j < 16; ++j) {
        const int k = kmap(map, h, j);
        a.b[j] = A[r * 64 + k];
        b.b[j] = B[k * 16 + r];
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a.v, b.v, c, 0, 0, 0);
    for (int g = 0; g < 4; ++g) C[(4 * h + g) * 16 + r] = c[g];
}

int main() {
    std::vector<int8_t> A(16 * 64), B(64 * 16);
    srand(11);
    for (auto &x : A) x = int8_t(rand() % 256 - 128);
    for (auto &x : B) x = int8_t(rand() % 256 - 128);
    int8_t *dA, *dB;
    int *dC;
    CK(hipMalloc(&dA, A.size()));
    CK(hipMalloc(&dB, B.size()));
    CK(hipMalloc(&dC, 256 * 4));
    CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
    for (int map = 0; map < 2; ++map) {
        k_layout<<<1, 64>>>(dA, dB, dC, map);
        CK(hipDeviceSynchronize());
        std::vector<int> C(256);
        CK(hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 16; ++i)
            for (int n = 0; n < 16; ++n) {
                int s = 0;
                for (int k = 0; k < 64; ++k) s += int(A[i * 64 + k]) * int(B[k * 16 + n]);
                bad += s != C[i * 16 + n];
            }
        printf("{\"probe\": \"layout_i8_16x16x64\", \"map\": %d, \"mismatches\": %d}\n", map, bad);
    }
    return 0;
}
