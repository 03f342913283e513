// Which SIMD each wave of a 512-thread workgroup lands on (HW_REG_HW_ID bits 5:4), for the ping-pong
// schedule of fthe_padic_m37 (the two waves of a SIMD must be in different halves of the workgroup).
// Build: hipcc --offload-arch=gfx950 -O2 tools/simd_map_probe.hip -o tools/bin/simd_map_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void probe(unsigned *out) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = id;
}
int main() {
    const int nb = 512;
    unsigned *d, h[nb * 8];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int same_half = 0, cross_half = 0;
    for (int b = 0; b < nb; b++) {
        if (b < 4) { printf("wg %d:", b); for (int w = 0; w < 8; w++) printf(" w%d->simd%u", w, (h[b * 8 + w] >> 4) & 3); printf("\n"); }
        for (int w = 0; w < 8; w++) for (int v = w + 1; v < 8; v++)
            if (((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + v] >> 4) & 3)) ((w >> 2) == (v >> 2) ? same_half : cross_half)++;
    }
    printf("{\"simd_pairs_same_half\": %d, \"simd_pairs_cross_half\": %d}\n", same_half, cross_half);
    return 0;
}
