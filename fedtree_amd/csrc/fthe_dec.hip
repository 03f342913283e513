// fthe_dec.hip -- the reference's decimal ciphertext wire format on the device.
//
// FedTree's distributed mode ships ciphertexts as decimal strings (GHEncBatch,
// fedtree.proto:82-99, written with mpz_get_str / read with mpz_set_str in
// distributed_server.cpp:37-54,1416-1433 and distributed_party.cpp:1267-1309).
// On the host that costs ~1.5 us per 4096-bit ciphertext per core (fthe_wire.cpp),
// several times the device encrypt rate; here the conversion runs on the GPU and
// produces exactly mpz_get_str's digits (no sign, no leading zeros, "0" for 0).
//
// Binary -> decimal: one thread per ciphertext keeps the number in registers and
// divides it by 10^9 repeatedly (a 64-by-32-bit division per limb); the 9-digit
// remainders land chunk-major in HBM.  After p divisions the value is below
// 2^(32W - 29.897 p), so 16-limb blocks above that bound are skipped (a uniform
// test: the bound depends on p only).  Lengths, an exclusive scan and a
// chunk-parallel writer then pack the strings back to back (offsets[count] = bytes).
// Decimal -> binary: one thread per string, acc = acc * 10^9 + chunk.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "fthe_glue.h"

namespace fthe {

constexpr uint32_t E9 = 1000000000u;

template <int W>
__global__ void __launch_bounds__(256) k_dec_chunks(const uint32_t *__restrict__ ct, int words, size_t count, int nch,
                             uint32_t *__restrict__ chunks) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= count) return;
    uint32_t x[W];
#pragma unroll
    for (int i = 0; i < W; i++) x[i] = i < words ? ct[g * (size_t)words + i] : 0u;
    for (int p = 0; p < nch; p++) {
        const int act = W - (int)((29.897352853986263 * p) / 32.0);     // limbs >= act are zero
        uint64_t rem = 0;
#pragma unroll
        for (int b = W / 16 - 1; b >= 0; b--) {
            if (b * 16 < act) {
#pragma unroll
                for (int i = 15; i >= 0; i--) {
                    const uint64_t cur = (rem << 32) | x[b * 16 + i];
                    const uint64_t q = cur / E9;
                    rem = cur - q * E9;
                    x[b * 16 + i] = (uint32_t)q;
                }
            }
        }
        chunks[(size_t)p * count + g] = (uint32_t)rem;
    }
}

__device__ __forceinline__ int ndigits(uint32_t v) {
    int d = 1;
    while (v >= 10u) { v /= 10u; d++; }
    return d;
}

// len[g] = decimal digits of ciphertext g; top[g] = its most significant non-zero chunk
__global__ void k_dec_len(const uint32_t *__restrict__ chunks, size_t count, int nch, int64_t *__restrict__ len,
                          int32_t *__restrict__ top) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g > count) return;
    if (g == count) { len[g] = 0; return; }         // scan sentinel: offsets[count] = total
    int t = nch - 1;
    while (t > 0 && chunks[(size_t)t * count + g] == 0u) t--;
    top[g] = t;
    len[g] = (int64_t)9 * t + ndigits(chunks[(size_t)t * count + g]);
}

// thread (c, g): chunk c of ciphertext g -> its digits at buf + off[g] + position
__global__ void k_dec_write(const uint32_t *__restrict__ chunks, size_t count, int nch,
                            const int64_t *__restrict__ off, const int32_t *__restrict__ top, char *__restrict__ buf) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)nch * count) return;
    const size_t g = t % count;
    const int c = (int)(t / count);
    const int tp = top[g];
    if (c > tp) return;
    uint32_t v = chunks[t];
    char *o = buf + off[g];
    if (c == tp) {                                  // leading chunk: no zero padding
        const int n = ndigits(v);
        for (int i = n - 1; i >= 0; i--) { o[i] = (char)('0' + v % 10u); v /= 10u; }
        return;
    }
    o += (off[g + 1] - off[g]) - 9 * (int64_t)(c + 1);
    for (int i = 8; i >= 0; i--) { o[i] = (char)('0' + v % 10u); v /= 10u; }
}

// decimal strings -> little-endian words; err != 0 on a malformed or oversized string
template <int W>
__global__ void __launch_bounds__(256) k_dec_parse(const char *__restrict__ buf, const int64_t *__restrict__ off, size_t count, int words,
                            int maxlen, uint32_t *__restrict__ ct, int *__restrict__ err) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= count) return;
    const int64_t b = off[g], n = off[g + 1] - b;
    uint32_t x[W];
#pragma unroll
    for (int i = 0; i < W; i++) x[i] = 0u;
    bool bad = n <= 0 || n > maxlen;
    uint32_t over = 0;
    if (!bad) {
        const char *s = buf + b;
        int64_t pos = 0;
        int first = (int)(n % 9);
        if (first == 0) first = 9;
        while (pos < n) {
            const int m = pos == 0 ? first : 9;
            uint32_t v = 0, mul = 1;
            for (int j = 0; j < m; j++) {
                const int d = s[pos + j] - '0';
                if (d < 0 || d > 9) bad = true;
                v = v * 10u + (uint32_t)(d & 15);
                mul *= 10u;
            }
            pos += m;
            uint64_t carry = v;                     // x = x * 10^m + v
#pragma unroll
            for (int i = 0; i < W; i++) {
                const uint64_t t = (uint64_t)x[i] * mul + carry;
                x[i] = (uint32_t)t;
                carry = t >> 32;
            }
            over |= (uint32_t)carry;
        }
    }
#pragma unroll
    for (int i = 0; i < W; i++)
        if (i >= words) over |= x[i];
    if (bad || over) { atomicOr(err, 1); return; }
#pragma unroll
    for (int i = 0; i < W; i++)
        if (i < words) ct[g * (size_t)words + i] = x[i];
}

static int dec_width(int words) { return words <= 32 ? 32 : words <= 64 ? 64 : words <= 128 ? 128 : 0; }

int dec_launch_chunks(const uint32_t *ct, int words, size_t count, int nch, uint32_t *chunks, hipStream_t st) {
    const dim3 grid((unsigned)((count + 255) / 256)), blk(256);
    switch (dec_width(words)) {
    case 32: hipLaunchKernelGGL(k_dec_chunks<32>, grid, blk, 0, st, ct, words, count, nch, chunks); break;
    case 64: hipLaunchKernelGGL(k_dec_chunks<64>, grid, blk, 0, st, ct, words, count, nch, chunks); break;
    case 128: hipLaunchKernelGGL(k_dec_chunks<128>, grid, blk, 0, st, ct, words, count, nch, chunks); break;
    default: return -1;
    }
    return 0;
}

int dec_launch_len_write(const uint32_t *chunks, size_t count, int nch, int64_t *len, int32_t *top, int pass,
                         const int64_t *off, char *buf, hipStream_t st) {
    if (pass == 0)
        hipLaunchKernelGGL(k_dec_len, dim3((unsigned)((count + 256) / 256)), dim3(256), 0, st, chunks, count, nch, len,
                           top);
    else
        hipLaunchKernelGGL(k_dec_write, dim3((unsigned)(((size_t)nch * count + 255) / 256)), dim3(256), 0, st, chunks,
                           count, nch, off, top, buf);
    return 0;
}

int dec_launch_parse(const char *buf, const int64_t *off, size_t count, int words, int maxlen, uint32_t *ct, int *err,
                     hipStream_t st) {
    const dim3 grid((unsigned)((count + 255) / 256)), blk(256);
    switch (dec_width(words)) {
    case 32: hipLaunchKernelGGL(k_dec_parse<32>, grid, blk, 0, st, buf, off, count, words, maxlen, ct, err); break;
    case 64: hipLaunchKernelGGL(k_dec_parse<64>, grid, blk, 0, st, buf, off, count, words, maxlen, ct, err); break;
    case 128: hipLaunchKernelGGL(k_dec_parse<128>, grid, blk, 0, st, buf, off, count, words, maxlen, ct, err); break;
    default: return -1;
    }
    return 0;
}

}  // namespace fthe
