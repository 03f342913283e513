// fthe_hist.hip -- device-side index work of the homomorphic histogram:
// the CSR of (feature, bin) segments built from dense_bin_id, and the pass
// planner of the segmented K-way product.  Integer bookkeeping only (the
// ciphertext products run in the montprog kernel); everything stays in HBM so
// a level's histogram never round-trips through the host.
//
// Reference loop being replaced (hist_tree_builder.cpp:565-595, :640-664):
//   for fid: for iid in node: bid = dense_bin_id[iid*n_column + fid];
//            if (bid != max_num_bin) hist[cut_col_ptr[fid] + bid] += gh[iid]
// Products mod n^2 commute, so the order of the members inside a segment does
// not change the result; the scatter below is atomic (unordered).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdint>
#include "fthe_glue.h"

namespace fthe {

// thread t = (r, f) over n_sel x n_col, f fastest (one instance's bin row is contiguous)
__device__ __forceinline__ bool hist_key(const uint8_t *__restrict__ bin, int n_col, const int32_t *__restrict__ cut,
                                         int max_bin, const int32_t *__restrict__ inst, size_t t, int64_t &iid,
                                         int64_t &key) {
    const size_t r = t / (size_t)n_col;
    const int f = (int)(t - r * (size_t)n_col);
    iid = inst ? (int64_t)inst[r] : (int64_t)r;
    const int bid = bin[(size_t)iid * n_col + f];
    key = (int64_t)cut[f] + bid;
    return bid != max_bin;
}

__global__ void k_hist_count(const uint8_t *__restrict__ bin, int n_col, const int32_t *__restrict__ cut, int max_bin,
                             const int32_t *__restrict__ inst, size_t n_sel, int planes, int64_t n_bins,
                             unsigned long long *__restrict__ cnt) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_sel * (size_t)n_col) return;
    int64_t iid, key;
    if (!hist_key(bin, n_col, cut, max_bin, inst, t, iid, key)) return;
    for (int p = 0; p < planes; p++) atomicAdd(&cnt[p * n_bins + key], 1ull);
}

__global__ void k_hist_scatter(const uint8_t *__restrict__ bin, int n_col, const int32_t *__restrict__ cut, int max_bin,
                               const int32_t *__restrict__ inst, size_t n_sel, int planes, int64_t n_bins, size_t count,
                               const int64_t *__restrict__ seg, unsigned long long *__restrict__ cursor,
                               int64_t *__restrict__ idx) {
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_sel * (size_t)n_col) return;
    int64_t iid, key;
    if (!hist_key(bin, n_col, cut, max_bin, inst, t, iid, key)) return;
    for (int p = 0; p < planes; p++) {
        const int64_t s = p * n_bins + key;
        const unsigned long long pos = atomicAdd(&cursor[s], 1ull);
        idx[seg[s] + (int64_t)pos] = iid + (int64_t)p * (int64_t)count;
    }
}

// groups of <= K members per segment (an empty segment still makes one group: the integer 1)
__global__ void k_group_counts(const int64_t *__restrict__ seg, size_t nseg, int K, int64_t *__restrict__ ng) {
    size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s > nseg) return;
    if (s == nseg) { ng[s] = 0; return; }
    const int64_t n = seg[s + 1] - seg[s];
    ng[s] = n > K ? (n + K - 1) / K : 1;
}

// gidx[j*G + g] = member j of group g (-1: none); members == nullptr -> identity
__global__ void k_plan_groups(const int64_t *__restrict__ seg, const int64_t *__restrict__ members, size_t nseg,
                              const int64_t *__restrict__ gptr, size_t G, int K, int64_t *__restrict__ gidx) {
    size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    size_t lo = 0, hi = nseg;                 // largest s with gptr[s] <= g (gptr strictly increasing)
    while (hi - lo > 1) {
        size_t mid = (lo + hi) / 2;
        if (gptr[mid] <= (int64_t)g) lo = mid; else hi = mid;
    }
    const int64_t q = (int64_t)g - gptr[lo];
    const int64_t b = seg[lo] + q * K, e = seg[lo + 1];
    for (int j = 0; j < K; j++) {
        const int64_t t = b + j;
        gidx[(size_t)j * G + g] = t < e ? (members ? members[t] : t) : -1;
    }
}

__global__ void k_u64_to_i64(const unsigned long long *__restrict__ a, int64_t *__restrict__ b, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = (int64_t)a[i];
}

// out[0..n) = exclusive prefix sums of in[0..n) (hipcub); tmp grows as needed
int exclusive_scan_i64(const int64_t *in, int64_t *out, size_t n, void *&tmp, size_t &tmp_bytes, hipStream_t st) {
    size_t need = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, need, in, out, n, st) != hipSuccess) return -2;
    if (need > tmp_bytes) {
        if (tmp) hipFree(tmp);
        tmp = nullptr; tmp_bytes = 0;
        if (hipMalloc(&tmp, need) != hipSuccess) return -6;
        tmp_bytes = need;
    }
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, st) == hipSuccess ? 0 : -2;
}

// The reference's first `hist[bin] = hist[bin] + gh[iid]` into an unencrypted zero encrypts that zero
// (GHPair::operator+, common.h:156-160), so a populated bin is Enc(0) * prod(members).
// ezm[s] = enc_zero[s] for a populated segment (seg[s+1] > seg[s]) and the integer 1 for an empty
// one, which keeps the reference's unencrypted zero; one thread per word.
__global__ void k_zero_first_rows(const uint32_t *__restrict__ ez, const int64_t *__restrict__ seg, size_t nseg,
                                  int cw, uint32_t *__restrict__ ezm) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * (size_t)cw) return;
    const size_t s = t / (size_t)cw, w = t - s * (size_t)cw;
    ezm[t] = seg[s + 1] > seg[s] ? ez[t] : (uint32_t)(w == 0);
}

}  // namespace fthe
