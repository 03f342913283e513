// fthe_glue.h -- declarations of the glue kernels (fthe_glue.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

namespace fthe {
struct RngKey { uint32_t k[8]; uint64_t nonce; };

constexpr int PACK_TILE = 64;       // ciphertexts per block of the tiled layout kernels
__global__ void k_pack_rows(const uint32_t *in, int win, const int64_t *idx, size_t count, int bit0, uint32_t *slot,
                            int S, int L, int rb);
__global__ void k_unpack_rows(uint32_t *x, const uint32_t *N, int S, int L, size_t count, uint32_t *out, int wout,
                              int rb);
__global__ void k_pack_u64(const uint64_t *m, size_t count, uint32_t *slot, int S, int L, int rb);
__global__ void k_copy_limbs(const uint32_t *src, int Ssrc, uint32_t *dst, int Sdst, int L);
__global__ void k_fill_const(const uint32_t *limbs, uint32_t *slot, int S, int L);
__global__ void k_canon(uint32_t *x, const uint32_t *N, int S, int L, int rb);
__global__ void k_crt_prep_q(uint32_t *cq, const uint32_t *q2, const uint32_t *kconst, uint32_t *v, int S, int L,
                             int rb);
__global__ void k_mul_add_out(const uint32_t *a, int na, const uint32_t *B, int nb, const uint32_t *h, int nh,
                              int L, size_t count, uint32_t *out, int wout, uint64_t *out_low, int rb);
// out = a + B h; the na = nb = nh = 37 / 74 forms on the register kernel (CRT recombination)
void mul_add_out(hipStream_t st, dim3 grid, const uint32_t *a, int na, const uint32_t *B, int nb, const uint32_t *h,
                 int nh, int L, size_t count, uint32_t *out, int wout, uint64_t *out_low, int rb);
__global__ void k_dec_lfunc(uint32_t *x, const uint32_t *P2, int S, const uint32_t *Pinv, int ky, uint32_t *y, int L, int rb);
__global__ void k_crt_dec_prep(uint32_t *mp, uint32_t *mq, const uint32_t *p, const uint32_t *q,
                               const uint32_t *two_p, uint32_t *d, int S, int L, int rb);
__global__ void k_rng_r(const uint32_t *n_words, int nw, int nbits, RngKey key, uint64_t index0, size_t count, uint32_t *r);
__global__ void k_rng_digits(RngKey key, uint64_t index0, size_t count, int nwin, int L, int bpd, int side, uint8_t *dig);
__global__ void k_alpha_digits(const uint32_t *alpha, int stride, int aw, size_t count, int nwin, int L, int bpd,
                               uint8_t *dig);
__global__ void k_slot_to_entries(const uint32_t *slot, int S, int L, size_t count, int ew, uint32_t *out);
// entries of nblk blocks of KB words, block h holding limbs [h K, h K + K) of the slot and KB - K zero pads
// (P-adic: 2 blocks, the digits; n-adic: 8 blocks, the four lane quarters of each digit)
__global__ void k_slot_to_digit_entries(const uint32_t *slot, int K, int KB, int nblk, int L, size_t count,
                                        uint32_t *out);
// fthe_hist.hip: histogram CSR and the segmented-product planner
__global__ void k_hist_count(const uint8_t *bin, int n_col, const int32_t *cut, int max_bin, const int32_t *inst,
                             size_t n_sel, int planes, int64_t n_bins, unsigned long long *cnt);
__global__ void k_hist_scatter(const uint8_t *bin, int n_col, const int32_t *cut, int max_bin, const int32_t *inst,
                               size_t n_sel, int planes, int64_t n_bins, size_t count, const int64_t *seg,
                               unsigned long long *cursor, int64_t *idx);
__global__ void k_group_counts(const int64_t *seg, size_t nseg, int K, int64_t *ng);
__global__ void k_plan_groups(const int64_t *seg, const int64_t *members, size_t nseg, const int64_t *gptr, size_t G,
                              int K, int64_t *gidx);
__global__ void k_zero_first_rows(const uint32_t *ez, const int64_t *seg, size_t nseg, int cw, uint32_t *ezm);
__global__ void k_u64_to_i64(const unsigned long long *a, int64_t *b, size_t n);
int exclusive_scan_i64(const int64_t *in, int64_t *out, size_t n, void *&tmp, size_t &tmp_bytes, hipStream_t st);
// fthe_dec.hip: decimal wire strings on the device
int dec_launch_chunks(const uint32_t *ct, int words, size_t count, int nch, uint32_t *chunks, hipStream_t st);
int dec_launch_len_write(const uint32_t *chunks, size_t count, int nch, int64_t *len, int32_t *top, int pass,
                         const int64_t *off, char *buf, hipStream_t st);
int dec_launch_parse(const char *buf, const int64_t *off, size_t count, int words, int maxlen, uint32_t *ct, int *err,
                     hipStream_t st);
__global__ void k_encode_fixed(const float *x, size_t count, uint64_t *m);
__global__ void k_decode_fixed(const uint64_t *m, size_t count, float *x);
}  // namespace fthe
