// Per-key context of fthe_addb_q152 (gen_addb.py), the Paillier-2048 ciphertext add with a matrix-core
// Barrett reduction: out = x y mod N, N = n^2 (paillier.cpp:92-105).  Restates tools/addb_model.py
// addb_image exactly (tests/test_addb_model.py compares the bytes through fthe_debug_addb_image):
//
//   mu = floor(2^8200 / N); mu' (515) and N' (513) = balanced base-256 digits (each in [-128, 127]);
//   copies: for output row m = 0..15 of an A tile, copy slot s(m) (rows 0-3, 12-15 -> 0..7, rows 4-11 ->
//     8..15: the ds_read_b128 lane groups then hit 64 distinct banks), byte y = c'[K_m - y] with
//     K_m = s_base + m + KO (product 1: c = mu, s_base = 512, KO = 64; product 2: c = N, 0, 560), 0 outside;
//   corrections (int32 per output column, the MFMAs' srcC): product 1 column s = 512 + i:
//     128 sum_{k < 516} mu'[s - k] (-2 at s = 515: the -2^4121 truncation bias), product 2 column s:
//     128 sum_{k < 512} N'[s - k];
//   then N as 128 little-endian dwords (the kernel's final conditional subtractions), then the integer 1 as a
//   128-dword row (the operand of a gathered index < 0).
// Layout constants: gen/addb_layout.h, written by fedtree_amd/build.py from gen_addb.py.
#pragma once
#include <gmp.h>
#include <cstdint>
#include <vector>

#include "gen/addb_layout.h"

namespace addb {

inline bool balanced(const mpz_t x, int n, std::vector<int> &d) {
    mpz_t t;
    mpz_init_set(t, x);
    d.assign(n, 0);
    int c = 0;
    for (int k = 0; k < n; k++) {
        int v = (int)(mpz_get_ui(t) & 255u) + c;
        mpz_fdiv_q_2exp(t, t, 8);
        if (v >= 128) { d[k] = v - 256; c = 1; } else { d[k] = v; c = 0; }
    }
    bool ok = mpz_sgn(t) == 0 && c == 0;
    mpz_clear(t);
    return ok;
}

inline int copy_slot(int m) { return m < 4 ? m : m < 12 ? m + 4 : m - 8; }

// n (n_words little-endian u32) -> the kctx bytes; false unless N = n^2 has 4095 or 4096 bits
inline bool build(const mpz_t n, std::vector<uint8_t> &img) {
    mpz_t N, mu;
    mpz_inits(N, mu, nullptr);
    mpz_mul(N, n, n);
    const size_t nb = mpz_sizeinbase(N, 2);
    bool ok = nb == 4095 || nb == 4096;
    std::vector<int> mud, Nd;
    if (ok) {
        mpz_ui_pow_ui(mu, 2, kAddbMuShift);
        mpz_fdiv_q(mu, mu, N);
        ok = balanced(mu, kAddbNd1, mud) && balanced(N, kAddbNd2, Nd);
    }
    if (ok) {
        img.assign(kAddbKctxBytes, 0);
        struct P { int off; const std::vector<int> *d; int sbase, ko; } ps[2] = {
            {kAddbA1Off, &mud, kAddbS1Base, kAddbKO1}, {kAddbA2Off, &Nd, 0, kAddbKO2}};
        for (const P &p : ps)
            for (int m = 0; m < 16; m++) {
                const int base = p.off + copy_slot(m) * kAddbCopy, km = p.sbase + m + p.ko;
                for (int y = 0; y < kAddbCopy; y++) {
                    const int i = km - y;
                    img[base + y] = (0 <= i && i < (int)p.d->size()) ? (uint8_t)((*p.d)[i] & 255) : 0;
                }
            }
        auto dig = [](const std::vector<int> &d, int i) { return (0 <= i && i < (int)d.size()) ? d[i] : 0; };
        auto put = [&](int off, int32_t v) {
            const uint32_t u = (uint32_t)v;
            for (int b = 0; b < 4; b++) img[off + b] = (uint8_t)(u >> (8 * b));
        };
        for (int i = 0; i < 16 * kAddbTiles1; i++) {
            const int s = kAddbS1Base + i;
            int32_t c = 0;
            for (int k = 0; k < 4 * kAddbNq1; k++) c += dig(mud, s - k);
            c *= 128;
            if (s == kAddbBiasCol) c += kAddbBiasDigit;
            put(kAddbCorr1Off + 4 * i, c);
        }
        for (int s = 0; s < 16 * kAddbTiles2; s++) {
            int32_t c = 0;
            for (int k = 0; k < 4 * kAddbNq3; k++) c += dig(Nd, s - k);
            put(kAddbCorr2Off + 4 * s, 128 * c);
        }
        size_t cnt = 0;
        mpz_export(img.data() + kAddbNOff, &cnt, -1, 4, 0, 0, N);
        img[kAddbOneOff] = 1;                                          // the row 1 (gathered index < 0)
    }
    mpz_clears(N, mu, nullptr);
    return ok;
}

}  // namespace addb
