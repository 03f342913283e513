// Per-key context of fthe_nadic_b76 (gen_nadicb.py), the parties' public-key encrypt r^n mod n^2 on base-n
// digits with matrix-core Barrett reductions by n (party.h:118-142 -> paillier.cpp:122-139).  Restates
// tools/nadicb_model.py nadicb_image exactly (tests/test_nadicb_model.py compares the bytes through
// fthe_debug_nadicb_image):
//
//   mu = floor(2^4128 / n); mu' (262) and n' (257) = balanced base-256 digits (each in [-128, 127]);
//   copies: for output row m = 0..15 of an A tile, copy slot s(m) (rows 0-3, 12-15 -> 0..7, rows 4-11 ->
//     8..15), byte y = c'[K_m - y] with K_m = s_base + m + KO (product 1: c = mu, s_base = 260; product 2:
//     c = n, 0), 0 outside;
//   corrections (int32 per output column, the MFMAs' srcC): product 1 column s = 260 + i:
//     128 sum_{k < 264} mu'[s - k] (-1 at s = 263: the -2^2104 truncation bias), product 2 column s:
//     128 sum_{k < 260} n'[s - k];
//   then n as 76 limbs of 27 bits (the kernel's CANON).
// Layout constants: gen/nadicb_layout.h, written by fedtree_amd/build.py from gen_nadicb.py.
#pragma once
#include <gmp.h>
#include <cstdint>
#include <vector>

#include "addb_image.hpp"
#include "gen/nadicb_layout.h"

namespace nadicb {

inline bool n_ok(const mpz_t n) {
    const size_t b = mpz_sizeinbase(n, 2);
    return mpz_odd_p(n) && b >= 2041 && b <= 2048;
}

inline bool build(const mpz_t n, std::vector<uint8_t> &img) {
    if (!n_ok(n)) return false;
    mpz_t mu;
    mpz_init(mu);
    mpz_ui_pow_ui(mu, 2, kNbA + kNbC);
    mpz_fdiv_q(mu, mu, n);
    std::vector<int> mud, nd;
    const bool ok = addb::balanced(mu, kNbNd1, mud) && addb::balanced(n, kNbNd2, nd);
    mpz_clear(mu);
    if (!ok) return false;
    img.assign(kNbCtxBytes, 0);
    struct P { int off; const std::vector<int> *d; int sbase, ko; } ps[2] = {
        {kNbA1Off, &mud, kNbS1Base, kNbKO1}, {kNbA2Off, &nd, 0, kNbKO2}};
    for (const P &p : ps)
        for (int m = 0; m < 16; m++) {
            const int base = p.off + addb::copy_slot(m) * kNbCopy, km = p.sbase + m + p.ko;
            for (int y = 0; y < kNbCopy; y++) {
                const int i = km - y;
                img[base + y] = (0 <= i && i < (int)p.d->size()) ? (uint8_t)((*p.d)[i] & 255) : 0;
            }
        }
    auto dig = [](const std::vector<int> &d, int i) { return (0 <= i && i < (int)d.size()) ? d[i] : 0; };
    auto put = [&](int off, uint32_t u) {
        for (int b = 0; b < 4; b++) img[off + b] = (uint8_t)(u >> (8 * b));
    };
    for (int i = 0; i < 16 * kNbTiles1; i++) {
        const int s = kNbS1Base + i;
        int32_t c = 0;
        for (int k = 0; k < 4 * kNbNq1; k++) c += dig(mud, s - k);
        c *= 128;
        if (s == kNbBiasCol) c += kNbBiasDigit;
        put(kNbCorr1Off + 4 * i, (uint32_t)c);
    }
    for (int s = 0; s < 16 * kNbTiles2; s++) {
        int32_t c = 0;
        for (int k = 0; k < 4 * kNbNq3; k++) c += dig(nd, s - k);
        put(kNbCorr2Off + 4 * s, (uint32_t)(128 * c));
    }
    mpz_t t;
    mpz_init(t);
    for (int j = 0; j < 76; j++) {                       // n limbs of 27 bits
        mpz_fdiv_q_2exp(t, n, 27 * j);
        put(kNbNOff + 4 * j, (uint32_t)(mpz_get_ui(t) & ((1u << 27) - 1)));
    }
    mpz_clear(t);
    return true;
}

}  // namespace nadicb
