// LDS tile image of fthe_padic_m37 (gen_padic_mfma.py): the A operands of its two matrix-core Barrett
// products, for one prime P (or P = n for the Paillier-1024 public form) of 1009..1030 bits.
// Restates tools/padic_mfma_model.py MfmaKey.tile_image exactly (tests/test_padic_mfma_model.py compares
// the two byte for byte).
//
//   product 1 (quotient, columns s = 112..271 of q1 mu): A1[s][i] = mu'[s - i] for i < 136 (the lane's
//     q1 bytes, fed as b - 128), A1[s][136] = g1'[s - 112] (the constant digit 1 of the B operand), 0 above;
//     g1 = (128 mu sum_{i<136} 256^i - 2^918) >> 896: the -128 offset's correction and the truncation bias;
//     A1[s][137] = mu'[s - 3]: the B digit 16 c there adds c 2^28 mu for the bit 28 of q1's lowest limb;
//   product 2 (remainder; matrix column s = 1 + the column of q3 P, s = 0..159): A2[s][0] = g2'[s - 1]
//     (constant digit), A2[s][i] = P'[s - i] for i >= 1 (q3's bytes from digit 1: a plain Toeplitz
//     matrix); g2 = 128 P sum_{j<132} 256^j mod 2^1040;
//   x' = balanced base-256 digits of x (each in [-128, 127], same value).
// Tile t (1 KB): lane l's 16 bytes at l * 16 are row r = l & 31, digits i = 16 (l >> 5) + j (the
// v_mfma_i32_32x32x32_i8 A map).  Order: product 1 Toeplitz m - k = -3..1 (k <= 3), product 1 k = 4 for
// m = 0..4, product 2 k = 0 for m = 0..4, product 2 Toeplitz m - k = 0..3 (k >= 1).  19 tiles, padded to
// 20 KB (the kernel's LDS fill).
#pragma once
#include <gmp.h>
#include <cstdint>
#include <vector>

namespace padic_tiles {

constexpr int kTiles = 19, kImageBytes = 20 * 1024, kS1Lo = 112, kNq1 = 136, kConst1 = 136, kNq3 = 132;

// n balanced base-256 digits of x >= 0; false if they do not hold x
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

// 128 * x * sum_{i<n} 256^i = 128 * x * (256^n - 1) / 255
inline void offset_sum(mpz_t out, const mpz_t x, int n) {
    mpz_t g;
    mpz_init(g);
    mpz_ui_pow_ui(g, 256, (unsigned long)n);
    mpz_sub_ui(g, g, 1);
    mpz_divexact_ui(g, g, 255);
    mpz_mul(out, g, x);
    mpz_mul_ui(out, out, 128);
    mpz_clear(g);
}

// the image for P (K = 37 digits: P of 1009..1030 bits); empty on failure
inline std::vector<uint8_t> build(const mpz_t P) {
    std::vector<uint8_t> img;
    if (mpz_sizeinbase(P, 2) < 1009 || mpz_sizeinbase(P, 2) > 1030) return img;
    mpz_t mu, c, b;
    mpz_inits(mu, c, b, nullptr);
    mpz_set_ui(mu, 1);
    mpz_mul_2exp(mu, mu, 56 * 37);
    mpz_fdiv_q(mu, mu, P);
    std::vector<int> mud, pd, g1, g2;
    bool ok = balanced(mu, 135, mud) && balanced(P, 130, pd);
    offset_sum(c, mu, kNq1);
    mpz_set_ui(b, 1);
    mpz_mul_2exp(b, b, 918);
    mpz_sub(c, c, b);
    mpz_fdiv_q_2exp(c, c, 8 * kS1Lo);
    ok = ok && balanced(c, 160, g1);
    offset_sum(c, P, kNq3);
    mpz_fdiv_r_2exp(c, c, 1040);
    ok = ok && balanced(c, 131, g2);
    mpz_clears(mu, c, b, nullptr);
    if (!ok) return img;
    g2.resize(130);
    auto a1 = [&](int s, int i) -> int {
        if (i == kConst1) return (s >= kS1Lo && s < kS1Lo + 160) ? g1[s - kS1Lo] : 0;
        if (i == kConst1 + 1) {                 // 16 c, c = bit 28 of q1's lowest limb: mu' shifted 3 bytes
            int j = s - 3;
            return (j >= 0 && j < (int)mud.size()) ? mud[j] : 0;
        }
        if (i > kConst1) return 0;
        int j = s - i;
        return (j >= 0 && j < (int)mud.size()) ? mud[j] : 0;
    };
    auto a2 = [&](int s, int i) -> int {
        if (i == 0) return (s >= 1 && s <= (int)g2.size()) ? g2[s - 1] : 0;
        int j = s - i;
        return (j >= 0 && j < (int)pd.size()) ? pd[j] : 0;
    };
    img.reserve(kImageBytes);
    auto tile = [&](int prod, int s_base, int m, int k) {
        for (int l = 0; l < 64; l++) {
            const int r = l & 31, h = l >> 5;
            for (int j = 0; j < 16; j++) {
                const int s = s_base + 32 * m + r, i = 32 * k + 16 * h + j;
                img.push_back((uint8_t)((prod == 1 ? a1(s, i) : a2(s, i)) & 255));
            }
        }
    };
    for (int d = -3; d <= 1; d++) tile(1, kS1Lo, d >= 0 ? d : 0, d >= 0 ? 0 : -d);
    for (int m = 0; m < 5; m++) tile(1, kS1Lo, m, 4);
    for (int m = 0; m < 5; m++) tile(2, 0, m, 0);
    for (int d = 0; d <= 3; d++) tile(2, 0, d + 1, 1);
    img.resize(kImageBytes, 0);
    return img;
}

}  // namespace padic_tiles
