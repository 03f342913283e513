// bn_host.hpp -- host-side big-integer helpers (GMP) for key set-up.
//
// Key material is derived once per key on the host (prime search, inverses,
// Montgomery constants, exponent schedules), exactly as the reference does it
// on the host with NTL/GMP (paillier.cpp:43-90, paillier_gmp.cpp:108-239).
// Nothing on the per-ciphertext path runs here.
#pragma once
#include <gmp.h>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace fthe {

constexpr int RADIX_BITS = 28;
constexpr uint32_t RADIX_MASK = (1u << RADIX_BITS) - 1;

// RAII wrapper around mpz_t.
struct Mpz {
    mpz_t v;
    Mpz() { mpz_init(v); }
    explicit Mpz(unsigned long x) { mpz_init_set_ui(v, x); }
    Mpz(const Mpz &o) { mpz_init_set(v, o.v); }
    Mpz &operator=(const Mpz &o) { if (this != &o) mpz_set(v, o.v); return *this; }
    ~Mpz() { mpz_clear(v); }
    operator mpz_ptr() { return v; }
    operator mpz_srcptr() const { return v; }
    __mpz_struct *operator->() { return v; }              // GMP macros use Z->_mp_size
    const __mpz_struct *operator->() const { return v; }
    size_t bits() const { return mpz_sgn(v) == 0 ? 0 : mpz_sizeinbase(v, 2); }
};

inline void mpz_from_words(mpz_t x, const uint32_t *w, int n) { mpz_import(x, (size_t)n, -1, 4, 0, 0, w); }
inline void mpz_to_words(const mpz_t x, uint32_t *w, int n) {
    std::memset(w, 0, (size_t)n * 4);
    size_t cnt = 0;
    if (mpz_sgn(x) == 0) return;
    if (mpz_sizeinbase(x, 2) > (size_t)n * 32) return;
    mpz_export(w, &cnt, -1, 4, 0, 0, x);
}
// radix-2^28 limbs (S of them)
inline std::vector<uint32_t> to_limbs(const mpz_t x, int S) {
    std::vector<uint32_t> l(S, 0);
    Mpz t; mpz_set(t, x);
    for (int k = 0; k < S; k++) {
        l[k] = (uint32_t)(mpz_get_ui(t) & RADIX_MASK);
        mpz_fdiv_q_2exp(t, t, RADIX_BITS);
    }
    return l;
}

// Montgomery modulus for the radix-2^28 program kernel with S limbs.
struct MontMod {
    int S = 0;
    Mpz N, R, R2, R3;
    uint32_t nprime = 0;
    std::vector<uint32_t> ctx;   // N limbs (S) + nprime: the kernel's ctx buffer
    void init(const mpz_t modulus, int limbs) {
        S = limbs;
        mpz_set(N, modulus);
        mpz_set_ui(R, 1); mpz_mul_2exp(R, R, (mp_bitcnt_t)RADIX_BITS * S);
        mpz_powm_ui(R2, R, 2, N);
        mpz_powm_ui(R3, R, 3, N);
        Mpz m2b, inv;
        mpz_set_ui(m2b, 1); mpz_mul_2exp(m2b, m2b, RADIX_BITS);
        mpz_invert(inv, N, m2b);
        mpz_sub(inv, m2b, inv);
        nprime = (uint32_t)mpz_get_ui(inv);
        ctx = to_limbs(N, S);
        ctx.push_back(nprime);
    }
    // x * R mod N (Montgomery form of x), as limbs
    std::vector<uint32_t> mont(const mpz_t x) const {
        Mpz t; mpz_mul(t, x, R); mpz_mod(t, t, N);
        return to_limbs(t, S);
    }
    std::vector<uint32_t> plain(const mpz_t x) const {
        Mpz t; mpz_mod(t, x, N);
        return to_limbs(t, S);
    }
};

// Smallest kernel limb count whose R = 2^(28 S) exceeds 4N with margin
// (the kernel keeps every intermediate < 2N without final subtractions).
inline int kernel_limbs_for_bits(int bits) {
    static const int avail[] = {37, 74};
    for (int s : avail)
        if (bits + 8 <= RADIX_BITS * s) return s;
    return 0;
}

// ---- uniform op program for the montprog kernel ---------------------------
enum Op : uint32_t { OP_END = 0, OP_LOADX = 1, OP_STOREX = 2, OP_SQR = 3, OP_MUL = 4,
                     OP_ADDSLOT = 5, OP_ADDSMALL = 6 };

struct Prog {
    std::vector<uint32_t> w;
    double montmuls = 0;   // Montgomery products per lane (roofline accounting)
    void op(Op o, uint32_t a) { w.push_back(o); w.push_back(a); }
    void loadx(int s) { op(OP_LOADX, s); }
    void storex(int s) { op(OP_STOREX, s); }
    void sqr(int n) { if (n > 0) { op(OP_SQR, n); montmuls += n; } }
    void mul(int s) { op(OP_MUL, s); montmuls += 1; }
    void addslot(int s) { op(OP_ADDSLOT, s); }
    void addsmall(uint32_t k) { op(OP_ADDSMALL, k); }
    void end() { op(OP_END, 0); }

    // X <- X^e (Montgomery domain), left-to-right sliding window of width w.
    // Uses slots tbl0 .. tbl0 + 2^(w-1) - 1 and sq_slot.  e > 0.
    void pow(const mpz_t e, int tbl0, int sq_slot, int w) {
        size_t nb = mpz_sizeinbase(e, 2);
        if (mpz_sgn(e) == 0) return;   // caller never asks for e == 0
        if (nb == 1) return;           // e == 1
        // largest odd window value needed
        int ntab = 1 << (w - 1);
        storex(tbl0);
        sqr(1);
        storex(sq_slot);
        loadx(tbl0);
        for (int k = 1; k < ntab; k++) { mul(sq_slot); storex(tbl0 + k); }
        long i = (long)nb - 1;
        auto bit = [&](long b) { return mpz_tstbit(e, (mp_bitcnt_t)b); };
        auto window = [&](long top, long &low, unsigned &val) {
            low = top - w + 1; if (low < 0) low = 0;
            while (!bit(low)) low++;
            val = 0;
            for (long b = top; b >= low; b--) val = (val << 1) | (unsigned)bit(b);
        };
        long low; unsigned v;
        window(i, low, v);
        loadx(tbl0 + (int)((v - 1) / 2));
        i = low - 1;
        int pend = 0;
        while (i >= 0) {
            if (!bit(i)) { pend++; i--; continue; }
            window(i, low, v);
            pend += (int)(i - low + 1);
            sqr(pend); pend = 0;
            mul(tbl0 + (int)((v - 1) / 2));
            i = low - 1;
        }
        sqr(pend);
    }
};

}  // namespace fthe
