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
// radix-2^B limbs (S of them)
inline std::vector<uint32_t> to_limbs(const mpz_t x, int S, int B = RADIX_BITS) {
    std::vector<uint32_t> l(S, 0);
    Mpz t; mpz_set(t, x);
    const uint32_t mask = (1u << B) - 1;
    for (int k = 0; k < S; k++) {
        l[k] = (uint32_t)(mpz_get_ui(t) & mask);
        mpz_fdiv_q_2exp(t, t, B);
    }
    return l;
}

// Kernel variants: limbs S of radix 2^B, lanes per ciphertext.  A modulus of
// `bits` bits needs R = 2^(B S) >= 2^8 N (almost-Montgomery headroom) and
// 2 S (2^B)^2 < 2^63 (64-bit column accumulators never overflow).
struct Shape { int S, B, lanes; };
inline Shape kernel_shape_for_bits(int bits) {
    static const Shape avail[] = {{37, 28, 1}, {74, 28, 1}, {152, 27, 4}};
    for (const Shape &s : avail)
        if (bits + 8 <= s.B * s.S) return s;
    return Shape{0, 0, 0};
}

// Montgomery modulus for the radix-2^28 program kernel with S limbs.
struct MontMod {
    Shape sh{0, 0, 0};
    int S = 0, B = RADIX_BITS;
    Mpz N, R, R2, R3;
    uint32_t nprime = 0;
    std::vector<uint32_t> ctx;   // N limbs (S) + nprime: the kernel's ctx buffer
    void init(const mpz_t modulus, Shape shape) {
        sh = shape; S = shape.S; B = shape.B;
        mpz_set(N, modulus);
        mpz_set_ui(R, 1); mpz_mul_2exp(R, R, (mp_bitcnt_t)B * S);
        mpz_powm_ui(R2, R, 2, N);
        mpz_powm_ui(R3, R, 3, N);
        Mpz m2b, inv;
        mpz_set_ui(m2b, 1); mpz_mul_2exp(m2b, m2b, B);
        mpz_invert(inv, N, m2b);
        mpz_sub(inv, m2b, inv);
        nprime = (uint32_t)mpz_get_ui(inv);
        ctx = to_limbs(N, S, B);
        ctx.push_back(nprime);
        // MULWC (four-lane kernel): quotient-estimate constants, doubles -k1 = -2^32 invN,
        // -k2 = -2^27 invN, -k3 = -2^59 invN and bias, invN <= 2^(B(S-2)) / N (rounded down).
        // Meaningful when N >= 2^(B S - 10) (classical_ok); zeros otherwise.
        double k[4] = {0, 0, 0, 0};
        if (classical_ok()) {
            Mpz t; mpz_fdiv_q_2exp(t, N, (mp_bitcnt_t)B * (S - 2) - 64);
            const double ntop = mpz_get_d(t) * (1.0 + 0x1p-50) * 0x1p-64;     // >= N / 2^(B(S-2))
            const double inv = 1.0 / ntop * (1.0 - 0x1p-50);
            k[0] = -inv * 0x1p32; k[1] = -inv * 0x1p27; k[2] = -inv * 0x1p59; k[3] = 0x1p-6;   // negated: -q
        }
        for (double d : k) {
            uint32_t w[2];
            std::memcpy(w, &d, 8);
            ctx.push_back(w[0]);
            ctx.push_back(w[1]);
        }
    }
    // the classical MSB-first product (OP_MULWC, tools/msb_model.py) needs the estimate's
    // ignored columns below 2^-8 of a quotient unit: N >= 2^(B S - 10)
    bool classical_ok() const { return sh.lanes == 4 && mpz_sizeinbase(N, 2) >= (size_t)(B * S - 10); }
    std::vector<uint32_t> limbs(const mpz_t x) const { return to_limbs(x, S, B); }
    // x * R mod N (Montgomery form of x), as limbs
    std::vector<uint32_t> mont(const mpz_t x) const {
        Mpz t; mpz_mul(t, x, R); mpz_mod(t, t, N);
        return to_limbs(t, S, B);
    }
};

inline int kernel_limbs_for_bits(int bits) { return kernel_shape_for_bits(bits).S; }

// ---- uniform op program for the montprog kernel ---------------------------
enum Op : uint32_t { OP_END = 0, OP_LOADX = 1, OP_STOREX = 2, OP_SQR = 3, OP_MUL = 4,
                     OP_ADDSLOT = 5, OP_ADDSMALL = 6,
                     // four-lane kernel only: canonical 128-word rows, kernarg row table entry t
                     OP_LOADW = 7, OP_MULW = 8, OP_STOREW = 9,
                     // gathered rows: row idx[g] of rows[0], idx (int64) at rows[t]; idx < 0 -> 1
                     OP_LOADWG = 10, OP_MULWG = 11,
                     // one-lane kernels only: LDS-DMA prefetch of the next multiplier
                     OP_PREFA = 12, OP_MULA = 13,
                     // fixed-base tables gathered by a per-lane digit (rows[0] table,
                     // rows[1] u8 digits [window][L]); one-lane: radix-2^B entries,
                     // four-lane: canonical 128-word rows
                     OP_LOADGD = 14, OP_MULGD = 15,
                     // the same with 16-bit windows (u16 digits, entry j*65536 + digit)
                     OP_LOADGD16 = 16, OP_MULGD16 = 17,
                     // four-lane kernel, row I/O: X <- row_t X mod N, classical MSB-first (no
                     // Montgomery factor); X canonical, N >= 2^(B S - 10)
                     OP_MULWC = 18,
                     // the same with the gathered row of MULWG t; CANON: X (< 4N) -> X mod N
                     OP_MULWGC = 19, OP_CANON = 20,
                     // P-adic kernel (gen_padic.py): plain X (2K limbs) <-> base-P digits;
                     // its LOADX / STOREX / SQR / MUL move and multiply digits
                     OP_LOADP = 22, OP_STOREP = 23 };

struct Prog {
    std::vector<uint32_t> w;
    double montmuls = 0;   // Montgomery products per lane (roofline accounting)
    double squarings = 0;  // of which squarings (the P-adic kernel's algorithmic MAC count differs)
    // one-lane kernels: pow()/pow_ones() prefetch each multiplier into LDS
    // (PREFA) ahead of the squarings that precede it, then MULA
    bool lds_a = false;
    void op(Op o, uint32_t a) { w.push_back(o); w.push_back(a); }
    void loadx(int s) { op(OP_LOADX, s); }
    void storex(int s) { op(OP_STOREX, s); }
    void sqr(int n) { if (n > 0) { op(OP_SQR, n); montmuls += n; squarings += n; } }
    void loadp(int s) { op(OP_LOADP, s); }
    void storep(int s) { op(OP_STOREP, s); }
    void mul(int s) { op(OP_MUL, s); montmuls += 1; }
    void addslot(int s) { op(OP_ADDSLOT, s); }
    void addsmall(uint32_t k) { op(OP_ADDSMALL, k); }
    void loadw(int t) { op(OP_LOADW, t); }
    void mulw(int t) { op(OP_MULW, t); montmuls += 1; }
    void storew(int t) { op(OP_STOREW, t); }
    void loadwg(int t) { op(OP_LOADWG, t); }
    void prefa(int s) { op(OP_PREFA, s); }
    void mula() { op(OP_MULA, 0); montmuls += 1; }
    // multiply by slot s, the squarings `n` before it (prefetch form when lds_a)
    void sqr_mul(int n, int s) {
        if (lds_a) { prefa(s); sqr(n); mula(); }
        else { sqr(n); mul(s); }
    }
    void mulwg(int t) { op(OP_MULWG, t); montmuls += 1; }
    // canon: canonical output (X < N), required when another MULWC / MULWGC follows
    void mulwc(int t, bool canon = false) { op(OP_MULWC, (uint32_t)t | (canon ? 0x100u : 0u)); montmuls += 1; }
    void mulwgc(int t, bool canon = false) { op(OP_MULWGC, (uint32_t)t | (canon ? 0x100u : 0u)); montmuls += 1; }
    void canon() { op(OP_CANON, 0); }
    void loadgd(int j) { op(OP_LOADGD, j); }
    void mulgd(int j) { op(OP_MULGD, j); montmuls += 1; }
    void loadgd16(int j) { op(OP_LOADGD16, j); }
    void mulgd16(int j) { op(OP_MULGD16, j); montmuls += 1; }
    void end() { op(OP_END, 0); }

    // X <- X^(2^j - 1) (Montgomery domain) by the all-ones addition chain:
    // 2^(2a)-1 = (2^a-1) 2^a + (2^a-1)  and  2^(a+1)-1 = 2 (2^a-1) + 1.
    // j-1 + popcount(j)-1 ... about log2(j) + popcount(j) multiplications and
    // j-1 squarings (the exponent 2^64-1 of GHPair::operator-: 63 + 6).
    void pow_ones(unsigned j, int base_slot, int tmp_slot) {
        if (j <= 1) return;
        storex(base_slot);
        int top = 31 - __builtin_clz(j);
        unsigned a = 1;
        for (int b = top - 1; b >= 0; b--) {
            storex(tmp_slot); sqr_mul((int)a, tmp_slot); a *= 2;          // 2^(2a)-1
            if ((j >> b) & 1) { sqr_mul(1, base_slot); a += 1; }          // 2^(a+1)-1
        }
    }

    // X <- X^e (Montgomery domain), left-to-right sliding window of width w.
    // Uses slots tbl0 .. tbl0 + 2^(w-1) - 1 and sq_slot.  e > 0.
    void pow(const mpz_t e, int tbl0, int sq_slot, int w) {
        size_t nb = mpz_sizeinbase(e, 2);
        if (mpz_sgn(e) == 0) return;   // caller never asks for e == 0
        if (nb == 1) return;           // e == 1
        if (nb >= 8 && mpz_popcount(e) == nb) { pow_ones((unsigned)nb, tbl0, sq_slot); return; }
        // largest odd window value needed
        int ntab = 1 << (w - 1);
        storex(tbl0);
        sqr(1);
        storex(sq_slot);
        if (lds_a) prefa(sq_slot);      // x^2 stays in the LDS A buffer for the whole table
        loadx(tbl0);
        for (int k = 1; k < ntab; k++) {
            if (lds_a) mula(); else mul(sq_slot);
            storex(tbl0 + k);
        }
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
            sqr_mul(pend, tbl0 + (int)((v - 1) / 2)); pend = 0;
            i = low - 1;
        }
        sqr(pend);
    }
};

}  // namespace fthe
