#!/usr/bin/env python3
"""Bit-exact model of the MFMA Barrett reduction of the P-adic kernel (fthe_padic_m37, gen_padic_mfma.py).

The P-adic kernel (tools/padic_model.py) spends ~60% of its multiply-adds in the two Barrett
reductions of every product mod P^2, and both of their products have a CONSTANT operand: the upper
half of q1 * mu and the lower half of q3 * P.  Over the 64 lanes of a wave (64 independent
ciphertext halves) each is a matrix product -- a Toeplitz matrix of the constant's base-256 digits
times the 64 lanes' digit vectors -- which is what the gfx950 matrix core computes:
v_mfma_i32_32x32x32_i8 multiplies a 32x32 i8 tile (the constant, read from LDS) by 32x32 i8 (32 lanes'
digits), accumulating exact int32 column sums.  The variable x variable products (x0^2, 2 x0 x1) stay
on the VALU; the lanes turn column sums back into 28-bit limbs with one v_mad_i64_i32 per column.

Digits.  The matrix core multiplies SIGNED bytes.  The constants are stored in balanced base-256 digits
(each in [-128, 127], same value); a lane's variable bytes b_i are fed as b_i ^ 0x80 = b_i - 128, and the
exact correction 128 * C * sum_i 256^i (a per-key constant) is added back through ONE extra digit
column: the B operand carries a constant digit 1 there and the A tiles that column's balanced digits of
the correction.  So no correction instruction runs on the VALU.

Product 1 (quotient):  q1 = floor(T / b^(K-1)) as bytes i < 136 (its 38 limbs, the lowest one allowed to
be < 2^29), constant digit at i = 136.  Columns s in [112, 272) are formed; the dropped columns s < 112
move the sum by less than 2^917.1, so a bias of -2^918 (inside the correction constant) makes the
computed numerator N satisfy  Pi - 2^920 < N < Pi  for Pi = q1 * mu, i.e. q3 = floor(N / b^(K+1)) is
Barrett's estimate or one below it.  N < 0 only when q1 = 0 (then Pi = 0, q3 = -1): the kernel clamps
q3 to 0 there (T < b^36 < P, so 0 is the exact quotient's lower bound and the remainder is T).
Product 2 (remainder):  r = (T - q3 P) mod b^K from columns s < 130 of q3 * P, exact (no truncation):
constant digit at i = 0, q3's bytes at i = 1..132; the matrix columns are s + 1, so that digit i meets
P'[s + 1 - i] (a plain Toeplitz matrix, zero above the diagonal band, as the skipped tiles assume).

This model computes the same column sums (as the tile x digit dot products the lanes feed the matrix
core), the same chunk accumulation (64-bit, arithmetic shifts) and the same clamping, and asserts every
bound (int32 column sums, 64-bit accumulators, digits < 5P).  It also builds the A tiles in the lane
order of the LDS image that the kernel reads (tile_image), which the host code must reproduce.

Run:  python tools/padic_mfma_model.py [seed] [trials]
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import padic_model as pm  # noqa: E402

B = pm.B
MASK = pm.MASK
K = 37
S1_LO, S1_HI = 112, 272          # product-1 columns (5 M-tiles of 32)
NQ1 = 136                        # q1 bytes (34 dwords, offset -128)
CONST1 = 136                     # product-1 constant digit position
NQ3 = 132                        # q3 bytes (33 dwords after the constant byte), offset -128
S2_HI = 160                      # product-2 columns 0..159 (only s < 130 are used)
BIAS_BITS = 918
QBIT = B * (K + 1)               # 1064: q3 = floor(N / 2^1064)
TILE_D1 = (-3, -2, -1, 0, 1)     # product-1 Toeplitz tiles (k <= 3), by d = m - k
TILE_D2 = (0, 1, 2, 3)           # product-2 Toeplitz tiles (k >= 1)


def s32(x):
    assert -(1 << 31) <= x < (1 << 31), "int32 column sum overflow"
    return x


def balanced(x, n):
    """n balanced base-256 digits (each in [-128, 127]) of x >= 0; asserts that they hold x exactly"""
    d = []
    c = 0
    for _ in range(n):
        v = (x & 255) + c
        x >>= 8
        if v >= 128:
            d.append(v - 256)
            c = 1
        else:
            d.append(v)
            c = 0
    assert x == 0 and c == 0, "balanced digits do not hold the value"
    return d


class MfmaKey(pm.PadicKey):
    def __init__(self, P):
        super().__init__(P, K)
        mu = pm.value(self.mu)
        self.mu_d = balanced(mu, 135)                       # mu < 2^1063: 134 digits + a carry digit
        self.P_d = balanced(P, 130)                         # P < 2^1031
        c1 = 128 * mu * sum(256 ** i for i in range(NQ1))
        g1 = (c1 - (1 << BIAS_BITS)) >> (8 * S1_LO)         # a multiple of 256^112: columns >= 112
        self.g1 = balanced(g1, S1_HI - S1_LO)
        c2 = 128 * P * sum(256 ** i for i in range(NQ3))
        self.g2 = balanced(c2 % (1 << 1040), 131)[:130]     # mod 2^1040 (columns < 130; 256^130 = 0 mod b^K)

    # A[s][i] of the two products (s: output column, i: B digit index)
    def a1(self, s, i):
        if i == CONST1:
            return self.g1[s - S1_LO] if S1_LO <= s < S1_HI else 0
        if i == CONST1 + 1:                     # 16 c for the bit 28 of q1's lowest limb (< 2^29)
            j = s - 3
            return self.mu_d[j] if 0 <= j < len(self.mu_d) else 0
        if i > CONST1:
            return 0
        j = s - i
        return self.mu_d[j] if 0 <= j < len(self.mu_d) else 0

    def a2(self, s, i):
        """product 2 in shifted columns: s = 1 + the column of q3 P (weight 256^(s - 1)), so that the
        q3 digit i (byte i - 1) meets P'[s - i]: a plain Toeplitz matrix, zero for i > s"""
        if i == 0:
            return self.g2[s - 1] if 1 <= s <= len(self.g2) else 0
        j = s - i
        return self.P_d[j] if 0 <= j < len(self.P_d) else 0

    def check_skipped_tiles(self):
        """the kernel forms only tiles (m, k) with m - k <= 1 (product 1) and m >= k (product 2): every
        other tile of the A matrices must be zero (and the Toeplitz tiles equal along m - k)"""
        for m in range(5):
            for k in range(5):
                for r in range(32):
                    for i in range(32 * k, 32 * k + 32):
                        if m - k > 1:
                            assert self.a1(S1_LO + 32 * m + r, i) == 0, (m, k)
                        if m < k:
                            assert self.a2(32 * m + r, i) == 0, (m, k)

    def tile_image(self):
        """the 19 A tiles as the kernel's LDS image: tile t is 1 KB, lane l's 16 bytes at l * 16
        (row r = l & 31, digits i = 16 (l >> 5) + j of the tile); order: product 1 Toeplitz d = -3..1
        (k = 0), product 1 k = 4 for m = 0..4, product 2 k = 0 for m = 0..4, product 2 Toeplitz d = 0..3
        (k = 1).  Entries are int8 as unsigned bytes."""
        out = bytearray()

        def tile(fn, s_base, m, k):
            for l in range(64):
                r, h = l & 31, l >> 5
                for j in range(16):
                    out.append(fn(s_base + 32 * m + r, 32 * k + 16 * h + j) & 255)
        for d in TILE_D1:                       # (m, k) = (d + 3, 3) is one of its instances... any will do
            m, k = (d, 0) if d >= 0 else (0, -d)
            tile(self.a1, S1_LO, m, k)
        for m in range(5):
            tile(self.a1, S1_LO, m, 4)
        for m in range(5):
            tile(self.a2, 0, m, 0)
        for d in TILE_D2:
            tile(self.a2, 0, d + 1, 1)
        return bytes(out)


def pack(limbs_, shift_bits, ndw):
    """the kernel's radix conversion: limb t (value < 2^30) lands at bit 28 t + shift_bits; dword w is
    acc's low word after the limbs that start in it; acc >>= 32 (acc < 2^64 asserted)"""
    dw = []
    acc = 0
    t = 0
    for w in range(ndw):
        while t < len(limbs_) and (B * t + shift_bits) // 32 == w:
            sh = B * t + shift_bits - 32 * w
            acc += limbs_[t] << sh
            assert acc < (1 << 64)
            t += 1
        dw.append(acc & 0xFFFFFFFF)
        acc >>= 32
    assert acc == 0 and t == len(limbs_), "packed value does not fit"
    return dw


def digits_of(dwords, xor_masks):
    """signed bytes the matrix core sees (dword i XOR xor_masks[i])"""
    out = []
    for w, m in zip(dwords, xor_masks):
        v = w ^ m
        for b in range(4):
            x = (v >> (8 * b)) & 255
            out.append(x - 256 if x >= 128 else x)
    return out


def orpack(limbs_, shift_bits, ndw):
    """the kernel's pack: dword w = (L_lo >> off) | (L_lo+1 << (28 - off)), normalised limbs (< 2^28)"""
    assert all(0 <= v < (1 << B) for v in limbs_)
    val = sum(v << (B * t + shift_bits) for t, v in enumerate(limbs_))
    assert val < (1 << (32 * ndw))
    return [(val >> (32 * w)) & 0xFFFFFFFF for w in range(ndw)]


def product1(key, q1):
    """q1: 38 limbs (q1[0] < 2^29, others < 2^28).  Returns (q3 limbs, clamped).  Bit 28 of q1[0] (c) is
    fed as the digit 16 c at position 137, whose A column is mu' shifted by 3 bytes."""
    c = q1[0] >> B
    assert c in (0, 1)
    dw = orpack([q1[0] & MASK] + list(q1[1:]), 0, 34) + [1 | (c << 12), 0, 0, 0, 0, 0]
    dig = digits_of(dw, [0x80808080] * 34 + [0] * 6)
    assert dig[CONST1] == 1 and dig[CONST1 + 1] == 16 * c
    col = {}
    for s in range(S1_LO, S1_HI):
        col[s] = s32(sum(key.a1(s, i) * dig[i] for i in range(160) if dig[i]))
    acc = 0
    q3 = []
    for t in range(-6, 40):
        for s in range(S1_LO, S1_HI):
            if (8 * s - QBIT) // B == t:
                acc = pm.s64(acc + (col[s] << (8 * s - QBIT - B * t)))
        if 0 <= t < K:
            q3.append(acc & MASK)
        acc >>= B
    assert acc in (0, -1)
    clamped = acc == -1
    if clamped:
        assert all(v == MASK for v in q3)
        q3 = [0] * K
    return q3, clamped


def product2(key, q3, T):
    """r = (T - q3 P) mod b^K (T: limbs 0..K-1, < 2^29 allowed)"""
    dw = orpack(q3, 8, 33)
    dw[0] |= 1
    dw += [0] * 7
    dig = digits_of(dw, [0x80808000] + [0x80808080] * 32 + [0x00000080] + [0] * 6)
    assert dig[0] == 1
    r = []
    acc = 0
    for t in range(K):
        acc = acc + T[t]
        for s in range(1, 131):
            if (8 * s - 8) // B == t:
                c = s32(sum(key.a2(s, i) * dig[i] for i in range(160) if dig[i]))
                acc = pm.s64(acc - (c << (8 * s - 8 - B * t)))
        r.append(acc & MASK)
        acc >>= B
    return r


def barrett(key, T, clamp=True):
    q1 = T[K - 1:2 * K]
    q3, clamped = product1(key, q1)
    r = product2(key, q3, T)
    assert pm.value(T) - pm.value(q3) * key.P == pm.value(r), "T = q3 P + r"
    return q3, r, clamped


pm_barrett = pm.barrett


def install():
    """route padic_model's sqr / mul / loadp through this Barrett"""
    pm.barrett = lambda key, T: barrett(key, T)[:2]


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rng = random.Random(seed)
    install()
    nclamp = 0
    for t in range(trials):
        bits = rng.choice([1009, 1010, 1023, 1024, 1024, 1029, 1030])
        P = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        key = MfmaKey(P)
        assert len(key.tile_image()) == 19 * 1024
        key.check_skipped_tiles()
        P2 = P * P
        # random and extreme digits through squaring / product
        for x0v, x1v in ((5 * P - 1, 5 * P - 1), (1, 0), (2, 0), (0, 1), (P - 1, P - 1),
                         (rng.randrange(5 * P), rng.randrange(5 * P))):
            x0, x1 = pm.limbs(x0v, K), pm.limbs(x1v, K)
            z0, z1 = pm.sqr(key, x0, x1)
            X = x0v + x1v * P
            assert (pm.value(z0) + pm.value(z1) * P) % P2 == X * X % P2
            pm.check_digit(key, z0)
            pm.check_digit(key, z1)
        a0, a1 = pm.limbs(rng.randrange(5 * P), K), pm.limbs(rng.randrange(5 * P), K)
        b0, b1 = pm.limbs(rng.randrange(5 * P), K), pm.limbs(rng.randrange(5 * P), K)
        z0, z1 = pm.mul(key, a0, a1, b0, b1)
        A = pm.value(a0) + pm.value(a1) * P
        Bv = pm.value(b0) + pm.value(b1) * P
        assert (pm.value(z0) + pm.value(z1) * P) % P2 == A * Bv % P2
        pm.check_digit(key, z0)
        pm.check_digit(key, z1)
        # LOADP of small and large plain values (clamp path for X < b^36)
        for X in (0, 1, 5, (1 << 1008) - 1, 1 << 1008, 50 * P2 - 1, rng.randrange(P2)):
            T = pm.limbs(X, 2 * K)
            q3, r, cl = barrett(key, T)
            nclamp += cl
            assert pm.value(r) < 5 * P and pm.value(q3) * P + pm.value(r) == X
        if t < 3:
            for X, e in ((rng.randrange(1, P), P), (rng.randrange(P2), P - 1), (1, P), (2, P - 1)):
                got = pm.value(pm.padic_pow(key, X, e))
                assert got % P2 == pow(X, e, P2), t
    print(f"ok: {trials} keys (squaring / product / LOADP through the MFMA Barrett, {nclamp} clamped quotients, "
          f"exponentiations)")


if __name__ == "__main__":
    main()
