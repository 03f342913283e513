#!/usr/bin/env python3
"""Bit-exact model of the n-adic public-key encrypt with matrix-core Barrett reductions (fthe_nadic_b76,
fedtree_amd/csrc/gen_nadicb.py).

A party's encrypt (Party::encrypt_histogram, party.h:118-142 -> paillier.cpp:122-139) is r^n mod n^2.  As in
gen_nadic.py the residue is kept as two base-n digits, X = x0 + x1 n, and a product is

    X Y == x0 y0 + (x0 y1 + x1 y0) n              (mod n^2)
    x0 y0 = u1 n + u0                              Barrett 1: quotient AND remainder
    Z = u0 + ((x0 y1 + x1 y0 + u1) mod n) n        Barrett 2: remainder only

The variable x variable products z1 = x0 y0 and z2 = x0 y1 + x1 y0 (a squaring: x0^2 and 2 x0 x1) stay on the
VALU (one quad of lanes per ciphertext, 76 limbs of 27 bits per digit, operand scanning); both Barrett
reductions have constant operands (mu, n) and run on v_mfma_i32_16x16x64_i8 over the 16 ciphertexts of a
wave, as the ciphertext add's reduction by n^2 does (tools/addb_model.py) -- half the size here: the Barretts
are by the 2048-bit n.

Barrett parameters (n of 2041..2048 bits; digits in [0, 3n); z < 19 n^2 < 2^4101):
    q1 = floor(z / 2^A),  A = 2016                 the z dwords 63..128: 66 dwords (264 bytes), q1 < 2^2085
    mu = floor(2^(A + C) / n),  C = 2112           mu < 2^2088: 262 balanced base-256 digits
    q3 = floor(q1 mu / 2^C)                        z/n - q1 mu/2^C < 2^A/n + q1/2^C < 2^-20: q or q - 1
Product 1 forms only the byte columns s >= 260 of q1 mu (17 tiles of 16 columns, 260..531); every |column|
< 264 * 128 * 255 < 2^23.05, so the dropped ones move the sum by less than 2^2103.05, and a bias of -2^2104
(digit -1 in column 263) makes the numerator N1 satisfy  Pi - 2^2105 < N1 <= Pi:  q3 = floor(N1 / 2^2112)
is q, q - 1 or q - 2, and r = z - q3 n lies in [0, 3n) -- the digit bound, so products chain with no
conditional subtraction (CANON reduces the digits at the end).  N1 < 0 only when Pi < 2^2104 (then z < n):
q3 is clamped to 0.  q3 < 19 n < 2^2053: 65 dwords.
Product 2 forms r2 = q3 n mod 2^2080 (byte columns 0..259 of 17 tiles), and r = (z - r2) mod 2^2080, exact
because r < 3n < 2^2050.

Matrix-core arithmetic (as addb_model.py): signed bytes -- the constants as balanced digits, the variable
bytes fed as b - 128 (b ^ 0x80), the correction 128 sum_k c[s - k] over the real input bytes (and product 1's
bias) as each column's initial accumulator; int32 column sums; each lane folds the 4 rows it holds of a tile
into an int64 group (4 adjacent columns = one dword position); the groups are normalised to dwords with a
signed carry in three chunks of tiles, chunk j on quad lane j (tiles 0..7 -> dwords 0..31, 8..15 -> 32..63,
16 -> 64..67), the chunk carry handed on by DPP -- so r2's dwords land on the lanes that hold the same dwords
of z (lane j: z dwords [32 j, 32 j + 32)), and q3's one dword below them (q3 dword i = group i + 1).

This model computes exactly those column sums (tile by tile, only the tiles whose constant entries are not
all zero), groups, chunk carries and the clamp, asserts every bound, and runs exponentiations through the
digit products against Python's pow.  The LDS image (nadicb_image) is compared byte for byte with the host
builder (fedtree_amd/csrc/nadicb_image.hpp) by tests/test_nadicb_model.py.
Run:  python tools/nadicb_model.py [seed] [trials]
"""
import os
import random
import sys

B = 27                          # limb radix bits of the VALU product
S = 76                          # limbs per digit (4 lanes x 19)
Q = S // 4
A_BITS, C_BITS = 2016, 2112
NZ = 129                        # z dwords (z < 2^4101): lane j holds [32 j, 32 j + 32), lane 3 also dword 128
Q1_DW0 = A_BITS // 32           # q1 = z dwords 63 .. 128
NQ1 = NZ - Q1_DW0               # 66
NQ3 = 65                        # q3 < 2^2053
R_DW = 65                       # r formed mod 2^2080
S1_BASE = 260                   # product-1 byte columns 260 .. 531
TILES1, TILES2 = 17, 17
KB1, KB2 = 5, 5                 # K-blocks of 64 bytes (q1: 264 real bytes, q3: 260)
BIAS_COL, BIAS_DIGIT = 263, -1  # -2^2104
ND1, ND2 = 262, 257             # balanced digits of mu and n
CHUNKS = (tuple(range(0, 8)), tuple(range(8, 16)), (16,))
N_BITS_MIN, N_BITS_MAX = 2041, 2048
FAST = [False]                  # column sums by convolution (exponentiations); the tile path otherwise


def s32(x):
    assert -(1 << 31) <= x < (1 << 31), "int32 column sum overflow"
    return x


def s64(x):
    assert -(1 << 63) <= x < (1 << 63), "int64 overflow"
    return x


def balanced(x, n):
    """n balanced base-256 digits (each in [-128, 127]) of x >= 0, asserting that they hold x exactly"""
    d, c = [], 0
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


def band(nd, s0, k0):
    """the 16 x 64 tile of output bytes [s0, s0 + 16) x input bytes [k0, k0 + 64) has a digit c[s - k], 0 <= s - k < nd"""
    lo, hi = s0 - k0 - 63, s0 + 15 - k0
    return not (hi < 0 or lo >= nd)


ACT1 = [[kb for kb in range(KB1) if band(ND1, S1_BASE + 16 * t, 64 * kb)] for t in range(TILES1)]
ACT2 = [[kb for kb in range(KB2) if band(ND2, 16 * t, 64 * kb)] for t in range(TILES2)]


class Key:
    """The per-key constants: balanced digits of mu and n, the column corrections (srcC initial values)."""

    def __init__(self, n):
        assert n % 2 == 1 and N_BITS_MIN <= n.bit_length() <= N_BITS_MAX, "n of 2041..2048 bits"
        self.n = n
        self.mu = (1 << (A_BITS + C_BITS)) // n
        assert self.mu < (1 << 2088)
        self.mud = balanced(self.mu, ND1)
        self.nd = balanced(n, ND2)
        self.corr1 = [128 * sum(self._dig(self.mud, s - k) for k in range(4 * NQ1))
                      for s in range(S1_BASE, S1_BASE + 16 * TILES1)]
        self.corr1[BIAS_COL - S1_BASE] += BIAS_DIGIT
        self.corr2 = [128 * sum(self._dig(self.nd, s - k) for k in range(4 * NQ3)) for s in range(16 * TILES2)]

    @staticmethod
    def _dig(d, i):
        return d[i] if 0 <= i < len(d) else 0

    def product(self, digits, act, base, tiles, nreal, feed, corr):
        """column sums of the constant times the fed bytes over the active tiles only (the MFMAs), from the
        corrections; checked against the full sum (the skipped tiles are all zero).  FAST: the same column
        sums as one integer convolution of the digits with the true bytes (the corrections cancel the -128
        offset exactly, which the tile path asserts), for long exponentiations."""
        if FAST[0]:
            import numpy as np
            b = np.array([f + 128 for f in feed[:nreal]], dtype=np.int64)
            full = np.convolve(np.array(digits, dtype=np.int64), b)
            cols = []
            for i in range(16 * tiles):
                s = base + i
                v = int(full[s]) if s < len(full) else 0
                cols.append(s32(v + (BIAS_DIGIT if (base == S1_BASE and s == BIAS_COL) else 0)))
            return cols
        cols = [s32(c) for c in corr]
        for t in range(tiles):
            for kb in act[t]:
                for r in range(16):
                    s = base + 16 * t + r
                    acc = sum(self._dig(digits, s - k) * (feed[k] if k < nreal else 0)
                              for k in range(64 * kb, 64 * kb + 64))
                    cols[16 * t + r] = s32(cols[16 * t + r] + acc)
        for i in range(16 * tiles):
            s = base + i
            assert cols[i] == corr[i] + sum(self._dig(digits, s - k) * feed[k] for k in range(nreal)), "skipped tile"
        return cols

    @staticmethod
    def groups(cols):
        out = []
        for g in range(len(cols) // 4):
            v = sum(cols[4 * g + i] << (8 * i) for i in range(4))
            assert abs(v) < (1 << 48)
            out.append(s64(v))
        return out

    @staticmethod
    def fold_chunks(groups):
        """chunk j (tiles CHUNKS[j], groups 4 t .. 4 t + 3) normalised by quad lane j: dwords with a signed
        carry (floor division by 2^32), the carry handed to the next chunk; returns the dwords and the final
        carry (lane 2's)"""
        dws, carry = [], 0
        for ch in CHUNKS:
            for t in ch:
                for h in range(4):
                    v = s64(groups[4 * t + h] + carry)
                    dws.append(v & 0xFFFFFFFF)
                    carry = v >> 32
                    assert abs(carry) < (1 << 31)
        return dws, carry

    def reduce(self, z, want_q=True):
        """z < 2^4104 -> (r in [0, 3n), q3), every step as the kernel computes it"""
        n = self.n
        assert 0 <= z < (1 << (32 * NZ)) and z < (1 << 4104)
        zd = [(z >> (32 * i)) & 0xFFFFFFFF for i in range(NZ)]
        q1d = zd[Q1_DW0:]
        q1 = z >> A_BITS
        assert q1 == sum(d << (32 * i) for i, d in enumerate(q1d)) and len(q1d) == NQ1
        feed1 = [((q1 >> (8 * i)) & 255) - 128 for i in range(4 * NQ1)] + [0] * (64 * KB1 - 4 * NQ1)
        cols1 = self.product(self.mud, ACT1, S1_BASE, TILES1, 4 * NQ1, feed1, self.corr1)
        dw1, carry1 = self.fold_chunks(self.groups(cols1))
        n1 = sum(d << (32 * i) for i, d in enumerate(dw1)) + (carry1 << (32 * len(dw1)))
        assert n1 == sum(cols1[i] << (8 * i) for i in range(len(cols1)))     # the fold is exact
        Pi = q1 * self.mu
        assert Pi - (1 << 2105) < (n1 << (8 * S1_BASE)) <= Pi, "bias / truncation bound"
        if carry1 < 0:                                      # N1 < 0: q3 clamped to 0
            assert Pi < (1 << 2105)
            q3 = 0
        else:
            assert carry1 == 0 and all(d == 0 for d in dw1[1 + NQ3:]), "q3 >= 2^2080"
            q3 = sum(dw1[1 + i] << (32 * i) for i in range(NQ3))
        q = z // n
        assert q - 2 <= q3 <= q, (q, q3)
        feed2 = [((q3 >> (8 * i)) & 255) - 128 for i in range(4 * NQ3)] + [0] * (64 * KB2 - 4 * NQ3)
        cols2 = self.product(self.nd, ACT2, 0, TILES2, 4 * NQ3, feed2, self.corr2)
        dw2, _ = self.fold_chunks(self.groups(cols2))
        r2 = sum(d << (32 * i) for i, d in enumerate(dw2[:R_DW]))
        assert r2 == (q3 * n) % (1 << (32 * R_DW))
        r = (sum(zd[i] << (32 * i) for i in range(R_DW)) - r2) % (1 << (32 * R_DW))
        assert r == z - q3 * n and 0 <= r < 3 * n
        return r, q3


# ---- the VALU product pass (operand scanning over the quad, two windows) -----------------------------------
def window_product(terms):
    """columns of sum_i a_i X b^i (terms: list over steps i of lists of (a, X limbs)) accumulated LSB-first as
    the kernel's ring does: at step i every column gets its a_i x_j terms, column i retires (split: hi into
    column i + 1).  Asserts the 64-bit column bound; returns z."""
    cols = [0] * (2 * S + 1)
    out = []
    carry = 0
    for i, tl in enumerate(terms):
        for a, X in tl:
            assert 0 <= a < (1 << 28) and all(0 <= x < (1 << B) for x in X)
            for j, x in enumerate(X):
                cols[i + j] += a * x
        c = cols[i] + carry
        assert c < (1 << 64), "column overflow"
        out.append(c & ((1 << B) - 1))
        carry = c >> B
    for i in range(len(terms), 2 * S):
        c = cols[i] + carry
        assert c < (1 << 64)
        out.append(c & ((1 << B) - 1))
        carry = c >> B
    assert carry == 0
    return sum(l << (B * k) for k, l in enumerate(out))


def limbs(x, k=S):
    assert 0 <= x < 1 << (B * k), x.bit_length()
    return [(x >> (B * i)) & ((1 << B) - 1) for i in range(k)]


class Digits:
    """X = x0 + x1 n with the kernel's ops (LOADX, SQR, MUL, CANON)"""

    def __init__(self, key, x0, x1):
        self.k, self.x0, self.x1 = key, x0, x1

    def check(self):
        assert 0 <= self.x0 < 3 * self.k.n and 0 <= self.x1 < 3 * self.k.n, "digit bound"

    def value(self):
        n = self.k.n
        return (self.x0 + self.x1 * n) % (n * n)

    def mul(self, y0, y1, sq=False):
        k = self.k
        X0, X1 = limbs(self.x0), limbs(self.x1)
        Y0, Y1 = limbs(y0), limbs(y1)
        if sq:
            z1 = window_product([[(Y0[i], X0)] for i in range(S)])
            z2 = window_product([[(2 * Y0[i], X1)] for i in range(S)])
        else:
            z1 = window_product([[(Y0[i], X0)] for i in range(S)])
            z2 = window_product([[(Y0[i], X1), (Y1[i], X0)] for i in range(S)])
        assert z1 == self.x0 * y0 and z2 == self.x0 * y1 + self.x1 * y0
        r1, q3 = k.reduce(z1)
        z2 += q3
        assert z2 < (1 << 4101)
        r2, _ = k.reduce(z2)
        self.x0, self.x1 = r1, r2
        self.check()

    def sqr(self):
        self.mul(self.x0, self.x1, sq=True)

    def canon(self):
        n = self.k.n
        while self.x0 >= n:
            self.x0 -= n
            self.x1 += 1
        while self.x1 >= n:
            self.x1 -= n


def encrypt(key, m, r, w=5):
    """(1 + m n) r^n mod n^2 through the digit products: LOADX r; CANON; pow(n) (left-to-right windows);
    MUL (1, m); CANON"""
    n = key.n
    X = Digits(key, r, 0)
    X.canon()
    X.check()
    tab = [None] * (1 << (w - 1))                    # odd powers X^(2t+1)
    tab[0] = (X.x0, X.x1)
    X2 = Digits(key, X.x0, X.x1)
    X2.sqr()
    for t in range(1, len(tab)):
        T = Digits(key, *tab[t - 1])
        T.mul(X2.x0, X2.x1)
        tab[t] = (T.x0, T.x1)
    bits = bin(n)[2:]
    i = 0
    acc = None
    while i < len(bits):
        if bits[i] == '0':
            acc.sqr()
            i += 1
            continue
        j = min(len(bits), i + w)
        while bits[j - 1] == '0':
            j -= 1
        v = int(bits[i:j], 2)
        if acc is None:
            acc = Digits(key, *tab[v >> 1])
        else:
            for _ in range(j - i):
                acc.sqr()
            acc.mul(*tab[v >> 1])
        i = j
    acc.mul(1, m)
    acc.canon()
    assert acc.x0 < n and acc.x1 < n
    return acc.x0 + acc.x1 * n


def rand_n(rng, bits=2048):
    while True:
        n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if n.bit_length() == bits:
            return n


def nadicb_image(n):
    """The per-key LDS image of fthe_nadic_b76 (gen_nadicb.py layout constants): 16 byte-shifted copies of
    mu's and of n's balanced digits (copy of output row m in slot copy_slot(m), byte y = digit[K_m - y],
    K_m = s_base + m + KO), then the column corrections of both products as int32."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fedtree_amd", "csrc"))
    import gen_nadicb as g
    assert (g.A_BITS, g.C_BITS, g.S1_BASE, g.TILES1, g.TILES2, g.KB1, g.KB2, g.NQ1, g.NQ3, g.BIAS_COL,
            g.BIAS_DIGIT, g.ND1, g.ND2) == (A_BITS, C_BITS, S1_BASE, TILES1, TILES2, KB1, KB2, NQ1, NQ3,
                                            BIAS_COL, BIAS_DIGIT, ND1, ND2)
    k = Key(n)
    img = bytearray(g.IMG_BYTES)
    for base, digits, sb, ko in ((g.A1_OFF, k.mud, S1_BASE, g.KO1), (g.A2_OFF, k.nd, 0, g.KO2)):
        for m in range(16):
            off = base + g.copy_slot(m) * g.COPY
            km = sb + m + ko
            for y in range(g.COPY):
                i = km - y
                img[off + y] = (digits[i] & 255) if 0 <= i < len(digits) else 0
    for off, corr in ((g.CORR1_OFF, k.corr1), (g.CORR2_OFF, k.corr2)):
        for i, c in enumerate(corr):
            img[off + 4 * i:off + 4 * i + 4] = (c & 0xFFFFFFFF).to_bytes(4, "little")
    return bytes(img)


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rng = random.Random(seed)
    keys = [rand_n(rng), rand_n(rng, 2047), rand_n(rng, 2041), (1 << 2040) + 1, (1 << 2048) - 1]
    for n in keys:
        k = Key(n)
        top = 3 * n - 1
        cases = [(0, 0), (1, 1), (top, top), (top, 0), (n, n), (n - 1, 2 * n + 5)]
        cases += [(rng.randrange(3 * n), rng.randrange(3 * n)) for _ in range(trials)]
        for a, b in cases:
            for z in (a * b, 2 * a * b + 19 * n - 1 if 2 * a * b + 19 * n - 1 < 19 * n * n else a * b):
                r, q3 = k.reduce(z)
                assert r == z % n + (z // n - q3) * n
        # products on digits at the bound, and squarings
        for _ in range(trials // 4 + 1):
            X = Digits(k, rng.randrange(3 * n), rng.randrange(3 * n))
            Y = (rng.randrange(3 * n), rng.randrange(3 * n))
            v = X.value() * (Y[0] + Y[1] * n) % (n * n)
            X.mul(*Y)
            assert X.value() == v
            v = X.value() ** 2 % (n * n)
            X.sqr()
            assert X.value() == v
        X = Digits(k, top, top)
        v = X.value() ** 2 % (n * n)
        X.sqr()
        assert X.value() == v
        print(f"n bits {n.bit_length()}: reductions and digit products ok; active tiles p1 "
              f"{sum(map(len, ACT1))} p2 {sum(map(len, ACT2))}")
    n = keys[0]
    k = Key(n)
    FAST[0] = True
    for m, r in ((0, 1), (2**64 - 1, n - 1), (12345, rng.randrange(1, n))):
        assert encrypt(k, m, r) == (1 + m * n) * pow(r, n, n * n) % (n * n)
    print("nadicb model OK (3 encrypts vs pow)")


if __name__ == "__main__":
    main()
