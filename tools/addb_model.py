#!/usr/bin/env python3
"""Bit-exact model of the Barrett ciphertext add on the matrix cores (fthe_addb_q152, gen_addb.py).

A pairwise add is z = x y mod N for N = n^2 of Paillier-2048 (4094 < log2 N <= 4096), canonical x, y < N
(paillier.cpp:92-105, paillier_gmp.cpp:16-21).  The four-lane row kernel forms the full product
z = x y (variable x variable: the VALU, 152 limbs of 27 bits per operand, one quad per ciphertext) and
reduces it by Barrett, whose two products have a constant operand (mu, N): over the 16 ciphertexts of a
wave they are matrix products, run on v_mfma_i32_16x16x64_i8 (16 output bytes x 16 ciphertexts per
instruction, K = 64 input bytes).

Barrett parameters (bit-level, HAC 14.42 with radix 2 and the cut points chosen on dword boundaries):
    q1 = floor(z / 2^A),  A = 4072        q1 < 2^(8192 - A) = 2^4120: 129 dwords (516 bytes)
    mu = floor(2^(A + C) / N),  C = 4128   mu < 2^4106: 515 balanced base-256 digits
    q3 = floor(q1 mu / 2^C)                z/N - q1 mu / 2^C < 2^(A - 4094) + q1 / 2^C < 2^-7, so
                                           q3 is floor(z / N) or one below it
    r  = z - q3 N  in [0, 2N)  (before the truncation below: [0, 3N) after it)
Product 1 forms only the columns s >= 512 (bytes) of q1 mu; the dropped columns move the sum by
|D| < 2^4120.02 (each |column| < 516 * 128 * 255 < 2^24.01), so a bias of -2^4121 (one digit -2 in
column 515) gives a numerator N1 with  Pi - 2^4122 < N1 <= Pi  for Pi = q1 mu: floor(N1 / 2^4128) is the
exact quotient estimate or one below it -> r in [0, 3N), two conditional subtractions at most.  N1 < 0
only when Pi < 2^4122 (z < 2^4072 N / 2^4106...): then q3 is clamped to 0 and r = z < N.
Product 2 forms r2 = q3 N mod 2^4104 (bytes s < 513), and r = (z - r2) mod 2^4104, exact because
0 <= r < 3N < 2^4098.

Matrix-core arithmetic.  The core multiplies SIGNED bytes: the constants are balanced base-256 digits
(each in [-128, 127]); the variable bytes b are fed as b - 128 (b ^ 0x80), and the correction
128 * sum_k c[s - k] of every output column s (a per-key constant, with product 1's bias) is the initial
accumulator (srcC) of the column's first MFMA, read from LDS.  Every column sum is exact in int32
(|C| < 2^24).  Each lane folds its four adjacent columns of a tile into one int64 group
P_G = sum_i C_{4G+i} 256^i (|P_G| < 2^48.1), and the groups are normalised to dwords with a signed
carry (floor division by 2^32), which gives q3's dwords (product 1: groups 1..128 over 2^4128) and r2's.

This model computes exactly those column sums (tile by tile, only the tiles whose constant entries are
not all zero), groups and carries, asserts every bound, and checks r against Python's integers.
Run:  python tools/addb_model.py [seed] [trials]
"""
import os
import random
import sys

A_BITS, C_BITS = 4072, 4128
NQ1 = 129                       # q1 dwords (516 bytes)
NQ3 = 129                       # q3 dwords (516 bytes: rows up to 2^4096 - 1 give q3 < 2^4098)
S1_BASE = 512                   # product-1 output byte columns 512 .. 512 + 16 * TILES1 - 1
TILES1 = 33
TILES2 = 33                     # product-2 output byte columns 0 .. 527 (only s < 513 are kept)
KB1, KB2 = 9, 9                 # K-blocks of 64 bytes (q1, q3: 516 bytes + 60 padding bytes, fed 0)
BIAS_COL, BIAS_DIGIT = 515, -2  # -2 * 256^515 = -2^4121
R_BITS = 4104                   # r is formed mod 2^4104 (= 27 * 152, the quad's limb range)


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


def _check_generator_constants():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fedtree_amd", "csrc"))
    import gen_addb as ga
    assert (ga.MU_SHIFT, ga.S1_BASE, ga.NQ1, ga.NQ3, ga.TILES1, ga.TILES2, ga.KB1, ga.KB2, ga.BIAS_COL,
            ga.BIAS_DIGIT) == (A_BITS + C_BITS, S1_BASE, NQ1, NQ3, TILES1, TILES2, KB1, KB2, BIAS_COL, BIAS_DIGIT)


class AddbKey:
    """The per-key constants: balanced digits of mu and N, the skipped-tile maps and the column
    corrections (srcC initial values) of both products."""

    def __init__(self, N):
        assert (1 << 4094) <= N < (1 << 4096), "the Barrett add covers N of 4095 or 4096 bits (n^2 of 2048-bit n)"
        self.N = N
        self.mu = (1 << (A_BITS + C_BITS)) // N
        assert self.mu < (1 << 4106)
        self.mud = balanced(self.mu, 515)
        self.Nd = balanced(N, 513)
        # active tiles: (t, kb) whose A entries c[s - k] are not all zero
        self.act1 = [(t, kb) for t in range(TILES1) for kb in range(KB1)
                     if self._band(self.mud, S1_BASE + 16 * t, 64 * kb)]
        self.act2 = [(t, kb) for t in range(TILES2) for kb in range(KB2)
                     if self._band(self.Nd, 16 * t, 64 * kb)]
        # column corrections: +128 * sum over the REAL input bytes k of c[s - k] (padding bytes are fed as 0)
        self.corr1 = [128 * sum(self._dig(self.mud, s - k) for k in range(4 * NQ1)) for s in
                      range(S1_BASE, S1_BASE + 16 * TILES1)]
        self.corr1[BIAS_COL - S1_BASE] += BIAS_DIGIT
        self.corr2 = [128 * sum(self._dig(self.Nd, s - k) for k in range(4 * NQ3)) for s in range(16 * TILES2)]

    @staticmethod
    def _dig(d, i):
        return d[i] if 0 <= i < len(d) else 0

    @staticmethod
    def _band(d, s0, k0):
        # entries d[s - k] for s in [s0, s0 + 16), k in [k0, k0 + 64)
        lo, hi = s0 - k0 - 63, s0 + 15 - k0
        return not (hi < 0 or lo >= len(d))

    def product(self, digits, act, base, tiles, nbytes_real, feed, corr):
        """Column sums of the constant (balanced digits) times the fed bytes, tile by tile over the
        active (t, kb) pairs only -- what the MFMAs accumulate -- starting from the corrections."""
        cols = [s32(c) for c in corr]
        for t, kb in act:
            for r in range(16):
                s = base + 16 * t + r
                acc = 0
                for k in range(64 * kb, 64 * kb + 64):
                    acc += self._dig(digits, s - k) * (feed[k] if k < nbytes_real else 0)
                cols[16 * t + r] = s32(cols[16 * t + r] + acc)
        # the skipped tiles contribute nothing: check against the full sum
        for idx in range(16 * tiles):
            s = base + idx
            full = corr[idx] + sum(self._dig(digits, s - k) * feed[k] for k in range(nbytes_real))
            assert cols[idx] == full, "a skipped tile was not all zero"
        return cols

    @staticmethod
    def groups(cols):
        """Four adjacent columns -> one int64 group (what a lane folds from its 4 accumulator registers)."""
        out = []
        for g in range(len(cols) // 4):
            v = sum(cols[4 * g + i] << (8 * i) for i in range(4))
            assert abs(v) < (1 << 49)
            out.append(s64(v))
        return out

    @staticmethod
    def fold(groups):
        """Groups at bit 32 G -> dwords with a signed carry (floor division), and the final carry."""
        dws, carry = [], 0
        for p in groups:
            v = s64(p + carry)
            dws.append(v & 0xFFFFFFFF)
            carry = v >> 32
            assert abs(carry) < (1 << 31)
        return dws, carry

    def reduce(self, z):
        """z < 2^8192 (any two 4096-bit rows: the reference reduces x y whatever x, y are) -> (r in [0, 3N),
        q3), every step as the kernel computes it."""
        N = self.N
        assert 0 <= z < (1 << 8192)
        q1 = z >> A_BITS
        assert q1 < (1 << (32 * NQ1))
        q1b = [(q1 >> (8 * i)) & 255 for i in range(4 * NQ1)]
        feed1 = [b - 128 for b in q1b] + [0] * (64 * KB1 - 4 * NQ1)
        cols1 = self.product(self.mud, self.act1, S1_BASE, TILES1, 4 * NQ1, feed1, self.corr1)
        g1 = self.groups(cols1)
        dw1, carry1 = self.fold(g1)
        n1 = sum(d << (32 * i) for i, d in enumerate(dw1)) + (carry1 << (32 * len(dw1)))
        n1_true = sum(cols1[i] << (8 * i) for i in range(len(cols1)))
        assert n1 == n1_true                                 # the fold is exact
        Pi = q1 * self.mu
        assert Pi - (1 << 4122) < (n1 << (8 * S1_BASE)) <= Pi, "bias / truncation bound"
        if carry1 < 0:                                       # N1 < 0: q3 clamped to 0
            assert Pi < (1 << 4122)
            q3 = 0
        else:
            assert carry1 == 0 and all(d == 0 for d in dw1[1 + NQ3:]), "q3 >= 2^4128"
            q3 = sum(dw1[1 + i] << (32 * i) for i in range(NQ3))
        q = z // N
        assert q - 2 <= q3 <= q, (q, q3)
        q3b = [(q3 >> (8 * i)) & 255 for i in range(4 * NQ3)]
        feed2 = [b - 128 for b in q3b] + [0] * (64 * KB2 - 4 * NQ3)
        cols2 = self.product(self.Nd, self.act2, 0, TILES2, 4 * NQ3, feed2, self.corr2)
        g2 = self.groups(cols2)
        dw2, _ = self.fold(g2)
        r2 = sum(d << (32 * i) for i, d in enumerate(dw2)) & ((1 << R_BITS) - 1)
        assert r2 == (q3 * N) & ((1 << R_BITS) - 1)
        r = ((z & ((1 << R_BITS) - 1)) - r2) & ((1 << R_BITS) - 1)
        assert r == z - q3 * N and 0 <= r < 3 * N
        return r, q3

    def add(self, x, y):
        r, _ = self.reduce(x * y)
        while r >= self.N:
            r -= self.N
        return r


def addb_image(N):
    """The per-key context of fthe_addb_q152 (kctx): the LDS image -- 16 byte-shifted copies of mu's and of
    N's balanced digits (copy of output row m in slot copy_slot(m), byte y = digit[K_m - y],
    K_m = s_base + m + KO), the column corrections of both products as int32 -- then N as 128 dwords.
    The host builder (fthe.hip addb_ctx) must produce the same bytes (tests/test_addb_model.py)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fedtree_amd", "csrc"))
    import gen_addb as ga
    _check_generator_constants()
    k = AddbKey(N)
    img = bytearray(ga.KCTX_BYTES)
    for base, digits, sb, ko in ((ga.A1_OFF, k.mud, S1_BASE, ga.KO1), (ga.A2_OFF, k.Nd, 0, ga.KO2)):
        for m in range(16):
            off = base + ga.copy_slot(m) * ga.COPY
            km = sb + m + ko
            for y in range(ga.COPY):
                i = km - y
                img[off + y] = (digits[i] & 255) if 0 <= i < len(digits) else 0
    for off, corr in ((ga.CORR1_OFF, k.corr1), (ga.CORR2_OFF, k.corr2)):
        for i, c in enumerate(corr):
            img[off + 4 * i:off + 4 * i + 4] = (c & 0xFFFFFFFF).to_bytes(4, "little")
    img[ga.N_OFF:ga.N_OFF + 512] = N.to_bytes(512, "little")
    img[ga.ONE_OFF] = 1                               # the row 1: a gathered index < 0
    return bytes(img)


def rand_n(rng, bits=2048):
    while True:
        n = rng.getrandbits(bits) | (3 << (bits - 2)) | 1
        if (n * n).bit_length() >= 4095:
            return n


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rng = random.Random(seed)
    keys = [rand_n(rng) for _ in range(3)]
    keys.append((1 << 2047) + 1)                       # smallest 2048-bit n: N of 4095 bits
    keys.append((1 << 2048) - 1)                       # largest: N just below 2^4096
    worst = 0
    for n in keys:
        k = AddbKey(n * n)
        N = k.N
        top = (1 << 4096) - 1
        cases = [(0, 0), (1, 1), (N - 1, N - 1), (N - 1, 1), (N - 2, N - 1), (1 << 2048, 1 << 2047),
                 (top, top), (N, N), (top, N - 1)]
        cases += [(rng.randrange(N), rng.randrange(N)) for _ in range(trials)]
        cases += [(rng.randrange(1 << 64), rng.randrange(N)) for _ in range(4)]
        for x, y in cases:
            r, q3 = k.reduce(x * y)
            worst = max(worst, r // N)
            assert k.add(x, y) == x * y % N
        print(f"n bits {n.bit_length()}: {len(cases)} adds ok; active tiles p1 {len(k.act1)} p2 {len(k.act2)}")
    print(f"addb model OK (max r/N before correction: {worst})")


if __name__ == "__main__":
    main()
