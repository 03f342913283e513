#!/usr/bin/env python3
"""Bit-exact model of the n-adic four-lane kernel (gen_nadic.py): the public-key encrypt's r^n mod n^2
with X = x0 + x1 n kept as two base-n digits, each product two fused classical MSB-first products mod n.

    X Y == x0 y0 + (x0 y1 + x1 y0) n   (mod n^2)
    x0 y0 = u1 n + u0                  classical product mod n: u0 its remainder, u1 the sum of its
                                       quotient digits (q1 of step t has weight b^(S-1-t))
    Z = u0 + ((x0 y1 + x1 y0 + u1) mod n) n

Both products run in lockstep over the same multiplier limbs (MSB first): window 1 accumulates
y0_i X0, window 2 accumulates y0_i X1 + y1_i X0 and, in its lowest column, window 1's quotient digit
of the same step -- so u1 is never stored.  A squaring is y = x with y0_i X1 + y1_i X0 = (2 x0_i) X1.
Per step and lane of a quad: 19 + 19 (squaring: + 19 + 19) multiply-adds against 38 + 38 for the
Montgomery product mod the 4096-bit n^2 (gen_montprog.py gen_quad), over 76 steps instead of 152.

Columns: radix-2^27 positions 0..S-1 plus the top TT, 64-bit two's complement (wrapped exactly as
v_mad_u64_u32 / v_mad_i64_i32 / v_lshl_add_u64 do).  Step t (i = S-1-t), per window:
  1. shift up one position; fold TT 2^27 into column S-1
  2. + the step's terms (window 2: + q1 into column 0)
  3. -q = trunc(bias - (col[S-1] 2^27 + hi32(col[S-2]) 2^32) invN) in double (fma chain, host
     constants of bn_host.hpp MontMod for N = n on 76 x 27-bit limbs; FTHE_GEN_NADIC_AB=fold: the 64-bit sum
     col[S-1] + (col[S-2] >> 27) formed with integer instructions, then a two-term chain)
  4. - q N
Checked invariants: 0 <= value < 2N after every step, |column| < 2^63, 0 <= q < 2^30.  Each product
ends with the signed normalisation and one conditional subtraction per digit, digit 0's carried into
digit 1: x0 in [0, N), x1 in [0, N] (the bounds need no more); CANON makes x1 < N for the output.
"""
import random
import sys
from fractions import Fraction

B = 27
BETA = 1 << B
M64 = (1 << 64) - 1
S = 76


# the kernel's quotient estimate: the three-term f64 chain over col[S-1] and hi32(col[S-2]) (default), or with
# FTHE_GEN_NADIC_AB=fold col[S-2] >> 27 folded into col[S-1] by two 64-bit integer instructions and one 64-bit
# value converted (5 f64 instructions; bit-exact too, but measured 1.2% slower)
FOLD = "fold" in __import__("os").environ.get("FTHE_GEN_NADIC_AB", "").split(",")


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def limbs(x, n=S):
    return [(x >> (B * k)) & (BETA - 1) for k in range(n)]


def fma(a, b, c):
    """IEEE fma: exact a*b + c, one rounding (Fraction -> float rounds to nearest even)"""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def consts(N):
    """bn_host.hpp MontMod (lanes 4): doubles k1, k2, k3 (negated) and the bias"""
    assert N.bit_length() >= B * S - 10
    t = N >> (B * (S - 2) - 64)
    bl = t.bit_length()
    if bl > 53:                                   # mpz_get_d truncates
        t = (t >> (bl - 53)) << (bl - 53)
    ntop = float(t) * (1.0 + 2.0 ** -50) * 2.0 ** -64
    inv = 1.0 / ntop * (1.0 - 2.0 ** -50)
    return -inv * 2.0 ** 32, -inv * 2.0 ** 27, -inv * 2.0 ** 59, 2.0 ** -6


class Window:
    def __init__(self):
        self.col = [0] * S
        self.tt = 0

    def shift(self):
        self.tt, self.col = self.col[S - 1], [0] + self.col[:S - 1]
        self.col[S - 1] = s64(self.col[S - 1] + s64(self.tt << B))   # fold (kernel: before the MADs)
        self.tt = 0

    def add(self, a, X):
        for j in range(S):
            self.col[j] = s64(self.col[j] + a * X[j])

    def estimate(self, k):
        k1, k2, k3, bias = k
        if FOLD:
            # y = col[S-1] + (col[S-2] >> 27) in 64-bit integers (V' = y 2^27: one conversion pair fewer)
            y = s64(self.col[S - 1] + (s64(self.col[S - 2]) >> B)) & M64
            lo, hi = y & 0xffffffff, y >> 32
            hi = hi - (1 << 32) if hi >> 31 else hi
            acc = fma(float(hi), k3, bias)
            acc = fma(float(lo), k2, acc)
            nq = int(acc)
            nq = max(min(nq, (1 << 31) - 1), -(1 << 31))
            return -nq
        c2, c1 = self.col[S - 2] & M64, self.col[S - 1] & M64
        hi2 = c2 >> 32
        hi2 = hi2 - (1 << 32) if hi2 >> 31 else hi2
        lo1 = c1 & 0xffffffff
        hi1 = c1 >> 32
        hi1 = hi1 - (1 << 32) if hi1 >> 31 else hi1
        acc = fma(float(hi2), k1, bias)
        acc = fma(float(lo1), k2, acc)
        acc = fma(float(hi1), k3, acc)
        nq = int(acc)                              # v_cvt_i32_f64: trunc toward zero (saturating)
        nq = max(min(nq, (1 << 31) - 1), -(1 << 31))
        return -nq

    def sub(self, q, NL):
        for j in range(S):
            self.col[j] = s64(self.col[j] - q * NL[j])

    def value(self):
        return sum(c * BETA ** k for k, c in enumerate(self.col))


def fused(y0, y1, x0, x1, N, k, sq=False, check=True, stats=None):
    """(x0 + x1 N)(y0 + y1 N) mod N^2 as two canonical digits; sq: y = x (window 2 takes 2 x0_i X1)"""
    assert 0 <= x0 < N and 0 <= x1 <= N and 0 <= y0 < N and 0 <= y1 <= N
    A0, A1, X0, X1, NL = limbs(y0), limbs(y1), limbs(x0), limbs(x1), limbs(N)
    w1, w2 = Window(), Window()
    u1 = 0
    for t in range(S):
        i = S - 1 - t
        w1.shift()
        w1.add(A0[i], X0)
        q1 = w1.estimate(k)
        w1.sub(q1, NL)
        w2.shift()
        if sq:
            w2.add(2 * A0[i], X1)
        else:
            w2.add(A0[i], X1)
            w2.add(A1[i], X0)
        w2.col[0] = s64(w2.col[0] + q1)
        q2 = w2.estimate(k)
        w2.sub(q2, NL)
        u1 = u1 * BETA + q1
        for q in (q1, q2):
            assert 0 <= q < 1 << 30, q
        if stats is not None:
            stats['q'] = max(stats.get('q', 0), q1, q2)
            stats['col'] = max(stats.get('col', 0), *(abs(c) for c in w1.col + w2.col))
        if check:
            for w in (w1, w2):
                v = w.value()
                assert 0 <= v < 2 * N, (t, v / N)
                assert all(-(1 << 63) < c < (1 << 63) for c in w.col)
    v1 = w1.value()
    assert x0 * y0 == v1 + u1 * N                  # window 1's quotient digits are u1
    f = int(v1 >= N)                               # digit 0's conditional subtraction carries into
    z0 = v1 - N * f                                # digit 1: window 2's column 0 before it is
    w2.col[0] = s64(w2.col[0] + f)                 # normalised
    v2 = w2.value()
    z1 = v2 - N if v2 >= N else v2                 # in [0, N]: N itself only from v2 = 2N - 1, f = 1
    return z0, z1


def pow_nadic(r, e, N, k, w=6):
    """r^e mod N^2 through the kernel's op program (bn_host.hpp Prog::pow, sliding window)"""
    x = (r % N, 0)

    def sq(x):
        return fused(x[0], x[1], x[0], x[1], N, k, sq=True, check=False)

    def mul(x, y):
        return fused(y[0], y[1], x[0], x[1], N, k, check=False)

    nb = e.bit_length()
    if nb == 1:
        return x
    ntab = 1 << (w - 1)
    tab = [x]
    x2 = sq(x)
    for _ in range(1, ntab):
        tab.append(mul(tab[-1], x2))
    bits = [(e >> b) & 1 for b in range(nb)]

    def window(top):
        low = max(top - w + 1, 0)
        while not bits[low]:
            low += 1
        val = 0
        for b in range(top, low - 1, -1):
            val = (val << 1) | bits[b]
        return low, val

    low, v = window(nb - 1)
    x = tab[(v - 1) // 2]
    i = low - 1
    pend = 0
    while i >= 0:
        if not bits[i]:
            pend += 1
            i -= 1
            continue
        low, v = window(i)
        pend += i - low + 1
        for _ in range(pend):
            x = sq(x)
        x = mul(x, tab[(v - 1) // 2])
        pend = 0
        i = low - 1
    for _ in range(pend):
        x = sq(x)
    return x


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rng = random.Random(seed)
    st = {}
    for t in range(trials):
        nb = rng.choice([2042, 2047, 2048, 2048, 2052])
        N = rng.getrandbits(nb) | (1 << (nb - 1)) | 1
        k = consts(N)
        kind = t % 4
        if kind == 0:
            xs = [rng.randrange(N) for _ in range(4)]
        elif kind == 1:
            xs = [N - 1] * 4
        elif kind == 2:
            xs = [N - 1 - rng.randrange(1 << 64) for _ in range(4)]
        else:
            xs = [rng.randrange(N), N - 1, rng.randrange(1 << 64), N - 1 - rng.randrange(1000)]
        x0, x1, y0, y1 = xs
        X, Y, N2 = x0 + x1 * N, y0 + y1 * N, N * N
        z0, z1 = fused(y0, y1, x0, x1, N, k, stats=st)
        assert z0 + z1 * N == X * Y % N2 and z0 < N and z1 <= N, t
        z0, z1 = fused(x0, x1, x0, x1, N, k, sq=True, stats=st)
        assert z0 + z1 * N == X * X % N2 and z0 < N and z1 <= N, t
        if kind == 1:                                   # digit 1 == N (an unreduced 0) as input
            z0, z1 = fused(y0, N, x0, N, N, k, stats=st)
            assert (z0 + z1 * N - (x0 + N * N) * (y0 + N * N)) % N2 == 0, t
    print(f"ok: {2 * trials} fused products, max q {st['q']} (< 2^{st['q'].bit_length()}), "
          f"max |column| < 2^{st['col'].bit_length()}")
    # exponentiations: r^e and the encrypt's (1 + m n) r^n
    for t in range(2):
        N = rng.getrandbits(2048) | (1 << 2047) | 1
        k = consts(N)
        r = rng.randrange(1, N)
        e = rng.getrandbits(96) | 1 if t == 0 else N
        if t == 1:
            e = rng.getrandbits(300) | (1 << 299)          # a shorter exponent keeps the model quick
        x0, x1 = pow_nadic(r, e, N, k)
        assert x0 + x1 * N == pow(r, e, N * N), t
        m = rng.getrandbits(64)
        z0, z1 = fused(1, m, x0, x1, N, k)
        z1 = z1 - N if z1 >= N else z1                  # CANON
        assert z0 + z1 * N == pow(r, e, N * N) * (1 + m * N) % (N * N)
    print("ok: exponentiations and the (1 + m n) product")


if __name__ == "__main__":
    main()
