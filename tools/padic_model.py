#!/usr/bin/env python3
"""Bit-exact model of the P-adic exponentiation kernel (fthe_padic_*): X mod P^2 kept as two base-P
digits, X = x0 + x1 P, so a product mod P^2 never forms a 4096-bit intermediate and never reduces
modulo the 2048-bit P^2:

    X Y = x0 y0 + (x0 y1 + x1 y0) P + x1 y1 P^2  ==  x0 y0 + (x0 y1 + x1 y0) P   (mod P^2)
    x0 y0 = u1 P + u0                                  (Barrett: quotient AND remainder)
    Z = u0 + ((x0 y1 + x1 y0 + u1) mod P) P           (second Barrett, remainder only)

Digits are radix-2^28 limbs, K = 37 limbs per digit (P of 1009..1030 bits, so that 5P and the quotients, below 50P, fit K limbs).  Digits are NOT reduced
below P: Barrett with a truncated quotient leaves them in [0, 5P), and every bound below holds for
inputs in that range, so the kernel never runs a correction loop.

Products are column-wise (product scanning): column c's 64-bit accumulator starts with the carry out
of column c-1, takes every term of weight c, and splits into limb (low 28 bits) + carry.  Terms are
28x28 -> 56-bit v_mad_u64_u32 (unsigned) or v_mad_i64_i32 (signed, the r = T - q P columns with -P in
SGPRs); this model wraps every accumulator mod 2^64 exactly as the hardware does and asserts that the
true value never needed more.

Costs (MADs, K = 37): squaring 2 x0 x1 (K^2) + x0^2 (K(K+1)/2) + 2 Barretts (~1.08 K^2 each) ~ 5,030
vs 8,251 for the radix-2^28 Montgomery squaring mod P^2 at S = 74 limbs; a general product ~7,030 vs
10,952.

Run:  python tools/padic_model.py [seed] [trials]
"""
import random
import sys

B = 28
BASE = 1 << B
MASK = BASE - 1
M64 = (1 << 64) - 1


def u64(x):
    assert 0 <= x < (1 << 64), "unsigned accumulator overflow"
    return x


def s64(x):
    assert -(1 << 63) <= x < (1 << 63), "signed accumulator overflow"
    return x


def limbs(x, n):
    assert 0 <= x < (1 << (B * n)), (x.bit_length(), n)
    return [(x >> (B * i)) & MASK for i in range(n)]


def value(ls):
    return sum(v << (B * i) for i, v in enumerate(ls))


class PadicKey:
    def __init__(self, P, K=37):
        assert P % 2 == 1
        self.K = K
        assert (1 << (B * (K - 1))) <= P < (1 << (B * K)), "Barrett needs b^(K-1) <= P < b^K"
        self.P = P
        self.NP = [-v for v in limbs(P, K)]                      # -P limbs (SGPRs, signed)
        self.mu = limbs((1 << (2 * B * K)) // P, K + 1)           # floor(b^2K / P), K+1 limbs (SGPRs)
        assert value(self.mu) == (1 << (2 * B * K)) // P


def col_product(a, b, ncols, init=None, double=False, square=False):
    """Product scanning of a x b into ncols normalised limbs (the last column keeps its carry-in)."""
    out = []
    carry = 0
    for c in range(ncols):
        if square:
            acc = 0
            for i in range(len(a)):
                j = c - i
                if i < j < len(a):
                    acc = u64(acc + a[i] * a[j])
            acc = u64((acc << 1) + carry)                       # v_lshl_add_u64 acc, 1, carry
            if c % 2 == 0 and c // 2 < len(a):
                acc = u64(acc + a[c // 2] * a[c // 2])
        else:
            acc = carry + (init[c] if init is not None and c < len(init) else 0)
            for i in range(len(a)):
                j = c - i
                if 0 <= j < len(b):
                    acc = u64(acc + a[i] * b[j])
            if double:
                raise NotImplementedError
        if c == ncols - 1:
            out.append(acc)
            assert acc < (1 << 32), "top limb must fit a VGPR"
        else:
            out.append(acc & MASK)
            carry = acc >> B
    return out


def barrett(key, T):
    """T: 2K limbs (limbs < 2^29 allowed in positions < K), T < b^2K.  Returns (q3, r) with
    T = q3 P + r exactly, 0 <= r < 5P, q3 <= T / P; both K normalised limbs."""
    K = key.K
    q1 = T[K - 1:2 * K]                                          # K+1 limbs, floor-ish of T / b^(K-1)
    # q2 = q1 mu, columns K-1 .. 2K+1 only (columns below K-1 dropped); q3 = columns K+1 .. 2K
    carry = 0
    q3 = []
    for c in range(K - 1, 2 * K + 1):
        acc = carry
        for i in range(K + 1):
            j = c - i
            if 0 <= j < K + 1:
                acc = u64(acc + q1[i] * key.mu[j])
        if c >= K + 1:
            q3.append(acc & MASK if c < 2 * K else acc)
        carry = acc >> B
    assert q3[-1] < BASE, "q3 fits K limbs"
    # r = (T - q3 P) mod b^K, signed columns
    r = []
    carry = 0
    for c in range(K):
        acc = carry + T[c]
        for i in range(K):
            j = c - i
            if 0 <= j < K:
                acc = s64(acc + q3[i] * key.NP[j])               # v_mad_i64_i32 q3_i, -P_j
        r.append(acc & MASK)
        carry = acc >> B                                          # arithmetic shift
    return q3, r


def check_digit(key, d):
    assert len(d) == key.K and all(0 <= v < BASE for v in d)
    assert value(d) < 5 * key.P, value(d) / key.P


def sqr(key, x0, x1):
    K = key.K
    # phase A: V = 2 x0 x1 (2K limbs, normalised)
    V = []
    carry = 0
    for c in range(2 * K):
        acc = 0
        for i in range(K):
            j = c - i
            if 0 <= j < K:
                acc = u64(acc + x0[i] * x1[j])
        acc = u64((acc << 1) + carry)
        if c == 2 * K - 1:
            V.append(acc)
        else:
            V.append(acc & MASK)
            carry = acc >> B
    # phase B: T = x0^2
    T = col_product(x0, x0, 2 * K, square=True)
    u1, u0 = barrett(key, T)
    for c in range(K):                                            # V += u1 (limbs < 2^29, no carry)
        V[c] += u1[c]
    _, z1 = barrett(key, V)
    return u0, z1


def mul(key, x0, x1, y0, y1):
    K = key.K
    W = []
    carry = 0
    for c in range(2 * K):                                        # W = x0 y1 + x1 y0
        acc = carry
        for i in range(K):
            j = c - i
            if 0 <= j < K:
                acc = u64(acc + x0[i] * y1[j])
                acc = u64(acc + x1[i] * y0[j])
        if c == 2 * K - 1:
            W.append(acc)
        else:
            W.append(acc & MASK)
            carry = acc >> B
    T = col_product(x0, y0, 2 * K)
    u1, u0 = barrett(key, T)
    for c in range(K):
        W[c] += u1[c]
    _, z1 = barrett(key, W)
    return u0, z1


def loadp(key, X):
    """plain X (2K limbs, X < b^2K) -> digits"""
    q3, r = barrett(key, limbs(X, 2 * key.K))
    return r, q3


def storep(key, x0, x1):
    """x0 + x1 P as 2K normalised limbs (< 6 P^2): v_mad_i64_i32 (-x1_i, -P_j)"""
    K = key.K
    out = []
    carry = 0
    nx1 = [-v for v in x1]
    for c in range(2 * K):
        acc = carry + (x0[c] if c < K else 0)
        for i in range(K):
            j = c - i
            if 0 <= j < K:
                acc = s64(acc + nx1[i] * key.NP[j])
        if c == 2 * K - 1:
            out.append(acc)
            assert 0 <= acc < BASE
        else:
            out.append(acc & MASK)
            carry = acc >> B
    return out


def padic_pow(key, X, e, w=6):
    """the host's left-to-right sliding window (bn_host.hpp Prog::pow) on digits"""
    P2 = key.P * key.P
    x0, x1 = loadp(key, X)
    val = lambda a, b: (value(a) + value(b) * key.P) % P2
    assert val(x0, x1) == X % P2
    tab = [(x0, x1)]
    s0, s1 = sqr(key, x0, x1)
    for _ in range((1 << (w - 1)) - 1):
        a, b = tab[-1]
        tab.append(mul(key, a, b, s0, s1))
    bits = bin(e)[2:]
    i = 0
    acc = None
    while i < len(bits):
        if bits[i] == '0':
            acc = sqr(key, *acc)
            i += 1
            continue
        j = min(len(bits), i + w)
        while bits[j - 1] == '0':
            j -= 1
        v = int(bits[i:j], 2)
        if acc is None:
            acc = tab[(v - 1) // 2]
        else:
            for _ in range(j - i):
                acc = sqr(key, *acc)
            acc = mul(key, *acc, *tab[(v - 1) // 2])
        for d in acc:
            check_digit(key, d)
        i = j
    return storep(key, *acc)


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rng = random.Random(seed)
    K = 37
    for t in range(trials):
        bits = rng.choice([1009, 1023, 1024, 1024, 1029, 1030])
        P = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        key = PadicKey(P, K)
        P2 = P * P
        # extreme digits: 5P - 1 both
        hi = limbs(5 * P - 1, K)
        z0, z1 = sqr(key, hi, hi)
        X = value(hi) + value(hi) * P
        assert (value(z0) + value(z1) * P) % P2 == X * X % P2
        check_digit(key, z0); check_digit(key, z1)
        a0, a1 = limbs(rng.randrange(5 * P), K), limbs(rng.randrange(5 * P), K)
        b0, b1 = limbs(rng.randrange(5 * P), K), limbs(rng.randrange(5 * P), K)
        z0, z1 = mul(key, a0, a1, b0, b1)
        A = value(a0) + value(a1) * P
        Bv = value(b0) + value(b1) * P
        assert (value(z0) + value(z1) * P) % P2 == A * Bv % P2
        check_digit(key, z0); check_digit(key, z1)
        if t < 6:
            X = rng.randrange(1, P) if t % 3 else rng.randrange(P2)    # y < P (encrypt) or c mod P^2 (decrypt)
            e = P if t % 2 == 0 else P - 1
            got = value(padic_pow(key, X, e))
            assert got % P2 == pow(X, e, P2), t
            assert got < 6 * P2
    print(f"ok: {trials} keys (squaring / product at the digit bounds, exponentiations)")


if __name__ == "__main__":
    main()
