#!/usr/bin/env python3
"""Bit-exact model of the Montgomery n-adic product (the LSB-first form of gen_nadic.py's fused product):
the public-key encrypt's r^n mod n^2 with X = x0 + x1 n kept as two base-n digits, each product two
interleaved Montgomery reductions mod the 2048-bit n instead of two classical MSB-first ones -- no
quotient estimate (the f64 chains, the overflow-column fold), q = col0 n' mod 2^27 on lane 0.

    R = 2^(27 S), S = 76 limbs;  Mont(X, Y) = X Y R^-1 mod n^2
    window 1:  R t1 = x0 y0 + Q1 n        (Q1 = sum q1_i b^i: its Montgomery quotient digits)
    so         X Y = R t1 + n (x0 y1 + x1 y0 - Q1)       exactly
    window 2:  R t2 = (x0 y1 + x1 y0 - Q1) + Q2 n       (-q1_i enters column 0 at step i)
    Mont(X, Y) == t1 + t2 n   (mod n^2)

Bounds (S = 76, n < 2^2049, so 8 n < R): with x0, x1, y0, y1 in [0, 2n) every output digit is in [0, 2n)
-- t1 < (4 n^2 + R n) / R < 2 n and t2 < (8 n^2 + R n) / R < 2 n, t2 > (-R) / R = -1 -- so the products
chain with no conditional subtraction ("almost Montgomery"); CANON reduces both digits at the end.

The exponentiation runs on the raw r as a Montgomery residue (the value r R^-1): its n-th power in that
domain is r^n R^(1-n); the encrypt's last two products are MUL (1, m) and MULK K with the per-key constant
K = R^(n+1) mod n^2, so c = r^n R^(1-n) (1 + m n) R^-1 K R^-1 = (1 + m n) r^n mod n^2.

Quad layout (as gen_montprog.py gen_quad's Montgomery step): lane k holds window positions
[kQ, kQ + Q), Q = 19.  Per step and window: columns += a_i X (19 v_mad_u64_u32 per lane); q from lane 0's
position 0 (v_mul_lo_u32 by n', mask, DPP broadcast); columns += q N; every lane splits its lowest
column c = lo + 2^27 hi (window 2: arithmetic shift, its columns are signed), keeps hi in its next column
and hands lo to the lane below as that lane's new top column (lane 0's lo is 0 after the Montgomery step,
so lane 3's fresh top column gets 0).  Columns are 64-bit two's complement, wrapped as the kernel wraps.
Checked: |column| < 2^63, q < 2^27, the digit bounds above, the identities.
"""
import random
import sys

B = 27
BETA = 1 << B
MASK = BETA - 1
M64 = (1 << 64) - 1
S = 76
LANES = 4
Q = S // LANES
R = 1 << (B * S)


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def limbs(x, n=S):
    assert 0 <= x < 1 << (B * n), x.bit_length()
    return [(x >> (B * k)) & MASK for k in range(n)]


def nprime(N):
    return (-pow(N, -1, BETA)) % BETA


class Window:
    """S columns, lane k at positions [kQ, kQ + Q)"""

    def __init__(self, signed):
        self.col = [0] * S
        self.signed = signed
        self.maxcol = 0

    def mad(self, a, X):
        for j in range(S):
            self.col[j] = s64(self.col[j] + a * X[j])

    def q(self, npr):
        return ((self.col[0] & 0xffffffff) * npr & 0xffffffff) & MASK     # v_mul_lo_u32, v_and

    def split_shift(self):
        """every lane: lowest column -> lo (to the lane below, its new top) + hi (its own next column)"""
        assert self.col[0] & MASK == 0
        lows = []
        for k in range(LANES):
            c = self.col[k * Q] & M64
            hi = s64(c) >> B if self.signed else c >> B
            lo = c & MASK
            lows.append(lo)
            self.col[k * Q + 1] = s64(self.col[k * Q + 1] + hi)
        new = [0] * S
        for k in range(LANES):
            for j in range(Q - 1):
                new[k * Q + j] = self.col[k * Q + j + 1]
            new[k * Q + Q - 1] = lows[(k + 1) % LANES]      # DPP quad_perm [1,2,3,0]; lane 0's lo is 0
        self.col = new
        self.maxcol = max(self.maxcol, *(abs(c) for c in self.col))

    def value(self):
        return sum(c * BETA ** k for k, c in enumerate(self.col))


def mont(y0, y1, x0, x1, N, sq=False, stats=None):
    """Mont((x0 + x1 N), (y0 + y1 N)) as two digits in [0, 2N); sq: y = x (window 2 takes 2 x0_i X1)"""
    assert all(0 <= v < 2 * N for v in (x0, x1, y0, y1))
    npr = nprime(N)
    A0, A1, X0, X1, NL = limbs(y0), limbs(y1), limbs(x0), limbs(x1), limbs(N)
    w1, w2 = Window(False), Window(True)
    Q1 = Q2 = 0
    for i in range(S):
        w1.mad(A0[i], X0)
        q1 = w1.q(npr)
        w1.mad(q1, NL)
        w1.split_shift()
        if sq:
            w2.mad(2 * A0[i], X1)
        else:
            w2.mad(A0[i], X1)
            w2.mad(A1[i], X0)
        w2.col[0] = s64(w2.col[0] - q1)                    # v_mad_i64_i32 col0, q1, (-1 on lane 0), col0
        q2 = w2.q(npr)
        w2.mad(q2, NL)
        w2.split_shift()
        Q1 += q1 << (B * i)
        Q2 += q2 << (B * i)
    t1, t2 = w1.value(), w2.value()
    assert R * t1 == x0 * y0 + Q1 * N
    W = (2 * x0 * x1) if sq else (x0 * y1 + x1 * y0)
    assert R * t2 == W - Q1 + Q2 * N
    assert 0 <= t1 < 2 * N and 0 <= t2 < 2 * N, (t1 / N, t2 / N)
    if stats is not None:
        stats['col'] = max(stats.get('col', 0), w1.maxcol, w2.maxcol)
    assert stats is None or stats['col'] < 1 << 63
    return t1, t2


def canon(z0, z1, N):
    if z0 >= N:
        z0 -= N
        z1 += 1
    while z1 >= N:
        z1 -= N
    return z0, z1


def pow_mont(r, e, N, w=6):
    """r^e R^(1-e) mod N^2 through the sliding-window program (bn_host.hpp Prog::pow), r < 2N raw"""
    x = (r, 0)

    def sq(x):
        return mont(x[0], x[1], x[0], x[1], N, sq=True)

    def mul(x, y):
        return mont(y[0], y[1], x[0], x[1], N)

    nb = e.bit_length()
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


def encrypt(m, r, N, e=None):
    """the public-key encrypt program: pow(e = N), MUL (1, m), MULK K, CANON"""
    e = N if e is None else e
    N2 = N * N
    K = pow(R, e + 1, N2)
    x = pow_mont(r, e, N)
    x = mont(1, m, x[0], x[1], N)
    x = mont(K % N, K // N, x[0], x[1], N)
    return canon(x[0], x[1], N)


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rng = random.Random(seed)
    st = {}
    Rinv = None
    for t in range(trials):
        nb = rng.choice([2042, 2047, 2048, 2048])
        N = rng.getrandbits(nb) | (1 << (nb - 1)) | 1
        N2 = N * N
        Rinv = pow(R, -1, N2)
        kind = t % 4
        if kind == 0:
            xs = [rng.randrange(2 * N) for _ in range(4)]
        elif kind == 1:
            xs = [2 * N - 1] * 4
        elif kind == 2:
            xs = [2 * N - 1 - rng.randrange(1 << 64) for _ in range(4)]
        else:
            xs = [rng.randrange(N), 2 * N - 1, rng.randrange(1 << 64), 0]
        x0, x1, y0, y1 = xs
        X, Y = x0 + x1 * N, y0 + y1 * N
        z0, z1 = mont(y0, y1, x0, x1, N, stats=st)
        assert (z0 + z1 * N) % N2 == X * Y * Rinv % N2, t
        z0, z1 = mont(x0, x1, x0, x1, N, sq=True, stats=st)
        assert (z0 + z1 * N) % N2 == X * X * Rinv % N2, t
    print(f"ok: {2 * trials} Montgomery n-adic products, max |column| < 2^{st['col'].bit_length()}")
    for t in range(3):
        N = rng.getrandbits(2048) | (1 << 2047) | 1
        r = [rng.randrange(1, N), 2 * N - 1, 1][t]
        e = rng.getrandbits(200) | (1 << 199)            # a shorter exponent keeps the model quick
        m = rng.getrandbits(64)
        z0, z1 = encrypt(m, r, N, e)
        assert z0 < N and z1 < N
        assert z0 + z1 * N == pow(r, e, N * N) * (1 + m * N) % (N * N), t
    print("ok: exponentiations and the (1 + m n) K products")


if __name__ == "__main__":
    main()
