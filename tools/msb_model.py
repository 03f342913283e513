#!/usr/bin/env python3
"""Bit-exact model of the classical (MSB-first, interleaved) modular product that the four-lane
montprog kernel runs for MULWC: X <- A * X mod N with no Montgomery factor, so a fresh pairwise
ciphertext add (paillier.cpp:103, x*y mod n^2) costs ONE 4096-bit product instead of a Montgomery
product plus the R^2 correction product.

Columns are radix-2^27 positions 0..S-1 plus the top TT (position S), each a 64-bit two's-complement
register (the model wraps every update mod 2^64 exactly as v_mad_i64_i32 / v_lshl_add_u64 do).
Step t (i = S-1-t, MSB first):
  1. shift up one position (ring relabel + one DPP hand-off per lane): old position S-1 becomes TT;
  2. column j += a_i * X_j                       (v_mad_u64_u32, 27x27-bit)
  3. W = TT * 2^27 + col[S-1]  (wraps; the true value is small), col[S-1] = W, TT = 0
  4. q = trunc(fma(W, 2^27, col[S-2]) * invN - bias)   in double, clamped at 0
     (invN = 1 / (N / 2^(27 (S-2))) rounded down; bias covers the ignored columns and rounding)
  5. column j -= q * N_j                          (v_mad_i64_i32 with -q)
Invariant (checked here): 0 <= value < 2N after every step, |column| < 2^63, q < 2^29.
The final signed normalisation + one conditional subtraction give X = A X mod N, canonical.
"""
import random
import struct
import sys

B = 27
BETA = 1 << B
M64 = (1 << 64) - 1


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def f64(x):
    """round to the nearest double, as v_cvt_f64_i32 / v_cvt_f64_u32 + fma would (value < 2^62)"""
    return struct.unpack("d", struct.pack("d", float(x)))[0]


def limbs(x, S):
    return [(x >> (B * k)) & (BETA - 1) for k in range(S)]


def msb_mulmod(a, x, N, S, check=True):
    A, X, NL = limbs(a, S), limbs(x, S), limbs(N, S)
    col = [0] * S
    TT = 0
    Ntop = (N >> (B * (S - 2) - 64)) / 2.0 ** 64  # N in units of the position S-2 column
    invN = (1.0 / Ntop) * (1 - 2.0 ** -45)        # rounded down
    bias = 2.0 ** -6                              # ignored columns (< 2^-9 of a unit of q) + rounding
    qmax = 0
    for t in range(S):
        i = S - 1 - t
        # 1. shift up: old S-1 -> TT (TT was folded to 0 at the previous step's estimate)
        assert TT == 0
        TT = col[S - 1]
        col = [0] + col[:S - 1]
        # 2. + a_i X
        for j in range(S):
            col[j] = s64(col[j] + A[i] * X[j])
        # 3. fold the top: W = TT 2^27 + col[S-1] (wrapping; true value small)
        W = s64((TT << B) + col[S - 1])
        col[S - 1] = W
        TT = 0
        # 4. quotient estimate (double)
        V = f64(W) * BETA + f64(col[S - 2])
        qd = V * invN - bias
        q = int(qd) if qd > 0 else 0
        q = min(q, (1 << 32) - 1)
        qmax = max(qmax, q)
        # 5. - q N
        for j in range(S):
            col[j] = s64(col[j] - q * NL[j])
        if check:
            val = sum(c * BETA ** k for k, c in enumerate(col))
            assert 0 <= val < 2 * N, (t, val >= 0, val / N)
            assert all(-(1 << 63) < c < (1 << 63) for c in col)
    val = sum(c * BETA ** k for k, c in enumerate(col))
    if val >= N:
        val -= N
    return val, qmax


def main():
    S = 152
    rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    qmax = 0
    for t in range(trials):
        nb = rng.choice([4095, 4096, 4096, 4095])      # n^2 of a 2048-bit n: >= 2^4094 (MULWC is used only then)
        N = rng.getrandbits(nb) | (1 << (nb - 1)) | 1
        kind = t % 4
        if kind == 0:
            a, x = rng.randrange(N), rng.randrange(N)
        elif kind == 1:
            a, x = N - 1, N - 1                 # extremes
        elif kind == 2:
            a, x = N - 1 - rng.randrange(1 << 64), rng.randrange(1 << 64)
        else:
            a, x = rng.randrange(N), N - 1 - rng.randrange(1000)
        got, qm = msb_mulmod(a, x, N, S)
        qmax = max(qmax, qm)
        assert got == a * x % N, t
    print(f"ok: {trials} products, max q {qmax} (< 2^{qmax.bit_length()})")


if __name__ == "__main__":
    main()
