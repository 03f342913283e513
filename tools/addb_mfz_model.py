#!/usr/bin/env python3
"""Bit-exact model of the add kernel's matrix-core product z = x y ("mfz", gen_addb.py section 2M): one
ciphertext at a time per wave, z's 1,024 byte columns as four 256-column blocks of v_mfma_i32_16x16x64_i8.

Both operands in balanced base-256 digits (x + 0x80..80, bytes XORed with 0x80: d_a in [-128, 128) for a < 512,
d_512 = the carry out in {0, 1}), so every i8 product is exact with no correction term.  Block u of z's columns
c = i + 16 j + 256 u (i, j < 16: the MFMA's row and column) accumulates over tiles t

    D_u[i][j] += sum_k A_t[i][k] B_tu[k][j],   A_t[i][k] = x_{i + 64 t + k - DELTA},  B_tu[k][j] = y_{c - a}

i.e. x's digits a = i + 64 t + k - DELTA (a Toeplitz window per row: row i starts i bytes later) and y's digits
b = 256 u + 16 j - 64 t - k + DELTA, which do not depend on i, so one B tile serves all 16 rows.  Only the
(t, u) whose window meets a valid (a, b) pair are issued (TILES below: 28).  x is read from LDS a dword-aligned
five-dword window per lane and funnel-shifted by the lane's byte offset (v_alignbyte_b32); y is stored byte-
reversed so that every B fragment is one aligned 16-byte read.  Column sums are int32 (|d| <= 128, 513 terms:
< 2^23.1); each lane folds its four rows (four consecutive columns) into an int64 group; the 256 groups of z are
normalised lane by lane (four groups per lane) with the carries handed from lane to lane.

Run: python tools/addb_mfz_model.py   (random and extreme operands vs Python integers)"""
import random

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fedtree_amd', 'csrc'))
from gen_addb import MZ_DELTA as DELTA, MZ_XOFF as XOFF, MZ_TILES as TILES, MZ_TS as TS  # noqa: E402
from gen_addb import MZ_RY as RY, MZ_XAREA as XAREA, MZ_YAREA as YAREA  # noqa: E402


def balanced(x):
    """513 balanced digits (i8 bytes) of x < 2^4096"""
    s = x + int('80' * 512, 16)
    b = s.to_bytes(513, 'little')
    d = [((v ^ 0x80) - 256 if (v ^ 0x80) > 127 else (v ^ 0x80)) for v in b[:512]] + [b[512]]
    assert sum(v << (8 * i) for i, v in enumerate(d)) == x
    return d


def stage(xd, yd):
    """the wave's x / yr staging areas as byte arrays (the kernel writes dwords; zeros elsewhere)"""
    xa = bytearray(XAREA)
    for a, v in enumerate(xd):
        xa[XOFF + a] = v & 0xff
    ya = bytearray(YAREA)
    for b, v in enumerate(yd):
        ya[RY - b] = v & 0xff
    return xa, ya


def a_frag(xa, lane, t):
    """lane l's 16 A bytes of tile t: the dword-aligned five-dword read and the byte funnel shift"""
    i, h = lane & 15, lane >> 4
    p0 = XOFF + i + 64 * t + 16 * h - DELTA
    d0, s = p0 >> 2, p0 & 3
    raw = xa[4 * d0:4 * d0 + 20]
    assert len(raw) == 20
    return bytes(raw[s:s + 16])


def b_frag(ya, lane, t, u):
    """lane l's 16 B bytes of tile (t, u): y digits b = 256 u + 16 j - 64 t - 16 h - q + DELTA, q = 0..15,
    at yr bytes RY - b: ascending in q, 16-byte aligned"""
    j, h = lane & 15, lane >> 4
    p0 = RY - (256 * u + 16 * j - 64 * t - 16 * h + DELTA)
    assert p0 % 16 == 0 and 0 <= p0 and p0 + 16 <= YAREA, (t, u, j, h, p0)
    return bytes(ya[p0:p0 + 16])


def s8(v):
    return v - 256 if v > 127 else v


def mfma16(afr, bfr, acc):
    """v_mfma_i32_16x16x64_i8 with the lane maps of tools/wave_emu.py: lane l holds A[l & 15][16 (l >> 4) + q]
    and B[16 (l >> 4) + q][l & 15]; register g of lane l is D[4 (l >> 4) + g][l & 15]"""
    A = [[0] * 64 for _ in range(16)]
    B = [[0] * 16 for _ in range(64)]
    for l in range(64):
        for q in range(16):
            A[l & 15][16 * (l >> 4) + q] = s8(afr[l][q])
            B[16 * (l >> 4) + q][l & 15] = s8(bfr[l][q])
    for l in range(64):
        for g in range(4):
            r, col = 4 * (l >> 4) + g, l & 15
            acc[l][g] += sum(A[r][k] * B[k][col] for k in range(64))


def product(x, y):
    xd, yd = balanced(x), balanced(y)
    xa, ya = stage(xd, yd)
    D = {u: [[0] * 4 for _ in range(64)] for u in range(4)}
    for t in TS:
        afr = [a_frag(xa, l, t) for l in range(64)]
        for u in range(4):
            if (t, u) in TILES:
                mfma16(afr, [b_frag(ya, l, t, u) for l in range(64)], D[u])
    groups = [0] * 256
    for u in range(4):
        for l in range(64):
            assert all(abs(v) < 1 << 24 for v in D[u][l])
            g = (l >> 4) + 4 * (l & 15) + 64 * u           # rows 4h'..4h'+3: columns 16 j + 4 h' + 256 u
            groups[g] = sum(D[u][l][r] << (8 * r) for r in range(4))
    # normalisation: lane l takes groups 4l..4l+3, chains them from carry 0, then the carries move lane to lane
    dw = [0] * 256
    carry = [0] * 64
    for l in range(64):
        c = 0
        for q in range(4):
            v = groups[4 * l + q] + c
            dw[4 * l + q] = v & 0xffffffff
            c = v >> 32                                   # signed
        carry[l] = c
        assert -(1 << 31) <= c < 1 << 31
    cin = [0] + carry[:63]
    rounds = 0
    while any(cin):
        rounds += 1
        out = [0] * 64
        for l in range(64):
            c = cin[l]
            for q in range(4):
                if not c:
                    break
                v = dw[4 * l + q] + c
                dw[4 * l + q] = v & 0xffffffff
                c = v >> 32
            out[l] = c
        cin = [0] + out[:63]
    z = sum(v << (32 * m) for m, v in enumerate(dw))
    return z, rounds


def main():
    rng = random.Random(11)
    print(f"tiles: {len(TILES)}  t range {TS[0]}..{TS[-1]}  per t: "
          + " ".join(f"{t}:{[u for tt, u in TILES if tt == t]}" for t in TS))
    cases = [(0, 0), (1, 1), ((1 << 4096) - 1, (1 << 4096) - 1), (int('80' * 512, 16), int('7f' * 512, 16)),
             (int('7f' * 512, 16), int('7f' * 512, 16)), (int('80' * 512, 16), int('80' * 512, 16))]
    cases += [(rng.getrandbits(4096), rng.getrandbits(4096)) for _ in range(40)]
    rmax = 0
    for x, y in cases:
        z, r = product(x, y)
        assert z == x * y, (hex(x)[:20], hex(y)[:20])
        rmax = max(rmax, r)
    print(f"{len(cases)} products exact; carry rounds after the first <= {rmax}")


if __name__ == '__main__':
    main()
