#!/usr/bin/env python3
"""GPU bring-up probe of fthe_nadic_b76 through fthe_debug_nadicb_prog: single ops on random digits in [0, 3n)
(LOADX/STOREX, CANON, one SQR, one MUL, SQR x3 + MUL), every ciphertext's output digits against
tools/nadicb_model.py's (the exact digits, not only the residue).  Prints one JSON line per test.
    python tools/nadicb_probe.py [count]"""
import ctypes
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import nadicb_model as nm  # noqa: E402
from fedtree_amd.paillier import Device, Paillier  # noqa: E402

S, B = 152, 27


def to_limbs(x0, x1):
    return [(x0 >> (B * j)) & ((1 << B) - 1) for j in range(76)] + [(x1 >> (B * j)) & ((1 << B) - 1) for j in range(76)]


def from_limbs(row):
    x0 = sum(int(row[j]) << (B * j) for j in range(76))
    x1 = sum(int(row[76 + j]) << (B * j) for j in range(76))
    return x0, x1


def main():
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 1536
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=7)
    n = pl.modulus
    key = nm.Key(n)
    nm.FAST[0] = True
    rng = random.Random(5)
    xs = [(rng.randrange(3 * n), rng.randrange(3 * n)) for _ in range(cnt)]
    ys = [(rng.randrange(3 * n), rng.randrange(3 * n)) for _ in range(cnt)]
    xs[:4] = [(0, 0), (1, 0), (3 * n - 1, 3 * n - 1), (n, n - 1)]
    lib = dev.lib

    def run(ops, slots, out_slot, nslots=4):
        inp = np.zeros((nslots, cnt, S), dtype=np.uint32)
        for s, vals in slots.items():
            inp[s] = np.array([to_limbs(a, b) for a, b in vals], dtype=np.uint32)
        prog = np.array(ops + [0, 0], dtype=np.uint32)
        out = np.zeros((cnt, S), dtype=np.uint32)
        rc = lib.fthe_debug_nadicb_prog(pl._key, dev.ctx, ctypes.c_void_p(prog.ctypes.data), len(prog),
                                        ctypes.c_void_p(inp.ctypes.data), nslots, cnt, out_slot,
                                        ctypes.c_void_p(out.ctypes.data))
        assert rc == 0, rc
        return [from_limbs(r) for r in out]

    def report(name, got, want):
        bad = [i for i in range(cnt) if got[i] != want[i]]
        info = {"test": name, "count": cnt, "bad": len(bad)}
        if bad:
            i = bad[0]
            info["first"] = i
            info["x0_ok_first"] = got[i][0] == want[i][0]
            info["x1_ok_first"] = got[i][1] == want[i][1]
            info["bad_ct_in_wave"] = sorted({b % 16 for b in bad})[:16]
            info["bad_waves"] = sorted({(b // 16) % 12 for b in bad})[:12]
            info["x0_bad"] = sum(got[b][0] != want[b][0] for b in bad)
            info["x1_bad"] = sum(got[b][1] != want[b][1] for b in bad)
            if got[i][0] != want[i][0]:
                d = got[i][0] ^ want[i][0]
                info["x0_diff_bits"] = [d.bit_length() - 1, (d & -d).bit_length() - 1]
            if got[i][1] != want[i][1]:
                d = got[i][1] ^ want[i][1]
                info["x1_diff_bits"] = [d.bit_length() - 1, (d & -d).bit_length() - 1]
        print(json.dumps(info), flush=True)
        return len(bad)

    total = 0
    got = run([1, 0, 2, 1], {0: xs}, 1)
    total += report("io", got, xs)
    got = run([1, 0, 20, 0, 2, 1], {0: xs}, 1)
    want = []
    for a, b in xs:
        D = nm.Digits(key, a, b)
        D.canon()
        want.append((D.x0, D.x1))
    total += report("canon", got, want)
    got = run([1, 0, 3, 1, 2, 2], {0: xs}, 2)
    want = []
    for a, b in xs:
        D = nm.Digits(key, a, b)
        D.sqr()
        want.append((D.x0, D.x1))
    total += report("sqr", got, want)
    got = run([1, 0, 4, 1, 2, 2], {0: xs, 1: ys}, 2)
    want = []
    for (a, b), (c, d) in zip(xs, ys):
        D = nm.Digits(key, a, b)
        D.mul(c, d)
        want.append((D.x0, D.x1))
    total += report("mul", got, want)
    got = run([1, 0, 3, 3, 4, 1, 2, 2], {0: xs, 1: ys}, 2)
    want = []
    for (a, b), (c, d) in zip(xs, ys):
        D = nm.Digits(key, a, b)
        for _ in range(3):
            D.sqr()
        D.mul(c, d)
        want.append((D.x0, D.x1))
    total += report("sqr3_mul", got, want)
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
