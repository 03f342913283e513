#!/usr/bin/env python3
"""A/B of the Paillier-2048 public-key encrypt: the matrix-core Barrett n-adic kernel fthe_nadic_b76
(the default at 2041..2048 bits) vs the Montgomery form fthe_nadic_m76 (FTHE_NADIC_MONT=1 at key set-up), same primes and plaintexts,
device-resident, variants round-robin; bit-identical outputs for injected r (and against the classical form and
the Montgomery s152 program).  Prints one JSON line.  python tools/nadicb_ab.py [ciphertexts] [reps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from fedtree_amd.paillier import Device, Paillier  # noqa: E402


def key_with(env, pa, dev):
    os.environ[env] = "1"
    try:
        return Paillier.from_primes(pa.p, pa.q, dev)
    finally:
        del os.environ[env]


def main():
    dev = Device(0)
    lib = dev.lib
    pa = Paillier(dev).keygen(2048, seed=7)
    pm = key_with("FTHE_NADIC_MONT", pa, dev)
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 393216
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    m = torch.arange(cnt, dtype=torch.int64, device="cuda:0")
    c = torch.empty((cnt, 2 * pa.n_words), dtype=torch.int32, device="cuda:0")
    out = {"ciphertexts": cnt, "key_bits": 2048}
    best = {"barrett": [], "mont": []}
    for key in (pa, pm):
        key.encrypt_u64_dev(m[:4096], c[:4096], seed=1, public=True)      # warm
    dev.sync()
    for rep in range(reps):
        for name, key in (("barrett", pa), ("mont", pm)):
            key.encrypt_u64_dev(m, c, seed=2 + rep, public=True)
            dev.sync()
            best[name].append(lib.fthe_last_kernel_ms(dev.ctx))
            print(json.dumps({"rep": rep, name: round(best[name][-1], 2)}), file=sys.stderr, flush=True)
    for name, ts in best.items():
        out[name + "_ms"] = [round(t, 2) for t in ts]
        out[name + "_per_s"] = round(cnt / (min(ts) * 1e-3))
    out["speedup"] = round(out["barrett_per_s"] / out["mont_per_s"], 3)
    low = torch.empty(cnt, dtype=torch.int64, device="cuda:0")
    pa.encrypt_u64_dev(m, c, seed=9, public=True)
    pa.decrypt_u64_dev(c, low)
    dev.sync()
    out["roundtrip_ok"] = bool(torch.equal(low, m))
    n = pa.modulus
    rng = np.random.default_rng(3)
    rs = [1, 2, n - 1, n - 2, n + 5, 2**2048 - 1] + [int.from_bytes(rng.bytes(256), "little") % n for _ in range(4090)]
    r = np.array([[(x >> (32 * j)) & 0xffffffff for j in range(pa.n_words)] for x in rs], dtype=np.uint32)
    mm = rng.integers(0, 2**64 - 1, len(rs), dtype=np.uint64)
    ca = pa.encrypt_u64(mm, r=r, public=True)
    out["injected_r_identical_mont"] = bool(np.array_equal(ca, pm.encrypt_u64(mm, r=r, public=True)))
    n2 = n * n
    got = [int.from_bytes(ca[i].tobytes(), "little") for i in range(8)]
    out["formula_ok_first8"] = all(got[i] == (1 + int(mm[i]) * n) * pow(rs[i], n, n2) % n2 for i in range(8))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
