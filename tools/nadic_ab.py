#!/usr/bin/env python3
"""A/B of the public-key encrypt: at Paillier-2048 the n-adic kernel (default) vs the Montgomery s152
program, at Paillier-1024 the P-adic kernel with P = n vs the Montgomery s74 program (FTHE_NO_NADIC=1 and
FTHE_NO_PADIC=1 at key set-up), device-resident, same key and plaintexts; bit-identical outputs for
injected r.  Prints one JSON line.   python tools/nadic_ab.py [ciphertexts] [key bits]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from fedtree_amd.paillier import Device, Paillier  # noqa: E402


def main():
    dev = Device(0)
    lib = dev.lib
    bits = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    pa = Paillier(dev).keygen(bits, seed=7)
    os.environ["FTHE_NO_NADIC"] = os.environ["FTHE_NO_PADIC"] = "1"
    pm = Paillier.from_primes(pa.p, pa.q, dev)
    del os.environ["FTHE_NO_NADIC"], os.environ["FTHE_NO_PADIC"]
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 393216
    m = torch.arange(cnt, dtype=torch.int64, device="cuda:0")
    c = torch.empty((cnt, 2 * pa.n_words), dtype=torch.int32, device="cuda:0")
    out = {"ciphertexts": cnt, "key_bits": bits}
    fast = "nadic" if bits > 1100 else "padic"
    for name, key in ((fast, pa), ("montgomery", pm)):
        key.encrypt_u64_dev(m[:4096], c[:4096], seed=1, public=True)      # warm
        dev.sync()
        best = None
        for rep in range(2):
            t0 = time.perf_counter()
            key.encrypt_u64_dev(m, c, seed=2 + rep, public=True)
            dev.sync()
            wall = time.perf_counter() - t0
            kms = lib.fthe_last_kernel_ms(dev.ctx)
            best = min(best or 1e9, kms)
        out[name + "_per_s"] = round(cnt / (best * 1e-3))
        out[name + "_ms"] = round(best, 2)
        out[name + "_wall_s"] = round(wall, 3)
    out["speedup"] = round(out[fast + "_per_s"] / out["montgomery_per_s"], 3)
    low = torch.empty(cnt, dtype=torch.int64, device="cuda:0")
    pa.encrypt_u64_dev(m, c, seed=9, public=True)
    pa.decrypt_u64_dev(c, low)
    dev.sync()
    out["roundtrip_ok"] = bool(torch.equal(low, m))
    r = np.random.default_rng(3).integers(1, 2**31, (2048, pa.n_words), dtype=np.uint32)
    mm = np.arange(2048, dtype=np.uint64)
    out["injected_r_identical"] = bool(np.array_equal(pa.encrypt_u64(mm, r=r, public=True),
                                                      pm.encrypt_u64(mm, r=r, public=True)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
