#!/usr/bin/env python3
"""Stress check of the public-key encrypt kernel fthe_nadic_b76 (the parties' default at 2048 bits): N
device-randomness public-key encrypts of one key holder's n (same seed) on b76 and on the Montgomery form
fthe_nadic_m76 (FTHE_NADIC_MONT=1 at key set-up), compared ciphertext for ciphertext, and every b76 ciphertext
decrypted back by the key holder.  Prints one JSON line.  Usage: python tools/b76_stress.py [N] [keys]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedtree_amd.paillier import Device, Paillier  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    keys = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = Device(0)
    out = {"ciphertexts_per_key": n, "keys": keys, "differing_vs_m76": 0, "decrypt_mismatches": 0}
    t0 = time.time()
    rng = np.random.default_rng(11)
    m = torch.from_numpy(rng.integers(0, 2**63, n, dtype=np.int64)).cuda()
    for kk in range(keys):
        pa = Paillier(dev).keygen(2048, seed=20261018 + kk)
        os.environ["FTHE_NADIC_MONT"] = "1"
        pm = Paillier.from_primes(pa.p, pa.q, dev)
        del os.environ["FTHE_NADIC_MONT"]
        cb = torch.empty((n, 2 * pa.n_words), dtype=torch.int32, device="cuda")
        cm = torch.empty_like(cb)
        low = torch.empty(n, dtype=torch.int64, device="cuda")
        pa.encrypt_u64_dev(m, cb, seed=77 + kk, public=True)
        pm.encrypt_u64_dev(m, cm, seed=77 + kk, public=True)
        pa.decrypt_u64_dev(cb, low)
        dev.sync()
        torch.cuda.synchronize()
        out["differing_vs_m76"] += int((cb != cm).any(dim=1).sum().item())
        out["decrypt_mismatches"] += int((low != m).sum().item())
        del cb, cm, low
    out["s"] = round(time.time() - t0, 1)
    print(json.dumps(out))
    return 1 if out["differing_vs_m76"] or out["decrypt_mismatches"] else 0


if __name__ == "__main__":
    sys.exit(main())
