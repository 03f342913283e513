#!/usr/bin/env python3
"""Stress check of the matrix-core Barrett kernel: N device-randomness Paillier-2048 encrypts (same seed) on
fthe_padic_m37 and on fthe_padic_k37 with the same primes, compared ciphertext for ciphertext, and every
m37 ciphertext decrypted back.  Prints one JSON line.  Usage: python tools/m37_stress.py [N]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedtree_amd.paillier import Device, Paillier  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    dev = Device(0)
    pa = Paillier(dev).keygen(2048, seed=20261017)
    os.environ["FTHE_NO_PADIC_MFMA"] = "1"
    pk = Paillier.from_primes(pa.p, pa.q, dev)
    del os.environ["FTHE_NO_PADIC_MFMA"]
    rng = np.random.default_rng(7)
    m = torch.from_numpy(rng.integers(0, 2**63, n, dtype=np.int64)).cuda()
    ca = torch.empty((n, 2 * pa.n_words), dtype=torch.int32, device="cuda")
    ck = torch.empty_like(ca)
    low = torch.empty(n, dtype=torch.int64, device="cuda")
    t0 = time.time()
    pa.encrypt_u64_dev(m, ca, seed=99)
    pk.encrypt_u64_dev(m, ck, seed=99)
    pa.decrypt_u64_dev(ca, low)
    dev.sync()
    torch.cuda.synchronize()
    diff = int((ca != ck).any(dim=1).sum().item())
    bad_dec = int((low != m).sum().item())
    print(json.dumps({"ciphertexts": n, "differing_vs_k37": diff, "decrypt_mismatches": bad_dec,
                      "s": round(time.time() - t0, 1)}))
    return 1 if diff or bad_dec else 0


if __name__ == "__main__":
    sys.exit(main())
