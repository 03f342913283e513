"""Rates of the exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT) vs the default
direct-y CRT encrypt, device-resident, Paillier-2048; one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda:0")
    c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    out = {}
    t0 = time.perf_counter()
    pl.set_fixed_base_exact(seed=0)
    dev.sync()
    out["table_build_s"] = round(time.perf_counter() - t0, 3)
    for name, kw in (("exact", dict(fixed_base_exact=True)), ("direct_y", {}), ("fixed_base", dict(fixed_base=True))):
        pl.encrypt_u64_dev(m[:4096], c[:4096], seed=1, **kw)
        dev.sync()
        pl.encrypt_u64_dev(m, c, seed=2, **kw)
        dev.sync()
        out[name + "_per_s"] = round(n / (dev.last_kernel_ms() * 1e-3))
        low = torch.empty_like(m)
        pl.decrypt_u64_dev(c, low)
        dev.sync()
        out[name + "_roundtrip_ok"] = bool(torch.equal(low, m))
    # one-generator exact mode: a key with factored P - 1 (FTHE_KEYGEN_KNOWN_ORDER)
    t0 = time.perf_counter()
    pk = Paillier(dev).keygen(2048, seed=20261016, known_order=True)
    out["known_order_keygen_s"] = round(time.perf_counter() - t0, 3)
    t0 = time.perf_counter()
    pk.set_fixed_base_exact(seed=0)
    dev.sync()
    out["known_order_table_build_s"] = round(time.perf_counter() - t0, 3)
    pk.encrypt_u64_dev(m[:4096], c[:4096], seed=1, fixed_base_exact=True)
    dev.sync()
    pk.encrypt_u64_dev(m, c, seed=2, fixed_base_exact=True)
    dev.sync()
    out["exact_known_order_per_s"] = round(n / (dev.last_kernel_ms() * 1e-3))
    low = torch.empty_like(m)
    pk.decrypt_u64_dev(c, low)
    dev.sync()
    out["exact_known_order_roundtrip_ok"] = bool(torch.equal(low, m))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
