"""Latency of one P-2048 ciphertext add through each entry point (GHPair operator cost).

  python tools/op_latency.py
Prints one JSON line: microseconds per single-row call for fthe_add_shared (the GHPair key's path),
fthe_add (host rows, context), fthe_add_dev (device rows, kernel + launch) and the kernel time alone."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from fedtree_amd import _lib
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    rows = pl.encrypt_u64(np.arange(1, 9, dtype=np.uint64), seed=3)
    out = {}
    n = 300

    def per_call(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        return round((time.perf_counter() - t0) / n * 1e6, 1)

    acc = rows[:1].copy()
    out["add_shared_us"] = per_call(lambda: pl.add_shared(acc, rows[1:2], out=acc))
    out["add_host_us"] = per_call(lambda: pl.add_batch(rows[:1], rows[1:2]))
    da = torch.from_numpy(rows[:1].view(np.int32)).cuda()
    db = torch.from_numpy(rows[1:2].view(np.int32)).cuda()
    do = torch.empty_like(da)
    out["add_dev_us_incl_sync"] = per_call(lambda: (pl.add_dev(da, db, do), dev.sync()))
    pl.add_dev(da, db, do)
    dev.sync()
    out["add_kernel_us"] = round(pl.lib.fthe_last_kernel_ms(dev.ctx) * 1e3, 1)
    for k in (8, 64, 512):
        a = np.repeat(rows[:1], k, axis=0)
        out[f"add_shared_{k}rows_us"] = per_call(lambda: pl.add_shared(a, a, out=a))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
