"""Device histogram timing: one node histogram (g and h planes) of n instances x
n_col features x 255 bins at Paillier-2048, everything resident in HBM.

  python tools/hist_rate.py [--n 1000000] [--cols 28]
Prints one JSON line (wall time of fthe_histogram_dev incl. the CSR build, and
members / s = instance-feature-plane products per second)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=28)
    a = ap.parse_args()
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    cw = 2 * pl.n_words
    n, nc = a.n, a.cols
    g = torch.Generator(device="cuda").manual_seed(1)
    m = torch.randint(0, 2**40, (2 * n,), dtype=torch.int64, device="cuda", generator=g)
    x = torch.empty((2 * n, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, x, seed=2, fixed_base=True)
    bins = torch.randint(0, 256, (n, nc), dtype=torch.uint8, device="cuda", generator=g)
    cut = (np.arange(nc + 1) * 255).astype(np.int32)
    nb = int(cut[-1])
    out = torch.empty((2 * nb, cw), dtype=torch.int32, device="cuda")
    pl.histogram_dev(x[:2 * 4096], 4096, 2, bins[:4096], cut, 255, out)      # warm-up
    dev.sync()
    res = {"instances": n, "features": nc, "bins": nb, "planes": 2}
    for name, inst in (("root", None), ("half_node", torch.arange(0, n, 2, dtype=torch.int32, device="cuda"))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pl.histogram_dev(x, n, 2, bins, cut, 255, out, inst=inst)
        dev.sync()
        dt = time.perf_counter() - t0
        sel = n if inst is None else inst.numel()
        members = int(2 * sel * nc * 255 / 256)
        res[name] = {"s": round(dt, 4), "member_products_per_s": round(members / dt),
                     "kernel_ms_products": round(dev.last_kernel_ms(), 2)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
