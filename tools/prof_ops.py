"""Small driver for kernel traces / counters of the mod-n^2 (four-lane) kernel:
one device-resident add of distinct rows (addsame: the same rows as both operands, half the unique bytes),
one 8-way reduce, one Montgomery-resident add, one party encrypt
from published bases and one histogram scatter at Paillier-2048 (--ops selects).

  python tools/prof_ops.py [--n 262144]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--ops", default="add,kway,hist")
    a = ap.parse_args()
    import torch
    from fedtree_amd.paillier import Device, Paillier, histogram_segments
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=5)
    cw = 2 * pl.n_words
    n = a.n
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
    c = torch.empty((n, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    dev.sync()
    if a.ops == "encrypt":
        return
    o = torch.empty_like(c)
    ops = a.ops.split(",")
    if "add" in ops:                                  # distinct operand rows (the bench's adds): 2 n rows read
        c2 = torch.empty_like(c)
        pl.encrypt_u64_dev(m, c2, seed=2)
        pl.add_dev(c, c2, o)
        dev.sync()
        print("add", n, "ms", dev.last_kernel_ms())
        del c2
    if "addsame" in ops:                              # x = y: each row read once for both operands (calibration)
        pl.add_dev(c, c, o)
        dev.sync()
        print("addsame", n, "ms", dev.last_kernel_ms())
    if "kway" in ops:
        x = torch.stack([c] * 8)
        for _ in range(3):                            # configs[3] at --n 2097152 (256 x 4096 bins x {g, h})
            pl.reduce_kway_dev(x, 8, o)
            dev.sync()
            print("kway8", n, "ms", dev.last_kernel_ms())
    if "mont" in ops:                                 # Montgomery-resident add (one product per add)
        mr = torch.empty_like(c)
        pl.to_mont_dev(c, mr)
        pl.add_mont_dev(mr, mr, o)
        dev.sync()
        print("add_mont", n, "ms", dev.last_kernel_ms())
    if "pbx" in ops:                                  # party encrypt from published bases (gathered products)
        party = pl.public(bases=pl.public_bases(seed=3))
        party.encrypt_u64_dev(m, o, seed=2, fixed_base_exact=True)
        dev.sync()
        print("public_exact", n, "ms", dev.last_kernel_ms())
    if "hist" in ops:
        rng = np.random.default_rng(1)
        ni = n // 2
        bins = rng.integers(0, 256, (ni, 8)).astype(np.uint8)
        cut = np.arange(9, dtype=np.int64) * 256
        seg, idx = histogram_segments(bins.reshape(-1), cut, 256)
        out = torch.empty((len(seg) - 1, cw), dtype=torch.int32, device="cuda")
        pl.reduce_segments_dev(c, seg, out, idx=idx)
        dev.sync()
        print("hist", len(idx), "ms", dev.last_kernel_ms())


if __name__ == "__main__":
    main()
