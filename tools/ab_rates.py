"""A/B helper: device-resident rates of one library build (FTHE_LIB selects it).

  FTHE_LIB=build/ab/libX.so python tools/ab_rates.py [--n 786432]
Prints one JSON line: CRT encrypt, add and sub rates (best of reps)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=786432)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    cw = 2 * pl.n_words
    m = torch.randint(0, 2**62, (a.n,), dtype=torch.int64, device="cuda")
    c = torch.empty((a.n, cw), dtype=torch.int32, device="cuda")
    o = torch.empty_like(c)

    def best(fn, units):
        fn(); dev.sync()
        t = 1e30
        for _ in range(a.reps):
            fn(); dev.sync()
            t = min(t, dev.last_kernel_ms())
        return round(units / (t * 1e-3))

    res = {"lib": os.environ.get("FTHE_LIB", "default")}
    res["encrypt"] = best(lambda: pl.encrypt_u64_dev(m, c, seed=1), a.n)
    res["add"] = best(lambda: pl.add_dev(c, c, o), a.n)
    if os.environ.get("FTHE_AB_ADD2") == "1":          # distinct operand rows (the bench's add)
        c2 = torch.empty_like(c)
        pl.encrypt_u64_dev(m, c2, seed=2)
        res["add_distinct"] = best(lambda: pl.add_dev(c, c2, o), a.n)
    if os.environ.get("FTHE_AB_FB", "1") == "1":
        pl.set_fixed_base(None)
        res["encrypt_fixed_base"] = best(lambda: pl.encrypt_u64_dev(m, c, seed=1, fixed_base=True), a.n)
        res["encrypt_public_fixed_base"] = best(lambda: pl.encrypt_u64_dev(m, c, seed=1, public=True, fixed_base=True), a.n)
        res["encrypt_public"] = best(lambda: pl.encrypt_u64_dev(m[:a.n // 4], c[:a.n // 4], seed=1, public=True), a.n // 4)
    k = a.n // 8
    res["sub"] = best(lambda: pl.sub_dev(c[:k], c[k:2 * k], o[:k]), k)
    if os.environ.get("FTHE_AB_KWAY") == "1":          # 8-party merge, a.n // 8 bins: adds/s
        x = c[:8 * k].reshape(8, k, cw)
        res["kway_adds"] = best(lambda: pl.reduce_kway_dev(x, 8, o[:k]), 7 * k)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
