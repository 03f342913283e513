"""A/B of the P-2048 pairwise add: the matrix-core Barrett kernel (fthe_addb_q152, default) against the
classical four-lane product (FTHE_ADD_NO_ADDB=1 at key set-up), same n, same rows, same process.
  python tools/addb_ab.py [n_adds] [reps]      -> one JSON line (best and median of reps, kernel time)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    os.environ["FTHE_ADD_NO_ADDB"] = "1"
    ref = Paillier.from_primes(pl.p, pl.q, dev)
    del os.environ["FTHE_ADD_NO_ADDB"]
    cw = 2 * pl.n_words
    m = torch.randint(0, 2**62, (2 * n,), dtype=torch.int64, device="cuda")
    c = torch.empty((2 * n, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    o1, o2 = torch.empty((n, cw), dtype=torch.int32, device="cuda"), torch.empty((n, cw), dtype=torch.int32, device="cuda")
    res = {"adds": n}
    for name, k, o in (("addb", pl, o1), ("classical", ref, o2), ("addb_again", pl, o1)):
        k.add_dev(c[:n], c[n:], o)
        dev.sync()
        ts = []
        for _ in range(reps):
            k.add_dev(c[:n], c[n:], o)
            dev.sync()
            ts.append(dev.last_kernel_ms())
        ts.sort()
        res[name] = {"best_per_s": round(n / (ts[0] * 1e-3)), "median_per_s": round(n / (ts[len(ts) // 2] * 1e-3)),
                     "ms": [round(t, 3) for t in ts]}
    res["same_rows"] = bool(torch.equal(o1, o2))
    res["speedup_median"] = round(res["addb"]["median_per_s"] / res["classical"]["median_per_s"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
