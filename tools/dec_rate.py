"""Device-resident Paillier-2048 CRT decrypt rates (full and short), one JSON line (FTHE_LIB selects the build)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1572864
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
    c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    out = {"lib": os.environ.get("FTHE_LIB", "default")}
    for name, short in (("decrypt", False), ("decrypt_short", True)):
        low = torch.empty_like(m)
        pl.decrypt_u64_dev(c[:4096], low[:4096], short=short)
        pl.decrypt_u64_dev(c, low, short=short)
        dev.sync()
        out[name + "_per_s"] = round(n / (dev.last_kernel_ms() * 1e-3))
        out[name + "_ok"] = bool(torch.equal(low, m))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
