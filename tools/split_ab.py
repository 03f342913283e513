"""Device-resident CRT encrypt / decrypt time by batch size for Paillier-1024 and -2048 (one JSON line per key
size): whether the mod-p and mod-q exponentiations run one after the other or on two streams (the split
path, <= FTHE_DEC_SPLIT lanes) matters where one half's launch leaves a partial round of waves.  Run it under
different FTHE_DEC_SPLIT values to compare."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COUNTS = {1024: (65536, 100000, 131072, 196608, 200000, 262144, 393216),
          2048: (65536, 131072, 200000, 262144, 393216)}


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    lib = dev.lib
    for bits, counts in COUNTS.items():
        pl = Paillier(dev).keygen(bits, seed=20261016 + bits)
        n = max(counts)
        m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
        c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda")
        out = {"bits": bits, "FTHE_DEC_SPLIT": os.environ.get("FTHE_DEC_SPLIT")}
        for cnt in counts:
            row = {}
            for name in ("encrypt", "decrypt"):
                ts = []
                low = torch.empty((cnt,), dtype=torch.int64, device="cuda")
                for i in range(4):
                    if name == "encrypt":
                        pl.encrypt_u64_dev(m[:cnt], c[:cnt], seed=5 + i)
                    else:
                        pl.decrypt_u64_dev(c[:cnt], low)
                    dev.sync()
                    ts.append(lib.fthe_last_kernel_ms(dev.ctx))
                if name == "decrypt":
                    assert torch.equal(low, m[:cnt]), (bits, cnt)
                ms = sorted(ts[1:])[1]
                row[name] = {"ms": round(ms, 3), "per_s": round(cnt / ms * 1e3)}
            out[cnt] = row
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
