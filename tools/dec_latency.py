"""Device-resident Paillier-2048 CRT decrypt time by batch size (the decrypt_gh / per-node regime,
server.h:69-111): one JSON line of {count: ms} for the full and short forms.  The small-batch paths
are chosen inside the library by count (s80 quad kernel <= FTHE_DEC_QUAD, two streams <=
FTHE_DEC_SPLIT lanes); run it under different env values to compare them."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COUNTS = (2, 64, 1024, 4096, 8192, 16384, 16385, 32768, 65536, 65537, 131072)


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    n = max(COUNTS)
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
    c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    out = {"env": {k: os.environ.get(k) for k in ("FTHE_DEC_QUAD", "FTHE_DEC_SPLIT")}}
    for name, short in (("decrypt", False), ("decrypt_short", True)):
        res = {}
        for cnt in COUNTS:
            low = torch.empty((cnt,), dtype=torch.int64, device="cuda")
            pl.decrypt_u64_dev(c[:cnt], low, short=short)
            dev.sync()
            reps = 5 if cnt <= 16385 else 2
            t0 = time.perf_counter()
            for _ in range(reps):
                pl.decrypt_u64_dev(c[:cnt], low, short=short)
            dev.sync()
            ms = (time.perf_counter() - t0) / reps * 1e3
            assert torch.equal(low, m[:cnt]), (name, cnt)
            res[cnt] = {"ms": round(ms, 2), "per_s": round(cnt / ms * 1e3)}
        out[name] = res
        print(json.dumps({name: res}), flush=True)
    res = {}
    for cnt in COUNTS:                       # device-randomness CRT encrypt (two streams <= FTHE_DEC_SPLIT)
        cc = torch.empty((cnt, 2 * pl.n_words), dtype=torch.int32, device="cuda")
        pl.encrypt_u64_dev(m[:cnt], cc, seed=5)
        dev.sync()
        reps = 5 if cnt <= 16385 else 2
        t0 = time.perf_counter()
        for _ in range(reps):
            pl.encrypt_u64_dev(m[:cnt], cc, seed=5)
        dev.sync()
        ms = (time.perf_counter() - t0) / reps * 1e3
        res[cnt] = {"ms": round(ms, 2), "per_s": round(cnt / ms * 1e3)}
    out["encrypt"] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
