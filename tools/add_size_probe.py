"""P-2048 add rate (fthe_addb_q152) by call size, cold and right after ~14 s of CRT encrypts (the bench times its
adds after the encrypt steps): does the 8M-add call of bench.py run slower than the 1M-add call of
tools/addb_ab.py because of the call size (row-I/O chunking) or because of the chip's state?
  python tools/add_size_probe.py          -> one JSON line"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    cw = 2 * pl.n_words
    N = 1 << 24
    m = torch.randint(0, 2**62, (N,), dtype=torch.int64, device="cuda")
    c = torch.empty((N, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    dev.sync()
    o = torch.empty((N // 2, cw), dtype=torch.int32, device="cuda")

    def rate(n, reps=5):
        pl.add_dev(c[:n], c[n:2 * n], o[:n])
        dev.sync()
        ts = []
        for _ in range(reps):
            pl.add_dev(c[:n], c[n:2 * n], o[:n])
            dev.sync()
            ts.append(dev.last_kernel_ms())
        ts.sort()
        return round(n / (ts[len(ts) // 2] * 1e-3))

    res = {"cold": {}, "after_encrypts": {}}
    for n in (1 << 20, 1 << 21, 1 << 22, 1 << 23):
        res["cold"][n] = rate(n)
    for n in (1 << 23, 1 << 20, 1 << 23):
        pl.encrypt_u64_dev(m[:N // 2 + N // 4], c[:N // 2 + N // 4], seed=2)     # ~4.4 s of m37
        pl.encrypt_u64_dev(m[:N // 2 + N // 4], c[:N // 2 + N // 4], seed=3)
        pl.encrypt_u64_dev(m[:N // 2 + N // 4], c[:N // 2 + N // 4], seed=4)
        dev.sync()
        res["after_encrypts"][f"{n}_{len(res['after_encrypts'])}"] = rate(n)
    res["rowio_chunk"] = os.environ.get("FTHE_ROWIO_CHUNK")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
