"""Device-resident rates of the other HE ops (secondary to bench.py's headline).

  python tools/bench_ops.py [--hist-bins 1048576] [--parties 8]

Prints one JSON object: Paillier-2048 public-key encrypt, CRT decrypt, add,
scalar mul (subtraction) and the config-4 histogram merge
(1,048,576 bins x {g,h} x 8 parties, BASELINE.json configs[3]).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hist-bins", type=int, default=256 * 4096)
    ap.add_argument("--parties", type=int, default=8)
    ap.add_argument("--hist-inst", type=int, default=100000)
    ap.add_argument("--hist-cols", type=int, default=28)
    ap.add_argument("--n", type=int, default=1 << 20, help="ciphertexts for the single-op rates")
    a = ap.parse_args()
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    lib = dev.lib
    pl = Paillier(dev).keygen(2048, seed=20261015)
    cw = 2 * pl.n_words
    res = {"key_bits": 2048}
    n = a.n
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
    c = torch.empty((n, cw), dtype=torch.int32, device="cuda")

    def timed(fn, units, reps=2):
        fn()
        dev.sync()
        best = 1e30
        for _ in range(reps):
            fn()
            dev.sync()
            best = min(best, lib.fthe_last_kernel_ms(dev.ctx))
        return units / (best * 1e-3), best

    res["crt_encrypt_per_s"], _ = timed(lambda: pl.encrypt_u64_dev(m, c, seed=1), n)
    c2 = torch.empty_like(c)
    k = min(n, 1 << 18)
    res["public_encrypt_per_s"], _ = timed(lambda: pl.encrypt_u64_dev(m[:k], c2[:k], seed=2, public=True), k, 1)
    low = torch.empty(n, dtype=torch.int64, device="cuda")
    res["crt_decrypt_per_s"], _ = timed(lambda: pl.decrypt_u64_dev(c, low), n)
    res["decrypt_roundtrip_ok"] = bool(torch.equal(low, m))
    o = torch.empty_like(c)
    res["add_per_s"], _ = timed(lambda: pl.add_dev(c, c2.flip(0).contiguous() if False else c, o), n)
    # scalar mul by 2^64-1 (operator-, common.h:311)
    def smul():
        from fedtree_amd import _lib
        _lib.check(lib.fthe_scalar_mul_u64_dev(pl._key, dev.ctx, ctypes.c_void_p(c.data_ptr()), 2**64 - 1, k,
                                               ctypes.c_void_p(o.data_ptr())))
    res["scalar_mul_minus1_per_s"], _ = timed(smul, k, 1)
    res["sub_per_s"], _ = timed(lambda: pl.sub_dev(c[:k], c[k:2 * k], o[:k]), k, 1)
    # per-feature prefix scan of a 256-bin x 1024-feature histogram (g, h)
    nsc = 2 * 256 * 1024
    if nsc <= n:
        seg = np.arange(0, nsc + 1, 256, dtype=np.int64)
        res["scan_256bin_per_s"], _ = timed(lambda: pl.scan_segments_dev(c[:nsc], seg, o[:nsc]), nsc, 1)
    del c2
    # config 4: k-party merge of 256 x 4096 bins x {g,h}
    bins = 2 * a.hist_bins
    P = a.parties
    x = torch.empty((P, bins, cw), dtype=torch.int32, device="cuda")
    src = c[: min(n, bins)]
    for p_ in range(P):
        for off in range(0, bins, src.shape[0]):
            e = min(bins, off + src.shape[0])
            x[p_, off:e] = src[: e - off]
    out = torch.empty((bins, cw), dtype=torch.int32, device="cuda")
    rate, ms = timed(lambda: pl.reduce_kway_dev(x, P, out), bins, 1)
    res["hist_merge"] = {"bins": a.hist_bins, "ciphertexts_out": bins, "parties": P, "ms": round(ms, 2),
                         "adds_per_s": round(bins * (P - 1) / (ms * 1e-3)),
                         "input_GB": round(x.numel() * 4 / 1e9, 2),
                         "hbm_GBps_boundary": round((x.numel() + out.numel()) * 4 / (ms * 1e-3) / 1e9, 1)}
    # histogram scatter (hist_tree_builder.cpp:574-595): n_inst x n_col members into bins, g and h
    from fedtree_amd.paillier import histogram_segments
    n_inst, n_col, nb = a.hist_inst, a.hist_cols, 256
    rng = np.random.default_rng(1)
    bins_ = rng.integers(0, nb, (n_inst, n_col)).astype(np.uint8)
    cut = np.arange(n_col + 1, dtype=np.int64) * nb
    t0 = time.perf_counter()
    seg_ptr, idx = histogram_segments(bins_.reshape(-1), cut, 255 + 1)
    t_csr = time.perf_counter() - t0
    gh = c[: 2 * n_inst] if 2 * n_inst <= n else c[:n].repeat((2 * n_inst + n - 1) // n, 1)[: 2 * n_inst]
    seg2 = np.concatenate([seg_ptr, seg_ptr[1:] + seg_ptr[-1]])
    idx2 = np.concatenate([idx, idx + n_inst])
    hout = torch.empty((2 * len(seg_ptr) - 2, cw), dtype=torch.int32, device="cuda")
    t0 = time.perf_counter()
    rate, ms = timed(lambda: pl.reduce_segments_dev(gh, seg2, hout, idx=idx2), len(idx2), 1)
    res["hist_build"] = {"instances": n_inst, "features": n_col, "bins": int(cut[-1]), "members": int(len(idx2)),
                         "kernel_ms": round(ms, 2), "members_per_s": round(rate), "csr_host_s": round(t_csr, 3),
                         "wall_s_2calls": round(time.perf_counter() - t0, 3)}
    for kk in list(res):
        if isinstance(res[kk], float):
            res[kk] = round(res[kk])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
