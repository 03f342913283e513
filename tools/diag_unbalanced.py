"""Diagnostic: unbalanced-prime keys, which operations disagree with the C oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle  # noqa: E402
from test_gpu_parity import _next_prime  # noqa: E402
from fedtree_amd.paillier import Device, Paillier  # noqa: E402

dev = Device(0)
o = pyoracle.COracle()
for shape in ["q_over_p_1.9", "p_over_q_1.9", "q_24_bits_longer", "q_over_p_1.3"]:
    rng = np.random.default_rng(len(shape))
    hw = 17
    base = int.from_bytes(rng.bytes(62), "little") | (1 << 495) | (1 << 511)
    base &= (1 << 512) - 1
    if shape == "q_24_bits_longer":
        p, q = _next_prime(base >> 12), _next_prime(base << 12)
    else:
        num = 19 if "1.9" in shape else 13
        a = _next_prime(base >> 1)
        b = _next_prime(a * num // 10)
        p, q = (b, a) if shape.startswith("p_over") else (a, b)
    pl = Paillier.from_primes(p, q, dev)
    ok = o.key(pyoracle.to_words(p, hw), pyoracle.to_words(q, hw))
    n = pl.modulus
    cnt = 64
    m = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    rs = [int.from_bytes(rng.bytes(pl.n_words * 4), "little") % (n - 1) + 1 for _ in range(cnt)]
    r = pyoracle.ints_to_words(rs, pl.n_words)
    r_or = np.zeros((cnt, 2 * hw), np.uint32)
    r_or[:, :pl.n_words] = r
    want = np.ascontiguousarray(ok.encrypt_batch(m, r_or)[:, :2 * pl.n_words])
    res = {"shape": shape, "pbits": p.bit_length(), "qbits": q.bit_length(), "nbits": n.bit_length()}
    c = pl.encrypt_u64(m, r=r)
    res["crt_bad"] = int((c != want).any(axis=1).sum())
    if res["crt_bad"]:
        i = int(np.nonzero((c != want).any(axis=1))[0][0])
        got, w = pyoracle.from_words(c[i]), pyoracle.from_words(want[i])
        res["crt_mod_p2_ok"] = got % (p * p) == w % (p * p)
        res["crt_mod_q2_ok"] = got % (q * q) == w % (q * q)
    try:
        cpub = pl.encrypt_u64(m, r=r, public=True)
        res["pub_bad"] = int((cpub != want).any(axis=1).sum())
    except Exception as e:  # noqa: BLE001
        res["pub"] = str(e)
    low = pl.decrypt_u64(want)
    res["dec_bad"] = int((low != m).sum())
    cd = pl.encrypt_u64(m, seed=4)
    res["direct_rt_bad"] = int((pl.decrypt_u64(cd) != m).sum())
    print(res, flush=True)
