"""BASELINE.json configs at full size on the device, through the C ABI.

* configs[1]: Paillier-1024 encrypt of 100k gradient pairs with injected r --
  bit-exact against the C/GMP oracle's ciphertexts of all 200k (SHA-256 of the
  fixture made by tests/golden/make_config1.py), CRT and public-key forms, plus
  the decrypt round trip of every ciphertext;
* configs[2]: Paillier-2048 encrypt + CRT decrypt of 10M gradient pairs (20M
  ciphertexts, 10.2 GB) device-resident with device randomness -- every
  plaintext round-trips, a sample decrypts identically under the C oracle;
* configs[3]: Paillier-2048 8-party merge of 256 x 4096 bins x {g, h} -- every
  merged bin decrypts to the plaintext sum (mod 2^64, the codec's wrap).
Integer work: every comparison is exact.
"""
import hashlib
import sys

import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN, load_golden

sys.path.insert(0, GOLDEN)
import make_config1 as cfg1   # noqa: E402

pytestmark = pytest.mark.gpu
SEED = 20261015


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_config1_p1024_100k_pairs_bit_exact(dev, coracle):
    from fedtree_amd.paillier import Paillier
    fix = load_golden("config1_p1024.json")
    pw, qw = cfg1.config1_key(coracle)
    p, q = pyoracle.from_words(pw), pyoracle.from_words(qw)
    m, r = cfg1.config1_inputs(p * q)
    assert _sha(m) == fix["m_sha256"] and _sha(r) == fix["r_sha256"]
    pl = Paillier.from_primes(p, q, dev)
    for public in (False, True):
        c = pl.encrypt_u64(m, r=r, public=public)
        assert c.shape == (len(m), fix["ct_words"])
        blocks = [_sha(c[i:i + fix["block"]]) for i in range(0, len(c), fix["block"])]
        bad = [i for i, (x, y) in enumerate(zip(blocks, fix["block_sha256"])) if x != y]
        assert not bad, f"public={public}: blocks {bad} differ from the oracle"
        assert _sha(c) == fix["ct_sha256"]
    assert np.array_equal(pl.decrypt_u64(c), m)


def test_config2_p2048_10M_pairs_roundtrip(dev, coracle):
    import torch
    from fedtree_amd import _lib
    import ctypes
    from fedtree_amd.paillier import Paillier, encode_fixed
    from fedtree_amd.synth import logistic_gradients
    pairs = 10_000_000
    pl = Paillier(dev).keygen(2048, seed=SEED)
    g, h = logistic_gradients(pairs, SEED)
    gh = np.concatenate([g, h])
    x = torch.from_numpy(gh).to("cuda:0")
    m = torch.empty(2 * pairs, dtype=torch.int64, device="cuda:0")
    dev.order_in()                   # direct C-ABI call: after torch's copy of x
    _lib.check(dev.lib.fthe_encode_fixed_dev(dev.ctx, ctypes.c_void_p(x.data_ptr()), 2 * pairs,
                                             ctypes.c_void_p(m.data_ptr())), "encode")
    dev.sync()
    m_host = encode_fixed(gh)
    assert np.array_equal(m.cpu().numpy().view(np.uint64), m_host)      # device codec == host codec
    del x
    c = torch.empty((2 * pairs, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.encrypt_u64_dev(m, c, seed=77)
    out = torch.empty_like(m)
    pl.decrypt_u64_dev(c, out)
    dev.sync()
    assert torch.equal(out, m)
    out.zero_()
    pl.decrypt_u64_dev(c, out, short=True)
    dev.sync()
    assert torch.equal(out, m)
    # a sample, decrypted by the oracle (full PowerMod, no CRT)
    idx = torch.arange(0, 2 * pairs, 2 * pairs // 48, device="cuda:0")
    sample = c[idx].cpu().numpy().view(np.uint32)
    ok = coracle.key(pyoracle.to_words(pl.p, pl.n_words // 2), pyoracle.to_words(pl.q, pl.n_words // 2))
    dec = ok.decrypt_batch(sample)
    assert [pyoracle.from_words(d) for d in dec] == [int(v) for v in m_host[idx.cpu().numpy()]]
    # fresh randomness: no repeated ciphertext among equal plaintexts of the sample
    assert len({s.tobytes() for s in sample}) == len(sample)
    # the timed path itself, bit for bit across the whole batch: 64 ciphertexts on each side of every 786,432-lane
    # launch boundary (the p and q halves of each chunk on two streams) and the batch's first and last 64, each
    # against the C oracle's full-PowerMod encrypt(m, r) with r rebuilt from the drawn (y_p, y_q)
    from test_gpu_direct_y import ENC_CHUNK, _check
    n = 2 * pairs
    edges = [0] + list(range(ENC_CHUNK, n, ENC_CHUNK)) + [n]
    idx = np.unique(np.concatenate([np.arange(max(0, b - 64), min(n, b + 64)) for b in edges]))
    rows = c[torch.from_numpy(idx).to("cuda:0")].cpu().numpy().view(np.uint32)
    _check(pl, ok, m_host[idx], rows, 77, idx)


def test_config3_p2048_8party_merge_full_size(dev):
    import torch
    from fedtree_amd.paillier import Paillier
    bins, parties = 2 * 256 * 4096, 8
    pl = Paillier(dev).keygen(2048, seed=SEED + 3)
    gen = torch.Generator(device="cuda:0").manual_seed(5)
    # codec-range plaintexts incl. negatives (two's complement wrap): |x| < 2^40
    m = torch.randint(-(1 << 40), 1 << 40, (parties, bins), dtype=torch.int64, device="cuda:0", generator=gen)
    c = torch.empty((parties, bins, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.encrypt_u64_dev(m.reshape(-1), c.reshape(parties * bins, -1), seed=9)
    merged = torch.empty((bins, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.reduce_kway_dev(c, parties, merged)
    del c
    out = torch.empty(bins, dtype=torch.int64, device="cuda:0")
    pl.decrypt_u64_dev(merged, out)
    dev.sync()
    assert torch.equal(out, m.sum(0))
