"""BASELINE configs[2] at full size on one GPU, checked through size-independent properties.

10M gradient pairs = 20M Paillier-2048 ciphertexts (10.24 GB, the bench's workload), device-resident:
* every ciphertext decrypts to its plaintext (CRT decrypt, all 20M compared, and the short p-half
  decrypt on a strided sample);
* the homomorphic sum of all 20M ciphertexts (one segmented product, the root-sum reduction of
  tree.cpp:20-34 at its largest) decrypts to the plaintext sum mod 2^64 -- a checksum of the whole batch;
* the same over the g plane alone, per 2^20-element segment (10 segment checksums, the last ragged);
* seeded determinism on a slice across the 393,216-lane chunk boundary.
The oracle's per-element bit-exactness is covered at smaller sizes (test_gpu_parity.py); these checks
are what the full size adds.  Integer work: every comparison is exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAIRS = 10_000_000


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


def test_fullsize_encrypt_decrypt_and_checksums(dev):
    import torch
    from fedtree_amd.paillier import Paillier, encode_fixed
    from fedtree_amd.synth import logistic_gradients
    pl = Paillier(dev).keygen(2048, seed=20261015)
    g, h = logistic_gradients(PAIRS)
    m_host = np.concatenate([encode_fixed(g), encode_fixed(h)])                  # 20M codec values
    n = len(m_host)
    m = torch.from_numpy(m_host.view(np.int64)).to("cuda:0")
    c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.encrypt_u64_dev(m, c, seed=77)
    low = torch.empty_like(m)
    pl.decrypt_u64_dev(c, low)
    assert torch.equal(low, m)                                                  # all 20M
    idx = torch.arange(0, n, 997, device="cuda:0")
    short = torch.empty(len(idx), dtype=torch.int64, device="cuda:0")
    pl.decrypt_u64_dev(c[idx].contiguous(), short, short=True)
    assert torch.equal(short, m[idx])
    # checksum of the whole batch: one 20M-term product decrypts to the plaintext sum mod 2^64
    seg = torch.tensor([0, n], dtype=torch.int64, device="cuda:0")
    tot = torch.empty((1, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.reduce_segments_csr_dev(c, seg, tot)
    s = torch.empty(1, dtype=torch.int64, device="cuda:0")
    pl.decrypt_u64_dev(tot, s)
    want = int(m_host.sum(dtype=np.uint64))                                     # wraps mod 2^64
    assert int(s.cpu().numpy().view(np.uint64)[0]) == want
    # 10 segment checksums over the g plane (2^20 elements each, the last one ragged)
    bounds = list(range(0, PAIRS, 1 << 20)) + [PAIRS]
    seg = torch.tensor(bounds, dtype=torch.int64, device="cuda:0")
    sums = torch.empty((len(bounds) - 1, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.reduce_segments_csr_dev(c[:PAIRS], seg, sums)
    ds = torch.empty(len(bounds) - 1, dtype=torch.int64, device="cuda:0")
    pl.decrypt_u64_dev(sums, ds)
    want_seg = [int(m_host[a:b].sum(dtype=np.uint64)) for a, b in zip(bounds[:-1], bounds[1:])]
    assert [int(x) for x in ds.cpu().numpy().view(np.uint64)] == want_seg
    # seeded determinism across the first chunk boundary
    k = 393216 + 4099
    again = torch.empty((k, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.encrypt_u64_dev(m[:k], again, seed=77)
    assert torch.equal(again, c[:k])
    del c, low, m
    torch.cuda.empty_cache()
