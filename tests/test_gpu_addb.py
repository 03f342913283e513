"""The P-2048 pairwise add on the matrix-core Barrett kernel (fthe_addb_q152, gen_addb.py; the default for
keys with a 2048-bit n): out = x y mod n^2 (paillier.cpp:92-105) bit-exact against Python's integers and
against the classical four-lane product (FTHE_ADD_NO_ADDB=1 at key set-up), across wave / workgroup /
chunk boundaries, with the extremes 0, 1, n^2 - 1, rows >= n^2 (the reference reduces them too), aliased
output and the host path.  Integer work: exact equality."""
import os

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu
SEED = 20261017


@pytest.fixture(scope="module")
def keys():
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=SEED)
    os.environ["FTHE_ADD_NO_ADDB"] = "1"
    try:
        ref = Paillier.from_primes(pl.p, pl.q, dev)          # the same n on the classical product
    finally:
        del os.environ["FTHE_ADD_NO_ADDB"]
    return dev, pl, ref


def _rows(vals, cw):
    return pyoracle.ints_to_words(vals, cw)


def test_addb_sizes_vs_classical_and_integers(keys):
    import torch
    dev, pl, ref = keys
    n2, cw = pl.n2, 2 * pl.n_words
    rng = np.random.default_rng(7)
    for cnt in (1, 15, 16, 17, 191, 192, 193, 4099):
        a = [int.from_bytes(rng.bytes(512), "little") % n2 for _ in range(cnt)]
        b = [int.from_bytes(rng.bytes(512), "little") % n2 for _ in range(cnt)]
        ad = torch.from_numpy(_rows(a, cw).view(np.int32)).cuda()
        bd = torch.from_numpy(_rows(b, cw).view(np.int32)).cuda()
        o1, o2 = torch.empty_like(ad), torch.empty_like(ad)
        pl.add_dev(ad, bd, o1)
        ref.add_dev(ad, bd, o2)
        dev.sync()
        assert torch.equal(o1, o2), cnt
        got = pyoracle.words_to_ints(o1.cpu().numpy().view(np.uint32))
        assert got == [x * y % n2 for x, y in zip(a, b)], cnt


def test_addb_extremes_and_noncanonical_rows(keys):
    import torch
    dev, pl, ref = keys
    n2, cw = pl.n2, 2 * pl.n_words
    ext = [0, 1, 2, n2 - 1, n2 - 2, n2 // 2, (1 << 4094) - 1, n2 - (1 << 64), 1 << 4000, (1 << 27) - 1,
           n2, n2 + 12345, (1 << 4096) - 1, (1 << 4072) - 1, 1 << 4072]
    a = [x for x in ext for _ in ext]
    b = [y for _ in ext for y in ext]
    ad = torch.from_numpy(_rows(a, cw).view(np.int32)).cuda()
    bd = torch.from_numpy(_rows(b, cw).view(np.int32)).cuda()
    o = torch.empty_like(ad)
    pl.add_dev(ad, bd, o)
    dev.sync()
    got = pyoracle.words_to_ints(o.cpu().numpy().view(np.uint32))
    bad = [(i, j) for i in range(len(ext)) for j in range(len(ext)) if got[i * len(ext) + j] != ext[i] * ext[j] % n2]
    assert not bad, bad[:8]


def test_addb_full_chunk_aliased_and_host(keys):
    """one chunk and a half of device rows (the launch loop), in place (out = a), and the host path"""
    import torch
    dev, pl, ref = keys
    cw = 2 * pl.n_words
    cnt = 600_000
    m = torch.randint(0, 2**62, (2 * cnt,), dtype=torch.int64, device="cuda")
    c = torch.empty((2 * cnt, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=3)
    want = torch.empty((cnt, cw), dtype=torch.int32, device="cuda")
    ref.add_dev(c[:cnt], c[cnt:], want)
    x = c[:cnt].clone()
    pl.add_dev(x, c[cnt:], x)                                # aliased output
    dev.sync()
    assert torch.equal(x, want)
    h = pl.add_batch(c[:5000].cpu().numpy().view(np.uint32), c[cnt:cnt + 5000].cpu().numpy().view(np.uint32))
    assert np.array_equal(h, want[:5000].cpu().numpy().view(np.uint32))
    # the sum decrypts to the plaintext sum (homomorphic add)
    low = torch.empty(cnt, dtype=torch.int64, device="cuda")
    pl.decrypt_u64_dev(x, low)
    dev.sync()
    assert torch.equal(low, m[:cnt] + m[cnt:])


def test_addb_beyond_one_launch(keys):
    """more rows than one launch addresses (4M: row offsets are 32-bit in the kernel): the launches split,
    and the rows around each split equal the classical product's"""
    import torch
    dev, pl, ref = keys
    cw = 2 * pl.n_words
    cnt = (1 << 22) + 1000
    m = torch.randint(0, 2**62, (2 * 8192,), dtype=torch.int64, device="cuda")
    c = torch.empty((2 * 8192, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=11)
    reps = (cnt + 8191) // 8192
    a = c[:8192].repeat(reps, 1)[:cnt]
    b = c[8192:].roll(1, 0).repeat(reps, 1)[:cnt]
    o = torch.empty_like(a)
    pl.add_dev(a, b, o)
    sl = torch.cat([torch.arange(0, 4096), torch.arange((1 << 22) - 4096, cnt)]).cuda()
    want = torch.empty((len(sl), cw), dtype=torch.int32, device="cuda")
    ref.add_dev(a[sl].contiguous(), b[sl].contiguous(), want)
    dev.sync()
    assert torch.equal(o[sl], want)
    del a, b, o
