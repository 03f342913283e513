"""Montgomery-resident rows (include/fthe.h fthe_to_mont_dev / fthe_from_mont_dev /
fthe_add_mont_dev) on the GPU.

The homomorphic add is x*y mod n^2 (paillier.cpp:103, paillier_gmp.cpp:16).  Rows
kept as x R mod n^2 multiply with one Montgomery product; converting back must give
exactly the ciphertext the reference's add gives.  Checked at the three golden key
sizes (one-lane n^2 kernels at 512/1023 bits, the four-lane row kernel at 2048):

* to_mont(x) = x R mod n^2 with R = to_mont(1), for edge rows 0, 1, n^2 - 1 and
  ciphertexts; from_mont(to_mont(x)) = x;
* from_mont(add_mont(to_mont(a), to_mont(b))) = a b mod n^2 (Python) = fthe_add_dev,
  bit-exact; aliasing (out = a);
* a 64-term chain of resident adds = the product of the 64 ciphertexts, decrypting
  to the plaintext sum (a tree sum, tree.cpp:20-34).
Integer work: every comparison is exact.
"""
import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN_KEYS, golden_key, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


def _t(rows):
    import torch
    return torch.from_numpy(np.ascontiguousarray(rows, dtype=np.uint32).view(np.int32)).to("cuda:0")


def _h(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_mont_rows_bit_exact(dev, name):
    import torch
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    n = p * q
    n2 = n * n
    pl = Paillier.from_primes(p, q, dev)
    cw = 2 * pl.n_words
    rng = np.random.default_rng(len(name) + 500)
    cnt = 1000
    m = rng.integers(0, 2**40, 2 * cnt, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=3)
    a, b = c[:cnt].copy(), c[cnt:].copy()
    a[0] = pyoracle.to_words(0, cw)
    a[1] = pyoracle.to_words(1, cw)
    a[2] = pyoracle.to_words(n2 - 1, cw)
    b[3] = pyoracle.to_words(n2 - 1, cw)
    da, db = _t(a), _t(b)
    ma, mb = torch.empty_like(da), torch.empty_like(db)
    pl.to_mont_dev(da, ma)
    pl.to_mont_dev(db, mb)
    one = torch.empty_like(da[:1])
    pl.to_mont_dev(_t(np.array([pyoracle.to_words(1, cw)])), one)
    R = pyoracle.from_words(_h(one)[0])
    assert 0 < R < n2
    ai, bi = pyoracle.words_to_ints(a), pyoracle.words_to_ints(b)
    assert pyoracle.words_to_ints(_h(ma)) == [x * R % n2 for x in ai]
    back = torch.empty_like(da)
    pl.from_mont_dev(ma, back)
    assert np.array_equal(_h(back), a)
    ms = torch.empty_like(da)
    pl.add_mont_dev(ma, mb, ms)
    Rinv = pow(R, -1, n2)
    assert pyoracle.words_to_ints(_h(ms)) == [x * y * R % n2 for x, y in zip(ai, bi)]
    s = torch.empty_like(da)
    pl.from_mont_dev(ms, s)
    want = [x * y % n2 for x, y in zip(ai, bi)]
    assert pyoracle.words_to_ints(_h(s)) == want
    ref = torch.empty_like(da)
    pl.add_dev(da, db, ref)
    assert torch.equal(ref, s)
    # aliasing: out = a
    pl.add_mont_dev(ma, mb, ma)
    assert torch.equal(ma, ms)
    assert Rinv * R % n2 == 1
    # decryptions of the resident sums (rows 4..: real ciphertexts)
    dec = pl.decrypt_u64(_h(s)[4:])
    assert np.array_equal(dec, (m[4:cnt] + m[cnt + 4:]))
    # zero count is a no-op
    pl.add_mont_dev(ma[:0], mb[:0], ms[:0])


@pytest.mark.parametrize("name", ["ref_gmp_L2048.json", "ref_gmp_L4096.json"])
def test_mont_rows_chain_sum(dev, name):
    """A 64-term sum kept resident: 64 conversions in, 63 one-product adds, 1 out."""
    import torch
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    pl = Paillier.from_primes(p, q, dev)
    terms, cnt = 64, 4096
    m = np.random.default_rng(8).integers(0, 2**32, (terms, cnt), dtype=np.uint64)
    c = pl.encrypt_u64(m.reshape(-1), seed=9).reshape(terms, cnt, -1)
    dc = _t(c.reshape(terms * cnt, -1)).reshape(terms, cnt, -1)
    res = torch.empty_like(dc)
    pl.to_mont_dev(dc, res)
    acc = res[0].clone()
    for j in range(1, terms):
        pl.add_mont_dev(acc, res[j], acc)
    out = torch.empty_like(acc)
    pl.from_mont_dev(acc, out)
    kway = torch.empty_like(acc)
    pl.reduce_kway_dev(dc, terms, kway)
    assert torch.equal(out, kway)
    assert np.array_equal(pl.decrypt_u64(_h(out)), m.sum(axis=0))
