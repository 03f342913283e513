"""Short-plaintext decryption (fthe_decrypt_short[_dev], include/fthe.h): the p
half of the CRT decryption (paillier.cpp:153-156 restricted to mod p).

* golden vectors of the reference's Paillier_GMP (plaintexts < 2^64 < p),
  bit-exact, at the three key sizes;
* sums and differences as FedTree makes them (8-party merge, a*b^(2^64-1)):
  equal to the full CRT decryption;
* a plaintext >= p decrypts to m mod p (the documented precondition).
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


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_short_decrypt_golden(dev, name):
    from fedtree_amd.paillier import Paillier
    g = load_golden(name)
    p, q = golden_key(g)
    pl = Paillier.from_primes(p, q, dev)
    cts = pyoracle.ints_to_words([int(c["c"], 16) for c in g["cases"]], 2 * g["n_words"])
    want = np.array([c["m"] for c in g["cases"]], dtype=np.uint64)
    low, full = pl.decrypt_u64(cts, full=True, short=True)
    assert np.array_equal(low, want)
    lf, ff = pl.decrypt_u64(cts, full=True)
    assert np.array_equal(full, ff)
    # FedTree-shaped derived plaintexts: k-way sums and subtractions
    rng = np.random.default_rng(3)
    m = rng.integers(0, 2**64, 4096, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=2)
    s = pl.reduce_kway(c.reshape(8, 512, -1))
    d = pl.sub_batch(c[:512], c[512:1024])
    for x in (s, d):
        assert np.array_equal(pl.decrypt_u64(x, short=True), pl.decrypt_u64(x))
    # precondition: a plaintext >= p comes back reduced mod p
    n = pl.modulus
    big = [p + 12345, n - 1]
    cb = pyoracle.ints_to_words([(1 + x * n) % (n * n) for x in big], 2 * pl.n_words)   # g^x with r = 1
    _, fb = pl.decrypt_u64(cb, full=True, short=True)
    assert [pyoracle.from_words(w) for w in fb] == [x % p for x in big]
