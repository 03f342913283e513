"""General plaintexts (fthe_encrypt_words[_dev]; Paillier::encrypt(const ZZ&),
paillier.cpp:122-139): bit-exact against the pure-Python oracle's
g^m r^n mod n^2 with the full PowerMod(g, m, n^2), including m >= n (the
identity g^m = 1 + m n mod n^2 holds for every m) and the largest m that fits;
decryption returns m mod n.  The single-value Paillier.encrypt no longer
truncates plaintexts above 2^64."""
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
def test_encrypt_words_vs_oracle(dev, name):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    pl = Paillier.from_primes(p, q, dev)
    key = pyoracle.keygen_from_primes(p, q)
    n = pl.modulus
    rng = np.random.default_rng(len(name) + 7)
    big = lambda: int.from_bytes(rng.bytes(pl.n_words * 4), "little")
    ms = [big() % n for _ in range(10)] + [0, 1, 2**64, n - 1, n, n + 5, 2**(32 * pl.n_words) - 1]
    rs = [big() % (n - 1) + 1 for _ in ms]
    want = [pyoracle.encrypt(key, m, r) for m, r in zip(ms, rs)]
    forms = [False] + ([True] if pl.lib.fthe_kernel_limbs(2 * pl.keyLength) else [])
    for public in forms:
        c = pl.encrypt_words(ms, r=rs, public=public)
        assert pyoracle.words_to_ints(c) == want, f"public={public}"
    _, full = pl.decrypt_u64(c, full=True)
    assert [pyoracle.from_words(w) for w in full] == [m % n for m in ms]
    # device randomness round trip, and the single-value API above 2^64
    cd = pl.encrypt_words(ms[:10], seed=3)
    _, full = pl.decrypt_u64(cd, full=True)
    assert [pyoracle.from_words(w) for w in full] == ms[:10]
    assert pl.decrypt(pl.encrypt(ms[0])) == ms[0]


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_mul_any_exponent_vs_oracle(dev, name):
    """Paillier::mul(x, y) = PowerMod(x, y, n^2) for exponents above 64 bits."""
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    pl = Paillier.from_primes(p, q, dev)
    key = pyoracle.keygen_from_primes(p, q)
    n, n2 = pl.modulus, pl.modulus ** 2
    x = pyoracle.encrypt(key, 12345, 777)
    for y in (2**64, 2**64 + 1, n - 1, 3 * n + 17, 2**(32 * pl.n_words) - 1):
        assert pl.mul(x, y) == pow(x, y, n2)
    assert pl.decrypt(pl.mul(x, 2**70 + 3)) == 12345 * (2**70 + 3) % n
