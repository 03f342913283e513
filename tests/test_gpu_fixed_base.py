"""Fixed-base randomizer mode (FTHE_ENC_FIXED_BASE, include/fthe.h) on the GPU.

Not a reference feature: an opt-in encryption mode.  A ciphertext is
c = (1 + m n) * hs^alpha mod n^2 with hs = h^n mod n^2, i.e. Paillier's
c = g^m r^n (paillier.cpp:134-137, g^m = 1 + m n) under r = h^alpha.  Checked:

* injected alpha: bit-exact against Python's pow for that formula, at the three
  golden key sizes, CRT (key holder) and public-key forms, incl. alpha = 0, 1 and
  the largest alpha the tables cover;
* device-drawn alpha: decryption by the unchanged CRT decrypt returns m, across a
  chunk boundary; seeded determinism; fresh ciphertexts; homomorphic add works;
* a public-only key encrypts, the private key decrypts.
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


def _key(dev, name):
    from fedtree_amd.paillier import Paillier
    g = load_golden(name)
    p, q = golden_key(g)
    return Paillier.from_primes(p, q, dev), p, q


def _want(n, hs, m, a):
    n2 = n * n
    return (1 + int(m) * n) % n2 * pow(hs, a, n2) % n2


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_fixed_base_injected_alpha_exact(dev, name):
    pl, p, q = _key(dev, name)
    n, n2 = pl.modulus, pl.modulus ** 2
    rng = np.random.default_rng(len(name))
    h = int.from_bytes(rng.bytes(pl.n_words * 4), "little") % (n - 2) + 2
    pl.set_fixed_base(h)
    bits_pub, bits_crt, hs = pl.fixed_base_info()
    assert hs == pow(h, n, n2)
    assert bits_crt >= max(p.bit_length(), q.bit_length()) + 64
    cnt = 40
    m = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    m[:3] = [0, 1, 2**64 - 1]
    forms = [(False, bits_crt)] + ([(True, bits_pub)] if bits_pub else [])
    for public, bits in forms:
        al = [int.from_bytes(rng.bytes(bits // 8), "little") for _ in range(cnt)]
        al[0], al[1], al[2] = 0, 1, (1 << bits) - 1
        c = pl.encrypt_u64(m, r=al, public=public, fixed_base=True)
        want = [_want(n, hs, x, a) for x, a in zip(m, al)]
        assert pyoracle.words_to_ints(c) == want, f"public={public}"
        assert np.array_equal(pl.decrypt_u64(c), m)


def test_fixed_base_random_alpha_roundtrip_p2048(dev):
    pl, p, q = _key(dev, "ref_gmp_L4096.json")
    pl.set_fixed_base(None)
    cnt = 393216 + 321                       # crosses the 393,216-lane chunk
    m = np.random.default_rng(5).integers(0, 2**64, cnt, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=99, fixed_base=True)
    assert np.array_equal(pl.decrypt_u64(c), m)
    # CRT path: every ciphertext lies in Z_{n^2}, fresh, and seeded runs repeat
    idx = np.arange(0, cnt, 4099)
    assert len({bytes(c[i]) for i in idx}) == len(idx)
    assert np.array_equal(pl.encrypt_u64(m[:2000], seed=99, fixed_base=True), c[:2000])
    assert not np.array_equal(pl.encrypt_u64(m[:2000], seed=98, fixed_base=True), c[:2000])
    # public-key form (four-lane kernel, row I/O)
    cp = pl.encrypt_u64(m[:50000], seed=7, public=True, fixed_base=True)
    assert np.array_equal(pl.decrypt_u64(cp), m[:50000])
    # homomorphic add of fixed-base ciphertexts
    s = pl.add_batch(c[:1000], cp[:1000])
    assert np.array_equal(pl.decrypt_u64(s), m[:1000] + m[:1000])
    # same message, same seed slot, different alpha -> different ciphertexts
    same = pl.encrypt_u64(np.full(64, 12345, np.uint64), seed=3, fixed_base=True)
    assert len({bytes(x) for x in same}) == 64


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_fixed_base_public_only_key(dev, name):
    from fedtree_amd.paillier import Paillier
    pl, p, q = _key(dev, name)
    pub = Paillier.from_public(pl.modulus, dev)
    if pub.lib.fthe_kernel_limbs(2 * pl.modulus.bit_length()) == 0:
        pytest.skip("n^2 size not built for the public-key form")
    m = np.random.default_rng(9).integers(0, 2**64, 3000, dtype=np.uint64)
    c = pub.encrypt_u64(m, seed=4, fixed_base=True)
    assert np.array_equal(pl.decrypt_u64(c), m)
