"""Exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT, include/fthe.h) on the GPU.

The reference draws r uniform in Z_n^* (paillier.cpp:127-133); r^n mod P^2 is then
uniform over G_P = {x^P mod P^2} (order P - 1) for P = p, q independently.  The
engine draws it as prod_i gam_i^y_i with three bases gam_i = t_i^P mod P^2 that
generate G_P and y_i uniform in [1, P).  Checked here:

* the bases: each gam_i lies in G_P, and at every small prime l | P - 1 not all
  three reduce to l-th powers mod P (so <gam_1, gam_2, gam_3> = G_P wherever P - 1
  factors over small primes -- completely so for the smooth-prime key below);
* injected exponents: bit-exact against (1 + m n) prod gam_i^y_i mod P^2 recombined
  by CRT (Python pow), at the three golden key sizes, incl. y = 0, 1 and the
  largest exponent the tables cover; decryption by the unchanged CRT decrypt;
* device-drawn exponents: round trips across a chunk boundary, seeded determinism,
  fresh ciphertexts, an oracle decryption sample, homomorphic add;
* public-only keys refuse the mode (it needs p, q).
Integer work: every comparison is exact.
"""
import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN_KEYS, golden_key, load_golden
from fedtree_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


def _primes_below(n):
    s = np.ones(n, bool)
    s[:2] = False
    for i in range(2, int(n ** 0.5) + 1):
        if s[i]:
            s[i * i::i] = False
    return [int(x) for x in np.nonzero(s)[0]]


SMALL = _primes_below(1 << 16)


def _check_bases(gam, P):
    P2 = P * P
    for g in gam:
        assert 1 < g < P2 and pow(g, P - 1, P2) == 1          # in G_P
    for l in SMALL:
        if (P - 1) % l == 0:
            assert not all(pow(g % P, (P - 1) // l, P) == 1 for g in gam), l


def _crt_want(p, q, m, ys, gam):
    n = p * q
    nb = len(gam[0])
    parts = []
    for P, yy, gg in ((p, ys[:nb], gam[0]), (q, ys[nb:], gam[1])):
        P2 = P * P
        v = (1 + int(m) * n) % P2
        for y, g in zip(yy, gg):
            v = v * pow(g, y, P2) % P2
        parts.append(v)
    cp, cq = parts
    p2, q2 = p * p, q * q
    return (cq + q2 * ((cp - cq) * pow(q2, -1, p2) % p2)) % (n * n)


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_exact_injected_exponents(dev, name):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    pl = Paillier.from_primes(p, q, dev)
    pl.set_fixed_base_exact(seed=7)
    gam, ew = pl.fixed_base_exact_info()
    assert ew == pl.n_words // 2
    _check_bases(gam[0], p)
    _check_bases(gam[1], q)
    rng = np.random.default_rng(len(name) + 100)
    ebits = 16 * ((max(p.bit_length(), q.bit_length()) + 15) // 16)
    cnt = 24
    m = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    m[:3] = [0, 1, 2**64 - 1]
    ys = [tuple(int.from_bytes(rng.bytes(ebits // 8), "little") for _ in range(6)) for _ in range(cnt)]
    ys[0] = (0,) * 6
    ys[1] = (1,) * 6
    ys[2] = ((1 << ebits) - 1,) * 6
    ys[3] = (p - 1, 0, 0, q - 1, 0, 0)                      # gam^(P-1) = 1
    assert len(gam[0]) == 3
    c = pl.encrypt_u64(m, r=ys, fixed_base_exact=True)
    want = [_crt_want(p, q, x, y, gam) for x, y in zip(m, ys)]
    assert pyoracle.words_to_ints(c) == want
    assert np.array_equal(pl.decrypt_u64(c), m)
    # y = 0 everywhere: the randomizer is 1 and c = 1 + m n
    assert pyoracle.from_words(c[0]) == 1 and pyoracle.from_words(c[1]) != 1 + p * q
    # seeded rebuild: same bases; another seed: different bases
    pl.set_fixed_base_exact(seed=7)
    assert pl.fixed_base_exact_info()[0] == gam
    pl.set_fixed_base_exact(seed=8)
    assert pl.fixed_base_exact_info()[0] != gam


def test_exact_random_roundtrip_p2048(dev, coracle):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden("ref_gmp_L4096.json"))
    pl = Paillier.from_primes(p, q, dev)
    cnt = 393216 + 321                                        # crosses the 393,216-lane chunk
    m = np.random.default_rng(6).integers(0, 2**64, cnt, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=21, fixed_base_exact=True)
    assert np.array_equal(pl.decrypt_u64(c), m)
    idx = np.arange(0, cnt, 4099)
    assert len({bytes(c[i]) for i in idx}) == len(idx)
    assert np.array_equal(pl.encrypt_u64(m[:2000], seed=21, fixed_base_exact=True), c[:2000])
    assert not np.array_equal(pl.encrypt_u64(m[:2000], seed=22, fixed_base_exact=True), c[:2000])
    same = pl.encrypt_u64(np.full(64, 4242, np.uint64), seed=3, fixed_base_exact=True)
    assert len({bytes(x) for x in same}) == 64
    ok = coracle.key(pyoracle.to_words(p, pl.n_words // 2), pyoracle.to_words(q, pl.n_words // 2))
    dec = ok.decrypt_batch(c[idx[:24]])
    assert [pyoracle.from_words(d) for d in dec] == [int(x) for x in m[idx[:24]]]
    s = pl.add_batch(c[:1000], c[1000:2000])
    assert np.array_equal(pl.decrypt_u64(s), m[:1000] + m[1000:2000])


def _is_prime(n, rng):
    if n < 2:
        return False
    for sp in SMALL[:50]:
        if n % sp == 0:
            return n == sp
    d, s = n - 1, 0
    while d % 2 == 0:
        d, s = d // 2, s + 1
    for _ in range(32):
        a = int(rng.integers(2, 2**62)) % (n - 3) + 2
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _smooth_prime(bits, rng):
    """P = prod(primes < 2^16) * 2 + 1 of `bits` bits: P - 1 factors completely over SMALL."""
    while True:
        x = 2
        while x.bit_length() < bits:
            x *= SMALL[int(rng.integers(1, len(SMALL)))]
        if x.bit_length() == bits and _is_prime(x + 1, rng):
            return x + 1


def test_exact_bases_generate_for_smooth_primes(dev):
    """p - 1, q - 1 fully factored over primes < 2^16: the engine's small-prime check
    is then complete, so <gam_1, gam_2, gam_3> = G_P exactly -- verified here at every
    prime factor -- and every encryption is exactly the reference's distribution."""
    from fedtree_amd.paillier import Paillier
    rng = np.random.default_rng(2026)
    while True:
        p, q = _smooth_prime(256, rng), _smooth_prime(256, rng)
        if p != q and (p * q).bit_length() == 512:            # gcd(n, phi(n)) = 1: p - 1, q - 1 are smooth
            break
    pl = Paillier.from_primes(p, q, dev)
    pl.set_fixed_base_exact(seed=11)
    gam, _ = pl.fixed_base_exact_info()
    for P, g in ((p, gam[0]), (q, gam[1])):
        rest = P - 1
        for l in SMALL:
            while rest % l == 0:
                rest //= l
        assert rest == 1                                       # fully factored
        _check_bases(g, P)
    m = np.arange(5000, dtype=np.uint64) * np.uint64(7919)
    c = pl.encrypt_u64(m, seed=5, fixed_base_exact=True)
    assert np.array_equal(pl.decrypt_u64(c), m)


def test_exact_needs_private_key(dev):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden("ref_gmp_L2048.json"))
    pub = Paillier.from_public(p * q, dev)
    with pytest.raises(RuntimeError):
        pub.encrypt_u64(np.arange(4, dtype=np.uint64), fixed_base_exact=True)
    with pytest.raises(RuntimeError):
        pub.set_fixed_base_exact(seed=1)
    assert _lib.FTHE_ENC_FIXED_BASE_EXACT == 4


def _factor_small(x):
    """x = prod(primes < 2^16)^e * rest; returns (distinct small primes, rest)."""
    fs = []
    for l in SMALL:
        if x % l == 0:
            fs.append(l)
            while x % l == 0:
                x //= l
    return fs, x


@pytest.mark.parametrize("bits", [1024, 2048])
def test_known_order_keygen_single_generator(dev, coracle, bits):
    """FTHE_KEYGEN_KNOWN_ORDER: P - 1 = 2 s P' with s smooth and P' prime, so the engine
    picks one generator per prime; verified here at every prime factor of P - 1, with
    injected exponents bit-exact and device-drawn round trips."""
    from fedtree_amd.paillier import Paillier
    pl = Paillier(dev).keygen(bits, seed=77, known_order=True)
    p, q, n = pl.p, pl.q, pl.modulus
    assert n.bit_length() == bits and p * q == n
    assert pl.p >= 3 << (bits // 2 - 2) and pl.q >= 3 << (bits // 2 - 2)
    pl.set_fixed_base_exact(seed=5)
    gam, ew = pl.fixed_base_exact_info()
    assert [len(g) for g in gam] == [1, 1]
    for P, (g,) in ((p, gam[0]), (q, gam[1])):
        fs, rest = _factor_small(P - 1)
        assert 2 in fs and rest > 2**64 and pow(3, rest - 1, rest) == 1      # P' a large (probable) prime
        for l in fs + [rest]:
            assert pow(g % P, (P - 1) // l, P) != 1, l                       # a generator of Z_P^*
        assert pow(g, P - 1, P * P) == 1                                       # in G_P
    rng = np.random.default_rng(bits)
    ebits = 16 * ((max(p.bit_length(), q.bit_length()) + 15) // 16)
    m = rng.integers(0, 2**64, 16, dtype=np.uint64)
    ys = [(int.from_bytes(rng.bytes(ebits // 8), "little"), int.from_bytes(rng.bytes(ebits // 8), "little"))
          for _ in range(16)]
    ys[0] = (0, 0)
    c = pl.encrypt_u64(m, r=ys, fixed_base_exact=True)
    assert pyoracle.words_to_ints(c) == [_crt_want(p, q, x, y, gam) for x, y in zip(m, ys)]
    mm = rng.integers(0, 2**64, 100_000, dtype=np.uint64)
    cc = pl.encrypt_u64(mm, seed=9, fixed_base_exact=True)
    assert np.array_equal(pl.decrypt_u64(cc), mm)
    ok = coracle.key(pyoracle.to_words(p, pl.n_words // 2), pyoracle.to_words(q, pl.n_words // 2))
    dec = ok.decrypt_batch(cc[:16])
    assert [pyoracle.from_words(d) for d in dec] == [int(x) for x in mm[:16]]
