"""Public exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT on a public key,
include/fthe.h fthe_key_public_bases / fthe_key_set_public_bases) on the GPU.

Parties encrypt their histograms with n alone (Party::encrypt_histogram,
party.h:118-142; public formula paillier.cpp:122-139, r uniform in Z_n^*).  The
key holder publishes bases hs_i = t_i^n mod n^2 with <t_i> = Z_n^*; a party draws
r^n as prod hs_i^y_i with y_i uniform below 2^(16 nwin) >= n 2^64.  Checked here:

* the published bases: each hs_i is an n-th residue mod n^2 (hs^phi(n) = 1), and
  hs_i mod p, mod q span every quotient Z_P^*/l-th powers for the small primes l
  dividing p-1 or q-1 (one non-l-th power where l divides one of them, rank 2 over
  GF(l) where it divides both) -- recomputed in Python from hs alone (t -> t^n is a
  bijection of Z_P^*, so the images carry the t_i's span);
* injected exponents: bit-exact against (1 + m n) prod hs_i^y_i mod n^2 (Python
  pow) at the three golden key sizes (one-lane n^2 kernels at 512/1023 bits, the
  four-lane row form at 2048), incl. y = 0, 1 and the largest exponent covered;
* device-drawn exponents: round trips, seeded determinism, fresh ciphertexts, the
  Server/Party histogram flow, known-order keys (2 bases);
* refusals: no bases (public key: FTHE_ERR_NOPRIV), bad bases, bases without p, q.
Integer work: every comparison is exact.
"""
import math

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


SMALL = _primes_below(1 << 12)
SMALL16 = _primes_below(1 << 16)


def _dlog(z, a, l, P):
    x = 1
    for d in range(l):
        if x == a:
            return d
        x = x * z % P
    raise AssertionError("not in <z>")


def _check_public_bases(hs, p, q, ls=SMALL):
    n = p * q
    n2 = n * n
    phi = (p - 1) * (q - 1)
    for h in hs:
        assert 1 < h < n2 and math.gcd(h, n) == 1 and pow(h, phi, n2) == 1
    for l in ls:
        inp, inq = (p - 1) % l == 0, (q - 1) % l == 0
        if not (inp or inq):
            continue
        a = [pow(h % p, (p - 1) // l, p) for h in hs] if inp else None
        b = [pow(h % q, (q - 1) // l, q) for h in hs] if inq else None
        if inp:
            assert any(x != 1 for x in a), l
        if inq:
            assert any(x != 1 for x in b), l
        if inp and inq and l < 1 << 12:
            i = next(i for i, x in enumerate(a) if x != 1)
            # rank 2: some j whose (log a_j, log b_j) is not a multiple of base i's
            assert any(pow(b[i], _dlog(a[i], a[j], l, p), q) != b[j] for j in range(len(hs)) if j != i), l


def _want(n, m, ys, hs):
    n2 = n * n
    v = (1 + int(m) * n) % n2
    for y, h in zip(ys, hs):
        v = v * pow(h, y, n2) % n2
    return v


@pytest.mark.parametrize("name", GOLDEN_KEYS)
def test_public_exact_injected_exponents(dev, name):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    n = p * q
    server = Paillier.from_primes(p, q, dev)
    hs = server.public_bases(seed=7)
    assert len(hs) == 3
    _check_public_bases(hs, p, q)
    assert server.public_bases(seed=7) == hs and server.public_bases(seed=8) != hs
    party = server.public(bases=hs)
    assert not party.has_private and party.has_public_bases
    nb, ew = party.public_bases_info()
    nwin = (n.bit_length() + 64 + 15) // 16
    assert nb == 3 and ew == [(nwin + 1) // 2] * 3 and hs.exp_bits == [16 * nwin] * 3
    ebits = 16 * nwin
    rng = np.random.default_rng(len(name) + 300)
    cnt = 24
    m = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    m[:3] = [0, 1, 2**64 - 1]
    ys = [tuple(int.from_bytes(rng.bytes(ebits // 8), "little") for _ in range(nb)) for _ in range(cnt)]
    ys[0] = (0,) * nb
    ys[1] = (1,) * nb
    ys[2] = ((1 << ebits) - 1,) * nb
    ys[3] = ((p - 1) * (q - 1), 0, 0)                        # hs^phi(n) = 1
    c = party.encrypt_u64(m, r=ys, fixed_base_exact=True)
    want = [_want(n, x, y, hs) for x, y in zip(m, ys)]
    assert pyoracle.words_to_ints(c) == want
    assert pyoracle.from_words(c[0]) == 1 and pyoracle.from_words(c[3]) == (1 + int(m[3]) * n) % (n * n)
    assert np.array_equal(server.decrypt_u64(c), m)
    # the key holder with the same bases, public form: identical ciphertexts
    server.set_public_bases(hs)
    assert np.array_equal(server.encrypt_u64(m, r=ys, public=True, fixed_base_exact=True), c)


@pytest.mark.parametrize("name", ["ref_gmp_L2048.json", "ref_gmp_L4096.json"])
def test_public_exact_random_roundtrip(dev, coracle, name):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden(name))
    server = Paillier.from_primes(p, q, dev)
    party = server.public(bases=server.public_bases())
    cnt = 200003
    m = np.random.default_rng(9).integers(0, 2**64, cnt, dtype=np.uint64)
    c = party.encrypt_u64(m, seed=31, fixed_base_exact=True)
    assert np.array_equal(server.decrypt_u64(c), m)
    idx = np.arange(0, cnt, 997)
    assert len({bytes(c[i]) for i in idx}) == len(idx)
    assert np.array_equal(party.encrypt_u64(m[:3000], seed=31, fixed_base_exact=True), c[:3000])
    assert not np.array_equal(party.encrypt_u64(m[:3000], seed=32, fixed_base_exact=True), c[:3000])
    same = party.encrypt_u64(np.full(64, 77, np.uint64), seed=4, fixed_base_exact=True)
    assert len({bytes(x) for x in same}) == 64
    ok = coracle.key(pyoracle.to_words(p, server.n_words // 2), pyoracle.to_words(q, server.n_words // 2))
    dec = ok.decrypt_batch(c[idx[:16]])
    assert [pyoracle.from_words(d) for d in dec] == [int(x) for x in m[idx[:16]]]
    s = party.add_batch(c[:1000], c[1000:2000])
    assert np.array_equal(server.decrypt_u64(s), m[:1000] + m[1000:2000])


def _full_factors(x):
    """Distinct primes of x = (primes < 2^16 part) * (at most one large prime cofactor), the shape of
    p - 1 for known-order keys (2 s P' with s a product of primes < 2^16); the cofactor is checked prime."""
    fs = []
    for l in SMALL16:
        if x % l == 0:
            fs.append(l)
            while x % l == 0:
                x //= l
    if x > 1:
        fs.append(x)
    return fs


@pytest.mark.parametrize("bits", [1024, 2048])
def test_public_exact_known_order_short_exponent(dev, bits):
    """FTHE_KEYGEN_KNOWN_ORDER keys: t_1 of order lcm(p-1, q-1) (a primitive root mod p and mod q,
    checked here at every prime factor) with a full exponent, t_2 generating the quotient Z_g,
    g = gcd(p-1, q-1), with a 128-bit exponent: 2 bases, 16 nwin + 128 exponent bits."""
    from fedtree_amd.paillier import Paillier
    rng = np.random.default_rng(bits)
    server = Paillier(dev).keygen(bits, seed=77, known_order=True)
    p, q = server.p, server.q
    n = p * q
    hs = server.public_bases(seed=3)
    nwin = (n.bit_length() + 64 + 15) // 16
    assert len(hs) == 2 and hs.exp_bits == [16 * nwin, 128]
    g = math.gcd(p - 1, q - 1)
    for P in (p, q):
        fs = _full_factors(P - 1)
        assert _is_prime_list(fs, rng)
        for l in fs:                                          # hs_1 mod P generates Z_P^* (t -> t^n bijective)
            assert pow(hs[0] % P, (P - 1) // l, P) != 1, l
    for l in _full_factors(g):                                 # t_2 generates Z_n^* / <t_1> = Z_g
        a = [pow(h % p, (p - 1) // l, p) for h in hs]
        b = [pow(h % q, (q - 1) // l, q) for h in hs]
        assert pow(b[0], _dlog(a[0], a[1], l, p), q) != b[1], l
    _check_public_bases(hs, p, q)
    party = server.public(bases=hs)
    nb, ew = party.public_bases_info()
    assert nb == 2 and ew == [(nwin + 1) // 2, 4]
    m = np.arange(20000, dtype=np.uint64) * np.uint64(1000003)
    c = party.encrypt_u64(m, seed=2, fixed_base_exact=True)
    assert np.array_equal(server.decrypt_u64(c), m)
    ys = [(5, 7), (0, 1), (2**(16 * nwin) - 1, 2**128 - 1), (2**1000 + 3, 2**100)]
    c = party.encrypt_u64(m[:4], r=ys, fixed_base_exact=True)
    assert pyoracle.words_to_ints(c) == [_want(n, x, y, hs) for x, y in zip(m[:4], ys)]
    # full-length exponents on the same bases (exp_bits omitted) still encrypt correctly
    full = server.public()
    full.set_public_bases(list(hs))
    assert full.public_bases_info() == (2, [(nwin + 1) // 2] * 2)
    assert np.array_equal(server.decrypt_u64(full.encrypt_u64(m[:500], seed=9, fixed_base_exact=True)), m[:500])


def _is_prime_list(fs, rng):
    def mr(x):
        if x < 4:
            return x in (2, 3)
        d, s = x - 1, 0
        while d % 2 == 0:
            d, s = d // 2, s + 1
        for _ in range(24):
            a = int(rng.integers(2, 2**62)) % (x - 3) + 2
            y = pow(a, d, x)
            if y in (1, x - 1):
                continue
            for _ in range(s - 1):
                y = y * y % x
                if y == x - 1:
                    break
            else:
                return False
        return True
    return all(mr(f) for f in fs)


def test_public_exact_histogram_flow(dev):
    """HEServer.send_key(bases=True) -> HEParty.encrypt_histogram(fixed_base_exact=True)
    -> merged by the party -> decrypted by the server (party.h:118-142, server.h:80-111)."""
    from fedtree_amd.paillier import GHPairs, HEParty, HEServer, Paillier
    srv = HEServer(dev)
    srv.paillier = Paillier.from_primes(*golden_key(load_golden("ref_gmp_L4096.json")), dev)
    parties = [HEParty(), HEParty()]
    for pt in parties:
        srv.send_key(pt, bases=True)
        assert pt.paillier.has_public_bases
    rng = np.random.default_rng(12)
    g = [rng.normal(size=300) for _ in parties]
    h = [rng.uniform(0.1, 1, size=300) for _ in parties]
    hists = [pt.encrypt_histogram(GHPairs(gg, hh), seed=i + 1, fixed_base_exact=True)
             for i, (pt, gg, hh) in enumerate(zip(parties, g, h))]
    total = (hists[0] + hists[1]).homo_decrypt(srv.paillier)
    want_g = (np.round(g[0] * 1e6).astype(np.int64) + np.round(g[1] * 1e6).astype(np.int64)) / 1e6
    assert np.allclose(total.g, want_g, atol=2e-6)
    # the short decrypt (p half only: plaintexts < p) decodes the same sums
    short = srv.decrypt_gh_pairs(hists[0] + hists[1], short=True)
    assert np.array_equal(short.g, total.g) and np.array_equal(short.h, total.h)
    # without published bases the flag falls back to the default public path
    plain = HEParty()
    srv.send_key(plain)
    enc = plain.encrypt_histogram(GHPairs(g[0], h[0]), seed=5, fixed_base_exact=True)
    assert np.allclose(enc.homo_decrypt(srv.paillier).g, np.round(g[0] * 1e6) / 1e6, atol=2e-6)


def test_public_exact_general_plaintexts(dev):
    """Paillier::encrypt(const ZZ&) plaintexts (any size < n) through the published-bases mode."""
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden("ref_gmp_L4096.json"))
    n = p * q
    server = Paillier.from_primes(p, q, dev)
    party = server.public(bases=server.public_bases(seed=5))
    rng = np.random.default_rng(41)
    ms = [0, 1, 2**64, 2**200 + 7, n - 1] + [int.from_bytes(rng.bytes(255), "little") for _ in range(11)]
    c = party.encrypt_words(ms, seed=3, fixed_base_exact=True)
    _, full = server.decrypt_u64(c, full=True)
    assert [pyoracle.from_words(x) for x in full] == [x % n for x in ms]
    assert len({bytes(x) for x in c}) == len(ms)


def test_public_exact_refusals(dev):
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden("ref_gmp_L2048.json"))
    n = p * q
    server = Paillier.from_primes(p, q, dev)
    pub = Paillier.from_public(n, dev)
    with pytest.raises(RuntimeError):                        # no bases: FTHE_ERR_NOPRIV
        pub.encrypt_u64(np.arange(4, dtype=np.uint64), fixed_base_exact=True)
    with pytest.raises(RuntimeError):                        # key holder, public form, no bases
        server.encrypt_u64(np.arange(4, dtype=np.uint64), public=True, fixed_base_exact=True)
    with pytest.raises(RuntimeError):                        # bases need p, q
        pub.public_bases()
    with pytest.raises(RuntimeError):
        pub.public_bases_info()
    for bad in ([n], [0], [n * n], [2, 3, 5, 7]):             # not a unit / out of range / nb > 3
        with pytest.raises(RuntimeError):
            pub.set_public_bases(bad)
    assert pub.lib.fthe_key_set_public_bases(pub._key, pub.dev.ctx, None, 0, None) == _lib.FTHE_ERR_ARG
    with pytest.raises(RuntimeError):                        # exponent bits not a multiple of 16 / too long
        pub.set_public_bases([2, 3], exp_bits=[100, 128])
    with pytest.raises(RuntimeError):
        pub.set_public_bases([2, 3], exp_bits=[16 * 200, 128])
    hs = server.public_bases(seed=1)
    pub.set_public_bases(hs)
    with pytest.raises(RuntimeError):                        # wrong injected exponent width
        pub.encrypt_u64(np.arange(2, dtype=np.uint64), r=np.zeros((2, 5), np.uint32), fixed_base_exact=True)
    c = pub.encrypt_u64(np.arange(4, dtype=np.uint64), seed=1, fixed_base_exact=True)
    assert np.array_equal(server.decrypt_u64(c), np.arange(4, dtype=np.uint64))


def test_public_exact_tables_shared_between_copies(dev):
    """Every party holds its own copy of the public key (party.h:181-185); copies with the same
    (device, n, bases) share one set of tables (13 GB at P-2048) instead of building their own."""
    import gc

    import torch
    from fedtree_amd.paillier import Paillier
    p, q = golden_key(load_golden("ref_gmp_L4096.json"))
    server = Paillier.from_primes(p, q, dev)
    hs = server.public_bases(seed=21)
    free0 = torch.cuda.mem_get_info(0)[0]
    a = server.public(bases=hs)
    dev.sync()
    free1 = torch.cuda.mem_get_info(0)[0]
    assert free0 - free1 > 12 << 30                           # the first copy builds the tables
    b = server.public(bases=hs)
    c2 = server.public(bases=hs)
    dev.sync()
    free2 = torch.cuda.mem_get_info(0)[0]
    assert free1 - free2 < 1 << 30                            # later copies share them
    m = np.arange(1000, dtype=np.uint64)
    y = [(3, 5, 7)] * 4
    ca = a.encrypt_u64(m[:4], r=y, fixed_base_exact=True)
    del a
    gc.collect()
    assert np.array_equal(b.encrypt_u64(m[:4], r=y, fixed_base_exact=True), ca)
    assert np.array_equal(server.decrypt_u64(c2.encrypt_u64(m, seed=4, fixed_base_exact=True)), m)
    other = server.public(bases=server.public_bases(seed=22))  # other bases: own tables
    dev.sync()
    assert torch.cuda.mem_get_info(0)[0] < free2 - (12 << 30)
    del b, c2, other
    gc.collect()
    dev.sync()
    assert torch.cuda.mem_get_info(0)[0] > free0 - (2 << 30)  # freed with the last copy
