"""The n-adic four-lane kernels behind the public-key encrypt at Paillier-2048 (Party::encrypt_histogram,
party.h:118-142 -> paillier.cpp:122-139): the matrix-core Barrett form fthe_nadic_b76 (gen_nadicb.py,
the default for n of 2041..2048 bits), the Montgomery form fthe_nadic_m76 (n of 1033..2040 bits; FTHE_NADIC_MONT=1
selects it everywhere) and the classical fthe_nadic_q76 (FTHE_NADIC_CLASSICAL=1): the
same ciphertexts as each other and as the Montgomery s152 program they replace (FTHE_NO_NADIC=1), every one of
them equal to the C oracle's (1 + m n) r^n mod n^2 on the sizes tested, for injected r at the extremes and random
r, u64 and word plaintexts, across a chunk boundary, on a public-only key too, and their launches really run.
Integer work: exact equality.
"""
import ctypes
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
    pa = Paillier(dev).keygen(2048, seed=SEED)
    os.environ["FTHE_NO_NADIC"] = "1"
    try:
        pm = Paillier.from_primes(pa.p, pa.q, dev)
    finally:
        del os.environ["FTHE_NO_NADIC"]
    return dev, pa, pm


def _nadic_launches(dev, fn):
    lib = dev.lib
    lib.fthe_prof_enable(dev.ctx, 1)
    try:
        out = fn()
        vals = [ctypes.c_double() for _ in range(7)]
        assert lib.fthe_prof_read(dev.ctx, *[ctypes.byref(v) for v in vals]) == 0
        launches = 0.0
        for variant in (2076, 2176, 2276):      # the classical, Montgomery and matrix-core Barrett forms
            ms, nl = ctypes.c_double(), ctypes.c_double()
            assert lib.fthe_prof_variant(dev.ctx, variant, ctypes.byref(ms), ctypes.byref(nl)) == 0
            launches += nl.value
    finally:
        lib.fthe_prof_enable(dev.ctx, 0)
    return out, launches


def _variant_launches(dev, fn, variant):
    lib = dev.lib
    lib.fthe_prof_enable(dev.ctx, 1)
    try:
        out = fn()
        vals = [ctypes.c_double() for _ in range(7)]
        assert lib.fthe_prof_read(dev.ctx, *[ctypes.byref(v) for v in vals]) == 0
        ms, nl = ctypes.c_double(), ctypes.c_double()
        assert lib.fthe_prof_variant(dev.ctx, variant, ctypes.byref(ms), ctypes.byref(nl)) == 0
    finally:
        lib.fthe_prof_enable(dev.ctx, 0)
    return out, nl.value


def test_three_forms_same_ciphertexts(keys):
    """fthe_nadic_b76 (matrix-core Barrett, the default at 2048 bits; tools/nadicb_model.py), fthe_nadic_m76
    (FTHE_NADIC_MONT=1) and fthe_nadic_q76 (FTHE_NADIC_CLASSICAL=1): identical ciphertexts for injected r at the
    extremes (r >= n included) and random, plaintexts up to 2^64 - 1, across a chunk boundary; each form's
    launches are its own kernel; 64 of them against the formula (every one against the oracle below)."""
    dev, pa, pm = keys
    from fedtree_amd.paillier import Paillier
    forms = {}
    for env, variant in (("FTHE_NADIC_MONT", 2176), ("FTHE_NADIC_CLASSICAL", 2076)):
        os.environ[env] = "1"
        try:
            forms[variant] = Paillier.from_primes(pa.p, pa.q, dev)
        finally:
            del os.environ[env]
    rng = np.random.default_rng(SEED + 5)
    n = pa.modulus
    cnt = 98304 + 1000                          # one launch's 98,304 ciphertexts + a partial one
    rs = [1, 2, n - 1, n - 2, n + 5, 2**2048 - 1, 2 * n - 1 if 2 * n < 2**2048 else n + 7] + \
        [int.from_bytes(rng.bytes(256), "little") % n for _ in range(cnt - 7)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    m[:3] = [0, 2**64 - 1, 1]
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    cb, lb = _variant_launches(dev, lambda: pa.encrypt_u64(m, r=rw, public=True), 2276)
    assert lb >= 2
    for variant, pl in forms.items():
        cv, lv = _variant_launches(dev, lambda: pl.encrypt_u64(m, r=rw, public=True), variant)
        assert lv == lb, variant
        assert np.array_equal(cb, cv), variant
    got = pyoracle.words_to_ints(cb[:64])
    n2 = n * n
    for i in range(64):
        assert got[i] == (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2, i


def test_injected_r_same_ciphertexts_as_montgomery(keys):
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED)
    n = pa.modulus
    cnt = 3000
    rs = [1, 2, n - 1, n - 2, n + 5, 2**2048 - 1] + \
        [int.from_bytes(rng.bytes(256), "little") % (n - 1) + 1 for _ in range(cnt - 6)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    m[:4] = [0, 1, 2**64 - 2, 2**63]
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    ca, launches = _nadic_launches(dev, lambda: pa.encrypt_u64(m, r=rw, public=True))
    assert launches == 1
    cm = pm.encrypt_u64(m, r=rw, public=True)
    assert np.array_equal(ca, cm)
    n2 = n * n
    for i in (0, 1, 2, 3, 4, 5, 17, cnt - 1):              # the formula, paillier.cpp:134-137
        want = (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2
        assert pyoracle.from_words(ca[i]) == want, i
    assert np.array_equal(pa.decrypt_u64(ca), m)


def test_words_plaintexts_and_device_randomness(keys):
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED + 1)
    n = pa.modulus
    ms = [0, 1, n - 1, n - 2, 2**64, 2**2047] + [int.from_bytes(rng.bytes(256), "little") % n for _ in range(250)]
    rs = [int.from_bytes(rng.bytes(256), "little") % (n - 1) + 1 for _ in ms]
    ca = pa.encrypt_words(ms, r=rs, public=True)
    assert np.array_equal(ca, pm.encrypt_words(ms, r=rs, public=True))
    lo, full = pa.decrypt_u64(ca, full=True)
    got = [pyoracle.from_words(row) for row in full]
    assert got == ms
    m = rng.integers(0, 2**64 - 1, 5000, dtype=np.uint64)
    c = pa.encrypt_u64(m, seed=SEED, public=True)
    assert np.array_equal(pa.decrypt_u64(c), m)


def test_chunk_boundary_and_public_only_key(keys):
    from fedtree_amd.paillier import Paillier
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED + 2)
    n = pa.modulus
    cnt = 98304 + 2048                              # one s152 chunk (393,216 lanes / 4) and a part
    rs = [int.from_bytes(rng.bytes(256), "little") % (n - 1) + 1 for _ in range(cnt)]
    raw = pyoracle.ints_to_words(rs, pa.n_words)
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    pub = Paillier.from_public(n, dev)
    cp, launches = _nadic_launches(dev, lambda: pub.encrypt_u64(m, r=raw))
    assert launches == 2
    idx = np.r_[0:64, 98304 - 64:98304 + 64, cnt - 64:cnt]
    assert np.array_equal(cp[idx], pm.encrypt_u64(m[idx], r=raw[idx], public=True))
    # and against the reference's formula PowerMod(g, m, n^2) PowerMod(r, n, n^2) (paillier.cpp:134-137), not
    # only against the other kernel: the 256 sampled ciphertexts on both sides of the launch boundary
    n2 = n * n
    got = pyoracle.words_to_ints(cp[idx])
    for j, i in enumerate(idx):
        assert got[j] == (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2, int(i)
    assert np.array_equal(pa.decrypt_u64(cp), m)


def _prime_of_bits(rng, bits):
    from test_gpu_parity import _next_prime
    while True:
        x = int.from_bytes(rng.bytes((bits + 7) // 8), "little") & ((1 << bits) - 1)
        x |= (1 << (bits - 1)) | (1 << (bits - 2))
        p = _next_prime(x)
        if p.bit_length() == bits:
            return p


def _key_of_bits(rng, nbits):
    while True:
        p = _prime_of_bits(rng, nbits // 2)
        q = _prime_of_bits(rng, nbits - nbits // 2)
        n = p * q
        if n.bit_length() == nbits and p != q:
            return p, q, n


# which kernel a party's key of n bits runs: the matrix-core Barrett form for n of 2041..2048 bits, the Montgomery
# form for 1033..2040 (n^2 on the s152 slots; no quotient estimate, so no lower bound of its own; FTHE_NADIC_MONT=1
# takes 2041..2048 too), below 1033 bits n^2 takes the s74 slots and neither n-adic form (1032: the Montgomery s74
# program, 1009..1030: the P-adic one)
@pytest.mark.parametrize("nbits,variant,mont", [(2048, 2276, False), (2048, 2176, True), (2045, 2276, False),
                                                (2042, 2176, True), (2041, 2276, False), (2040, 2176, False),
                                                (2030, 2176, False), (1536, 2176, False), (1033, 2176, False),
                                                (1032, None, False)])
def test_modulus_range_edges(nbits, variant, mont):
    """every ciphertext of a party's public-key encrypt (600 per size, injected r incl. 1 and n - 1) equals the
    C oracle's full formula PowerMod(g, m, n^2) PowerMod(r, n, n^2) (paillier.cpp:134-137), on the kernel the
    size selects; all decrypt back"""
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    rng = np.random.default_rng(nbits)
    p, q, n = _key_of_bits(rng, nbits)
    if mont:
        os.environ["FTHE_NADIC_MONT"] = "1"
    try:
        pl = Paillier.from_public(n, dev)
    finally:
        os.environ.pop("FTHE_NADIC_MONT", None)
    cnt = 600
    rs = [1, n - 1] + [int.from_bytes(rng.bytes(260), "little") % (n - 1) + 1 for _ in range(cnt - 2)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    m[:2] = [0, 2**64 - 1]
    rw = pyoracle.ints_to_words(rs, pl.n_words)
    c, launches = _nadic_launches(dev, lambda: pl.encrypt_u64(m, r=rw))
    if variant is None:
        assert launches == 0
    else:
        _, lv = _variant_launches(dev, lambda: pl.encrypt_u64(m, r=rw), variant)
        assert launches == 1 and lv == 1
    if pl.n_words % 2 == 0:                                  # the C oracle (GMP, threads): p, q of n_words / 2
        o = pyoracle.COracle()
        ok = o.key(pyoracle.to_words(p, pl.n_words // 2), pyoracle.to_words(q, pl.n_words // 2))
        assert np.array_equal(c, ok.encrypt_batch(m, rw))
    else:
        n2 = n * n
        got = pyoracle.words_to_ints(c)
        for i in range(cnt):
            assert got[i] == pow(n + 1, int(m[i]), n2) * pow(rs[i], n, n2) % n2, i
    full = Paillier.from_primes(p, q, dev)
    assert np.array_equal(full.decrypt_u64(c), m)


@pytest.mark.parametrize("nbits,classical", [(2042, True), (2041, False)])
def test_classical_form_range(nbits, classical):
    """FTHE_NADIC_CLASSICAL=1: fthe_nadic_q76 from n of 2042 bits, the Montgomery s152 program one bit below"""
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    rng = np.random.default_rng(nbits + 7)
    while True:
        p = _prime_of_bits(rng, nbits // 2)
        q = _prime_of_bits(rng, nbits - nbits // 2)
        n = p * q
        if n.bit_length() == nbits:
            break
    os.environ["FTHE_NADIC_CLASSICAL"] = "1"
    try:
        pl = Paillier.from_public(n, dev)
    finally:
        del os.environ["FTHE_NADIC_CLASSICAL"]
    cnt = 300
    rs = [1, n - 1] + [int.from_bytes(rng.bytes(260), "little") % (n - 1) + 1 for _ in range(cnt - 2)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    rw = pyoracle.ints_to_words(rs, pl.n_words)
    c, launches = _variant_launches(dev, lambda: pl.encrypt_u64(m, r=rw), 2076)
    assert launches == (1 if classical else 0)
    n2 = n * n
    for i in (0, 1, 2, cnt - 1):
        assert pyoracle.from_words(c[i]) == (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2, i
