"""The n-adic four-lane kernel (fthe_nadic_q76, gen_nadic.py) behind the public-key encrypt
at Paillier-2048 (Party::encrypt_histogram, party.h:118-142 -> paillier.cpp:122-139): the same
ciphertexts as the Montgomery s152 program it replaces (FTHE_NO_NADIC=1 at key set-up restores that),
for injected r at the extremes and random r, u64 and word plaintexts, across a chunk boundary, on a
public-only key too, and its launches really run.  Integer work: exact equality.
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
        for variant in (2076, 2176):            # the classical and the Montgomery form (default)
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


def test_montgomery_form_same_ciphertexts_as_classical(keys):
    """fthe_nadic_m76 (Montgomery n-adic, default; tools/nadic_mont_model.py) against fthe_nadic_q76
    (FTHE_NADIC_CLASSICAL=1) and the oracle's formula: injected r at the extremes (r >= n included) and
    random, plaintexts up to 2^64 - 1, across a chunk boundary; each form's launches are its own kernel."""
    dev, pa, pm = keys
    from fedtree_amd.paillier import Paillier
    os.environ["FTHE_NADIC_CLASSICAL"] = "1"
    try:
        pc = Paillier.from_primes(pa.p, pa.q, dev)
    finally:
        del os.environ["FTHE_NADIC_CLASSICAL"]
    rng = np.random.default_rng(SEED + 5)
    n = pa.modulus
    cnt = 98304 + 1000                          # one launch's 98,304 ciphertexts + a partial one
    rs = [1, 2, n - 1, n - 2, n + 5, 2**2048 - 1, 2 * n - 1 if 2 * n < 2**2048 else n + 7] + \
        [int.from_bytes(rng.bytes(256), "little") % n for _ in range(cnt - 7)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    m[:3] = [0, 2**64 - 1, 1]
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    ca, la = _variant_launches(dev, lambda: pa.encrypt_u64(m, r=rw, public=True), 2176)
    cc, lc = _variant_launches(dev, lambda: pc.encrypt_u64(m, r=rw, public=True), 2076)
    assert la == lc and la >= 2
    assert np.array_equal(ca, cc)
    got = pyoracle.words_to_ints(ca[:64])
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
    assert np.array_equal(pa.decrypt_u64(cp), m)


def _prime_of_bits(rng, bits):
    from test_gpu_parity import _next_prime
    while True:
        x = int.from_bytes(rng.bytes((bits + 7) // 8), "little") & ((1 << bits) - 1)
        x |= (1 << (bits - 1)) | (1 << (bits - 2))
        p = _next_prime(x)
        if p.bit_length() == bits:
            return p


# the Montgomery form (default) runs every n of 1033..2048 bits (n^2 on the s152 slots); the classical form
# needs n >= 2^(27*76 - 10) for its quotient estimate (n of 2042..2048), below that FTHE_NADIC_CLASSICAL=1
# keys fall back to the Montgomery s152 program (tests/test_gpu_nadic.py::test_classical_form_range)
@pytest.mark.parametrize("nbits,nadic", [(2042, True), (2045, True), (2041, True), (2030, True), (1536, True)])
def test_modulus_range_edges(nbits, nadic):
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    rng = np.random.default_rng(nbits)
    while True:
        p = _prime_of_bits(rng, nbits // 2)
        q = _prime_of_bits(rng, nbits - nbits // 2)
        n = p * q
        if n.bit_length() == nbits:
            break
    pl = Paillier.from_public(n, dev)
    cnt = 600
    rs = [1, n - 1] + [int.from_bytes(rng.bytes(260), "little") % (n - 1) + 1 for _ in range(cnt - 2)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    rw = pyoracle.ints_to_words(rs, pl.n_words)
    c, launches = _nadic_launches(dev, lambda: pl.encrypt_u64(m, r=rw))
    assert launches == (1 if nadic else 0)
    n2 = n * n
    for i in (0, 1, 2, cnt - 1):                         # paillier.cpp:134-137 with g = n + 1
        assert pyoracle.from_words(c[i]) == (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2, i
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
