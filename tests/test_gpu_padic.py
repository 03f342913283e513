"""The VALU P-adic exponentiation kernel (fthe_padic_k37; the key holder's default is its
MFMA-Barrett variant fthe_padic_m37, tests/test_gpu_padic_mfma.py, so these keys set FTHE_NO_PADIC_MFMA) behind the key holder's CRT encrypt
and decrypt at Paillier-2048: the same ciphertexts and plaintexts as the Montgomery s74 programs it
replaces (FTHE_NO_PADIC=1 at key set-up restores those), for injected r at the extremes and random r,
and its launches really run (profiling counters of the variant).  Integer work: exact equality.
"""
import ctypes
import os

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu

SEED = 20261016


@pytest.fixture(scope="module", params=[2048, 1024])
def keys(request):
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    os.environ["FTHE_NO_PADIC_MFMA"] = "1"
    try:
        pa = Paillier(dev).keygen(request.param, seed=SEED)
    finally:
        del os.environ["FTHE_NO_PADIC_MFMA"]
    os.environ["FTHE_NO_PADIC"] = "1"
    try:
        pm = Paillier.from_primes(pa.p, pa.q, dev)
    finally:
        del os.environ["FTHE_NO_PADIC"]
    return dev, pa, pm


def _r_words(pl, rs):
    return pyoracle.ints_to_words(rs, pl.n_words)


def test_injected_r_same_ciphertexts_as_montgomery(keys, coracle):
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED)
    n = pa.modulus
    cnt = 3000
    rs = [1, 2, n - 1, n - 2] + [int.from_bytes(rng.bytes(256), "little") % (n - 1) + 1 for _ in range(cnt - 4)]
    m = rng.integers(0, 2**63, cnt, dtype=np.uint64)
    m[:4] = [0, 1, 2**63 - 1, 2**62]
    rw = _r_words(pa, rs)
    ca = pa.encrypt_u64(m, r=rw)
    cm = pm.encrypt_u64(m, r=rw)
    assert np.array_equal(ca, cm)
    pw = (max(pa.p.bit_length(), pa.q.bit_length()) + 31) // 32
    ok = coracle.key(pyoracle.to_words(pa.p, pw), pyoracle.to_words(pa.q, pw))
    idx = np.r_[0:8, cnt - 8:cnt]
    assert np.array_equal(ca[idx], ok.encrypt_batch(m[idx], rw[idx]))
    assert np.array_equal(pa.decrypt_u64(ca), m)
    assert np.array_equal(pm.decrypt_u64(ca), m)


def test_device_randomness_same_as_montgomery_and_decrypts(keys):
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED + 1)
    for cnt in (40000, 397312):                  # the split path (one chunk) and the chunked one
        m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
        ca = pa.encrypt_u64(m, seed=SEED + cnt)
        cm = pm.encrypt_u64(m, seed=SEED + cnt)
        assert np.array_equal(ca, cm), cnt
        assert np.array_equal(pa.decrypt_u64(ca), m)
        assert np.array_equal(pa.decrypt_u64(ca, short=True), m)
        la, fa = pa.decrypt_u64(ca, full=True)
        lm, fm = pm.decrypt_u64(ca, full=True)
        assert np.array_equal(la, lm) and np.array_equal(fa, fm)
        assert np.array_equal(fa[:, :2].copy().view(np.uint64).ravel(), m) and not fa[:, 2:].any()


def test_padic_launches_run(keys):
    dev, pa, pm = keys
    lib = dev.lib
    m = np.arange(70000, dtype=np.uint64)
    lib.fthe_prof_enable(dev.ctx, 1)
    pa.encrypt_u64(m, seed=3)
    x = ctypes.c_double()
    assert lib.fthe_prof_exec_macs(dev.ctx, ctypes.byref(x)) == 0
    vals = [ctypes.c_double() for _ in range(7)]
    assert lib.fthe_prof_read(dev.ctx, *[ctypes.byref(v) for v in vals]) == 0
    ms, nl = ctypes.c_double(), ctypes.c_double()
    big = pa.modulus.bit_length() > 1100
    assert lib.fthe_prof_variant(dev.ctx, 1037 if big else 1019, ctypes.byref(ms), ctypes.byref(nl)) == 0
    lib.fthe_prof_enable(dev.ctx, 0)
    assert nl.value == 2 and ms.value > 0                 # y_p^p and y_q^q, one launch each
    # v_mad per lane and prime: 1,024 squarings x 5,108 + ~180 products x 7,143 + LOADP / STOREP at
    # K = 37; 512 x 1,427 + ~100 x 1,959 + ... at K = 19
    per_lane = x.value / (2 * 70000)
    lo, hi = (6.0e6, 7.0e6) if big else (0.85e6, 1.05e6)
    assert lo < per_lane < hi, per_lane


def test_multi_chunk_injected_r_paillier1024(coracle):
    """Paillier-1024 with injected r across a chunk boundary: stage A (small-limb kernel) and the K = 19
    P-adic kernel share c->slots1 in separate regions, so the stage-A constants of the second chunk are
    intact; sampled ciphertexts on both sides of the boundary equal the C oracle's encrypt(m, r)."""
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(1024, seed=SEED + 7)
    rng = np.random.default_rng(SEED + 7)
    cnt = 393216 + 4096
    n = pl.modulus
    raw = rng.integers(0, 2**32, (cnt, pl.n_words + 2), dtype=np.uint32)
    rs = [int.from_bytes(row.tobytes(), "little") % (n - 1) + 1 for row in raw]     # uniform-ish in [1, n)
    rw = pyoracle.ints_to_words(rs, pl.n_words)
    m = rng.integers(0, 2**63, cnt, dtype=np.uint64)
    c = pl.encrypt_u64(m, r=rw)
    pw = (max(pl.p.bit_length(), pl.q.bit_length()) + 31) // 32
    ok = coracle.key(pyoracle.to_words(pl.p, pw), pyoracle.to_words(pl.q, pw))
    idx = np.r_[0:32, 393216 - 32:393216 + 32, cnt - 32:cnt]
    assert np.array_equal(c[idx], ok.encrypt_batch(m[idx], rw[idx]))
    assert np.array_equal(pl.decrypt_u64(c), m)


def _padic_launches(dev, fn):
    """fn's result and its P-adic launches per variant (profiling counters of the context)."""
    lib = dev.lib
    lib.fthe_prof_enable(dev.ctx, 1)
    try:
        out = fn()
        vals = [ctypes.c_double() for _ in range(7)]
        assert lib.fthe_prof_read(dev.ctx, *[ctypes.byref(v) for v in vals]) == 0
        launches = {}
        for v in (1037, 1019, 1137):
            ms, nl = ctypes.c_double(), ctypes.c_double()
            assert lib.fthe_prof_variant(dev.ctx, v, ctypes.byref(ms), ctypes.byref(nl)) == 0
            launches[v] = nl.value
    finally:
        lib.fthe_prof_enable(dev.ctx, 0)
    return out, launches


def _prime_of_bits(rng, bits):
    """A probable prime of exactly `bits` bits (test keys only)."""
    from test_gpu_parity import _next_prime
    while True:
        x = int.from_bytes(rng.bytes((bits + 7) // 8), "little") & ((1 << bits) - 1)
        x |= (1 << (bits - 1)) | (1 << (bits - 2))
        p = _next_prime(x)
        if p.bit_length() == bits:
            return p


# Prime sizes at the edges of the P-adic digit ranges (fthe.hip padic_digits): K = 37 takes P of
# 1009..1030 bits, K = 19 P of 505..514 bits (P of 515-516 bits puts the key's CRT halves on the s74
# shape, kernel_shape_for_bits); one bit outside, the key runs the Montgomery programs.
# (K = 37 keys run the MFMA-Barrett variant fthe_padic_m37 = 1137 by default: the edges hold for it too)
@pytest.mark.parametrize("pbits,qbits,variant", [
    (1009, 1030, 1137), (1030, 1030, 1137), (1008, 1030, None), (1030, 1031, None),
    (505, 514, 1019), (514, 514, 1019), (504, 514, None), (505, 515, None)])
def test_digit_range_edges_vs_c_oracle(coracle, pbits, qbits, variant):
    """Keys whose primes sit on (or one bit past) the P-adic kernel's range: the largest P has the
    tightest digit bounds ([0, 5P) digits, 50 P < b^K).  Injected r at the extremes and random r are
    bit-exact against the C oracle, decrypts (low and full) match it, device randomness and the exact
    fixed-base randomizer decrypt back, and the P-adic kernel runs exactly when both primes are in range."""
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    rng = np.random.default_rng(pbits * 7919 + qbits)
    p, q = _prime_of_bits(rng, pbits), _prime_of_bits(rng, qbits)
    pl = Paillier.from_primes(p, q, dev)
    n = pl.modulus
    hw = (qbits + 31) // 32
    ok = coracle.key(pyoracle.to_words(p, hw), pyoracle.to_words(q, hw))
    cnt = 20000                                    # above the small-batch (s80) decrypt threshold
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    m[:3] = [0, 1, 2**64 - 2]
    rs = [1, 2, n - 1, n - 2] + [int.from_bytes(rng.bytes(pl.n_words * 4), "little") % (n - 1) + 1
                                 for _ in range(cnt - 4)]
    r = pyoracle.ints_to_words(rs, pl.n_words)
    c, launches = _padic_launches(dev, lambda: pl.encrypt_u64(m, r=r))
    (low, full), dl = _padic_launches(dev, lambda: pl.decrypt_u64(c, full=True))
    cd, el = _padic_launches(dev, lambda: pl.encrypt_u64(m, seed=11))      # device randomness (direct y)
    for got in (launches, dl, el):                 # y_p^p and y_q^q, or c^(p-1) and c^(q-1)
        want = {1037: 0, 1019: 0, 1137: 0}
        if variant is not None:
            want[variant] = 2
        assert got == want, got
    assert np.array_equal(low, m)
    idx = np.r_[0:48, cnt - 16:cnt]
    r_or = np.zeros((len(idx), 2 * hw), np.uint32)
    r_or[:, :pl.n_words] = r[idx]
    want_or = ok.encrypt_batch(m[idx], r_or)
    assert not want_or[:, 2 * pl.n_words:].any()
    assert np.array_equal(c[idx], want_or[:, :2 * pl.n_words])
    assert np.array_equal(full[idx], ok.decrypt_batch(want_or)[:, :pl.n_words])
    ld, fd = pl.decrypt_u64(cd, full=True)
    assert np.array_equal(ld, m) and not fd[:, 2:].any()
    if pbits > 1000:                               # exact fixed-base tables (digit form when P-adic)
        assert np.array_equal(pl.decrypt_u64(pl.encrypt_u64(m, seed=12, fixed_base_exact=True)), m)


def test_public_encrypt_padic_paillier1024(keys):
    """Paillier-1024 public-key encrypt (n of 1009..1030 bits) runs on the K = 37 P-adic kernel with P = n:
    the same ciphertexts as the Montgomery s74 program for injected r at the extremes and random r, and
    decrypts back; at Paillier-2048 the n-adic kernel serves it (tests/test_gpu_nadic.py)."""
    dev, pa, pm = keys
    if pa.modulus.bit_length() > 1100:
        pytest.skip("Paillier-2048: n-adic kernel")
    rng = np.random.default_rng(SEED + 3)
    n = pa.modulus
    cnt = 3000
    rs = [1, 2, n - 1, n - 2, n + 7, 2**1024 - 1] + \
        [int.from_bytes(rng.bytes(128), "little") % (n - 1) + 1 for _ in range(cnt - 6)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    m[:3] = [0, 1, 2**64 - 2]
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    ca, launches = _padic_launches(dev, lambda: pa.encrypt_u64(m, r=rw, public=True))
    assert launches == {1037: 1, 1019: 0, 1137: 0}
    assert np.array_equal(ca, pm.encrypt_u64(m, r=rw, public=True))
    n2 = n * n
    for i in (0, 1, 2, 3, 4, 5, cnt - 1):             # paillier.cpp:134-137 with g = n + 1
        assert pyoracle.from_words(ca[i]) == (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2, i
    assert np.array_equal(pa.decrypt_u64(ca), m)
    ms = [0, n - 1, 2**64, 2**1000 + 3]
    assert np.array_equal(pa.encrypt_words(ms, r=rs[:4], public=True), pm.encrypt_words(ms, r=rs[:4], public=True))
    c = pa.encrypt_u64(m, seed=SEED, public=True)
    assert np.array_equal(pa.decrypt_u64(c), m)
