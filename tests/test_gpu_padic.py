"""The P-adic exponentiation kernel (fthe_padic_k37) behind the key holder's CRT encrypt
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
    pa = Paillier(dev).keygen(request.param, seed=SEED)
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
    for cnt in (40000, 70000):                   # the split path (<= 65,536 lanes) and the chunked one
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
