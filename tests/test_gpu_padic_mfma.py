"""The matrix-core Barrett P-adic kernel (fthe_padic_m37, the key holder's default at Paillier-2048)
through the engine: the same Paillier-2048 ciphertexts and plaintexts as the Montgomery s74 programs
(FTHE_NO_PADIC=1) for injected r at the extremes and random r, device randomness that decrypts, the
Paillier-1024 public form with P = n, and its launches really run on the variant (profiling counters).
Integer work: exact equality."""
import ctypes
import os

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu

SEED = 20261017


def _key_with(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def keys():
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pa = _key_with({}, lambda: Paillier(dev).keygen(2048, seed=SEED))
    pm = _key_with({"FTHE_NO_PADIC": "1"}, lambda: Paillier.from_primes(pa.p, pa.q, dev))
    return dev, pa, pm


def test_mfma_injected_r_same_ciphertexts_as_montgomery(keys, coracle):
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED)
    n = pa.modulus
    cnt = 3000
    rs = [1, 2, n - 1, n - 2] + [int.from_bytes(rng.bytes(256), "little") % (n - 1) + 1 for _ in range(cnt - 4)]
    m = rng.integers(0, 2**63, cnt, dtype=np.uint64)
    m[:4] = [0, 1, 2**63 - 1, 2**62]
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    ca = pa.encrypt_u64(m, r=rw)
    assert np.array_equal(ca, pm.encrypt_u64(m, r=rw))
    pw = (max(pa.p.bit_length(), pa.q.bit_length()) + 31) // 32
    ok = coracle.key(pyoracle.to_words(pa.p, pw), pyoracle.to_words(pa.q, pw))
    idx = np.r_[0:8, cnt - 8:cnt]
    assert np.array_equal(ca[idx], ok.encrypt_batch(m[idx], rw[idx]))
    assert np.array_equal(pa.decrypt_u64(ca), m)                   # c^(P-1) mod P^2 on the MFMA kernel


def test_mfma_device_randomness_decrypts(keys):
    dev, pa, pm = keys
    rng = np.random.default_rng(SEED + 1)
    for cnt in (40000, 397312):                  # the split path (one chunk) and the chunked one
        m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
        c = pa.encrypt_u64(m, seed=SEED + cnt)
        assert np.array_equal(pm.decrypt_u64(c), m)
        assert np.array_equal(pa.decrypt_u64(c), m)


def test_mfma_launches_run(keys):
    dev, pa, pm = keys
    lib = dev.lib
    lib.fthe_prof_enable(dev.ctx, 1)
    pa.encrypt_u64(np.arange(70000, dtype=np.uint64), seed=3)
    vals = [ctypes.c_double() for _ in range(7)]
    assert lib.fthe_prof_read(dev.ctx, *[ctypes.byref(v) for v in vals]) == 0
    got = {}
    for S in (1037, 1137):
        ms, nl = ctypes.c_double(), ctypes.c_double()
        assert lib.fthe_prof_variant(dev.ctx, S, ctypes.byref(ms), ctypes.byref(nl)) == 0
        got[S] = nl.value
    lib.fthe_prof_enable(dev.ctx, 0)
    assert got == {1037: 0.0, 1137: 2.0}                     # y_p^p and y_q^q on fthe_padic_m37


def test_mfma_public_paillier1024_p_equals_n():
    """Paillier-1024 public-key encrypt runs r^n mod n^2 on the K = 37 P-adic kernel with P = n: on the MFMA
    kernel too, with the same ciphertexts as the Montgomery program and the formula of paillier.cpp:134-137"""
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pa = _key_with({}, lambda: Paillier(dev).keygen(1024, seed=SEED + 2))
    pm = _key_with({"FTHE_NO_PADIC": "1"}, lambda: Paillier.from_primes(pa.p, pa.q, dev))
    rng = np.random.default_rng(SEED + 3)
    n = pa.modulus
    rs = [1, 2, n - 1, 2**1024 - 1] + [int.from_bytes(rng.bytes(128), "little") % (n - 1) + 1 for _ in range(996)]
    m = rng.integers(0, 2**63, 1000, dtype=np.uint64)
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    c = pa.encrypt_u64(m, r=rw, public=True)
    assert np.array_equal(c, pm.encrypt_u64(m, r=rw, public=True))
    n2 = n * n
    for i in (0, 1, 2, 3, 999):
        assert pyoracle.from_words(c[i]) == (1 + int(m[i]) * n) * pow(rs[i], n, n2) % n2, i
    assert np.array_equal(pa.decrypt_u64(c), m)


def test_mfma_million_ciphertexts_identical_to_valu_kernel(keys):
    """2^20 device-randomness encrypts (same seed, so the same y_p, y_q per ciphertext) on the MFMA kernel and
    on fthe_padic_k37 with the same primes: every ciphertext bit-identical (the intermediate digits differ --
    the matrix-core quotient may be one lower -- the canonical results may not), and the decrypts agree."""
    from fedtree_amd.paillier import Paillier
    dev, pa, pm = keys
    pk = _key_with({"FTHE_NO_PADIC_MFMA": "1"}, lambda: Paillier.from_primes(pa.p, pa.q, dev))
    rng = np.random.default_rng(SEED + 9)
    m = rng.integers(0, 2**64 - 1, 1 << 20, dtype=np.uint64)
    ca = pa.encrypt_u64(m, seed=SEED + 11)
    ck = pk.encrypt_u64(m, seed=SEED + 11)
    assert np.array_equal(ca, ck)
    assert np.array_equal(pa.decrypt_u64(ck), m)


@pytest.mark.parametrize("pq", [
    (int("80" * 128, 16), int("7f" * 128, 16) | (1 << 1023)),           # balanced-digit carries in every byte
    ((1 << 1030) - (1 << 600), (1 << 1008) + (1 << 500)),              # the largest and smallest P of the range
], ids=["x80-x7f", "max-min"])
def test_mfma_structured_primes_vs_valu_kernel_and_oracle(pq, coracle):
    """Primes next to byte-structured values (0x80 / 0x7f runs: the balanced-digit tiles carry everywhere) and
    at both ends of the 1009..1030-bit range: injected r bit-exact against the C oracle and identical to
    fthe_padic_k37, device randomness identical to it, decrypts back."""
    from test_gpu_parity import _next_prime
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    p, q = (_next_prime(x) for x in pq)
    pa = _key_with({}, lambda: Paillier.from_primes(p, q, dev))
    pk = _key_with({"FTHE_NO_PADIC_MFMA": "1"}, lambda: Paillier.from_primes(p, q, dev))
    n = pa.modulus
    rng = np.random.default_rng(SEED + 13)
    cnt = 20000
    rs = [1, 2, n - 1, n - 2] + [int.from_bytes(rng.bytes(pa.n_words * 4), "little") % (n - 1) + 1
                                 for _ in range(cnt - 4)]
    m = rng.integers(0, 2**64 - 1, cnt, dtype=np.uint64)
    rw = pyoracle.ints_to_words(rs, pa.n_words)
    ca = pa.encrypt_u64(m, r=rw)
    assert np.array_equal(ca, pk.encrypt_u64(m, r=rw))
    hw = (max(p.bit_length(), q.bit_length()) + 31) // 32
    ok = coracle.key(pyoracle.to_words(p, hw), pyoracle.to_words(q, hw))
    idx = np.r_[0:16, cnt - 16:cnt]
    r_or = np.zeros((len(idx), 2 * hw), np.uint32)
    r_or[:, :pa.n_words] = rw[idx]
    want = ok.encrypt_batch(m[idx], r_or)
    assert np.array_equal(ca[idx], want[:, :2 * pa.n_words])
    cd = pa.encrypt_u64(m, seed=SEED + 17)
    assert np.array_equal(cd, pk.encrypt_u64(m, seed=SEED + 17))
    assert np.array_equal(pa.decrypt_u64(cd), m)
    assert np.array_equal(pa.decrypt_u64(ca), m)
