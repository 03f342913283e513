"""Decrypt of arbitrary ciphertext rows -- not ones the engine produced -- against the reference's formula
m = L(c^lambda mod n^2) mu mod n (paillier.cpp:141-156, Paillier_GMP::decrypt paillier_gmp.cpp:75-85, whose
mpz_powm reduces c mod n^2 first): uniform rows over the whole 2 n_words-word range (so also c >= n^2,
unreduced), the edges 1, 2, n^2 - 1, n^2 + 1, 1 + n, 2^(64 n_words) - 1, on the three decrypt paths (the
four-lane s80 one for small batches, the split p/q one for one chunk, the chunked one beyond) and on every
exponentiation kernel of a key: the matrix-core P-adic kernel (default), the VALU P-adic kernel
(FTHE_NO_PADIC_MFMA) and the Montgomery programs (FTHE_NO_PADIC).  The short form is m mod p.  Integer work: exact equality."""
import math
import os

import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu

SEED = 20261016
PATH_COUNTS = (48, 40000, 397312)       # s80 quad path (<= 16,384), split p/q (one chunk), chunked
KERNEL_ENV = [{}, {"FTHE_NO_PADIC_MFMA": "1"}, {"FTHE_NO_PADIC": "1"}]


def _with_env(env, fn):
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


def _ref_decrypt(c, n, lam, mu):
    """paillier.cpp:153-156: L(u) = (u - 1) / n on u = c^lambda mod n^2 (c reduced by the powm)"""
    n2 = n * n
    return (pow(c % n2, lam, n2) - 1) // n * mu % n


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


@pytest.mark.parametrize("bits", [2048, 1024])
def test_decrypt_arbitrary_rows_vs_reference_formula(dev, bits):
    from fedtree_amd.paillier import Paillier
    base = Paillier(dev).keygen(bits, seed=SEED + bits)
    keys = [_with_env(env, lambda: Paillier.from_primes(base.p, base.q, dev)) for env in KERNEL_ENV]
    n, p = base.modulus, base.p
    lam, mu = base.lambda_, base.u
    cw = 2 * base.n_words
    top = (1 << (32 * cw)) - 1
    assert top >= n * n
    rng = np.random.default_rng(SEED + bits + 1)
    edges = [1, 2, n * n - 1, n * n + 1, 1 + n, top]
    cts = rng.integers(0, 2**32, (max(PATH_COUNTS), cw), dtype=np.uint32)
    cts[:len(edges)] = pyoracle.ints_to_words(edges, cw)
    sample = list(range(48)) + list(range(max(PATH_COUNTS) - 16, max(PATH_COUNTS)))
    rows = {i: pyoracle.from_words(cts[i]) for i in sample}
    for i in sample:
        assert math.gcd(rows[i], n) == 1, i                 # valid ciphertexts (fails with prob. ~2^-1000)
    want = {i: _ref_decrypt(rows[i], n, lam, mu) for i in sample}
    assert want[0] == want[2] == want[3] == 0 and want[4] == 1
    for env, k in zip(KERNEL_ENV, keys):
        full_by_count = {}
        for cnt in PATH_COUNTS:
            low, full = k.decrypt_u64(cts[:cnt], full=True)
            for i in sample:
                if i < cnt:
                    assert pyoracle.from_words(full[i]) == want[i], (env, cnt, i)
                    assert int(low[i]) == want[i] % 2**64, (env, cnt, i)
            full_by_count[cnt] = full
        for cnt in PATH_COUNTS[:-1]:                         # every path agrees on every row
            assert np.array_equal(full_by_count[cnt], full_by_count[PATH_COUNTS[-1]][:cnt]), (env, cnt)
        for cnt in (PATH_COUNTS[0], PATH_COUNTS[-1]):
            _, short = k.decrypt_u64(cts[:cnt], full=True, short=True)
            for i in sample:
                if i < cnt:
                    assert pyoracle.from_words(short[i]) == want[i] % p, (env, cnt, i)
