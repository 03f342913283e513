"""Error behaviour of the C ABI on a live context (the reference aborts through
CHECK / exit(1), common.h:47-52, paillier_gpu.cu:13-16; the engine returns status
codes and leaves the context usable).  Each failing call is followed by a good one."""
import ctypes

import numpy as np
import pytest

from fedtree_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(1024, seed=3)
    pub = Paillier.from_public(pl.modulus, dev)
    return dev, pl, pub


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def test_bad_arguments_return_codes(env):
    dev, pl, pub = env
    lib, ctx, key = dev.lib, dev.ctx, pl._key
    cw = 2 * pl.n_words
    m = np.arange(8, dtype=np.uint64)
    c = np.zeros((8, cw), np.uint32)
    r = np.ones((8, pl.n_words + 1), np.uint32)
    E = _lib
    # r wider than n
    assert lib.fthe_encrypt_u64(key, ctx, _p(m), 8, _p(r), pl.n_words + 1, 0, _p(c), 0) == E.FTHE_ERR_ARG
    # null output with a count
    assert lib.fthe_encrypt_u64(key, ctx, _p(m), 8, None, 0, 0, None, 0) == E.FTHE_ERR_ARG
    # private operations on a public-only key
    low = np.zeros(8, np.uint64)
    assert lib.fthe_decrypt(pub._key, ctx, _p(c), 8, _p(low), None) == E.FTHE_ERR_NOPRIV
    assert lib.fthe_encrypt_u64(pub._key, ctx, _p(m), 8, None, 0, 0, _p(c), E.FTHE_ENC_FIXED_BASE_EXACT) \
        == E.FTHE_ERR_NOPRIV
    assert lib.fthe_key_fixed_base_exact(pub._key, ctx, 1) == E.FTHE_ERR_NOPRIV
    # k-way with k out of range
    x = np.zeros((65, 1, cw), np.uint32)
    assert lib.fthe_reduce_kway(key, ctx, _p(x), 65, 1, _p(c)) == E.FTHE_ERR_ARG
    assert lib.fthe_reduce_kway(key, ctx, _p(x), 0, 1, _p(c)) == E.FTHE_ERR_ARG
    # invalid key material
    out = ctypes.c_void_p()
    w = np.array([7, 0], np.uint32)
    assert lib.fthe_key_from_primes(ctx, _p(w), _p(w), 2, ctypes.byref(out)) == E.FTHE_ERR_KEY      # p == q
    ev = np.array([8, 0], np.uint32)
    assert lib.fthe_key_from_primes(ctx, _p(ev), _p(w), 2, ctypes.byref(out)) == E.FTHE_ERR_KEY     # even p
    assert lib.fthe_key_generate(ctx, 1023, 0, ctypes.byref(out)) == E.FTHE_ERR_ARG                 # odd bits
    assert lib.fthe_strerror(E.FTHE_ERR_NOPRIV)
    # the context still works
    got = pl.encrypt_u64(m, seed=1)
    assert np.array_equal(pl.decrypt_u64(got), m)
    assert np.array_equal(pl.decrypt_u64(pub.encrypt_u64(m, seed=2)), m)


def test_zero_counts_are_no_ops(env):
    dev, pl, pub = env
    cw = 2 * pl.n_words
    e = np.zeros((0, cw), np.uint32)
    assert pl.encrypt_u64(np.zeros(0, np.uint64)).shape == (0, cw)
    assert pl.decrypt_u64(e).shape == (0,)
    assert pl.add_batch(e, e).shape == (0, cw)
    assert pl.encrypt_u64(np.zeros(0, np.uint64), fixed_base_exact=True).shape == (0, cw)
    m = np.arange(3, dtype=np.uint64)
    assert np.array_equal(pl.decrypt_u64(pl.encrypt_u64(m, seed=4)), m)
