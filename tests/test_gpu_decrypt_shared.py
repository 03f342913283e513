"""fthe_decrypt_shared: the coalescing decrypt for concurrent callers of one key
(Server::decrypt_gh per node from OpenMP threads, server.h:69-78, FLtrainer.cpp:758-764).

Many threads on ONE Paillier object, mixed full / short / full-plaintext requests of
different sizes: every caller gets exactly its own plaintexts (the batches are merged
and scattered back), the same as fthe_decrypt; argument errors as the other decrypts.
"""
import threading

import numpy as np
import pytest

from conftest import golden_key, load_golden

pytestmark = pytest.mark.gpu


def _run_all(work, T, timeout=120):
    """Daemon threads; a queue that deadlocks fails the test instead of hanging pytest."""
    th = [threading.Thread(target=work, args=(i,), daemon=True) for i in range(T)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=timeout)
    assert not any(t.is_alive() for t in th), "shared queue deadlocked"


@pytest.fixture(scope="module")
def pl():
    from fedtree_amd.paillier import Device, Paillier
    g = load_golden("ref_gmp_L2048.json")
    p, q = golden_key(g)
    return Paillier.from_primes(p, q, Device(0))


def test_shared_matches_decrypt(pl):
    rng = np.random.default_rng(5)
    m = rng.integers(0, 2**64, 300, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=9)
    lo, full = pl.decrypt_u64_shared(c, full=True)
    assert np.array_equal(lo, m)
    assert np.array_equal(full, pl.decrypt_u64(c, full=True)[1])
    assert np.array_equal(pl.decrypt_u64_shared(c, short=True), m)
    assert len(pl.decrypt_u64_shared(c[:0])) == 0


def test_shared_many_threads(pl):
    rng = np.random.default_rng(6)
    T, R = 24, 3
    sizes = [2 if i % 3 else int(rng.integers(1, 40)) for i in range(T)]
    ms = [rng.integers(0, 2**64, s, dtype=np.uint64) for s in sizes]
    cs = [pl.encrypt_u64(m, seed=100 + i) for i, m in enumerate(ms)]
    # sums decrypt to plaintexts above 2^64: full plaintexts must come back per caller too
    sums = [pl.add_batch(c, c) for c in cs]
    bad = []
    go = threading.Barrier(T)

    def work(i):
        try:
            go.wait()
            for r in range(R):
                kind = (i + r) % 3
                if kind == 0:
                    ok = np.array_equal(pl.decrypt_u64_shared(cs[i]), ms[i])
                elif kind == 1:
                    ok = np.array_equal(pl.decrypt_u64_shared(cs[i], short=True), ms[i])
                else:
                    _, f = pl.decrypt_u64_shared(sums[i], full=True)
                    want = [2 * int(x) for x in ms[i]]
                    got = [int.from_bytes(w.astype("<u4").tobytes(), "little") for w in f]
                    ok = got == want
                if not ok:
                    bad.append((i, r))
        except Exception as e:
            bad.append((i, repr(e)))

    _run_all(work, T)
    assert not bad, bad


def test_encrypt_shared_many_threads(pl):
    """fthe_encrypt_shared: 24 threads on one key, CRT and public-key requests merged per flags;
    every ciphertext decrypts to its own caller's plaintexts."""
    from fedtree_amd.paillier import Paillier
    pub = Paillier.from_public(pl.modulus, pl.dev)
    rng = np.random.default_rng(8)
    T = 24
    ms = [rng.integers(0, 2**64, 2 if i % 4 else 17, dtype=np.uint64) for i in range(T)]
    outs, bad = [None] * T, []
    go = threading.Barrier(T)

    def work(i):
        try:
            go.wait()
            outs[i] = (pub if i % 5 == 0 else pl).encrypt_u64_shared(ms[i], public=(i % 3 == 0))
        except Exception as e:
            bad.append((i, repr(e)))

    _run_all(work, T)
    assert not bad, bad
    for i in range(T):
        assert np.array_equal(pl.decrypt_u64(outs[i]), ms[i]), i
    # fresh randomness: equal plaintexts give different ciphertexts
    a = pl.encrypt_u64_shared(np.zeros(4, dtype=np.uint64))
    assert len({bytes(r.tobytes()) for r in a}) == 4


def test_shared_public_key_rejected(pl):
    from fedtree_amd import _lib
    from fedtree_amd.paillier import Paillier
    pub = Paillier.from_public(pl.modulus, pl.dev)
    c = pl.encrypt_u64(np.array([1], dtype=np.uint64), seed=1)
    with pytest.raises(_lib.FtheError):
        pub.decrypt_u64_shared(c)


def test_shared_errors_do_not_block_other_callers(pl):
    """Requests that fail inside a merged batch of one key's queue (public-form exact
    fixed-base without published bases -> FTHE_ERR_UNSUPPORTED) return their error; the other
    callers of the same batches still get their ciphertexts and nobody hangs."""
    from fedtree_amd import _lib
    rng = np.random.default_rng(11)
    T = 16
    ms = [rng.integers(0, 2**64, 3, dtype=np.uint64) for _ in range(T)]
    status, outs = [None] * T, [None] * T
    go = threading.Barrier(T)

    def work(i):
        go.wait()
        try:
            if i % 4 == 1:        # bad flags for this key: public-form exact fixed-base, no bases published
                m = np.ascontiguousarray(ms[i])
                out = np.zeros((len(m), 2 * pl.n_words), np.uint32)
                status[i] = pl.lib.fthe_encrypt_shared(pl._key, m.ctypes.data, len(m), out.ctypes.data,
                                                       _lib.FTHE_ENC_FIXED_BASE_EXACT | _lib.FTHE_ENC_PUBLIC)
            else:
                outs[i] = pl.encrypt_u64_shared(ms[i])
                status[i] = 0
        except Exception as e:    # noqa: BLE001
            status[i] = repr(e)

    _run_all(work, T)
    for i in range(T):
        if i % 4 == 1:
            assert status[i] == _lib.FTHE_ERR_UNSUPPORTED, (i, status[i])
        else:
            assert status[i] == 0, (i, status[i])
            assert np.array_equal(pl.decrypt_u64(outs[i]), ms[i])


def test_add_mul_shared_many_threads_alias_safe(pl):
    """fthe_add_shared / fthe_scalar_mul_u64_shared (GHPair::operator+, +=, - of the USE_HIP build):
    24 threads on one key, each accumulating in place (out aliases a, the call shape of
    `paillier.add(g_enc, g_enc, rhs.g_enc)`, common.h:207-229) and subtracting with the all-ones
    scalar; the results equal the golden reference adds and the batch engine's."""
    gold = load_golden("ref_gmp_L2048.json")
    import pyoracle
    cw = 2 * pl.n_words
    cts = pyoracle.ints_to_words([int(c["c"], 16) for c in gold["cases"]], cw)
    adds = gold["adds"]
    T = 24
    res, bad = [None] * T, []

    def work(i):
        try:
            a = adds[i % len(adds)]
            acc = np.ascontiguousarray(cts[a["i"]][None].copy())
            pl.add_shared(acc, cts[a["j"]][None], out=acc)           # in place: acc = acc * c_j
            neg = pl.scalar_mul_shared(cts[a["j"]][None], 2**64 - 1)
            back = pl.add_shared(acc, neg)                             # acc * c_j^-1 (low 64 bits)
            res[i] = (acc.copy(), back)
        except Exception as e:  # noqa: BLE001
            bad.append((i, repr(e)))

    _run_all(work, T)
    assert not bad, bad
    for i in range(T):
        a = adds[i % len(adds)]
        assert pyoracle.from_words(res[i][0][0]) == int(a["c"], 16), i
        want_back = pl.add_batch(res[i][0], pl.scalar_mul(cts[a["j"]][None], 2**64 - 1))
        assert np.array_equal(res[i][1], want_back), i
        assert int(pl.decrypt_u64(res[i][1])[0]) == gold["cases"][a["i"]]["m"] % 2**64
