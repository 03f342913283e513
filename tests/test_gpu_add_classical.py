"""The pairwise ciphertext add x*y mod n^2 (paillier.cpp:103) of a Paillier-2048 key runs as ONE
classical MSB-first product on the four-lane kernel (OP_MULWC, tools/msb_model.py) instead of a
Montgomery product plus the R^2 correction.  Exact against Python big-int products: random pairs
across the launch boundaries, the extremes 0, 1, n^2-1, values just below n^2, in-place (aliased)
output, and the host path.  Integer work: exact equality."""
import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pl():
    """the classical product on the four-lane kernel: FTHE_ADD_NO_ADDB=1 at key set-up keeps the pairwise add
    off the matrix-core Barrett kernel (tests/test_gpu_addb.py compares the two)"""
    import os
    from fedtree_amd.paillier import Device, Paillier
    os.environ["FTHE_ADD_NO_ADDB"] = "1"
    try:
        return Paillier(Device(0)).keygen(2048, seed=20261016)
    finally:
        del os.environ["FTHE_ADD_NO_ADDB"]


def _rows(vals, cw):
    return pyoracle.ints_to_words(vals, cw)


def test_classical_add_random_and_extremes(pl):
    import torch
    n2 = pl.n2
    cw = 2 * pl.n_words
    assert n2.bit_length() >= 4094
    rng = np.random.default_rng(5)
    cnt = 20000
    a = [int.from_bytes(rng.bytes(512), "little") % n2 for _ in range(cnt)]
    b = [int.from_bytes(rng.bytes(512), "little") % n2 for _ in range(cnt)]
    # extremes, incl. rows >= n^2 (not ciphertexts, but the reference still returns x y mod n^2)
    ext = [0, 1, 2, n2 - 1, n2 - 2, n2 // 2, (1 << 4094) - 1, n2 - (1 << 64), 1 << 4000, (1 << 27) - 1,
           n2, n2 + 12345, (1 << 4096) - 1]
    for i, x in enumerate(ext):
        for j, y in enumerate(ext):
            a[i * len(ext) + j], b[i * len(ext) + j] = x, y
    ad = torch.from_numpy(_rows(a, cw).view(np.int32)).cuda()
    bd = torch.from_numpy(_rows(b, cw).view(np.int32)).cuda()
    out = torch.empty_like(ad)
    pl.add_dev(ad, bd, out)
    pl.dev.sync()
    got = pyoracle.words_to_ints(out.cpu().numpy().view(np.uint32))
    bad = [i for i in range(cnt) if got[i] != a[i] * b[i] % n2]
    assert all(x < n2 for x in got)
    assert not bad, (len(bad), bad[:5])
    # in place: out aliases a
    pl.add_dev(ad, bd, ad)
    pl.dev.sync()
    assert pyoracle.words_to_ints(ad.cpu().numpy().view(np.uint32)) == got


def test_classical_add_host_path_and_golden(pl):
    from conftest import golden_key, load_golden
    from fedtree_amd.paillier import Paillier
    g = load_golden("ref_gmp_L4096.json")
    p, q = golden_key(g)
    gp = Paillier.from_primes(p, q, pl.dev)
    cw = 2 * gp.n_words
    cts = _rows([int(c["c"], 16) for c in g["cases"]], cw)
    out = gp.add_batch(cts[[x["i"] for x in g["adds"]]], cts[[x["j"] for x in g["adds"]]])
    assert [pyoracle.from_words(x) for x in out] == [int(x["c"], 16) for x in g["adds"]]
    # a chain of in-place host adds (sum of many ciphertexts) decrypts to the plaintext sum
    m = np.arange(1, 301, dtype=np.uint64) * 1000003
    c = gp.encrypt_u64(m, seed=3)
    acc = c[:1].copy()
    for i in range(1, len(c)):
        acc = gp.add_batch(acc, c[i:i + 1])
    assert int(gp.decrypt_u64(acc)[0]) == int(m.sum())


def test_classical_add_large_launch_matches_mont_rows(pl):
    """Across rowio chunk boundaries (4 x 393,216 rows per launch): add == from_mont(add_mont(to_mont))."""
    import torch
    cw = 2 * pl.n_words
    n = 393216 * 4 + 1000
    m = torch.randint(0, 2**62, (2 * n,), dtype=torch.int64, device="cuda")
    c = torch.empty((2 * n, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=9)
    o = torch.empty((n, cw), dtype=torch.int32, device="cuda")
    pl.add_dev(c[:n], c[n:], o)
    mr = torch.empty_like(c)
    pl.to_mont_dev(c, mr)
    om = torch.empty_like(o)
    pl.add_mont_dev(mr[:n], mr[n:], om)
    ref = torch.empty_like(o)
    pl.from_mont_dev(om, ref)
    pl.dev.sync()
    assert torch.equal(o, ref)
    low = torch.empty(n, dtype=torch.int64, device="cuda")
    pl.decrypt_u64_dev(o, low, short=True)
    pl.dev.sync()
    assert torch.equal(low, m[:n] + m[n:])
