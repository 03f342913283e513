"""Device-resident homomorphic histogram (fthe_histogram_dev) and the device-CSR
segmented product (fthe_reduce_segments_csr_dev), through the C ABI.

* bit-exact against the oracle's restatement of the reference scatter loop
  (hist_tree_builder.cpp:574-595; pyoracle.histogram) for the root (all
  instances) and for a node's instance subset (:640-664), at P-1024 (one-lane
  n^2 kernel) and P-2048 (four-lane row-I/O kernel), with missing values;
* the device-CSR segmented product equals the host-CSR one (ragged segments:
  empty, singletons, a multi-pass segment);
* full size (200,000 instances x 8 features x 256 bins, P-2048): every bin
  decrypts to the sum of its members' encoded gradients.
Integer work: every comparison is exact.
"""
import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


def _pl(dev, coracle, nbits, seed):
    from fedtree_amd.paillier import Paillier
    rng = np.random.default_rng(seed)
    hw = nbits // 64
    pw, qw = [coracle.next_prime(rng.integers(0, 2**32, hw, dtype=np.uint64).astype(np.uint32)) for _ in range(2)]
    return Paillier.from_primes(pyoracle.from_words(pw), pyoracle.from_words(qw), dev)


def _bins(rng, n_inst, n_col, max_bin):
    per = rng.integers(1, max_bin + 1, n_col)
    cut = np.concatenate([[0], np.cumsum(per)]).astype(np.int32)
    bins = np.stack([np.where(rng.random(n_inst) < 0.05, max_bin, rng.integers(0, per[f], n_inst))
                     for f in range(n_col)], 1).astype(np.uint8)
    return cut, bins


@pytest.mark.parametrize("nbits", [1024, 2048])
def test_histogram_dev_vs_reference_loop(dev, coracle, nbits):
    import torch
    pl = _pl(dev, coracle, nbits, 71 + nbits)
    key = pyoracle.keygen_from_primes(pl.p, pl.q)
    rng = np.random.default_rng(nbits)
    n_inst, n_col, max_bin = 600, 5, 32
    cut, bins = _bins(rng, n_inst, n_col, max_bin)
    m = rng.integers(0, 2**40, 2 * n_inst, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=3)                                   # g plane then h plane
    cw = 2 * pl.n_words
    xd = torch.from_numpy(c.view(np.int32)).cuda()
    bd = torch.from_numpy(bins).cuda()
    n_bins = int(cut[-1])
    out = torch.empty((2 * n_bins, cw), dtype=torch.int32, device="cuda")
    cts = pyoracle.words_to_ints(c)
    for inst in (None, np.sort(rng.choice(n_inst, 217, replace=False)).astype(np.int32)):
        idev = None if inst is None else torch.from_numpy(inst).cuda()
        pl.histogram_dev(xd, n_inst, 2, bd, cut, max_bin, out, inst=idev)
        pl.dev.sync()
        got = pyoracle.words_to_ints(out.cpu().numpy().view(np.uint32))
        rows = np.arange(n_inst) if inst is None else inst
        for p in range(2):
            want = pyoracle.histogram(key, [cts[p * n_inst + i] for i in rows], bins[rows].reshape(-1),
                                      [int(x) for x in cut], max_bin)
            assert got[p * n_bins:(p + 1) * n_bins] == [1 if w is None else w for w in want], (inst is None, p)


@pytest.mark.parametrize("nbits", [1024, 2048])
def test_reduce_segments_csr_dev_equals_host_csr(dev, coracle, nbits):
    import torch
    pl = _pl(dev, coracle, nbits, 81 + nbits)
    rng = np.random.default_rng(nbits + 9)
    cnt = 1500
    c = pl.encrypt_u64(rng.integers(0, 2**50, cnt, dtype=np.uint64), seed=5)
    lens = np.concatenate([[0, 1, 0, 700, 9, 8, 17, 64, 65, 1, 0], rng.integers(0, 20, 40)])
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    idx = rng.integers(0, cnt, seg[-1]).astype(np.int64)
    want = pl.reduce_segments(c, seg, idx)
    xd = torch.from_numpy(c.view(np.int32)).cuda()
    out = torch.empty((len(lens), c.shape[1]), dtype=torch.int32, device="cuda")
    pl.reduce_segments_csr_dev(xd, torch.from_numpy(seg).cuda(), out, idx=torch.from_numpy(idx).cuda())
    pl.dev.sync()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    seg_c = np.array([0, 3, 3, 600, cnt], np.int64)                  # identity members
    out2 = torch.empty((4, c.shape[1]), dtype=torch.int32, device="cuda")
    pl.reduce_segments_csr_dev(xd, torch.from_numpy(seg_c).cuda(), out2)
    pl.dev.sync()
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), pl.reduce_segments(c, seg_c))


def test_histogram_dev_full_size_p2048(dev, coracle):
    import torch
    pl = _pl(dev, coracle, 2048, 91)
    rng = np.random.default_rng(11)
    n_inst, n_col = 200_000, 8
    cut = (np.arange(n_col + 1) * 255).astype(np.int32)             # 255 bins per feature, 255 = missing
    bins = rng.integers(0, 256, (n_inst, n_col)).astype(np.uint8)
    bins[rng.random((n_inst, n_col)) < 0.3] = 0                       # a heavy bin per feature
    m = rng.integers(0, 2**40, 2 * n_inst, dtype=np.uint64)
    md = torch.from_numpy(m.view(np.int64)).cuda()
    cw = 2 * pl.n_words
    xd = torch.empty((2 * n_inst, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(md, xd, seed=13)
    bd = torch.from_numpy(bins).cuda()
    n_bins = int(cut[-1])
    out = torch.empty((2 * n_bins, cw), dtype=torch.int32, device="cuda")
    pl.histogram_dev(xd, n_inst, 2, bd, cut, 255, out)
    pl.dev.sync()
    low = pl.decrypt_u64(out.cpu().numpy().view(np.uint32))
    want = np.zeros(2 * n_bins, np.uint64)
    for f in range(n_col):
        b = bins[:, f].astype(np.int64)
        ok = b != 255
        for p in range(2):
            np.add.at(want, p * n_bins + cut[f] + b[ok], m[p * n_inst:(p + 1) * n_inst][ok])
    assert np.array_equal(low, want)


@pytest.mark.parametrize("nbits", [1024, 2048])
def test_histogram_zero_first_matches_reference_sequence(dev, coracle, nbits):
    """Q10: the reference's bin is Enc(0) * prod(members) -- its accumulator is an unencrypted zero and
    the first + encrypts it (common.h:156-160).  With one Enc(0) for every bin (the GMP build's encrypt
    draws the same r on every call) the engine reproduces pyoracle.histogram(...,
    enc_zero=E0) bit-exactly; with a distinct Enc(0) per bin (fresh randomness, the NTL build) each
    populated bin is its own E0_b * prod; empty bins stay the unencrypted zero (the integer 1)."""
    import torch
    pl = _pl(dev, coracle, nbits, 171 + nbits)
    key = pyoracle.keygen_from_primes(pl.p, pl.q)
    rng = np.random.default_rng(nbits + 3)
    n_inst, n_col, max_bin = 300, 4, 24
    cut, bins = _bins(rng, n_inst, n_col, max_bin)
    for f, per in enumerate(np.diff(cut)):                         # the last bin of each feature stays empty
        if per >= 2:
            bins[bins[:, f] == per - 1, f] = 0
    m = rng.integers(0, 2**40, 2 * n_inst, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=23)
    cw = 2 * pl.n_words
    n_bins = int(cut[-1])
    xd = torch.from_numpy(c.view(np.int32)).cuda()
    bd = torch.from_numpy(bins).cuda()
    out = torch.empty((2 * n_bins, cw), dtype=torch.int32, device="cuda")
    cts = pyoracle.words_to_ints(c)
    r0 = int.from_bytes(rng.bytes(pl.n_words * 4), "little") % (pl.modulus - 1) + 1
    e0 = pyoracle.encrypt(key, 0, r0)
    ez_shared = torch.from_numpy(np.tile(pyoracle.to_words(e0, cw), (2 * n_bins, 1)).view(np.int32)).cuda()
    ez_fresh_h = pl.encrypt_u64(np.zeros(2 * n_bins, np.uint64), seed=29)
    ez_fresh = torch.from_numpy(ez_fresh_h.view(np.int32)).cuda()
    fresh = pyoracle.words_to_ints(ez_fresh_h)
    for inst in (None, np.sort(rng.choice(n_inst, 111, replace=False)).astype(np.int32)):
        idev = None if inst is None else torch.from_numpy(inst).cuda()
        rows = np.arange(n_inst) if inst is None else inst
        pl.histogram_dev(xd, n_inst, 2, bd, cut, max_bin, out, inst=idev, enc_zero=ez_shared)
        pl.dev.sync()
        got = pyoracle.words_to_ints(out.cpu().numpy().view(np.uint32))
        plain = []
        for p in range(2):
            want = pyoracle.histogram(key, [cts[p * n_inst + i] for i in rows], bins[rows].reshape(-1),
                                      [int(x) for x in cut], max_bin, enc_zero=e0)
            assert got[p * n_bins:(p + 1) * n_bins] == [1 if w is None else w for w in want], (inst is None, p)
            plain += pyoracle.histogram(key, [cts[p * n_inst + i] for i in rows], bins[rows].reshape(-1),
                                        [int(x) for x in cut], max_bin)
        assert any(w is None for w in plain)                        # some bins stay empty
        pl.histogram_dev(xd, n_inst, 2, bd, cut, max_bin, out, inst=idev, enc_zero=ez_fresh)
        pl.dev.sync()
        got = pyoracle.words_to_ints(out.cpu().numpy().view(np.uint32))
        assert got == [1 if w is None else pyoracle.add(key, fresh[b], w) for b, w in enumerate(plain)]
    # the host-CSR segmented product with the same semantics, ragged segments incl. empty ones
    lens = np.array([0, 1, 0, 19, 8, 9, 0, 3])
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    idx = rng.integers(0, len(c), seg[-1]).astype(np.int64)
    ez = torch.from_numpy(ez_fresh_h[:len(lens)].view(np.int32)).cuda()
    o2 = torch.empty((len(lens), cw), dtype=torch.int32, device="cuda")
    pl.reduce_segments_zero_first_dev(xd, seg, ez, o2, idx=idx)
    pl.dev.sync()
    plain = pl.reduce_segments(c, seg, idx)
    want = [1 if lens[s] == 0 else pyoracle.add(key, fresh[s], pyoracle.from_words(plain[s])) for s in range(len(lens))]
    assert pyoracle.words_to_ints(o2.cpu().numpy().view(np.uint32)) == want
