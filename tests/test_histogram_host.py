"""Host logic of the histogram scatter (hist_tree_builder.cpp:574-595): the CSR
segments built by fedtree_amd.paillier.histogram_segments, folded by the
oracle's segment product, equal the oracle's restatement of the reference loop.
Tiny keys, pure Python: no GPU."""
import numpy as np
import pytest

import pyoracle
from fedtree_amd.paillier import histogram_segments


def _key():
    return pyoracle.keygen_from_primes(1000003, 1000033)


@pytest.mark.parametrize("n_inst,n_col,max_bin,seed", [(0, 3, 8, 0), (1, 1, 4, 1), (57, 4, 6, 2), (300, 7, 16, 3)])
def test_segments_match_reference_loop(n_inst, n_col, max_bin, seed):
    rng = np.random.default_rng(seed)
    key = _key()
    nbins_per = rng.integers(1, max_bin + 1, n_col)
    cut = np.concatenate([[0], np.cumsum(nbins_per)]).astype(np.int64)
    # bin ids in [0, nbins_per[fid]) or max_bin (missing)
    bins = np.zeros((n_inst, n_col), np.uint8)
    for f in range(n_col):
        b = rng.integers(0, nbins_per[f], n_inst)
        b[rng.random(n_inst) < 0.1] = max_bin
        bins[:, f] = b
    cts = [pyoracle.encrypt(key, int(m), int(r)) for m, r in
           zip(rng.integers(0, 2**40, n_inst), rng.integers(1, 2**30, n_inst))]
    want = pyoracle.histogram(key, cts, bins.reshape(-1), list(cut), max_bin)
    seg_ptr, idx = histogram_segments(bins.reshape(-1), cut, max_bin)
    assert len(seg_ptr) == cut[-1] + 1
    got = pyoracle.segment_product(key, cts, list(seg_ptr), list(idx))
    for b in range(cut[-1]):
        if want[b] is None:
            assert seg_ptr[b + 1] == seg_ptr[b] and got[b] == 1
        else:
            assert got[b] == want[b]
    # members in instance order within each bin
    for b in range(cut[-1]):
        s = idx[seg_ptr[b]:seg_ptr[b + 1]]
        assert np.all(np.diff(s) > 0)


def test_enc_zero_promotion_preserves_plaintext():
    """The reference's first add promotes the zero accumulator with Enc(0)
    (common.h:156-160): same plaintext as the plain product."""
    key = _key()
    cts = [pyoracle.encrypt(key, m, 17 + m) for m in (5, 7, 11)]
    bins = np.array([0, 0, 1], np.uint8)
    ez = pyoracle.encrypt(key, 0, 12345)
    a = pyoracle.histogram(key, cts, bins, [0, 2], 2, enc_zero=ez)
    b = pyoracle.histogram(key, cts, bins, [0, 2], 2)
    assert [pyoracle.decrypt(key, x) for x in a] == [pyoracle.decrypt(key, x) for x in b] == [12, 11]
