"""BASELINE.json configs[0] plumbing on the engine: the credit vertical 2-party
example (examples/credit/credit_vertical_p{0,1}.conf: 30,000 instances, party 1
holds 10 features, max_num_bin = 16, key_length = 512 -- parser.cpp:50) with HE.

One boosting round's HE traffic, in the reference's order:
  server (party 0, labels) homo_init(512) and encrypt_gh_pairs (server.h:58-67,
  113-135) of the logistic gradients at the initial prediction;
  party 1 builds the encrypted root histogram of its features on the device
  (hist_tree_builder.cpp:565-595), then level 1: the smaller child's histogram
  from its instance list (:640-664) and the sibling as father - child (:670-680),
  then the per-feature prefix (:695-708);
  the server decrypts (server.h:80-111).
Checks: every decrypted bin equals the exact sum of the members' fixed-point
codes (common.h:81-86) -- an integer identity, so bit-exact -- and the decoded
floats match float64 sums of the gradients within the codec quantum.
Data: tests/golden/credit_bins.npz (make_credit_fixture.py; labels and a
quantile binning of the reference's credit CSVs).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "credit_bins.npz")


def test_credit_vertical_he_round():
    import torch
    from fedtree_amd.paillier import GHPairs, HEParty, HEServer, decode_fixed, encode_fixed
    d = np.load(FIX)
    y, bins, nb = d["y"], d["bins_p1"], d["nbins_p1"].astype(np.int64)
    n, n_col = bins.shape
    max_num_bin = 16
    cut = np.concatenate([[0], np.cumsum(nb)]).astype(np.int32)
    n_bins = int(cut[-1])

    server = HEServer()
    server.homo_init(512, seed=20261015)
    party = HEParty()
    server.send_key(party)
    assert server.paillier.keyLength == 512 and not party.paillier.has_private

    p = np.full(n, 0.5, np.float32)                      # sigmoid(0): the first tree
    g = (p - y.astype(np.float32)).astype(np.float32)
    h = np.maximum(p * (1 - p), 1e-16).astype(np.float32)
    enc = server.encrypt_gh_pairs(GHPairs(g, h), seed=1)
    cw = 2 * party.paillier.n_words
    x = torch.from_numpy(np.concatenate([enc.g_enc, enc.h_enc]).view(np.int32)).cuda()
    bd = torch.from_numpy(np.ascontiguousarray(bins)).cuda()
    eg, eh = encode_fixed(g), encode_fixed(h)

    def want(rows):
        w = np.zeros(2 * n_bins, np.uint64)
        for f in range(n_col):
            b = bins[rows, f].astype(np.int64)
            np.add.at(w, cut[f] + b, eg[rows])
            np.add.at(w, n_bins + cut[f] + b, eh[rows])
        return w

    def run(inst):
        out = torch.empty((2 * n_bins, cw), dtype=torch.int32, device="cuda")
        party.paillier.histogram_dev(x, n, 2, bd, cut, max_num_bin, out,
                                     inst=None if inst is None else torch.from_numpy(inst).cuda())
        party.paillier.dev.sync()
        return out.cpu().numpy().view(np.uint32)

    root = run(None)
    low = server.paillier.decrypt_u64(root)
    assert np.array_equal(low, want(np.arange(n)))
    gsum = np.zeros(n_bins)
    for f in range(n_col):
        np.add.at(gsum, cut[f] + bins[:, f], g.astype(np.float64))
    assert np.allclose(decode_fixed(low[:n_bins]), gsum, atol=n * 1.5e-6)

    # level 1: split on party 1's feature 4 at its median bin; compute the smaller child
    left = bins[:, 4] < nb[4] // 2
    small = np.nonzero(left if left.sum() <= (~left).sum() else ~left)[0].astype(np.int32)
    big = np.setdiff1d(np.arange(n, dtype=np.int32), small)
    child = run(small)
    sib = party.paillier.sub_batch(root, child)              # father - computed
    assert np.array_equal(server.paillier.decrypt_u64(child), want(small))
    assert np.array_equal(server.paillier.decrypt_u64(sib), want(big))

    # per-feature prefix over the sibling histogram (inclusive_scan_by_key)
    seg = np.concatenate([cut, cut[1:] + n_bins]).astype(np.int64)
    pre = party.paillier.scan_segments(sib, seg)
    wb = want(big)
    wpre = np.concatenate([np.concatenate([np.cumsum(wb[s:e], dtype=np.uint64)
                                           for s, e in zip(seg[:-1], seg[1:])])])
    assert np.array_equal(server.paillier.decrypt_u64(pre), wpre)
