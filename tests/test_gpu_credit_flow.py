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


def test_credit_vertical_he_10_trees_depth_6():
    """configs[0] at its stated size: 10 trees of depth 6 (credit_vertical_p*.conf).
    Per tree, as the vertical simulation does (FLtrainer.cpp:556 re-keys, server.h:58-67, 113-135): a fresh
    Paillier-512 key, the server encrypts the 30,000 gradient pairs at the current prediction; then per level
    (0..5) party 1 builds the smaller child's histogram on the device from its instance list
    (hist_tree_builder.cpp:640-664; the root from all instances), the sibling as father - child (:670-680), the
    per-feature prefix (:695-708), and the server decrypts every prefix bin of every node of the level
    (server.h:80-111).  Every decrypted bin is checked by integer identity against the members' fixed-point codes
    (common.h:81-86).  Splits: the best gain over party 1's features from the decrypted sums (lambda = 1,
    min_child_weight = 1, the GBDTParam defaults); leaves -G / (H + lambda) update the prediction, so every
    tree encrypts new gradients."""
    import time

    from fedtree_amd.paillier import GHPairs, HEParty, HEServer, encode_fixed
    d = np.load(FIX)
    y, bins, nb = d["y"], d["bins_p1"], d["nbins_p1"].astype(np.int64)
    n, n_col = bins.shape
    max_num_bin, depth, trees, lam = 16, 6, 10, 1.0
    cut = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
    n_bins = int(cut[-1])
    seg = np.concatenate([cut, cut[1:] + n_bins]).astype(np.int64)
    server, party = HEServer(), HEParty()
    bd = torch_dev(np.ascontiguousarray(bins))
    pred = np.zeros(n, np.float32)
    t0 = time.perf_counter()
    stats = dict(encrypts=0, histograms=0, siblings=0, decrypts=0, nodes=0, leaves=0)
    for tree in range(trees):
        server.homo_init(512, seed=20261015 + tree)
        server.send_key(party)
        p = (1.0 / (1.0 + np.exp(-pred.astype(np.float64)))).astype(np.float32)
        g = (p - y.astype(np.float32)).astype(np.float32)
        h = np.maximum(p * (1 - p), 1e-16).astype(np.float32)
        enc = server.encrypt_gh_pairs(GHPairs(g, h), seed=tree + 1)
        stats["encrypts"] += 2 * n
        x = torch_dev(np.concatenate([enc.g_enc, enc.h_enc]).view(np.int32))
        eg, eh = encode_fixed(g), encode_fixed(h)
        cw = 2 * party.paillier.n_words

        def want(rows):
            w = np.zeros(2 * n_bins, np.uint64)
            for f in range(n_col):
                b = cut[f] + bins[rows, f].astype(np.int64)
                np.add.at(w, b, eg[rows])
                np.add.at(w, n_bins + b, eh[rows])
            return w

        def run(inst):
            import torch
            out = torch.empty((2 * n_bins, cw), dtype=torch.int32, device="cuda")
            party.paillier.histogram_dev(x, n, 2, bd, cut.astype(np.int32), max_num_bin, out,
                                         inst=None if inst is None else torch_dev(inst))
            party.paillier.dev.sync()
            stats["histograms"] += 1
            return out.cpu().numpy().view(np.uint32)

        level = [(np.arange(n, dtype=np.int32), run(None))]          # (instances, encrypted histogram)
        for lv in range(depth):
            pres = [party.paillier.scan_segments(hist, seg) for _, hist in level]
            dec = server.paillier.decrypt_u64(np.concatenate(pres))
            stats["decrypts"] += len(dec)
            nxt = []
            for k, (rows, hist) in enumerate(level):
                got = dec[k * 2 * n_bins:(k + 1) * 2 * n_bins]
                wb = want(rows)
                wpre = np.concatenate([np.cumsum(wb[s:e], dtype=np.uint64) for s, e in zip(seg[:-1], seg[1:])])
                assert np.array_equal(got, wpre), (tree, lv, k)
                stats["nodes"] += 1
                sg = got.view(np.int64).astype(np.float64) / 1e6            # signed fixed point (Q6, Q9)
                G, H = sg[cut[1] - 1], sg[n_bins + cut[1] - 1]
                best = (0.0, None)
                for f in range(n_col):
                    for b in range(int(cut[f]), int(cut[f + 1]) - 1):
                        GL, HL = sg[b], sg[n_bins + b]
                        GR, HR = G - GL, H - HL
                        if HL < 1.0 or HR < 1.0:
                            continue
                        gain = GL * GL / (HL + lam) + GR * GR / (HR + lam) - G * G / (H + lam)
                        if gain > best[0] + 1e-12:
                            best = (gain, (f, b - int(cut[f])))
                if best[1] is None:
                    pred[rows] += np.float32(-G / (H + lam))
                    stats["leaves"] += 1
                    continue
                f, b = best[1]
                left = rows[bins[rows, f] <= b]
                right = rows[bins[rows, f] > b]
                if lv == depth - 1:                                      # children at depth 6 are leaves
                    GL, HL = sg[int(cut[f]) + b], sg[n_bins + int(cut[f]) + b]
                    pred[left] += np.float32(-GL / (HL + lam))
                    pred[right] += np.float32(-(G - GL) / (H - HL + lam))
                    stats["leaves"] += 2
                    continue
                small, big = (left, right) if len(left) <= len(right) else (right, left)
                child = run(small)
                sib = party.paillier.sub_batch(hist, child)              # father - computed
                stats["siblings"] += 1
                nxt += [(small, child), (big, sib)]
            level = nxt
            if not level:
                break
    el = time.perf_counter() - t0
    print(f"configs[0]: {trees} trees x depth {depth}: {stats}, {el:.1f} s")
    assert stats["leaves"] >= trees and stats["nodes"] >= trees * depth
    # the trees fit: the training loss fell
    p = 1.0 / (1.0 + np.exp(-pred.astype(np.float64)))
    loss = -np.mean(y * np.log(p + 1e-12) + (1 - y) * np.log(1 - p + 1e-12))
    assert loss < np.log(2) - 0.02, loss


def torch_dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()
