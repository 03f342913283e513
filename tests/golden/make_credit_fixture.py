"""Make tests/golden/credit_bins.npz from the reference's credit example data
(dataset/credit/credit_vertical_p{0_withlabel,1}.csv, the data of
examples/credit/credit_vertical_p{0,1}.conf -- BASELINE.json configs[0]).

Stored: labels y (uint8, p0's `y` column) and per-party bin ids (uint8,
instance-major) from a per-feature quantile binning into <= max_num_bin = 16
bins (the conf's value).  The binning is this script's, not FedTree's
HistCut: the HE plumbing test needs a realistic bin layout of the real data
shape, not the reference's exact cut points.  Rows are aligned by `id`.

  python tests/golden/make_credit_fixture.py /root/reference/dataset/credit
"""
import os
import sys

import numpy as np

MAX_NUM_BIN = 16


def load(path):
    head = open(path).readline().strip().split(",")
    a = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.float64)
    return head, a


def bins_of(x):
    out = np.zeros(x.shape, np.uint8)
    cuts = []
    for f in range(x.shape[1]):
        q = np.unique(np.quantile(x[:, f], np.linspace(0, 1, MAX_NUM_BIN + 1)[1:-1]))
        out[:, f] = np.searchsorted(q, x[:, f], side="right")
        cuts.append(len(q) + 1)
    return out, np.array(cuts, np.int32)


def main(d):
    h0, a0 = load(os.path.join(d, "credit_vertical_p0_withlabel.csv"))
    h1, a1 = load(os.path.join(d, "credit_vertical_p1.csv"))
    a1 = a1[np.argsort(a1[:, 0])]
    a0 = a0[np.argsort(a0[:, 0])]
    assert np.array_equal(a0[:, 0], a1[:, 0])
    y = a0[:, h0.index("y")].astype(np.uint8)
    x0 = a0[:, 2:]
    x1 = a1[:, 1:]
    b0, n0 = bins_of(x0)
    b1, n1 = bins_of(x1)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "credit_bins.npz")
    np.savez_compressed(out, y=y, bins_p0=b0, bins_p1=b1, nbins_p0=n0, nbins_p1=n1)
    print(out, y.shape, b0.shape, b1.shape, n0, n1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/dataset/credit")
