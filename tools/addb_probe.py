"""Bring-up probe of fthe_addb_q152: adds of several sizes in a fresh process, each row checked against
Python's x y mod n^2; prints per size the rows that differ (zero rows counted apart).
  python tools/addb_probe.py 15 1 15 16 17 193"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))


def main():
    import torch
    import pyoracle
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261017)
    n2, cw = pl.n2, 2 * pl.n_words
    rng = np.random.default_rng(7)
    for cnt in [int(x) for x in sys.argv[1:]]:
        a = [int.from_bytes(rng.bytes(512), "little") % n2 for _ in range(cnt)]
        b = [int.from_bytes(rng.bytes(512), "little") % n2 for _ in range(cnt)]
        ad = torch.from_numpy(pyoracle.ints_to_words(a, cw).view(np.int32)).cuda()
        bd = torch.from_numpy(pyoracle.ints_to_words(b, cw).view(np.int32)).cuda()
        o = torch.full_like(ad, 7)
        torch.cuda.synchronize()
        pl.add_dev(ad, bd, o)
        dev.sync()
        torch.cuda.synchronize()
        got = pyoracle.words_to_ints(o.cpu().numpy().view(np.uint32))
        want = [x * y % n2 for x, y in zip(a, b)]
        bad = [i for i in range(cnt) if got[i] != want[i]]
        untouched = [i for i in bad if got[i] == sum(7 << (32 * k) for k in range(cw))]
        print(json.dumps({"count": cnt, "bad": len(bad), "untouched": len(untouched), "first_bad": bad[:8]}),
              flush=True)


if __name__ == "__main__":
    main()
