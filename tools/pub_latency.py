"""Latency of small public-key encrypts (a party without published bases, party.h:118-142): Paillier-2048,
default formula on the s152 four-lane kernel, host in/out.  One JSON line {count: ms}."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    key = Paillier(dev).keygen(2048, seed=20261015)
    pub = Paillier.from_public(key.modulus, dev)
    out = {}
    for cnt in (2, 64, 1024, 16384):
        m = np.arange(cnt, dtype=np.uint64)
        c = pub.encrypt_u64(m)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            c = pub.encrypt_u64(m)
        ms = (time.perf_counter() - t0) / reps * 1e3
        assert np.array_equal(key.decrypt_u64(c), m)
        out[cnt] = {"ms": round(ms, 2), "per_s": round(cnt / ms * 1e3)}
    print(json.dumps({"public_encrypt_latency": out}), flush=True)


if __name__ == "__main__":
    main()
