"""The key's shared queues under concurrent single-element callers (bench.py's concurrent_decrypt_gh and
ghpair_operator_add loops, longer): 32 Python threads on one Paillier-2048 key, decrypt_gh through
fthe_decrypt_shared (server.h:69-78) and ciphertext adds through fthe_add_shared.  One JSON line; run it
under different FTHE_LINGER_US values to compare."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _run(nthr, fn):
    go = threading.Barrier(nthr + 1)

    def body(i):
        go.wait()
        fn(i)
    ths = [threading.Thread(target=body, args=(i,)) for i in range(nthr)]
    for t in ths:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    for t in ths:
        t.join()
    return time.perf_counter() - t0


def main():
    import numpy as np
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261016)
    nthr, rounds, per = 32, 12, 100
    cts = [pl.encrypt_u64(np.array([7 * i, 11 * i], dtype=np.uint64), seed=50 + i) for i in range(nthr)]
    ok = [True] * nthr

    def dgh(i):
        for _ in range(rounds):
            ok[i] &= bool(np.array_equal(pl.decrypt_u64_shared(cts[i]), [7 * i, 11 * i]))
    s = _run(nthr, dgh)
    rows = pl.encrypt_u64(np.arange(1, 65, dtype=np.uint64), seed=77)
    accs = [rows[i:i + 1].copy() for i in range(nthr)]

    def adds(i):
        for j in range(per):
            pl.add_shared(accs[i], rows[(i + j) % 64:(i + j) % 64 + 1], out=accs[i])
    sa = _run(nthr, adds)
    # every accumulator decrypts to its plaintext sum
    want = [(i + 1) + sum((i + j) % 64 + 1 for j in range(per)) for i in range(nthr)]
    ok_add = bool(np.array_equal(pl.decrypt_u64(np.concatenate(accs)), np.array(want, dtype=np.uint64)))
    print(json.dumps({"FTHE_LINGER_US": os.environ.get("FTHE_LINGER_US"), "threads": nthr,
                      "decrypt_gh_ms_per_round": round(s * 1e3 / rounds, 2), "decrypt_ok": all(ok),
                      "adds_per_s": round(nthr * per / sa), "adds_ok": ok_add}), flush=True)


if __name__ == "__main__":
    main()
