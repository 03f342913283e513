"""decrypt_gh from OpenMP threads (FLtrainer.cpp:758-764, server.h:69-78): T host threads, each with its
own engine context and a copy of one Paillier-2048 key, decrypt one GHPair (2 ciphertexts, host in/out)
R times concurrently.  One JSON line: wall ms per round and pairs/s for each T, every result checked."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    from fedtree_amd.paillier import Device, Paillier
    base = Paillier(Device(0)).keygen(2048, seed=20261015)
    p, q = base.p, base.q
    out = {}
    R = 4
    shared = os.environ.get("FTHE_CP_SHARED") == "1"    # all threads on one key through fthe_decrypt_shared
    out["mode"] = "decrypt_shared (one key, coalesced)" if shared else "decrypt per thread context"
    for T in (1, 2, 4, 8, 16, 32):
        c_shared = [base.encrypt_u64(np.array([1000 + i, 2000 + i], dtype=np.uint64), seed=7 + i)
                    for i in range(T)] if shared else None
        ready = threading.Barrier(T + 1)
        done = threading.Barrier(T + 1)
        errs = []

        def work(i):
            try:
                m = np.array([1000 + i, 2000 + i], dtype=np.uint64)
                if shared:
                    pl = base
                    c = c_shared[i]
                    dec = pl.decrypt_u64_shared
                else:
                    dev = Device(0)
                    pl = Paillier.from_primes(p, q, dev)
                    c = pl.encrypt_u64(m, seed=7 + i)
                    dec = pl.decrypt_u64
                dec(c)
                ready.wait()
                for _ in range(R):
                    if not np.array_equal(dec(c), m):
                        errs.append(i)
                done.wait()
            except Exception as e:      # keep the barriers from hanging
                errs.append(repr(e))
                ready.abort()
                done.abort()

        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        for t in th:
            t.start()
        ready.wait()
        t0 = time.perf_counter()
        done.wait()
        ms = (time.perf_counter() - t0) * 1e3 / R
        for t in th:
            t.join()
        assert not errs, errs
        out[T] = {"ms_per_round": round(ms, 2), "pairs_per_s": round(T / ms * 1e3)}
        print(json.dumps({T: out[T]}), flush=True)
    print(json.dumps({"concurrent_decrypt_gh": out, "rounds": R}), flush=True)


if __name__ == "__main__":
    main()
