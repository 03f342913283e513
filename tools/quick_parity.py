"""Quick GPU bring-up: engine vs oracle at P-512/1024/2048 + a timing probe."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from fedtree_amd import _lib  # noqa: E402
import pyoracle  # noqa: E402


def splitmix(seed):
    s = seed
    while True:
        s = (s + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        yield z ^ (z >> 31)


def det_primes(nbits, seed, o):
    g = splitmix(seed)
    hw = nbits // 64
    ps = []
    for _ in range(2):
        w = np.array([next(g) & 0xFFFFFFFF for _ in range(hw)], dtype=np.uint32)
        ps.append(o.next_prime(w))
    return ps


def p(x):
    return ctypes.c_void_p(x.ctypes.data)


def main():
    lib = _lib.load()
    o = pyoracle.COracle()
    ctx = ctypes.c_void_p()
    _lib.check(lib.fthe_ctx_create(0, ctypes.byref(ctx)), "ctx")
    ok = True
    for nbits in (512, 1024, 2048):
        pw, qw = det_primes(nbits, 20261015 + nbits, o)
        key = ctypes.c_void_p()
        _lib.check(lib.fthe_key_from_primes(ctx, p(pw), p(qw), len(pw), ctypes.byref(key)), "key")
        nw = lib.fthe_key_n_words(key)
        okey = o.key(pw, qw)
        pk = pyoracle.keygen_from_primes(pyoracle.from_words(pw), pyoracle.from_words(qw))
        n = pk["n"]
        rng = np.random.default_rng(nbits)
        cnt = 300
        m = rng.integers(0, 2**63, cnt, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, cnt, dtype=np.uint64)
        m[:5] = np.array([0, 1, 2**64 - 1, 2**63 - 1, 2**63], dtype=np.uint64)
        rs = [int.from_bytes(rng.bytes(nw * 4), "little") % (n - 1) + 1 for _ in range(cnt)]
        rs[0] = 1
        rs[1] = n - 1
        r = pyoracle.ints_to_words(rs, nw)
        want = okey.encrypt_batch(m, r)
        for flags in (0, 1):
            c = np.zeros((cnt, 2 * nw), dtype=np.uint32)
            st = lib.fthe_encrypt_u64(key, ctx, p(m), cnt, p(r), nw, 0, p(c), flags)
            if st == _lib.FTHE_ERR_UNSUPPORTED:
                print(f"P-{nbits} flags={flags}: unsupported")
                continue
            _lib.check(st, "encrypt")
            same = np.array_equal(c, want)
            ok &= same
            print(f"P-{nbits} encrypt flags={flags}: {'OK' if same else 'MISMATCH'}"
                  f" ({np.sum(np.any(c != want, axis=1))} rows differ)")
        mlow = np.zeros(cnt, dtype=np.uint64)
        mfull = np.zeros((cnt, nw), dtype=np.uint32)
        _lib.check(lib.fthe_decrypt(key, ctx, p(want), cnt, p(mlow), p(mfull)), "decrypt")
        same = np.array_equal(mlow, m)
        okfull = all(pyoracle.from_words(mfull[i]) == int(m[i]) for i in range(cnt))
        ok &= same and okfull
        print(f"P-{nbits} decrypt: low64 {'OK' if same else 'MISMATCH'} full {'OK' if okfull else 'MISMATCH'}")
        # add / kway / scalar mul (public path only)
        out = np.zeros_like(want)
        rev = np.ascontiguousarray(want[::-1])
        st = lib.fthe_add(key, ctx, p(want), p(rev), cnt, p(out))
        if st == _lib.FTHE_OK:
            w2 = okey.add_batch(want, rev)
            print(f"P-{nbits} add: {'OK' if np.array_equal(out, w2) else 'MISMATCH'}")
            ok &= np.array_equal(out, w2)
            k = 5
            xs = np.ascontiguousarray(np.concatenate([np.roll(want, j, axis=0) for j in range(k)]))
            out = np.zeros_like(want)
            _lib.check(lib.fthe_reduce_kway(key, ctx, p(xs), k, cnt, p(out)), "kway")
            acc = want.copy()
            for j in range(1, k):
                acc = okey.add_batch(acc, np.roll(want, j, axis=0))
            print(f"P-{nbits} kway: {'OK' if np.array_equal(out, acc) else 'MISMATCH'}")
            ok &= np.array_equal(out, acc)
            out = np.zeros_like(want)
            _lib.check(lib.fthe_scalar_mul_u64(key, ctx, p(want), 2**64 - 1, cnt, p(out)), "smul")
            w3 = np.stack([okey.mul_u64(want[i], 2**64 - 1) for i in range(cnt)])
            print(f"P-{nbits} scalar_mul: {'OK' if np.array_equal(out, w3) else 'MISMATCH'}")
            ok &= np.array_equal(out, w3)
        else:
            print(f"P-{nbits} add: status {st}")
        # timing probe: device RNG CRT encrypt
        if nbits == 2048:
            cnt2 = int(os.environ.get("QP_COUNT", "262144"))
            m2 = rng.integers(0, 2**64, cnt2, dtype=np.uint64)
            c2 = np.zeros((cnt2, 2 * nw), dtype=np.uint32)
            for rep in range(2):
                t0 = time.time()
                _lib.check(lib.fthe_encrypt_u64(key, ctx, p(m2), cnt2, None, 0, 7, p(c2), 0), "enc2")
                t1 = time.time()
                ms = lib.fthe_last_kernel_ms(ctx)
                mm = lib.fthe_last_montmuls(ctx)
                print(f"P-2048 CRT encrypt {cnt2}: wall {t1 - t0:.3f}s kernel {ms:.1f} ms -> "
                      f"{cnt2 / (ms * 1e-3):.0f} enc/s; montmuls/ct {mm / cnt2:.0f}; "
                      f"{mm / (ms * 1e-3):.3e} MontMul/s")
            # check a sample of the RNG ciphertexts: decrypt with the oracle
            sample = c2[:: max(1, cnt2 // 64)][:64]
            dec = okey.decrypt_batch(sample)
            good = all(pyoracle.from_words(dec[i]) == int(m2[:: max(1, cnt2 // 64)][i]) for i in range(len(sample)))
            print(f"P-2048 RNG ciphertexts decrypt (oracle) {'OK' if good else 'MISMATCH'}")
            ok &= good
            mlow = np.zeros(cnt2, dtype=np.uint64)
            _lib.check(lib.fthe_decrypt(key, ctx, p(c2), cnt2, p(mlow), None), "dec2")
            ms = lib.fthe_last_kernel_ms(ctx)
            same = np.array_equal(mlow, m2)
            ok &= same
            print(f"P-2048 CRT decrypt {cnt2}: {ms:.1f} ms -> {cnt2 / (ms * 1e-3):.0f} dec/s; roundtrip "
                  f"{'OK' if same else 'MISMATCH'}")
        lib.fthe_key_destroy(key)
    lib.fthe_ctx_destroy(ctx)
    print("ALL OK" if ok else "FAILURES")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
