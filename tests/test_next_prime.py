"""The keygen's prime search (fthe_next_prime, host only).

Key generation draws a random start with the top two bits set and takes the next
prime (GenPrimePair, paillier.cpp:43-62; paillier_gmp.cpp:108-239 via mpz_nextprime).
The engine sieves windows of odd candidates and tests them on up to 16 host threads;
the result must be the smallest prime above the start, i.e. what mpz_nextprime returns.
Checked here in Python: the result is prime (Miller-Rabin, 32 random bases) and every
odd number between the start and the result is composite.  Runs on the CPU.
"""
import numpy as np

import pyoracle
from fedtree_amd import _lib


def _is_probable_prime(n, rng):
    if n < 4:
        return n in (2, 3)
    if n % 2 == 0:
        return False
    d, s = n - 1, 0
    while d % 2 == 0:
        d, s = d // 2, s + 1
    for _ in range(32):
        a = int.from_bytes(rng.bytes(16), "little") % (n - 3) + 2
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _next_prime(start, words):
    lib = _lib.load()
    w = np.asarray(pyoracle.to_words(start, words), dtype=np.uint32)
    out = np.zeros(words + 1, dtype=np.uint32)
    rc = lib.fthe_next_prime(w.ctypes.data, words, out.ctypes.data, words + 1)
    assert rc == 0
    return pyoracle.from_words(out)


def test_next_prime_is_the_smallest_prime_above_start():
    rng = np.random.default_rng(556)
    for bits in (40, 256, 512, 1024):
        for _ in range(3 if bits < 1024 else 2):
            start = int.from_bytes(rng.bytes(bits // 8), "little") | (3 << (bits - 2))
            start >>= max(0, start.bit_length() - bits)
            words = (bits + 31) // 32
            p = _next_prime(start, words)
            assert p > start and _is_probable_prime(p, rng), (bits, start)
            x = start + 1 + (start % 2 == 1)                 # odd numbers in (start, p)
            x |= 1
            while x < p:
                assert not _is_probable_prime(x, rng), (bits, x)
                x += 2


def test_next_prime_small_and_edge_starts():
    assert _next_prime(1 << 20, 1) == 1048583
    assert _next_prime((1 << 31) - 1, 1) == 2147483659               # crosses 2^31
    assert _next_prime(1048583, 1) == 1048589                          # start prime: strictly greater
    lib = _lib.load()
    out = np.zeros(1, dtype=np.uint32)
    w = np.asarray([0xFFFFFFFB], dtype=np.uint32)                       # next prime > 2^32 - 5 needs 2 words
    assert lib.fthe_next_prime(w.ctypes.data, 1, out.ctypes.data, 1) == _lib.FTHE_ERR_ARG
    assert lib.fthe_next_prime(None, 1, out.ctypes.data, 1) == _lib.FTHE_ERR_ARG
