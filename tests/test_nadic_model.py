"""CPU checks of the n-adic public-encrypt kernel's arithmetic: the bit-exact model
(tools/nadic_model.py) at the bounds of n and of the digits, and the generated gfx950 assembly run on the
quad emulator (tools/quad_emu.py) -- LOADX of a raw r, CANON, SQR, MUL by the (1, m) digits, STOREX --
against Python integers (r^e (1 + m n) mod n^2, paillier.cpp:134-137 with g = n + 1)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "fedtree_amd", "csrc"))

import nadic_model as nm  # noqa: E402


def test_model_products_at_bounds():
    rng = random.Random(5)
    for bits in (2042, 2048, 2050):
        n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        k = nm.consts(n)
        n2 = n * n
        cases = [[n - 1] * 4, [rng.randrange(n) for _ in range(4)], [0, n - 1, 1, n - 1],
                 [n - 1 - rng.randrange(1 << 64) for _ in range(4)]]
        for x0, x1, y0, y1 in cases:
            X, Y = x0 + x1 * n, y0 + y1 * n
            z0, z1 = nm.fused(y0, y1, x0, x1, n, k)
            assert z0 + z1 * n == X * Y % n2 and z0 < n and z1 <= n
            z0, z1 = nm.fused(x0, x1, x0, x1, n, k, sq=True)
            assert z0 + z1 * n == X * X % n2 and z0 < n and z1 <= n
        # digit 1 == n (an unreduced 0, the one non-canonical product output) as input
        z0, z1 = nm.fused(n - 1, n, n - 1, n, n, k)
        assert (z0 + z1 * n - (n - 1) ** 2) % n2 == 0


def test_model_exponentiation():
    rng = random.Random(6)
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    k = nm.consts(n)
    r = rng.randrange(1, n)
    e = rng.getrandbits(64) | (1 << 63)
    x0, x1 = nm.pow_nadic(r, e, n, k)
    assert x0 + x1 * n == pow(r, e, n * n)


def test_generated_assembly_on_quad_emulator():
    import quad_emu
    cwd = os.getcwd()
    os.chdir(ROOT)
    try:
        quad_emu.selftest(trials=1, ebits=6)
    finally:
        os.chdir(cwd)


def test_gathered_digit_entries_on_quad_emulator():
    """LOADGD / MULGD (8-bit windows) and LOADGD16 / MULGD16 from digit-form table entries (the
    published-bases public encrypt's gathered products) on the emulated quad"""
    import quad_emu
    cwd = os.getcwd()
    os.chdir(ROOT)
    try:
        quad_emu.selftest_gather(False)
        quad_emu.selftest_gather(True)
    finally:
        os.chdir(cwd)


def test_montgomery_model_bounds_and_encrypt():
    """tools/nadic_mont_model.py: the Montgomery n-adic product (fthe_nadic_m76) at digits up to 2n - 1
    (the chained bound), squarings, and the encrypt program pow / MUL (1, m) / MUL K / CANON vs pow()"""
    import nadic_mont_model as mm
    rng = random.Random(5)
    st = {}
    for nb in (1033, 1536, 2042, 2048):
        n = rng.getrandbits(nb) | (1 << (nb - 1)) | 1
        n2 = n * n
        rinv = pow(mm.R, -1, n2)
        for xs in ([2 * n - 1] * 4, [rng.randrange(2 * n) for _ in range(4)], [0, 2 * n - 1, 1, 0]):
            x0, x1, y0, y1 = xs
            z0, z1 = mm.mont(y0, y1, x0, x1, n, stats=st)
            assert (z0 + z1 * n) % n2 == (x0 + x1 * n) * (y0 + y1 * n) * rinv % n2
            z0, z1 = mm.mont(x0, x1, x0, x1, n, sq=True, stats=st)
            assert (z0 + z1 * n) % n2 == (x0 + x1 * n) ** 2 * rinv % n2
    assert st['col'] < 1 << 62
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    e = rng.getrandbits(40) | (1 << 39)
    m = rng.getrandbits(64)
    for r in (2 * n - 1, rng.randrange(1, n)):
        z0, z1 = mm.encrypt(m, r, n, e)
        assert z0 + z1 * n == pow(r, e, n * n) * (1 + m * n) % (n * n)


def test_montgomery_assembly_on_quad_emulator():
    """the generated fthe_nadic_m76 (gen_nadic.py mont=True) on the emulated quad: LOADX of a raw r,
    CANON, pow, MUL (1, m), MUL K, CANON, STOREX against pow(r, e, n^2) (1 + m n)"""
    import quad_emu
    cwd = os.getcwd()
    os.chdir(ROOT)
    try:
        quad_emu.selftest(trials=2, ebits=6, mont=True)
    finally:
        os.chdir(cwd)
