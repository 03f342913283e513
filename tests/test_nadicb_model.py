"""The matrix-core Barrett form of the n-adic public-key encrypt (fthe_nadic_b76), checked on the CPU before the
GPU sees it:
* tools/nadicb_model.py's reductions (tile by tile, every int32 / int64 bound, the chunked normalisation, the clamp)
  at the digit bound, and a full encrypt through the digit products against pow;
* the host builder of the per-key context in the library (nadicb_image.hpp, through the fthe_debug_nadicb_image
  hook) byte for byte against the model's, and its refusal outside n of 2041..2048 bits;
* the generated kernel run on the wave emulator (tools/wave_emu.py: LOADX, CANON, STOREX, SQR, MUL of unreduced
  digits, CANON -> r^7 mod n^2 for 16 ciphertexts) against Python integers."""
import ctypes
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "fedtree_amd", "csrc"))

import nadicb_model as nm  # noqa: E402


def test_generator_constants_match_model():
    import gen_nadicb as g
    assert (g.A_BITS, g.C_BITS, g.S1_BASE, g.TILES1, g.TILES2, g.KB1, g.KB2, g.NQ1, g.NQ3, g.BIAS_COL,
            g.BIAS_DIGIT, g.ND1, g.ND2, g.CHUNKS) == (nm.A_BITS, nm.C_BITS, nm.S1_BASE, nm.TILES1, nm.TILES2,
                                                    nm.KB1, nm.KB2, nm.NQ1, nm.NQ3, nm.BIAS_COL, nm.BIAS_DIGIT,
                                                    nm.ND1, nm.ND2, nm.CHUNKS)
    assert g.ACT1 == nm.ACT1 and g.ACT2 == nm.ACT2
    assert g.lds_bytes() <= 160 * 1024


@pytest.mark.parametrize("bits", [2048, 2041])
def test_reduction_tiles_and_bounds(bits):
    rng = random.Random(bits)
    n = nm.rand_n(rng, bits)
    k = nm.Key(n)
    nm.FAST[0] = False
    try:
        top = 3 * n - 1
        for z in (0, top * top, 2 * top * top + 19 * n - 1, n * n - 1, rng.randrange(19 * n * n)):
            z = min(z, 19 * n * n - 1)
            r, q3 = k.reduce(z)
            assert r == z - q3 * n and 0 <= r < 3 * n
    finally:
        nm.FAST[0] = False


def test_encrypt_through_digit_products():
    rng = random.Random(3)
    n = nm.rand_n(rng, 2048)
    k = nm.Key(n)
    nm.FAST[0] = True
    try:
        r = rng.randrange(1, n)
        m = 2**64 - 1
        assert nm.encrypt(k, m, r) == (1 + m * n) * pow(r, n, n * n) % (n * n)
    finally:
        nm.FAST[0] = False


def test_host_image_matches_model():
    from fedtree_amd import _lib
    lib = _lib.load()
    rng = random.Random(11)
    for bits in (2048, 2047, 2041):
        n = nm.rand_n(rng, bits)
        nw = np.frombuffer(n.to_bytes(256, "little"), dtype=np.uint32).copy()
        ln = ctypes.c_size_t(0)
        assert lib.fthe_debug_nadicb_image(ctypes.c_void_p(nw.ctypes.data), 64, None, ctypes.c_size_t(0),
                                           ctypes.byref(ln)) == 0
        buf = np.zeros(ln.value, dtype=np.uint8)
        assert lib.fthe_debug_nadicb_image(ctypes.c_void_p(nw.ctypes.data), 64, ctypes.c_void_p(buf.ctypes.data),
                                           ctypes.c_size_t(ln.value), ctypes.byref(ln)) == 0
        import gen_nadicb as g
        img = nm.nadicb_image(n)
        assert bytes(buf[:g.IMG_BYTES]) == img
        limbs = [(n >> (27 * j)) & ((1 << 27) - 1) for j in range(76)]
        assert list(buf[g.N_OFF:g.N_OFF + 304].view(np.uint32)) == limbs
    for bad in ((1 << 2039) + 1, (1 << 2048) + 1, (1 << 2047) + 2):    # 2040 bits, 2049 bits, even n
        nw = np.frombuffer(bad.to_bytes(260, "little"), dtype=np.uint32).copy()
        ln = ctypes.c_size_t(0)
        assert lib.fthe_debug_nadicb_image(ctypes.c_void_p(nw.ctypes.data), len(nw), None, ctypes.c_size_t(0),
                                           ctypes.byref(ln)) != 0


def test_kernel_on_wave_emulator():
    import wave_emu
    assert wave_emu.nadicb_selftest(waves=2) == 0          # two waves: per-wave LDS areas and rows
