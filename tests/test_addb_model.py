"""The matrix-core Barrett add (fthe_addb_q152, fedtree_amd/csrc/gen_addb.py) without a GPU:

* tools/addb_model.py, the bit-exact model of its arithmetic (Barrett cut points, truncated product with
  its bias, int32 column sums, signed group folds), against Python's x y mod N -- the reference's add
  (paillier.cpp:92-105, paillier_gmp.cpp:16-21) -- on random and extreme operands, n of 2048 bits at both
  ends of the range;
* the host builder of the per-key context in the library (addb_image.hpp, through the
  fthe_debug_addb_image hook) byte for byte against the model's;
* the generated gfx950 assembly itself, run on tools/wave_emu.py (64-lane wavefronts: DPP, EXEC/VCC,
  LDS, v_mfma_i32_16x16x64_i8 with the lane map measured on the GPU), one workgroup of adds vs x y mod N.
"""
import ctypes
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "fedtree_amd", "csrc"))

import addb_model as am  # noqa: E402

KEYS = [None, (1 << 2047) + 1, (1 << 2048) - 1]


def _n(i):
    return KEYS[i] if KEYS[i] else am.rand_n(random.Random(4))


@pytest.mark.parametrize("ki", [0, 1, 2])
def test_model_reduces_exactly(ki):
    n = _n(ki)
    k = am.AddbKey(n * n)
    N = k.N
    rng = random.Random(ki)
    top = (1 << 4096) - 1                             # rows >= N: not ciphertexts, reduced all the same
    cases = [(N - 1, N - 1), (0, N - 1), (1, 1), (N - 1, 1), (1 << 2048, (1 << 2048) - 1), (top, top), (N, N),
             (top, 1)]
    cases += [(rng.randrange(N), rng.randrange(N)) for _ in range(3)]
    for x, y in cases:
        r, q3 = k.reduce(x * y)                       # asserts every bound and q3 in [q - 2, q]
        assert 0 <= r < 3 * N
        assert k.add(x, y) == x * y % N


def test_model_rejects_short_moduli():
    with pytest.raises(AssertionError):
        am.AddbKey(((1 << 2046) + 1) ** 2)            # n of 2047 bits: N below 2^4094


@pytest.mark.parametrize("ki", [0, 1, 2])
def test_host_context_matches_model(ki):
    lib = ctypes.CDLL(os.path.join(ROOT, "fedtree_amd", "libfthe.so"))
    n = _n(ki)
    nw = np.frombuffer(n.to_bytes(256, "little"), dtype=np.uint32).copy()
    ln = ctypes.c_size_t()
    assert lib.fthe_debug_addb_image(ctypes.c_void_p(nw.ctypes.data), 64, None, ctypes.c_size_t(0),
                                     ctypes.byref(ln)) == 0
    buf = np.zeros(ln.value, np.uint8)
    assert lib.fthe_debug_addb_image(ctypes.c_void_p(nw.ctypes.data), 64, ctypes.c_void_p(buf.ctypes.data),
                                     ctypes.c_size_t(buf.size), ctypes.byref(ln)) == 0
    assert bytes(buf) == am.addb_image(n * n)


def test_host_context_refuses_short_n():
    lib = ctypes.CDLL(os.path.join(ROOT, "fedtree_amd", "libfthe.so"))
    n = (1 << 2040) + 7
    nw = np.frombuffer(n.to_bytes(256, "little"), dtype=np.uint32).copy()
    ln = ctypes.c_size_t()
    assert lib.fthe_debug_addb_image(ctypes.c_void_p(nw.ctypes.data), 64, None, ctypes.c_size_t(0),
                                     ctypes.byref(ln)) == -4          # FTHE_ERR_UNSUPPORTED


def test_generated_kernel_on_wave_emulator():
    """the gfx950 assembly of fthe_addb_q152, one workgroup: a full wave of 16 adds (N - 1 squared,
    0 (N - 1), 1 1 and random rows) and a partly live wave (13 of 16), every row vs x y mod N"""
    import wave_emu
    wave_emu.selftest()


def test_slow_path_ripples_carry_real_values():
    """the normalisation's rare slow paths (gen_addb.py norm_two_chains: chain A's carry into chain B's
    lowest dword; lane_delivery: a lane's carry into the next lane's chunk) must be run with nonzero carries, not
    only with the slowall build's carry 0.  The emulator selftest's structured rows ((N - 1)^2, 0 (N - 1), rows >= N
    under n = 2^2047 + 1) overflow both joins: every slow-path multiply-add is counted with the lanes whose carry
    register is nonzero, and the results stay exact.  The one ripple no input reaches is lane 3's four extra dwords
    (N1 dwords 128..131, only after dwords 113..127 saturate): the same generated ripple code under one more EXEC
    mask; structured quotients (4 special moduli x 96 patterns, x = 1 and y = k 2^4072 + e) never overflowed there."""
    import collections
    import gen_addb as ga
    import wave_emu
    asm = ga.gen_addb('fthe_addb_q152')
    ins = [s for s in (ln.split('//')[0].strip() for ln in asm.splitlines())
           if s and not s.endswith(':') and not s.startswith('.')]
    carry = f"v{166 + 1}"                                   # gen_addb: X = CR + 1, the rippled carry
    ripple = {i for i, s in enumerate(ins) if s.startswith('v_mad_i64_i32') and f", {carry}, 1," in s}
    assert ripple
    hits = collections.Counter()
    orig = wave_emu.Wave.step

    def step(self, op, a):
        if self.pc - 1 in ripple:
            hits[self.pc - 1] += sum(1 for ln in self.lanes() if self.vget(ln, a[2]) != 0)
        return orig(self, op, a)
    wave_emu.Wave.step = step
    try:
        wave_emu.selftest()                                 # asserts every row exact
    finally:
        wave_emu.Wave.step = orig
    assert sum(hits.values()) > 100 and len([pc for pc, h in hits.items() if h]) > 30, hits


def test_matrix_core_product_model():
    """tools/addb_mfz_model.py (the "mfz" product of gen_addb.py section 2M): z = x y from the 28 i8 MFMA tiles over
    balanced digits, the dword-aligned A windows with their byte funnel shift, the reversed y staging, the groups and
    the lane-to-lane carries, against Python integers on extreme and random operands"""
    import addb_mfz_model as mm
    import gen_addb as ga
    assert (mm.DELTA, mm.XOFF, mm.TILES, mm.RY) == (ga.MZ_DELTA, ga.MZ_XOFF, ga.MZ_TILES, ga.MZ_RY)
    rng = random.Random(23)
    for x, y in [((1 << 4096) - 1, (1 << 4096) - 1), (int('80' * 512, 16), int('7f' * 512, 16)), (0, 3)] + \
            [(rng.getrandbits(4096), rng.getrandbits(4096)) for _ in range(4)]:
        assert mm.product(x, y)[0] == x * y


def test_matrix_core_product_kernel_on_wave_emulator(monkeypatch):
    """the "mfz" build of fthe_addb_q152 (the product on the matrix cores, a measured A/B variant: bit-exact on the
    GPU, slower) on the emulator: 16 adds incl. (N - 1)^2, 0 y, 1 1 and the all-ones rows >= N"""
    import gen_addb as ga
    import wave_emu
    monkeypatch.setenv("FTHE_GEN_ADDB_DBG", "mfz")
    asm = ga.gen_addb('fthe_addb_q152')
    assert '.Lmz_ct' in asm
    rng = random.Random(29)
    n = am.rand_n(rng)
    N = n * n
    xs = [N - 1, 0, 1, (1 << 4096) - 1] + [rng.randrange(N) for _ in range(12)]
    ys = [N - 1, 5, 1, (1 << 4096) - 1] + [rng.randrange(N) for _ in range(12)]
    out = wave_emu.addb_run(n, xs, ys, asm)
    assert out == [x * y % N for x, y in zip(xs, ys)]
