"""CPU checks of the P-adic kernel's arithmetic: the bit-exact model (tools/padic_model.py)
at the digit bounds, and the generated gfx950 assembly itself run on the single-lane emulator
(tools/asm_emu.py) for LOADP / SQR / MUL / STOREP against Python integers and the model."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "fedtree_amd", "csrc"))

import padic_model as pm  # noqa: E402

import pytest  # noqa: E402

K = 37


def _key(rng, bits, k=K):
    return pm.PadicKey(rng.getrandbits(bits) | (1 << (bits - 1)) | 1, k)


def test_model_products_at_digit_bounds():
    rng = random.Random(11)
    for k, bits in ((37, 1009), (37, 1024), (37, 1030), (19, 505), (19, 512), (19, 516)):
        key = _key(rng, bits, k)
        K = k
        P, P2 = key.P, key.P * key.P
        hi = pm.limbs(5 * P - 1, K)
        for a0, a1, b0, b1 in ((hi, hi, hi, hi),
                               tuple(pm.limbs(rng.randrange(5 * P), K) for _ in range(4))):
            A = pm.value(a0) + pm.value(a1) * P
            B = pm.value(b0) + pm.value(b1) * P
            z0, z1 = pm.mul(key, a0, a1, b0, b1)
            assert (pm.value(z0) + pm.value(z1) * P) % P2 == A * B % P2
            pm.check_digit(key, z0)
            pm.check_digit(key, z1)
            z0, z1 = pm.sqr(key, a0, a1)
            assert (pm.value(z0) + pm.value(z1) * P) % P2 == A * A % P2
            pm.check_digit(key, z0)
            pm.check_digit(key, z1)


@pytest.mark.parametrize("K,bits", [(37, 1024), (19, 512)])
def test_generated_assembly_on_emulator(K, bits):
    from asm_emu import Emu, M32
    from gen_padic import gen_padic
    asm = gen_padic(K, 28, f"fthe_padic_k{K}")
    rng = random.Random(5)
    key = _key(rng, bits, K)
    P, P2 = key.P, key.P * key.P
    S, L = 2 * K, 256
    KA, CTX, PROG, SLOTS = 0x100, 0x1000, 0x2000, 0x100000
    X, Y = rng.randrange(P2), rng.randrange(P2)
    # LOADP 0 -> STOREX 2; LOADP 1 -> MUL 2 -> SQR 1 -> STOREX 3; STOREP 4
    prog = [22, 0, 2, 2, 22, 1, 4, 2, 3, 1, 2, 3, 23, 4, 0, 0]
    em = Emu(asm)
    for i, v in enumerate([SLOTS, 0, PROG, 0, CTX, 0, L * 4, S * L * 4, L, 0]):
        em.mem[KA + 4 * i] = v
    pad = ((20 + K + 3) & ~3) - 20 - K                          # zero words before mu (gen_padic.py)
    for i, w in enumerate([(-x) & M32 for x in pm.limbs(P, K)] + [0] * pad + key.mu):
        em.mem[CTX + 4 * i] = w
    for i, w in enumerate(prog):
        em.mem[PROG + 4 * i] = w
    for slot, val in ((0, X), (1, Y)):
        for k, limb in enumerate(pm.limbs(val, S)):
            em.mem[SLOTS + slot * S * L * 4 + k * L * 4] = limb
    em.s[0], em.s[1], em.s[2] = KA, 0, 0
    em.v[0] = 0
    em.run(f"fthe_padic_k{K}")
    rd = lambda slot: [em.mem.get(SLOTS + slot * S * L * 4 + k * L * 4, 0) for k in range(S)]
    x0, x1 = pm.loadp(key, X)
    assert rd(2) == x0 + x1                                    # raw digits of LOADP, as the model's
    y0, y1 = pm.loadp(key, Y)
    z0, z1 = pm.sqr(key, *pm.mul(key, y0, y1, x0, x1))
    assert rd(3) == z0 + z1                                    # MUL then SQR, limb for limb
    out = pm.value(rd(4))
    assert out % P2 == (X * Y) ** 2 % P2 and out < 6 * P2      # STOREP: x0 + x1 P


def test_gathered_table_products_on_emulator():
    """LOADXGD / MULGD (8-bit and 16-bit digits): table entries in the register-bank layout
    (x0 limbs, pad, x1 limbs, pad) gathered by a per-lane digit, multiplied as the model does."""
    from asm_emu import Emu, M32
    from gen_padic import gen_padic
    K = 37
    KB = K + (K & 1)
    EW = 2 * KB
    asm = gen_padic(K, 28, "fthe_padic_k37")
    rng = random.Random(9)
    key = _key(rng, 1024, K)
    P = key.P
    S, L = 2 * K, 256
    KA, CTX, PROG, SLOTS, TAB, DIG = 0x100, 0x1000, 0x2000, 0x100000, 0x4000000, 0x8000000
    for wide in (False, True):
        W = 16 if wide else 8
        d0, d1 = rng.randrange(1 << W), rng.randrange(1 << W)
        e0 = [pm.limbs(rng.randrange(5 * P), K) for _ in range(2)]
        e1 = [pm.limbs(rng.randrange(5 * P), K) for _ in range(2)]
        em = Emu(asm)
        for i, v in enumerate([SLOTS, 0, PROG, 0, CTX, 0, L * 4, S * L * 4, L, 0, TAB, 0, DIG, 0]):
            em.mem[KA + 4 * i] = v
        for i, w in enumerate([(-x) & M32 for x in pm.limbs(P, K)] + [0, 0, 0] + key.mu):
            em.mem[CTX + 4 * i] = w
        code = 16 if wide else 14
        for i, w in enumerate([code, 0, code + 1, 1, 2, 2, 0, 0]):     # LOADXGD 0; MULGD 1; STOREX 2
            em.mem[PROG + 4 * i] = w
        for j, (d, (x0, x1)) in enumerate(((d0, e0), (d1, e1))):
            base = TAB + ((j << W) | d) * EW * 4
            for k, limb in enumerate(x0 + [0] + x1 + [0]):
                em.mem[base + 4 * k] = limb
            # digit of lane 0 for window j: byte / halfword at DIG + j*L*size
            sz = 2 if wide else 1
            a = DIG + j * L * sz
            em.mem[a & ~3] = (em.mem.get(a & ~3, 0) & ~((0xffff if wide else 0xff) << (8 * (a & 3)))) | (d << (8 * (a & 3)))
        em.s[0], em.s[1], em.s[2] = KA, 0, 0
        em.v[0] = 0
        em.run("fthe_padic_k37")
        out = [em.mem.get(SLOTS + 2 * S * L * 4 + k * L * 4, 0) for k in range(S)]
        z0, z1 = pm.mul(key, e0[0], e0[1], e1[0], e1[1])
        assert out == z0 + z1, wide
