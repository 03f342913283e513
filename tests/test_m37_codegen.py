"""CPU checks of the generated fthe_padic_m37 assembly (gen_padic_mfma.py) that need no GPU:

* the register budget (two waves per SIMD) and the per-squaring instruction count of the default schedule;
* the pre-flipped operand bytes: the limbs that only reach the matrix cores leave the column tails and chunk
  folds XORed with a per-limb pattern, and the packing applies only the residual byte flips.  The packing
  instructions the generator emits for Barrett 1 (T's upper half -> the q1 operand dwords) are executed here,
  one lane, on pre-flipped limbs, and must give exactly the dwords of the unflipped limbs with bit 7 of every
  byte flipped (what the i8 matrix product expects: b ^ 0x80 = b - 128);
* the v_bitop3_b32 truth tables the generator uses, under the operand order the compiler's own output shows
  (bit index = src0 << 2 | src1 << 1 | src2);
* the whole kernel, one wave on the CPU emulator (tools/wave_emu.py), against Python integers."""
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fedtree_amd", "csrc"))
import gen_padic_mfma as g  # noqa: E402

M32 = (1 << 32) - 1
PAT = (0x00808080, 0x08080808)       # limb t of a packed number (at bit 28 t): bits j with 28 t + j = 7 mod 8


def _asm():
    return g.gen_padic_mfma("fthe_padic_m37")


def _sections(asm):
    sec, out = None, {}
    for line in asm.split(".rodata")[0].splitlines():
        m = re.match(r"^(\.L\w+):", line)
        if m:
            sec = m.group(1)
            continue
        t = line.strip()
        if t and not t.startswith("."):
            out.setdefault(sec, []).append(t)
    return out


def test_register_budget_and_instruction_count():
    asm = _asm()
    nv = int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", asm).group(1))
    assert nv <= 256, nv                                   # two waves per SIMD (512 VGPRs per lane slot)
    body = asm.split(".rodata")[0]
    top = max(int(b or a) for a, b in re.findall(r"v(?:\[\d+:(\d+)\]|(\d+))", body) if (a or b))
    assert top < nv
    s = _sections(asm)
    valu = sum(1 for ins in s[".Lsqr_loop"] + s[".Lreduce"] if ins.startswith("v_") and "mfma" not in ins)
    mfma = sum(1 for ins in s[".Lreduce"] if "v_mfma" in ins)
    assert mfma == 136
    assert valu <= 4076, valu                              # round 3: 4,392 -> 4,102; round 5 (Karatsuba) 4,076


def _run(lines, regs, sregs):
    """one lane of the packing subset"""
    def val(tok):
        tok = tok.strip()
        if tok.startswith("v"):
            return regs[int(tok[1:])]
        if tok.startswith("s"):
            return sregs[int(tok[1:])]
        return int(tok, 0) & M32
    for ins in lines:
        op, rest = ins.split(None, 1)
        a = [x.strip() for x in rest.split(",")]
        d = int(a[0][1:])
        if op == "v_lshlrev_b32_e32":
            r = val(a[2]) << (val(a[1]) & 31)
        elif op == "v_lshrrev_b32_e32":
            r = val(a[2]) >> (val(a[1]) & 31)
        elif op == "v_lshl_or_b32":
            r = (val(a[1]) << (val(a[2]) & 31)) | val(a[3])
        elif op == "v_xor_b32_e32":
            r = val(a[1]) ^ val(a[2])
        elif op == "v_bfi_b32":
            r = (val(a[1]) & val(a[2])) | (~val(a[1]) & val(a[3]))
        elif op == "v_bfe_u32":
            r = (val(a[1]) >> (val(a[2]) & 31)) & ((1 << (val(a[3]) & 31)) - 1)
        elif op == "v_mov_b32_e32":
            r = val(a[1])
        else:
            raise AssertionError(f"unexpected instruction in the packing: {ins}")
        regs[d] = r & M32


def test_preflipped_q1_packing_matches_the_flipped_bytes():
    s = _sections(_asm())[".Lreduce"]
    # Barrett 1's operand packing: from the reduction's entry up to its first lane exchange
    pack = []
    for ins in s:
        if ins.startswith("v_permlane32_swap") or ins.startswith("s_nop"):
            break
        if ins.startswith("v_"):
            pack.append(ins)
    assert pack and not any("bitop3" in x for x in pack)
    K, TT, XB = 37, 100, 60
    rng = random.Random(7)
    for trial in range(200):
        limbs = [rng.getrandbits(28) for _ in range(2 * K)]
        limbs[K - 1] = rng.getrandbits(29)                 # T[36] may carry a bit 28 (u1 added)
        limbs[2 * K - 1] = rng.getrandbits(22)
        if trial == 0:
            limbs = [(1 << 28) - 1] * (2 * K)
            limbs[2 * K - 1] = (1 << 22) - 1
        regs = [0] * 256
        for i, x in enumerate(limbs):                      # T[37..73] as the product tails leave them
            regs[TT + i] = x ^ PAT[(i - (K - 1)) % 2] if i >= K else x
        _run(pack, regs, {35: (1 << 28) - 1})
        q1 = sum((limbs[K - 1 + t] & ((1 << 28) - 1 if t == 0 else M32)) << (28 * t) for t in range(K + 1))
        for w in range(34):
            want = ((q1 >> (32 * w)) & M32) ^ 0x80808080
            assert regs[XB + w] == want, (trial, w, hex(regs[XB + w]), hex(want))
        assert regs[XB + 34] == (((limbs[K - 1] >> 28) & 1) << 12 | 1)   # digit 16 c at byte 137, digit 1 at 136


def _bitop3(a, b, c, tbl):
    r = 0
    for i in range(32):
        idx = ((a >> i) & 1) << 2 | ((b >> i) & 1) << 1 | ((c >> i) & 1)
        r |= ((tbl >> idx) & 1) << i
    return r


def test_bitop3_tables():
    rng = random.Random(3)
    for _ in range(100):
        x, m, p = rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(32)
        assert _bitop3(x, m, p, 0x6A) == (x & m) ^ p               # column tail / chunk out: (x & mask) ^ pat
        assert _bitop3(x, m, p, 0xE2) == ((x ^ p) & m) ^ p         # q1 = 0 clamp on a pre-flipped limb
        assert _bitop3(m, p, x, 0x6C) == (x & m) ^ p               # hipcc's own encoding of (a & b) ^ c
    src = open(os.path.join(ROOT, "fedtree_amd", "csrc", "gen_padic_mfma.py")).read()
    assert "bitop3:0x6a" in src and "bitop3:0xe2" in src


@pytest.mark.parametrize("bits", [1009, 1030])
def test_wave_emulation_of_the_kernel(bits):
    """one wave of the generated fthe_padic_m37 on the CPU (tools/wave_emu.py: the MFMA and permlane32 lane
    maps measured on the GPU): LOADP, STOREX, SQR, MUL, STOREP = x^3 mod P^2 on 64 lanes, P at the ends of the
    kernel's range, x incl. 0, 1, P - 1, P and P^2 - 1"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import wave_emu
    assert wave_emu.m37_selftest(seed=bits, bits=bits) == 0


@pytest.mark.parametrize("bits", [1009, 1030])
def test_wave_emulation_extreme_digits(bits):
    """the squaring's Karatsuba cross term (gen_padic_mfma.py kara_cross) at the largest digits the kernel
    admits (all-ones limbs, each digit < 5P), zero halves and random digits: two squarings from raw digits"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import wave_emu
    assert wave_emu.m37_digits_selftest(seed=bits, bits=bits) == 0
    assert wave_emu.m37_digits_selftest(seed=bits, bits=bits, ab="nokara") == 0
