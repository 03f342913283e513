#!/usr/bin/env python3
"""Generator of the n-adic public-key encrypt kernel with matrix-core Barrett reductions (gfx950 assembly):
fthe_nadic_b76, r^n mod n^2 for the parties' encrypt (Party::encrypt_histogram, party.h:118-142 ->
paillier.cpp:122-139) with X = x0 + x1 n kept as two base-n digits, one ciphertext per quad of lanes, for n
of 2041..2048 bits.  tools/nadicb_model.py is the bit-exact model of the arithmetic (Barrett cut points, bias,
column corrections, chunked normalisation, every bound); this file lays it out on the machine.

A product X Y (a squaring, or a general product with digits y0, y1 from a slot) is
  1. the VALU pass: z1 = x0 y0 and z2 = x0 y1 + x1 y0 (SQR: x0^2 and 2 x0 x1) by operand scanning over the
     76 multiplier limbs, two rings of 64-bit columns (19 v_mad_u64_u32 per lane and window per step; no
     reduction inside: the per-step overhead is the split of each window's lowest column, the hand-off of its
     low 27 bits one lane down and the retirement of lane 0's limb into the A-column row it has consumed);
  2. z1, z2 -> dwords in the add kernel's quad layout (lane j: dwords [32 j, 32 j + 32), lane 3 also dword 128):
     the retired low limbs from LDS on lanes 0, 1, the window's limbs moved to lanes 2, 3 by DPP;
  3. Barrett 1 on z1 (quotient AND remainder) and Barrett 2 on z2 + q3_1 (remainder only), each two i8 matrix
     products with a constant operand -- q1 mu (17 tiles, 61 MFMAs) and q3 n (17 tiles, 45 MFMAs) on
     v_mfma_i32_16x16x64_i8 over the wave's 16 ciphertexts -- exactly the scheme of the add kernel
     (gen_addb.py: byte-shifted constant copies in LDS, -128 offset corrections as srcC, int64 groups, chunked
     signed normalisation), at 2048 bits;
  4. r = (z - q3 n) mod 2^2080 in [0, 3n) becomes the new digit's 27-bit limbs through a staging row.
Digits stay in [0, 3n) between products (no conditional subtraction); CANON reduces them at the end.
The q1 mu / q3 n multiply-adds the Montgomery form (fthe_nadic_m76) runs on the VALU -- half of its 76 per
step -- go to the matrix cores.

Ops (uint32 pairs, bn_host.hpp Prog; the classical n-adic program of fthe_nadic_q76):
    0 END, 1 LOADX slot, 2 STOREX slot, 3 SQR count, 4 MUL slot, 20 CANON
Kernel arguments: those of gen_montprog.py (slots, prog, ctx, limb stride, slot stride); ctx = the LDS image
(IMG_BYTES: mu copies, n copies, corrections; nadicb_image.hpp) then n as 76 limbs of 27 bits (N_OFF).
Workgroups of WAVES waves (12: one per CU, 3 waves per SIMD; the image is loaded into LDS once per CU), 16
ciphertexts per wave: the launch covers L ciphertexts with L a multiple of 16 * WAVES.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_montprog import _descriptor  # noqa: E402

S, Q, B = 76, 19, 27
MASK = (1 << B) - 1
WAVES = int(os.environ.get("FTHE_GEN_NADICB_WAVES", "12"))   # timing builds only (FTHE_GEN_*: never in-tree)
CT_PER_WAVE = 16
RB = 76                          # A-column row: 16 ciphertexts x 4 B + pad; 19 dwords: a quad's four write_rows
                                 # lanes 19 x 19 k = 9 k dwords apart (68 B rows: 3 k, 2- to 3-way conflicts) and
                                 # to_dwords' two lanes 18 apart (tools/lds_conflicts.py)
ROWS = 2 * S                     # rows 0..75: y0 / x0 (then z1's retired limbs), 76..151: y1 (then z2's)
# ---- Barrett constants (tools/nadicb_model.py) -------------------------------------------------------------
A_BITS, C_BITS = 2016, 2112
NZ = 129
Q1_DW0 = A_BITS // 32            # 63
NQ1, NQ3 = NZ - Q1_DW0, 65       # 66, 65
S1_BASE = 260
TILES1, TILES2 = 17, 17
KB1, KB2 = 5, 5
BIAS_COL, BIAS_DIGIT = 263, -1
ND1, ND2 = 262, 257
CHUNKS = (tuple(range(0, 8)), tuple(range(8, 16)), (16,))


def band(nd, s0, k0):
    lo, hi = s0 - k0 - 63, s0 + 15 - k0
    return not (hi < 0 or lo >= nd)


ACT1 = [[kb for kb in range(KB1) if band(ND1, S1_BASE + 16 * t, 64 * kb)] for t in range(TILES1)]
ACT2 = [[kb for kb in range(KB2) if band(ND2, 16 * t, 64 * kb)] for t in range(TILES2)]
# copy offsets: the A read of tile t, K-block kb, lane half h is at KO + 16 (4 kb - t) + 16 h of row m's copy
KO1 = 16 * max(t - 4 * kb for t in range(TILES1) for kb in ACT1[t])
KO2 = 16 * max(t - 4 * kb for t in range(TILES2) for kb in ACT2[t])
_span = max(KO1 + 16 * max(4 * kb - t for t in range(TILES1) for kb in ACT1[t]),
            KO2 + 16 * max(4 * kb - t for t in range(TILES2) for kb in ACT2[t])) + 64
COPY = 32 + 256 * ((_span - 32 + 255) // 256)        # == 32 mod 256: the b128 lane groups hit distinct banks
A1_OFF = 0
A2_OFF = 16 * COPY
CORR1_OFF = 32 * COPY
CORR2_OFF = CORR1_OFF + TILES1 * 64
IMG_BYTES = CORR2_OFF + TILES2 * 64
N_OFF = IMG_BYTES                                     # n limbs (76 x u32) in ctx, not copied to LDS
CTX_BYTES = N_OFF + 4 * S
QROW = 400                       # q / r staging row: 80 dwords used; 100 dwords == 4 mod 32 (4-way stores:
                                 # the quad layout's lanes 32 dwords apart; 416 would free the B reads but make
                                 # the 32-lane ds_write_b32 8-way, tools/lds_conflicts.py)
GROW = 568                       # group staging row: a product's 68 int64 groups (every chunk at once); 142
                                 # dwords == 2 (mod 4): the folds' 16-lane ds_write_b64 hit 32 distinct banks
CSTRIDE = 264                    # chunk k's groups at 264 k: with GROW = 568 the normalisation's ds_read_b64
                                 # are conflict-free too (16-byte rows for ds_read_b128 cannot give conflict-free
                                 # writes; tools/lds_conflicts.py)
QST_OFF = 0                      # staging areas inside the wave area (the A column is dead in the Barretts); the
GST_OFF = 0                      # groups overlap the q staging, which the B operands have left before the MFMAs
WAVE_AREA = max(ROWS * RB, QST_OFF + 16 * QROW, GST_OFF + 16 * GROW)
M_A = (0, 1, 2, 3, 12, 13, 14, 15)
M_B = (4, 5, 6, 7, 8, 9, 10, 11)
assert IMG_BYTES % 16 == 0 and WAVE_AREA % 16 == 0 and (QROW // 4) % 32 == 4


def lds_bytes(waves=WAVES):
    """the image, the wave areas and the workgroup's batch counter (one dword, 16-byte slot)"""
    return IMG_BYTES + waves * WAVE_AREA + 16


assert lds_bytes() <= 160 * 1024


def copy_slot(m):
    return M_A.index(m) if m in M_A else 8 + M_B.index(m)


def layout_header():
    """gen/nadicb_layout.h: the constants of the host image builder (nadicb_image.hpp) and launcher"""
    vals = dict(kNbA=A_BITS, kNbC=C_BITS, kNbNd1=ND1, kNbNd2=ND2, kNbS1Base=S1_BASE, kNbTiles1=TILES1,
                kNbTiles2=TILES2, kNbNq1=NQ1, kNbNq3=NQ3, kNbBiasCol=BIAS_COL, kNbBiasDigit=BIAS_DIGIT,
                kNbKO1=KO1, kNbKO2=KO2, kNbCopy=COPY, kNbA1Off=A1_OFF, kNbA2Off=A2_OFF, kNbCorr1Off=CORR1_OFF,
                kNbCorr2Off=CORR2_OFF, kNbImgBytes=IMG_BYTES, kNbNOff=N_OFF, kNbCtxBytes=CTX_BYTES,
                kNbWaves=WAVES, kNbPerWg=WAVES * CT_PER_WAVE, kNbLdsBytes=lds_bytes())
    lines = ["// generated by fedtree_amd/build.py from gen_nadicb.py -- layout of fthe_nadic_b76", "#pragma once"]
    lines += [f"constexpr int {k} = {v};" for k, v in vals.items()]
    return "\n".join(lines) + "\n"


def gen_nadicb(name: str, waves: int = WAVES) -> str:
    # timing-only switches (wrong results; fedtree_amd/build.py never lets FTHE_GEN_* reach the in-tree library):
    # noprod (no VALU product steps), nobarrett (no reductions), nomfma (no MFMAs), noconv (no z -> dword moves),
    # nonorm (no group normalisation)
    DBG = set(os.environ.get("FTHE_GEN_NADICB_DBG", "").split(","))
    DPP = "row_mask:0xf bank_mask:0xf"
    LDSB = lds_bytes(waves)
    LDS_CNT = LDSB - 16                 # the workgroup's batch counter
    # ---- VGPRs ---------------------------------------------------------------------------------------------
    V_LANE = 0                        # lane (0..63) * 4 after the prologue (tid at entry)
    V_ROW, V_LDSI, V_LDSW, V_SH = 1, 2, 3, 4     # (g, k) slot code; A column base; lane k's row base; 2 k
    V_A1, V_A2, V_C, V_B, V_G, V_GR, V_QW = 5, 6, 7, 8, 9, 10, 11
    V_TMP = 12                        # pair 12:13
    X0B, X1B = 14, 33                 # digit limbs (19 each)
    T1B, T2B = 52, 96                 # two rings of NT 64-bit columns (product pass)
    NT = Q + 3                        # even: the a_i double buffer keeps its parity across trips
    V_AI, V_BI, V_A2X = (140, 141), (142, 143), 144
    # Barrett-phase plan (the product registers are dead): z dwords, MFMA operands, fold / norm scratch
    Z1B, Z2B = 14, 47                 # 33 dwords each (lane 3's dword 128 in local 32)
    BQ = 80                           # B operands, KB x 4 = v80..v99
    ACC = (100, 104)                  # two accumulator sets (the third of the MFMA phase: GB)
    AOP = (108, 112, 116, 120)        # four A-operand buffers (reads two MFMAs ahead, as gen_addb)
    DQ = 124                          # chunk dwords v124..v155 (the carry rides in DQ + g + 1 until g + 1 is done)
    GB = 156                          # group read buffers: 2 x (2 int64) = v156..v163, ds_read_b128 each
    PG = FV = 164                     # int64 pair (the fold's group; the normalisation's odd-group sum)
    ACCS = ACC + (GB,) if "acc2" not in DBG else ACC   # MFMA accumulator sets (GB is free until the norm)
    NACC = len(ACCS)
    XDL_WAIT = 19                     # wait states after an MFMA before a VALU reads its result (as before)
    CR = 166                          # chunk carry
    NVGPR = 168
    assert T2B + 2 * NT <= V_AI[0] and V_A2X < NVGPR
    # conversion / CANON scratch (product registers dead or not yet live)
    # z -> dwords conversions run in place on 38 limbs: z1 at Z1B (the digits are dead), z2 at Z2B (z1's
    # window, dead by then); z2's window (the T2 ring) is read by DPP while z1 converts
    NV, DD = 80, 100                  # CANON: n's quarter (19), difference (19)
    YT = 52                           # MUL: the y digits loaded from the slot (38, ring area)

    def pair(n):
        return f"v[{n}:{n + 1}]"

    def quad4(n):
        return f"v[{n}:{n + 3}]"

    def X0(k):
        return f"v{X0B + k}"

    def X1(k):
        return f"v{X1B + k}"

    tmp = pair(V_TMP)
    # ---- SGPRs ---------------------------------------------------------------------------------------------
    # s[0:1] kernarg, s2 wg id, s[4:5] slots, s[6:7] prog, s[8:9] ctx, s10 limb stride, s11 slot stride,
    # s[14:15] op / arg, s[16:17] address scratch, s18 trip counter, s19 SQR counter, lane masks s[20:21] quad
    # lane 3, s[22:23] lane 0, s[24:25] lane 1, s[26:27] lane 2, s[28:29] lanes 0-1, s30 = 256, s31 = 65536,
    # s32 = 2^24, s33 = 0x80808080, s[34:35] saved exec, s36 ctx lo + N_OFF, s[40:41] the program's first op,
    # s42 workgroups launched, s43 batches of 16 ciphertexts, s44 scratch
    LANE_MASK = {3: "s[20:21]", 0: "s[22:23]", 1: "s[24:25]", 2: "s[26:27]"}
    NSGPR = 72 if "stamp" in DBG else 46

    o = []
    e = o.append
    e('.amdgcn_target "amdgcn-amd-amdhsa--gfx950"')
    e('.amdhsa_code_object_version 5')
    e('.text')
    e(f'.globl {name}')
    e('.p2align 8')
    e(f'.type {name},@function')
    e(f'{name}:')
    e('  s_load_dwordx2 s[4:5], s[0:1], 0x0')
    e('  s_load_dwordx2 s[6:7], s[0:1], 0x8')
    e('  s_load_dwordx2 s[8:9], s[0:1], 0x10')
    e('  s_load_dwordx2 s[10:11], s[0:1], 0x18')
    for j, pat in ((3, 0x88888888), (0, 0x11111111), (1, 0x22222222), (2, 0x44444444)):
        lo, hi = LANE_MASK[j][2:-1].split(':')
        e(f'  s_mov_b32 s{lo}, {hex(pat)}')
        e(f'  s_mov_b32 s{hi}, {hex(pat)}')
    e('  s_mov_b32 s28, 0x33333333')
    e('  s_mov_b32 s29, 0x33333333')
    e('  s_movk_i32 s30, 0x100')
    e('  s_mov_b32 s31, 0x10000')
    e('  s_mov_b32 s32, 0x1000000')
    e('  s_mov_b32 s33, 0x80808080')
    e('  s_waitcnt lgkmcnt(0)')
    # ---- constant image -> LDS: every thread copies 16 B per pass -----------------------------------------
    e(f'  v_lshlrev_b32_e32 v{V_ROW}, 4, v{V_LANE}')
    per = 64 * waves * 16
    for p in range((IMG_BYTES + per - 1) // per):
        off = p * per
        part = off + per > IMG_BYTES
        if part:
            e(f'  v_cmp_gt_u32_e32 vcc, {hex(IMG_BYTES - off)}, v{V_ROW}')
            e('  s_and_saveexec_b64 s[34:35], vcc')
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(off)}, v{V_ROW}')
        e(f'  global_load_dwordx4 v[{X0B}:{X0B + 3}], v{V_LDSI}, s[8:9]')
        e('  s_waitcnt vmcnt(0)')
        e(f'  ds_write_b128 v{V_LDSI}, v[{X0B}:{X0B + 3}]')
        if part:
            e('  s_mov_b64 exec, s[34:35]')
    e(f'  v_cmp_eq_u32_e32 vcc, 0, v{V_LANE}')                            # thread 0: batch counter = 0
    e('  s_and_saveexec_b64 s[34:35], vcc')
    e(f'  v_mov_b32_e32 v{V_TMP}, {hex(LDS_CNT)}')
    e(f'  v_mov_b32_e32 v{V_TMP + 1}, 0')
    e(f'  ds_write_b32 v{V_TMP}, v{V_TMP + 1}')
    e('  s_mov_b64 exec, s[34:35]')
    e('  s_load_dwordx2 s[42:43], s[0:1], 0x20')                         # live ciphertexts, workgroups launched
    e('  s_waitcnt lgkmcnt(0)')
    e('  s_barrier')
    # desyncN (timing knob): the waves w, w + 4, w + 8 of a workgroup share a SIMD; the second and third start
    # N and 2N s_sleep 127 (~8K cycles each) late, so their matrix phases meet the others' product passes.
    # Measured neutral to slower (659-661 vs 657.6-658.1 ms per 393,216, profiles/r05t_nadicb_desync_ab.jsonl):
    # the persistent waves' batch draws already spread their phases, so off
    DSN = next((int(t[6:]) for t in DBG if t.startswith('desync') and t[6:].isdigit()), 0)
    if DSN:
        e(f'  v_readfirstlane_b32 s44, v{V_LANE}')
        e('  s_lshr_b32 s44, s44, 8')                                         # wave / 4 = slot on its SIMD
        for k in (1, 2):
            e(f'  s_cmp_lt_u32 s44, {k}')
            e(f'  s_cbranch_scc1 .Ldesync_{k}')
            for _ in range(DSN):
                e('  s_sleep 127')
            e(f'.Ldesync_{k}:')
    e('// @stampinit')
    e('  s_add_u32 s44, s42, 15')
    e('  s_lshr_b32 s44, s44, 4')                                         # batches of 16 ciphertexts
    e('  s_mov_b32 s42, s43')
    e('  s_mov_b32 s43, s44')
    e('  s_mov_b64 s[40:41], s[6:7]')
    # ---- per-lane constants ----------------------------------------------------------------------------------
    e(f'  v_lshrrev_b32_e32 v{V_TMP}, 6, v{V_LANE}')                    # wave
    e(f'  v_mul_u32_u24_e32 v{V_TMP}, {WAVE_AREA}, v{V_TMP}')
    e(f'  v_add_u32_e32 v{V_TMP}, {IMG_BYTES}, v{V_TMP}')              # wave area base
    e(f'  v_mov_b32_e32 v{V_A2X}, v{V_TMP}')                           # (kept for V_G, V_B below)
    e(f'  v_and_b32_e32 v{V_LANE}, 63, v{V_LANE}')                     # lane
    e(f'  v_lshrrev_b32_e32 v{V_TMP + 1}, 2, v{V_LANE}')               # c (ciphertext of the wave)
    e(f'  v_lshl_add_u32 v{V_LDSI}, v{V_TMP + 1}, 2, v{V_TMP}')        # area + 4 c
    e(f'  v_mul_u32_u24_e32 v{V_QW}, {QROW}, v{V_TMP + 1}')
    e(f'  v_add_u32_e32 v{V_QW}, v{V_QW}, v{V_TMP}')                   # staging row of c (QST_OFF = 0)
    e(f'  v_mul_u32_u24_e32 v{V_GR}, {GROW}, v{V_TMP + 1}')
    e(f'  v_add_u32_e32 v{V_GR}, v{V_GR}, v{V_TMP}')
    e(f'  v_add_u32_e32 v{V_GR}, {GST_OFF}, v{V_GR}')                 # group row of c
    e(f'  v_and_b32_e32 v{V_SH}, 3, v{V_LANE}')                        # k
    e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {CSTRIDE}, v{V_SH}')
    e(f'  v_add_u32_e32 v{V_GR}, v{V_GR}, v{V_TMP + 1}')               # + CSTRIDE k: quad lane k's chunk (norm reads)
    e(f'  v_and_b32_e32 v{V_SH}, 3, v{V_LANE}')                        # k (quad lane)
    e(f'  v_mul_u32_u24_e32 v{V_LDSW}, {Q * RB}, v{V_SH}')
    e(f'  v_add_u32_e32 v{V_LDSW}, v{V_LDSW}, v{V_LDSI}')              # area + 4 c + 19 k RB
    # MFMA layout: lane l, m = l & 15 (B column: ciphertext), h = l >> 4
    e(f'  v_and_b32_e32 v{V_TMP + 1}, 15, v{V_LANE}')                  # m
    e(f'  v_lshrrev_b32_e32 v{V_B}, 4, v{V_LANE}')
    e(f'  v_lshlrev_b32_e32 v{V_B}, 4, v{V_B}')                        # 16 h
    e(f'  v_add_u32_e32 v{V_A1}, 4, v{V_TMP + 1}')
    e(f'  v_subrev_u32_e32 v{V_A2}, 8, v{V_TMP + 1}')
    e(f'  v_cmp_gt_u32_e32 vcc, 12, v{V_TMP + 1}')
    e(f'  v_cndmask_b32_e32 v{V_A1}, v{V_A2}, v{V_A1}, vcc')
    e(f'  v_cmp_gt_u32_e32 vcc, 4, v{V_TMP + 1}')
    e(f'  v_cndmask_b32_e32 v{V_A1}, v{V_A1}, v{V_TMP + 1}, vcc')      # copy slot of row m
    e(f'  v_mul_u32_u24_e32 v{V_A1}, {COPY}, v{V_A1}')
    e(f'  v_add_u32_e32 v{V_A1}, v{V_A1}, v{V_B}')                     # slot*COPY + 16 h
    e(f'  v_add_u32_e32 v{V_A2}, {A2_OFF}, v{V_A1}')
    e(f'  v_add_u32_e32 v{V_C}, {CORR1_OFF}, v{V_B}')                  # corrections + 16 h
    e(f'  v_lshrrev_b32_e32 v{V_G}, 1, v{V_B}')                        # 8 h
    e(f'  v_mul_u32_u24_e32 v{V_TMP}, {GROW}, v{V_TMP + 1}')
    e(f'  v_add_u32_e32 v{V_G}, v{V_G}, v{V_TMP}')
    e(f'  v_add_u32_e32 v{V_G}, {GST_OFF}, v{V_G}')                   # group row m + 8 h (area added below)
    e(f'  v_mul_u32_u24_e32 v{V_TMP}, {QROW}, v{V_TMP + 1}')
    e(f'  v_add_u32_e32 v{V_B}, v{V_B}, v{V_TMP}')                    # staging row m + 16 h (area below)
    e(f'  v_add_u32_e32 v{V_G}, v{V_G}, v{V_A2X}')                    # + the wave's area
    e(f'  v_add_u32_e32 v{V_B}, v{V_B}, v{V_A2X}')
    e(f'  v_lshlrev_b32_e32 v{V_SH}, 1, v{V_SH}')                      # 2 k
    e(f'  v_lshlrev_b32_e32 v{V_LANE}, 7, v{V_LANE}')                  # lane * 128: ROW = g*512 + k*128
    if "ldsfree" in DBG:
        # timing knock-out (wrong results): the staging / group addresses spread so that no LDS access of the
        # Barrett phases has a bank conflict -- the same instructions at conflict-free addresses (the potential
        # of a conflict-free staging layout)
        e(f'  v_lshrrev_b32_e32 v{V_TMP}, 7, v{V_LANE}')                 # lane
        e(f'  v_lshl_add_u32 v{V_QW}, v{V_TMP}, 3, v{V_A2X}')            # area + 8 lane (+ 128 k at the sites)
        e(f'  v_lshl_add_u32 v{V_B}, v{V_TMP}, 4, v{V_A2X}')             # area + 16 lane
        e(f'  v_lshl_add_u32 v{V_G}, v{V_TMP}, 3, v{V_A2X}')             # area + 8 lane
        e(f'  v_lshl_add_u32 v{V_GR}, v{V_TMP}, 4, v{V_A2X}')            # area + 16 lane
    e('  s_add_u32 s36, s8, ' + hex(N_OFF))
    e('  s_addc_u32 s37, s9, 0')

    # ---- persistent waves: workgroup wg owns the batches wg, wg + nwg, ... of 16 ciphertexts; its waves draw
    #      them from the LDS counter (a wave the SIMD's arbiter favours runs more of them, as fthe_addb_q152),
    #      and run the whole program on each (the END op draws the next) ----------------------------------------
    e('// @phase batch')
    e('.Lnext_batch:')
    e('  s_mov_b64 exec, 1')
    e(f'  v_mov_b32_e32 v{V_TMP}, {hex(LDS_CNT)}')
    e(f'  v_mov_b32_e32 v{V_TMP + 1}, 1')
    e(f'  ds_add_rtn_u32 v{V_TMP}, v{V_TMP}, v{V_TMP + 1}')
    e('  s_waitcnt lgkmcnt(0)')
    e('  s_mov_b64 exec, -1')
    e('  s_nop 1')
    e(f'  v_readfirstlane_b32 s44, v{V_TMP}')
    e('  s_mul_i32 s44, s44, s42')
    e('  s_add_u32 s44, s44, s2')                                          # batch
    e('  s_cmp_ge_u32 s44, s43')
    e('  s_cbranch_scc1 .Lend')
    e('  s_lshl_b32 s44, s44, 13')                                         # 16 ciphertexts x 512
    e(f'  v_add_u32_e32 v{V_ROW}, s44, v{V_LANE}')
    e('  s_mov_b64 s[6:7], s[40:41]')
    e('.Lprog:')
    e('// @phase ops')
    e('  s_load_dwordx2 s[14:15], s[6:7], 0x0')
    e('  s_add_u32 s6, s6, 8')
    e('  s_addc_u32 s7, s7, 0')
    e('  s_waitcnt lgkmcnt(0)')
    for code, lab in ((1, '.Lloadx'), (2, '.Lstorex'), (3, '.Lsqr'), (4, '.Lmul'), (20, '.Lcanon')):
        e(f'  s_cmp_eq_u32 s14, {code}')
        e(f'  s_cbranch_scc1 {lab}')
    e('  s_branch .Lnext_batch')

    # ---- slot access: limb j of this lane's quarter of digit d at slot limb d*S + k*Q + j ---------------
    def slot_addr():
        e('  s_mul_i32 s16, s15, s11')
        e('  s_mul_hi_u32 s17, s15, s11')
        e('  s_add_u32 s16, s4, s16')
        e('  s_addc_u32 s17, s5, s17')

    def step_addr(times=None):
        if times is None:
            e('  s_add_u32 s16, s16, s10')
        else:
            e(f'  s_mul_i32 s14, s10, {times}')
            e('  s_add_u32 s16, s16, s14')
        e('  s_addc_u32 s17, s17, 0')

    def goff(dst):
        e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')            # g
        e(f'  v_lshlrev_b32_e32 v{V_TMP}, 2, v{V_TMP}')            # g*4
        e(f'  v_bfe_u32 v{V_TMP + 1}, v{V_ROW}, 7, 2')             # k
        e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {Q}, v{V_TMP + 1}')  # k*Q
        e(f'  v_mul_lo_u32 v{V_TMP + 1}, v{V_TMP + 1}, s10')       # k*Q*L*4
        e(f'  v_add_u32_e32 v{dst}, v{V_TMP}, v{V_TMP + 1}')

    V_GO = V_AI[0]

    def digits_io(d0, d1, store):
        goff(V_GO)
        slot_addr()
        for dig, f in enumerate((d0, d1)):
            for j in range(Q):
                if store:
                    e(f'  global_store_dword v{V_GO}, {f(j)}, s[16:17]')
                else:
                    e(f'  global_load_dword {f(j)}, v{V_GO}, s[16:17]')
                if j != Q - 1:
                    step_addr()
            if dig == 0:
                step_addr(S - Q + 1)
        e('  s_waitcnt vmcnt(0)')

    # ---- quad helpers -----------------------------------------------------------------------------------
    def ripple_quad(lab, vals, nv, signed=False, width=B):
        """vals(k) limbs (k < nv) of `width` bits, this lane's pending 64-bit carry-out in tmp: carries move to
        the next lane's limb 0 (lane 0 gets none) and ripple until none is left; lane 3's is dropped"""
        shr = 'v_ashrrev_i64' if signed else 'v_lshrrev_b64'
        a0, a1 = V_AI
        e(f'{lab}_loop:')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{a0}, v{V_TMP} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_mov_b32_dpp v{a1}, v{V_TMP + 1} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, v{a0}, 0, s[22:23]')
        e(f'  v_cndmask_b32_e64 v{V_TMP + 1}, v{a1}, 0, s[22:23]')
        e(f'  v_or_b32_e32 v{a0}, v{V_TMP}, v{V_TMP + 1}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{a0}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        for k in range(nv):
            e(f'  v_mad_u64_u32 {tmp}, vcc, {vals(k)}, 1, {tmp}')
            e(f'  v_and_b32_e32 {vals(k)}, {hex((1 << width) - 1)}, v{V_TMP}')
            e(f'  {shr} {tmp}, {width}, {tmp}')
            if k == 1 and nv > 2:                # a carry absorbed by limbs 0, 1 everywhere (the usual case):
                e(f'  v_or_b32_e32 v{a0}, v{V_TMP}, v{V_TMP + 1}')   # no carry-out changes, nothing to hand on
                e(f'  v_cmp_ne_u32_e32 vcc, 0, v{a0}')
                e('  s_nop 4')
                e(f'  s_cbranch_vccz {lab}_done')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    def canon_once(X, tag):
        """X (19 normalised limbs per lane, < 2^2052) -> X - n when X >= n, across the quad; leaves vcc =
        (X was >= n) on every lane.  n's quarter in NV, scratch DD."""
        bo, fin, t1 = f"v{V_AI[0]}", f"v{V_AI[1]}", f"v{V_TMP}"
        for j in range(Q):
            e(f'  v_sub_u32_e32 v{DD + j}, {X(j)}, v{NV + j}')
            if j:
                e(f'  v_add_u32_e32 v{DD + j}, v{DD + j}, {bo}')
            e(f'  v_ashrrev_i32_e32 {bo}, 31, v{DD + j}')
            e(f'  v_and_b32_e32 v{DD + j}, {hex(MASK)}, v{DD + j}')
        e(f'  v_mov_b32_e32 {fin}, 0')
        lab = f'.L{tag}_borrow'
        e(f'{lab}_loop:')
        e(f'  v_cndmask_b32_e64 {t1}, 0, {bo}, s[20:21]')
        e(f'  v_or_b32_e32 {fin}, {fin}, {t1}')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp {t1}, {bo} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 {bo}, {t1}, 0, s[22:23]')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, {bo}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        for j in range(Q):
            e(f'  v_add_u32_e32 v{DD + j}, v{DD + j}, {bo}')
            e(f'  v_ashrrev_i32_e32 {bo}, 31, v{DD + j}')
            e(f'  v_and_b32_e32 v{DD + j}, {hex(MASK)}, v{DD + j}')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp {t1}, {fin} quad_perm:[3,3,3,3] {DPP}')
        e(f'  v_cmp_eq_u32_e32 vcc, 0, {t1}')
        for j in range(Q):
            e(f'  v_cndmask_b32_e32 {X(j)}, {X(j)}, v{DD + j}, vcc')

    # ---- LOADX / STOREX / CANON ---------------------------------------------------------------------------
    e('.Lloadx:')
    digits_io(X0, X1, False)
    e('  s_branch .Lprog')
    e('.Lstorex:')
    digits_io(X0, X1, True)
    e('  s_branch .Lprog')

    e('.Lcanon:')
    # n's quarter: limbs [19 k, 19 k + 19) from ctx + N_OFF
    e(f'  v_bfe_u32 v{V_TMP}, v{V_ROW}, 7, 2')
    e(f'  v_mul_u32_u24_e32 v{V_TMP}, {4 * Q}, v{V_TMP}')
    for j in range(Q):
        e(f'  global_load_dword v{NV + j}, v{V_TMP}, s[36:37] offset:{4 * j}')
    e('  s_waitcnt vmcnt(0)')
    # x0 in [0, 3n): two rounds, each carrying 1 into x1 (digit bound: x1 + 2 < 3n + 2 -> three rounds)
    for rnd in range(2):
        canon_once(X0, f'cx0{rnd}')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, 1, vcc')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, v{V_TMP}, s[22:23]')           # lane 0 only
        e(f'  v_add_u32_e32 {X1(0)}, {X1(0)}, v{V_TMP}')
        e(f'  v_mov_b64_e32 {tmp}, 0')
        for k in range(Q):
            e(f'  v_mad_u64_u32 {tmp}, vcc, {X1(k)}, 1, {tmp}')
            e(f'  v_and_b32_e32 {X1(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
        ripple_quad(f'.Lcr{rnd}', X1, Q)
    for rnd in range(3):
        canon_once(X1, f'cx1{rnd}')
    e('  s_branch .Lprog')

    # ---- A operand -> LDS -------------------------------------------------------------------------------
    def write_rows(src, row0):
        for k in range(Q):
            e(f'  ds_write_b32 v{V_LDSW}, {src(k)} offset:{(row0 + k) * RB}')
        e('  s_waitcnt lgkmcnt(0)')

    e('.Lmul:')
    digits_io(lambda j: f"v{YT + j}", lambda j: f"v{YT + Q + j}", False)
    write_rows(lambda j: f"v{YT + j}", 0)
    write_rows(lambda j: f"v{YT + Q + j}", S)
    e('  s_mov_b32 s19, 0')
    e('  s_branch .Lprod_mul')

    e('.Lsqr:')
    e('  s_mov_b32 s19, s15')
    e('.Lsqr_loop:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    write_rows(X0, 0)
    e('  s_branch .Lprod_sq')

    # ---- the product pass (two windows, LSB-first operand scanning) ---------------------------------------
    def T(tb, k):
        k %= NT
        return f"v[{tb + 2 * k}:{tb + 2 * k + 1}]"

    def Tlo(tb, k):
        return f"v{tb + 2 * (k % NT)}"

    def Thi(tb, k):
        return f"v{tb + 2 * (k % NT) + 1}"

    def emit_product(sq):
        lab = '.Lprod_sq' if sq else '.Lprod_mul'

        # the retired column's low 27 bits go to the lane below by one v_and_b32 with DPP into a fixed pair per
        # window whose high dword stays 0 (lane 3 masked to 0), and the next step's multiply-add into that
        # column takes the pair as its addend: no fresh ring column to clear (as fthe_addb_q152); lane 0's
        # product limb is stored unmasked and masked when to_dwords reads it back
        HO = {T1B: 146, T2B: 148}            # in the Barretts' DQ registers (dead in the product pass)
        VMK = 150

        def top(tb, u, j):
            return pair(HO[tb]) if j == Q - 1 else T(tb, u + j)

        def split(tb, u, t):
            """the lowest column: hi -> the lane's next column, lo (lane 0: the product limb) kept in place"""
            e(f'  v_lshrrev_b64 {t}, {B}, {T(tb, u)}')
            e(f'  v_lshl_add_u64 {T(tb, u + 1)}, {t}, 0, {T(tb, u + 1)}')

        def retire(tb, u, row):
            """lane 0's lo is the product limb: written to A-column row `row` (its multiplier is consumed)"""
            e('  s_mov_b64 exec, s[22:23]')
            e(f'  ds_write_b32 v{V_LDSI}, {Tlo(tb, u)} offset:{row * RB}')
            e('  s_mov_b64 exec, -1')

        def handoff(tb, u):
            """lo & (2^27 - 1) to the lane below (lane 3: 0) in the window's pair; >= 5 wait states after the
            EXEC writes of retire() (the schedule below keeps MADs between), after the step's last read of
            the pair"""
            e(f'  v_and_b32_dpp v{HO[tb]}, {Tlo(tb, u)}, v{VMK} quad_perm:[1,2,3,0] {DPP}')

        def step(u, i, last):
            ai, nai = f"v{V_AI[u % 2]}", f"v{V_AI[(u + 1) % 2]}"
            bi, nbi = f"v{V_BI[u % 2]}", f"v{V_BI[(u + 1) % 2]}"
            for j in range(Q):
                e(f'  v_mad_u64_u32 {T(T1B, u + j)}, vcc, {ai}, {X0(j)}, {top(T1B, u, j)}')
                if j == 2:
                    split(T1B, u, pair(V_TMP))
                if j == 6 and not last:
                    e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(i + 1) * RB}')
                    if not sq:
                        e(f'  ds_read_b32 {nbi}, v{V_LDSI} offset:{(S + i + 1) * RB}')
                if j == 8:
                    retire(T1B, u, i)
            for j in range(Q):
                if sq:                               # x0_i (2 x1): X1 doubled once per squaring
                    e(f'  v_mad_u64_u32 {T(T2B, u + j)}, vcc, {ai}, {X1(j)}, {top(T2B, u, j)}')
                else:
                    e(f'  v_mad_u64_u32 {T(T2B, u + j)}, vcc, {ai}, {X1(j)}, {top(T2B, u, j)}')
                    e(f'  v_mad_u64_u32 {T(T2B, u + j)}, vcc, {bi}, {X0(j)}, {T(T2B, u + j)}')
                if j == 0:
                    handoff(T1B, u)
                if j == 2:
                    split(T2B, u, pair(V_TMP))
                if j == 8:
                    retire(T2B, u, S + i)
            handoff(T2B, u)
            if not last:
                e('  s_waitcnt lgkmcnt(2)')                      # the prefetch reads (issued before the writes)

        e(f'{lab}:')
        e('// @phase product')
        if "prio" in DBG:                        # timing knobs: the product pass at low / high priority
            e('  s_setprio 0')
        if "prioinv" in DBG:
            e('  s_setprio 3')
        for k in range(NT):
            e(f'  v_mov_b64_e32 {T(T1B, k)}, 0')
            e(f'  v_mov_b64_e32 {T(T2B, k)}, 0')
        e(f'  v_mov_b64_e32 {pair(HO[T1B])}, 0')
        e(f'  v_mov_b64_e32 {pair(HO[T2B])}, 0')
        e(f'  v_mov_b32_e32 v{VMK}, {hex(MASK)}')
        e(f'  v_cndmask_b32_e64 v{VMK}, v{VMK}, 0, s[20:21]')
        if sq:                                   # window 2 of a squaring is 2 x0 x1: double x1's limbs (< 2^28)
            for j in range(Q):                   # once instead of 2 x0_i at every step; x1 is dead after the pass
                e(f'  v_lshlrev_b32_e32 {X1(j)}, 1, {X1(j)}')
        e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI}')
        if not sq:
            e(f'  ds_read_b32 v{V_BI[0]}, v{V_LDSI} offset:{S * RB}')
        e('  s_waitcnt lgkmcnt(0)')
        # steps i = 0..75: NTRIP trips of NT steps (the ring relabels every step; the LDS cursor moves per
        # trip), then TL steps
        NTRIP, TL = S // NT, S % NT
        assert NT % 2 == 0 and TL > 0
        if "noprod" in DBG:
            e(f'  s_branch {lab}_skip')
        e(f'  s_mov_b32 s18, {NTRIP}')
        e(f'{lab}_trip:')
        for u in range(NT):
            step(u, u, False)
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(NT * RB)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_cmp_lg_u32 s18, 0')
        e(f'  s_cbranch_scc1 {lab}_trip')
        for u in range(TL):
            step(u, u, u == TL - 1)
        e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(NTRIP * NT * RB)}, v{V_LDSI}')
        if "noprod" in DBG:
            e(f'{lab}_skip:')
        e('  s_waitcnt lgkmcnt(0)')
        e('// @phase window')
        if "prio" in DBG:
            e('  s_setprio 3')
        if "prioinv" in DBG:
            e('  s_setprio 0')
        # ---- normalise both windows: positions TL .. TL + 18 -> 19 limbs (z limbs 76 + 19 k + j) --------
        for tb, tag in ((T1B, 'n1'), (T2B, 'n2')):
            e(f'  v_mov_b64_e32 {tmp}, 0')
            for k in range(Q):                   # the top column is in the window's hand-off pair
                e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {T(tb, TL + k) if k < Q - 1 else pair(HO[tb])}')
                e(f'  v_and_b32_e32 {Tlo(tb, TL + k)}, {hex(MASK)}, v{V_TMP}')
                e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
            ripple_quad(f'{lab}_{tag}', lambda k, tb=tb: Tlo(tb, TL + k), Q)
        e('// @phase conv')
        # ---- z1, z2 -> dwords Z1, Z2 (quad layout of the add kernel) ----------------------------------------
        for tb, zb, row0, tag in ((T1B, Z1B, 0, 'z1'), (T2B, Z2B, S, 'z2')):
            if "noconv" not in DBG:
                to_dwords(zb, row0, lambda k, tb=tb: Tlo(tb, TL + k))
        e('  s_branch .Lbarrett')

    def to_dwords(zb, row0, W):
        """z (low 76 limbs in A-column rows row0.., high 76 in W(k) on lane k) -> dwords zb[0..32]: lane j
        holds z limbs [38 j, 38 j + 38) in ZL (lanes 0, 1 from LDS, lanes 2, 3 by DPP from the window), then
        the add kernel's limbs_to_words (2j-bit funnel) and lane 3's dword 128"""
        ZL = zb                                        # in place: dword i overwrites limb i (never read after)
        e('  s_nop 1')
        for k in range(Q):
            e(f'  v_mov_b32_dpp v{ZL + k}, {W(k)} quad_perm:[0,1,0,2] {DPP}')
            e(f'  v_mov_b32_dpp v{ZL + Q + k}, {W(k)} quad_perm:[0,1,1,3] {DPP}')
        # lanes 0, 1: rows row0 + 38 j + k of column c (V_LDSW = area + 4c + 19 j RB, so + 19 j RB more)
        e(f'  v_add_u32_e32 v{V_TMP}, v{V_LDSW}, v{V_LDSW}')
        e(f'  v_sub_u32_e32 v{V_TMP}, v{V_TMP}, v{V_LDSI}')                  # area + 4 c + 38 j RB
        e('  s_mov_b64 exec, s[28:29]')
        for k in range(2 * Q):
            e(f'  ds_read_b32 v{ZL + k}, v{V_TMP} offset:{(row0 + k) * RB}')
        e('  s_mov_b64 exec, -1')
        e('  s_waitcnt lgkmcnt(0)')
        # product limbs were stored with their carries above bit 27: a limb's first use takes bits [s, 27) by
        # v_bfe_u32, a last use shifts the carries out of the dword; only the limbs that end inside a dword
        # (and limb 37, whose top bits go to the next lane and dword 128) are masked
        dw = [(32 * i - B * (32 * i // B), 32 * i // B, min((32 * i + 31) // B, 2 * Q - 1)) for i in range(32)]
        mid = sorted({jj for i, (s, j0, j1) in enumerate(dw) for jj in range(j0 + 1, j1 + 1)
                      if B * jj - 32 * i + B < 32} | {2 * Q - 1})
        for k in mid:
            e(f'  v_and_b32_e32 v{ZL + k}, {hex(MASK)}, v{ZL + k}')
        U = lambda i: f"v{zb + i}"
        t1, bo = f"v{V_AI[0]}", f"v{V_AI[1]}"
        for i, (s, j0, j1) in enumerate(dw):
            lo = 32 * i
            e(f'  v_bfe_u32 {U(i)}, v{ZL + j0}, {s}, {B - s}')
            for jj in range(j0 + 1, j1 + 1):
                e(f'  v_lshl_or_b32 {U(i)}, v{ZL + jj}, {B * jj - lo}, {U(i)}')
        e(f'  v_sub_u32_e32 {bo}, 32, v{V_SH}')
        e(f'  v_and_b32_e32 {bo}, 31, {bo}')                          # 32 - 2j (lane 0: 0)
        for i in range(31, 0, -1):                     # (U(i) << 2j) | (U(i-1) >> 32 - 2j); lane 0 keeps U(i)
            e(f'  v_alignbit_b32 {t1}, {U(i)}, {U(i - 1)}, {bo}')
            e(f'  v_cndmask_b32_e64 {U(i)}, {t1}, {U(i)}, s[22:23]')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp {t1}, v{ZL + 2 * Q - 1} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_sub_u32_e32 {bo}, {B}, v{V_SH}')                     # lane 0: shift 27 -> no bits
        e(f'  v_lshrrev_b32_e32 {t1}, {bo}, {t1}')
        e(f'  v_lshl_or_b32 {U(0)}, {U(0)}, v{V_SH}, {t1}')
        e(f'  v_lshrrev_b32_e32 {U(32)}, 19, v{ZL + 2 * Q - 1}')       # lane 3: bits 4096..4103 (limb 151 >> 19)

    for sq in (True, False):
        emit_product(sq)

    # ---- the two Barrett reductions ------------------------------------------------------------------------
    def stage_off(t):
        """byte offset of tile t's groups in the staging row: chunk k at CSTRIDE k"""
        k = next(i for i, ch in enumerate(CHUNKS) if t in ch)
        return CSTRIDE * k + 32 * (t - CHUNKS[k][0])

    def fold_tile(acc, off):
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc}, 1, 0')
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 1}, s30, {pair(PG)}')
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 2}, s31, {pair(PG)}')
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 3}, s32, {pair(PG)}')
        e(f'  ds_write_b64 v{V_G}, {pair(PG)} offset:{off}')

    def mfma_consts(prod):
        """A-copy base register, its K offset, the active K-blocks per tile, the corrections' offset"""
        return ((V_A1, KO1, ACT1, 0) if prod == 1 else (V_A2, KO2, ACT2, CORR2_OFF - CORR1_OFF))

    def first_reads(prod, issue):
        """chunk 0's first corrections and A operands: constant image rows, independent of the staging, so the
        stage issues them ahead of its own writes (preload) and their round trip overlaps the staging's"""
        A, KO, act, corr = mfma_consts(prod)
        tiles = CHUNKS[0]
        ops = [(n, t, kb) for n, t in enumerate(tiles) for kb in act[t]]
        for n in range(min(NACC, len(tiles))):
            issue(('c', n), f'  ds_read_b128 {quad4(ACCS[n % NACC])}, v{V_C} offset:{corr + 64 * tiles[n]}')
        for x in range(min(3, len(ops))):
            n, t, kb = ops[x]
            off = KO + 16 * (4 * kb - t)
            assert 0 <= off and off + 64 <= COPY
            issue(('a', x), f'  ds_read_b128 {quad4(AOP[x % 4])}, v{A} offset:{off}')

    def preload(prod):
        if "nopreload" not in DBG:
            first_reads(prod, lambda tag, ins: e(ins))

    def mfma_product(prod):
        e(f'// @phase mfma{prod}')
        A, KO, act, corr = mfma_consts(prod)
        e(f'  v_mov_b32_e32 v{CR}, 0')
        # all 17 tiles as one stream (the folds stage each tile's groups at its chunk's offset): no drain of the
        # MFMA pipeline and no exposed operand round trip at the chunk boundaries (chunkloop: one loop per chunk)
        for j, tiles in enumerate(CHUNKS if "chunkloop" in DBG else [tuple(t for ch in CHUNKS for t in ch)]):
            ops = [(n, t, kb) for n, t in enumerate(tiles) for kb in act[t]]
            q = []

            def issue(tag, ins):
                e(ins)
                q.append(tag)

            def wait_for(tag):
                if tag not in q:
                    return
                i = q.index(tag)
                e(f'  s_waitcnt lgkmcnt({min(len(q) - i - 1, 15)})')
                del q[:i + 1]

            def read_a(x):
                n, t, kb = ops[x]
                off = KO + 16 * (4 * kb - t)
                assert 0 <= off and off + 64 <= COPY
                issue(('a', x), f'  ds_read_b128 {quad4(AOP[x % 4])}, v{A} offset:{off}')

            def read_corr(n, t):
                issue(('c', n), f'  ds_read_b128 {quad4(ACCS[n % NACC])}, v{V_C} offset:{corr + 64 * t}')

            # A operands are read three MFMAs ahead into four buffers (the buffer re-filled after MFMA x is MFMA
            # x - 1's, whose operands were read at its issue).  Three accumulator sets: tile n - 2 is folded right after tile n's first MFMA, so its results have
            # long been written (tile n - 1's MFMAs and reads in between) and the fold needs no s_nop padding
            # unless the instructions since its last MFMA number under XDL_WAIT; tile n + 1's corrections (srcC,
            # the set tile n - 2 used) are read right after that fold
            last_mfma = {}

            def settle(n):
                """wait states before a VALU read of tile n's accumulators: one per instruction issued since"""
                since = sum(1 for ln in o[last_mfma[n] + 1:] if ln.startswith('  '))
                need = XDL_WAIT - since
                while need > 0:
                    e(f'  s_nop {min(need, 8) - 1}')
                    need -= 8

            if j > 0 or "nopreload" in DBG:              # chunk 0's arrived with the stage (its lgkmcnt(0))
                for n in range(min(NACC, len(tiles))):
                    read_corr(n, tiles[n])
                for x in range(min(3, len(ops))):
                    read_a(x)
            for x, (n, t, kb) in enumerate(ops):
                first = x == 0 or ops[x - 1][0] != n
                if first:
                    wait_for(('c', n))
                wait_for(('a', x))
                if "nomfma" not in DBG:
                    e(f'  v_mfma_i32_16x16x64_i8 {quad4(ACCS[n % NACC])}, {quad4(AOP[x % 4])}, '
                      f'{quad4(BQ + 4 * kb)}, {quad4(ACCS[n % NACC])}')
                last_mfma[n] = len(o) - 1
                if x + 3 < len(ops):
                    read_a(x + 3)
                if first and n >= NACC - 1:
                    m = n - (NACC - 1)
                    settle(m)
                    fold_tile(ACCS[m % NACC], stage_off(tiles[m]))              # every chunk staged
                    q.append(('w', m))
                    if m + NACC < len(tiles):
                        read_corr(m + NACC, tiles[m + NACC])
            for m in range(max(0, len(tiles) - (NACC - 1)), len(tiles)):
                settle(m)
                fold_tile(ACCS[m % NACC], stage_off(tiles[m]))
        e('  s_waitcnt lgkmcnt(0)')
        if "nonorm" not in DBG:
            normalise_chunks()

    def normalise_chunks():
        """Every chunk at once: quad lane k normalises chunk k's groups (k = 0, 1: 32 groups, k = 2: 4; lane 3 has
        none) with carry-in 0 -- one chain instead of three after each other, itself split in two interleaved
        halves joined like the chunks -- and then the chunks' carries are
        delivered: lane k + 1 adds lane k's carry-out to its lowest dword; the signed overflow of that add (rare:
        |carry| < 2^18 against a uniform dword) ripples through the lane's dwords on a slow path and changes its
        carry-out, which is delivered the same way until no lane receives one.  CR: every lane's final carry."""
        e('// @phase norm')
        sizes = [4 * len(ch) for ch in CHUNKS]
        assert sizes[:2] == [32, 32] and sizes[2] == 4 and len(sizes) == 3
        L012, L01 = "s[34:35]", "s[28:29]"
        e('  s_mov_b32 s34, 0x77777777')
        e('  s_mov_b32 s35, 0x77777777')
        e(f'  s_mov_b64 exec, {L012}')
        # two chains per lane, interleaved: groups 0..15 (A) and 16..31 (B, carry-in 0) -- half the dependent
        # v_mad_i64_i32 latency; A's carry then goes into B's lowest dword like the chunks' carries between lanes.
        # Lane 2 (4 groups) runs B's first steps on don't-care rows; its dwords 16..19 are cleared after.
        H = 16
        chains = ((0, GB, FV), (H, AOP[0], ACC[0]))      # (first group, read double buffer, odd-step pair)
        cvs = [None, None]

        def rd(c, p):                                     # pair p (groups 2 p, 2 p + 1) of chain c
            g0c, buf, _ = chains[c]
            for hh in (0, 1):                             # two ds_read_b64 (8-byte rows, conflict-free)
                b = buf + 4 * (p % 2) + 2 * hh
                e(f'  ds_read_b64 v[{b}:{b + 1}], v{V_GR} offset:{8 * (g0c + 2 * p + hh)}')
        npair = H // 2
        for p in (0, 1):
            rd(0, p)
            rd(1, p)
        for p in range(npair):
            if 2 * p == sizes[2]:                         # lane 2's chunk ends: its carry stays in FV + 1
                e(f'  s_mov_b64 exec, {L01}')
            e(f'  s_waitcnt lgkmcnt({4 if p + 1 < npair else 0})')
            for h in (0, 1):                              # even group of A, of B, then the odd groups
                for c in (0, 1):
                    g0c, buf, fp = chains[c]
                    g = g0c + 2 * p + h
                    src = pair(buf + 4 * (p % 2) + 2 * h)
                    cin = cvs[c] if cvs[c] else '0'
                    if h == 0:
                        e(f'  v_mad_i64_i32 {pair(DQ + g)}, vcc, {cin}, 1, {src}' if cvs[c] else
                          f'  v_mov_b64_e32 {pair(DQ + g)}, {src}')
                        cvs[c] = f"v{DQ + g + 1}"
                    else:
                        e(f'  v_mad_i64_i32 {pair(fp)}, vcc, {cin}, 1, {src}')
                        cvs[c] = f"v{fp + 1}"
            for c in (0, 1):
                g0c, _, fp = chains[c]
                e(f'  v_mov_b32_e32 v{DQ + g0c + 2 * p + 1}, v{fp}')
            if p + 2 < npair:
                rd(0, p + 2)
                rd(1, p + 2)
        FB = chains[1][2]
        assert cvs == [f"v{FV + 1}", f"v{FB + 1}"]
        # lanes 0, 1: dword 16 += A's carry; the rare signed overflow ripples through dwords 17..31 into B's carry
        TP = V_TMP
        lab = f'.Lch{len(o)}'
        e(f'  v_mov_b32_e32 v{TP}, v{DQ + H}')
        e(f'  v_mov_b32_e32 v{TP + 1}, 0')
        e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{FV + 1}, 1, {pair(TP)}')
        e(f'  v_mov_b32_e32 v{DQ + H}, v{TP}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{TP + 1}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        e('  s_and_saveexec_b64 s[38:39], vcc')
        for i in range(H + 1, 2 * H):
            e(f'  v_mov_b32_e32 v{TP}, v{DQ + i}')
            e(f'  v_mov_b32_e32 v{FV}, v{TP + 1}')
            e(f'  v_mov_b32_e32 v{TP + 1}, 0')
            e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{FV}, 1, {pair(TP)}')
            e(f'  v_mov_b32_e32 v{DQ + i}, v{TP}')
        e(f'  v_add_u32_e32 v{FB + 1}, v{TP + 1}, v{FB + 1}')
        e('  s_mov_b64 exec, s[38:39]')
        e(f'{lab}_done:')
        e(f'  v_mov_b32_e32 v{CR}, v{FB + 1}')            # lanes 0, 1: B's carry-out (exec is L01)
        e('  s_mov_b64 exec, s[26:27]')
        e(f'  v_mov_b32_e32 v{CR}, v{FV + 1}')            # lane 2: A's (its only chain); its dwords 16..19
        e(f'  v_mov_b64_e32 {pair(DQ + H)}, 0')           # from B's first steps back to 0 (q3_1 is added to z2
        e(f'  v_mov_b64_e32 {pair(DQ + H + 2)}, 0')       # dword by dword, lane 2 included)
        e('  s_mov_b64 exec, -1')
        # delivery: DL = the carries (or their changes) still to deliver, lane k -> lane k + 1 (k = 0, 1)
        DL, X, TP = GB, CR + 1, V_TMP
        lab = f'.Lcd{len(o)}'
        e(f'  v_mov_b32_e32 v{DL}, v{CR}')
        e(f'{lab}_loop:')
        e('  s_nop 4')                                    # EXEC / VALU writes -> DPP
        e(f'  v_mov_b32_dpp v{X}, v{DL} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{X}, v{X}, 0, s[22:23]')     # lane 0 receives none
        e(f'  v_cndmask_b32_e64 v{X}, v{X}, 0, s[20:21]')     # lane 3 has no chunk
        e(f'  v_mov_b32_e32 v{TP}, v{DQ}')
        e(f'  v_mov_b32_e32 v{TP + 1}, 0')
        e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{X}, 1, {pair(TP)}')   # lowest dword + carry (signed)
        e(f'  v_mov_b32_e32 v{DQ}, v{TP}')
        e(f'  v_mov_b32_e32 v{DL}, 0')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{TP + 1}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        # slow path, the lanes whose add overflowed: the signed overflow P ripples through dwords 1.. (lane 2:
        # 1..3, then it is lane 2's carry change); lane 1's final P changes its carry, delivered next round
        e('  s_and_saveexec_b64 s[34:35], vcc')
        P = X
        e(f'  v_mov_b32_e32 v{P}, v{TP + 1}')
        for i in range(1, 32):
            if i == sizes[2]:
                e(f'  v_add_u32_e32 v{TP}, v{P}, v{CR}')
                e(f'  v_cndmask_b32_e64 v{CR}, v{CR}, v{TP}, s[26:27]')   # lane 2: carry += P
                e(f'  v_cndmask_b32_e64 v{P}, v{P}, 0, s[26:27]')         # and nothing more to ripple
            e(f'  v_mov_b32_e32 v{TP}, v{DQ + i}')
            e(f'  v_mov_b32_e32 v{TP + 1}, 0')
            e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{P}, 1, {pair(TP)}')
            e(f'  v_mov_b32_e32 v{DQ + i}, v{TP}')
            e(f'  v_mov_b32_e32 v{P}, v{TP + 1}')
        e(f'  v_add_u32_e32 v{CR}, v{P}, v{CR}')          # lane 1: carry += P (lane 2: P = 0 here)
        e(f'  v_mov_b32_e32 v{DL}, v{P}')
        e('  s_mov_b64 exec, s[34:35]')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    def stage_q1(zb):
        """q1 = z dwords 63..128 (raw) -> staging positions 0..65, 0x80 bytes at 66..79; B operands (read_b).
        Lane k's local dword i is z dword 32 k + i -> position 32 k - 63 + i: lanes 2, 3 all of theirs (lane 3
        also local 32 = dword 128), lane 1 its local 31 (position 0)."""
        e('// @phase stage')
        preload(1)
        t = zb                                                   # raw dwords: the B operands are XORed after the read
        e(f'  v_bfe_u32 v{V_TMP}, v{V_ROW}, 7, 2')
        e(f'  v_lshlrev_b32_e32 v{V_TMP}, 7, v{V_TMP}')
        e(f'  v_add_u32_e32 v{V_TMP}, v{V_TMP}, v{V_QW}')                 # row + 128 k
        e(f'  v_subrev_u32_e32 v{V_TMP + 1}, {4 * Q1_DW0}, v{V_TMP}')     # position 32 k - 63
        e('  s_mov_b64 exec, s[24:25]')
        e(f'  ds_write_b32 v{V_TMP + 1}, v{t + 31} offset:{4 * 31}')       # lane 1: position 0
        e('  s_mov_b32 s34, 0xcccccccc')
        e('  s_mov_b32 s35, 0xcccccccc')
        e('  s_mov_b64 exec, s[34:35]')                                    # lanes 2, 3 (odd bases 1, 33)
        e(f'  ds_write_b32 v{V_TMP + 1}, v{t}')
        for i in range(1, 31, 2):
            e(f'  ds_write2_b32 v{V_TMP + 1}, v{t + i}, v{t + i + 1} offset0:{i} offset1:{i + 1}')
        e(f'  ds_write_b32 v{V_TMP + 1}, v{t + 31} offset:{4 * 31}')
        e('  s_mov_b64 exec, s[20:21]')
        e(f'  ds_write_b32 v{V_TMP + 1}, v{t + 32} offset:{4 * 32}')       # lane 3: dword 128 -> position 65
        e('  s_mov_b64 exec, s[22:23]')                  # lane 0: positions 66..79 = 0x80 bytes (0 after the XOR)
        e(f'  v_mov_b32_e32 v{V_TMP}, s33')
        for d in range(NQ1, 16 * KB1):
            e(f'  ds_write_b32 v{V_QW}, v{V_TMP} offset:{4 * d}')
        e('  s_mov_b64 exec, -1')
        read_b(KB1)

    def read_b(kbs):
        """the B operands (staged raw) -> registers, XOR 0x80 per byte: u8 -> u8 - 128 as i8 (20 XORs instead of
        one per staged dword)"""
        e('  s_waitcnt lgkmcnt(0)')
        for kb in range(kbs):
            e(f'  ds_read_b128 {quad4(BQ + 4 * kb)}, v{V_B} offset:{64 * kb}')
        for kb in range(kbs):
            e(f'  s_waitcnt lgkmcnt({kbs - 1 - kb})')
            for i in range(4):
                e(f'  v_xor_b32_e32 v{BQ + 4 * kb + i}, s33, v{BQ + 4 * kb + i}')

    def clear_dq():
        for i in range(32):
            e(f'  v_mov_b32_e32 v{DQ + i}, 0')

    def stage_q3():
        """q3 dword d = N1 dword d + 1: lane k holds N1 dwords [32 k, 32 k + 32) in DQ -> positions 32 k - 1 + i
        (lane 0 from i = 1), raw; lane 2 sets positions 65..79 to 0x80 bytes, which read_b's XOR makes 0"""
        e('// @phase stage')
        preload(2)
        e('  s_mov_b32 s34, 0x77777777')
        e('  s_mov_b32 s35, 0x77777777')
        e('  s_mov_b64 exec, s[34:35]')                                    # lanes 0..2
        e(f'  v_bfe_u32 v{V_TMP}, v{V_ROW}, 7, 2')
        e(f'  v_lshlrev_b32_e32 v{V_TMP}, 7, v{V_TMP}')
        e(f'  v_add_u32_e32 v{V_TMP}, v{V_TMP}, v{V_QW}')                 # row + 128 k = position 32 k
        for i in range(1, 31, 2):
            e(f'  ds_write2_b32 v{V_TMP}, v{DQ + i}, v{DQ + i + 1} offset0:{i - 1} offset1:{i}')
        e(f'  ds_write_b32 v{V_TMP}, v{DQ + 31} offset:{4 * 30}')
        e('  s_mov_b64 exec, s[26:27]')                  # lane 2: positions 65..79 = 0x80 bytes (0 after the XOR)
        e(f'  v_mov_b32_e32 v{V_TMP + 1}, s33')
        for d in range(65, 16 * KB2 - 1, 2):
            e(f'  ds_write2_b32 v{V_TMP}, v{V_TMP + 1}, v{V_TMP + 1} offset0:{d - 64} offset1:{d - 63}')
        e(f'  ds_write_b32 v{V_TMP}, v{V_TMP + 1} offset:{4 * (16 * KB2 - 1 - 64)}')
        e('  s_mov_b32 s34, 0x66666666')
        e('  s_mov_b32 s35, 0x66666666')
        e('  s_mov_b64 exec, s[34:35]')                                    # lanes 1, 2: N1 dword 32 k -> pos 32 k - 1
        e(f'  v_subrev_u32_e32 v{V_TMP}, 4, v{V_TMP}')
        e(f'  ds_write_b32 v{V_TMP}, v{DQ}')
        e('  s_mov_b64 exec, -1')
        read_b(KB2)

    def unxor_q3():
        e('  s_mov_b64 exec, s[28:29]')
        for i in range(2, 32):
            e(f'  v_xor_b32_e32 v{DQ + i}, s33, v{DQ + i}')
        e('  s_mov_b32 s34, 0x77777777')
        e('  s_mov_b32 s35, 0x77777777')
        e('  s_mov_b64 exec, s[34:35]')
        e(f'  v_xor_b32_e32 v{DQ}, s33, v{DQ}')
        e(f'  v_xor_b32_e32 v{DQ + 1}, s33, v{DQ + 1}')
        e('  s_mov_b64 exec, -1')

    def clamp(lab):
        """N1 < 0 (lane 2's final carry) -> q3 = 0"""
        e('  s_nop 4')
        e(f'  v_mov_b32_dpp v{V_TMP}, v{CR} quad_perm:[2,2,2,2] {DPP}')
        e(f'  v_cmp_gt_i32_e32 vcc, 0, v{V_TMP}')
        e('  s_and_saveexec_b64 s[34:35], vcc')
        e(f'  s_cbranch_execz {lab}')
        clear_dq()
        e(f'{lab}:')
        e('  s_mov_b64 exec, s[34:35]')

    def carry_ripple(lab, R, n, ci, cin):
        """lane k (k < 3) hands its carry ci (0/1, out of its dword n - 1) to lane k + 1, which adds it to its
        dwords R(0..n-1); repeated until no lane receives one.  Lane 3's carry goes into its dword R(n) (the
        number's top dword, 128)."""
        e('  s_mov_b64 exec, s[20:21]')
        e(f'  v_add_u32_e32 v{R + n}, v{R + n}, v{ci}')
        e('  s_mov_b64 exec, -1')
        e(f'{lab}_loop:')
        e('  s_nop 4')                                                  # EXEC written by SALU -> DPP
        e(f'  v_mov_b32_dpp v{cin}, v{ci} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{cin}, v{cin}, 0, s[22:23]')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{cin}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        e(f'  v_add_co_u32_e32 v{R}, vcc, v{R}, v{cin}')
        e(f'  v_mov_b32_e32 v{ci}, 0')                                   # the carries handed on are delivered
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')                               # absorbed by dword 0 everywhere (usual)
        e('  s_and_saveexec_b64 s[34:35], vcc')                         # the lanes whose dword 0 carried
        for i in range(1, n):
            e(f'  v_addc_co_u32_e32 v{R + i}, vcc, 0, v{R + i}, vcc')
        e(f'  v_cndmask_b32_e64 v{ci}, 0, 1, vcc')
        e('  s_and_b64 exec, exec, s[20:21]')                            # lane 3: into its top dword
        e(f'  v_add_u32_e32 v{R + n}, v{R + n}, v{ci}')
        e('  s_mov_b64 exec, s[34:35]')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    def borrow_ripple(lab, R, n, bo, bin_):
        e(f'{lab}_loop:')
        e('  s_nop 4')
        e(f'  v_mov_b32_dpp v{bin_}, v{bo} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{bin_}, v{bin_}, 0, s[22:23]')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{bin_}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        e(f'  v_sub_co_u32_e32 v{R}, vcc, v{R}, v{bin_}')
        e(f'  v_mov_b32_e32 v{bo}, 0')                                   # the borrows handed on are delivered
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')                               # absorbed by dword 0 everywhere (usual)
        e('  s_and_saveexec_b64 s[34:35], vcc')                         # the lanes whose dword 0 borrowed
        for i in range(1, n):
            e(f'  v_subb_co_u32_e64 v{R + i}, vcc, v{R + i}, 0, vcc')
        e(f'  v_cndmask_b32_e64 v{bo}, 0, 1, vcc')
        e('  s_mov_b64 exec, s[34:35]')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    def remainder_to_digit(zb, X, tag):
        """r = (z - r2) mod 2^2080 (lane j: dwords [32 j, 32 j + 32), lane 2: dword 64 only) -> staging row
        positions 0..64 -> lane k reads positions [16 k, 16 k + 17), funnel-shifts by k, 19 limbs of 27 bits"""
        e('// @phase remainder')
        e(f'  v_sub_co_u32_e32 v{zb}, vcc, v{zb}, v{DQ}')
        for i in range(1, 32):
            e(f'  v_subb_co_u32_e32 v{zb + i}, vcc, v{zb + i}, v{DQ + i}, vcc')
        e(f'  v_cndmask_b32_e64 v{V_AI[0]}, 0, 1, vcc')
        borrow_ripple(f'.L{tag}_rb', zb, 32, V_AI[0], V_AI[1])
        # stage: lanes 0, 1 all 32, lane 2 local 0 (position 64)
        e(f'  v_bfe_u32 v{V_TMP}, v{V_ROW}, 7, 2')
        e(f'  v_lshlrev_b32_e32 v{V_TMP + 1}, 7, v{V_TMP}')
        e(f'  v_add_u32_e32 v{V_TMP + 1}, v{V_TMP + 1}, v{V_QW}')         # position 32 k
        e('  s_mov_b32 s34, 0x77777777')
        e('  s_mov_b32 s35, 0x77777777')
        e('  s_mov_b64 exec, s[34:35]')
        e(f'  ds_write_b32 v{V_TMP + 1}, v{zb}')
        e('  s_mov_b64 exec, s[28:29]')
        for i in range(1, 31, 2):
            e(f'  ds_write2_b32 v{V_TMP + 1}, v{zb + i}, v{zb + i + 1} offset0:{i} offset1:{i + 1}')
        e(f'  ds_write_b32 v{V_TMP + 1}, v{zb + 31} offset:{4 * 31}')
        e('  s_mov_b64 exec, -1')
        e('  s_waitcnt lgkmcnt(0)')
        # lane k: positions 16 k .. 16 k + 16 into W (zb area is free now: r is staged)
        W = BQ                                                            # free after product 2
        if "ldsfree" in DBG:                                              # timing knock-out: aligned, spread
            e(f'  v_mov_b32_e32 v{V_TMP + 1}, v{V_B}')
        else:
            e(f'  v_lshlrev_b32_e32 v{V_TMP + 1}, 6, v{V_TMP}')
            e(f'  v_add_u32_e32 v{V_TMP + 1}, v{V_TMP + 1}, v{V_QW}')     # position 16 k
        for i in range(4):
            e(f'  ds_read_b128 v[{W + 4 * i}:{W + 4 * i + 3}], v{V_TMP + 1} offset:{16 * i}')
        e(f'  ds_read_b32 v{W + 16}, v{V_TMP + 1} offset:64')
        e('  s_waitcnt lgkmcnt(0)')
        # bits [513 k, 513 k + 513) = positions 16 k.. shifted right by k
        for i in range(16):
            e(f'  v_alignbit_b32 v{W + i}, v{W + i + 1}, v{W + i}, v{V_TMP}')
        e(f'  v_lshrrev_b32_e32 v{W + 16}, v{V_TMP}, v{W + 16}')
        for jj in range(Q):
            a, sh = (B * jj) >> 5, (B * jj) & 31
            if sh + B <= 32:
                e(f'  v_bfe_u32 {X(jj)}, v{W + a}, {sh}, {B}')
            else:
                e(f'  v_alignbit_b32 {X(jj)}, v{W + a + 1}, v{W + a}, {sh}')
                e(f'  v_and_b32_e32 {X(jj)}, {hex(MASK)}, {X(jj)}')

    e('.Lbarrett:')
    if "nobarrett" in DBG:
        e('  s_branch .Lbarrett_end')
    # ---- Barrett 1: z1 -> q3_1, r1 (new x0) ---------------------------------------------------------------
    stage_q1(Z1B)
    clear_dq()
    mfma_product(1)
    clamp('.Lnoclamp1')
    e('// @phase q3add')
    # z2 += q3_1: Z2 local i += DQ[i + 1] (i < 31), local 31 += the next lane's DQ[0]
    _dbg_noq3 = os.environ.get("FTHE_GEN_NADICB_DBG") == "noq3"
    if _dbg_noq3:
        e('  s_branch .Ldbg_skip_q3')
    e('  s_nop 4')                                                      # EXEC written by SALU (clamp) -> DPP
    e(f'  v_mov_b32_dpp v{V_TMP}, v{DQ} quad_perm:[1,2,3,3] {DPP}')
    e(f'  v_cndmask_b32_e64 v{V_TMP}, v{V_TMP}, 0, s[20:21]')          # lane 3: none
    e(f'  v_add_co_u32_e32 v{Z2B}, vcc, v{Z2B}, v{DQ + 1}')
    for i in range(1, 31):
        e(f'  v_addc_co_u32_e32 v{Z2B + i}, vcc, v{Z2B + i}, v{DQ + i + 1}, vcc')
    e(f'  v_addc_co_u32_e32 v{Z2B + 31}, vcc, v{Z2B + 31}, v{V_TMP}, vcc')
    e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, 1, vcc')                       # carry out of local 31
    carry_ripple('.Lzc', Z2B, 32, V_TMP, V_TMP + 1)
    if _dbg_noq3:
        e('.Ldbg_skip_q3:')
    stage_q3()
    mfma_product(2)
    remainder_to_digit(Z1B, X0, 'b1')
    # ---- Barrett 2: z2 + q3_1 -> r2 (new x1) --------------------------------------------------------------
    stage_q1(Z2B)
    clear_dq()
    mfma_product(1)
    clamp('.Lnoclamp2')
    stage_q3()
    mfma_product(2)
    remainder_to_digit(Z2B, X1, 'b2')
    e('.Lbarrett_end:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    e('  s_sub_u32 s19, s19, 1')
    e('  s_branch .Lsqr_loop')

    e('.Lend:')
    e('// @stampout')
    e('  s_endpgm')
    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    if "stamp" in DBG:
        o = stamp_pass(o, waves)
    o.extend(_descriptor(name, LDSB, NVGPR, NSGPR, max_wg=64 * waves).splitlines())
    return "\n".join(o) + "\n"


STAMP_PHASES = ['batch', 'ops', 'product', 'window', 'conv', 'stage', 'mfma1', 'norm', 'q3add', 'mfma2', 'remainder']


def stamp_pass(o, waves):
    """timing build (FTHE_GEN_NADICB_DBG=stamp, tools/nadicb_stamps.py): at every `// @phase` marker the
    s_memtime ticks since the last one go to the accumulator of the phase that ran (s50, runtime: the op loop
    jumps, so the textual order is not the running order; SGPR-relative s_movrels / s_movreld on M0); after the
    last batch lane 0 writes 16 dwords per wave at kernarg rows[15] + 64 (waves wg + wave): the 11 sums, the
    batches, the s_memrealtime of the first and the last stamp, 0, 0"""
    ids = {ph: i for i, ph in enumerate(STAMP_PHASES)}
    acc0 = 52
    out = []

    def stamp(new_id):
        return ['  s_memtime s[48:49]', '  s_waitcnt lgkmcnt(0)', '  s_sub_u32 s51, s48, s46', '  s_mov_b32 m0, s50',
                '  s_nop 0', f'  s_movrels_b32 s45, s{acc0}', '  s_add_u32 s51, s51, s45', f'  s_movreld_b32 s{acc0}, s51',
                f'  s_mov_b32 s50, {new_id}', '  s_mov_b64 s[46:47], s[48:49]']
    for line in o:
        if line.startswith('// @phase'):
            ph = line.split()[2]
            out += stamp(ids[ph])
            if ph == 'batch':
                out.append('  s_add_u32 s64, s64, 1')
            out.append(line)
        elif line == '// @stampinit':
            out += [f'  s_mov_b32 s{acc0 + i}, 0' for i in range(len(STAMP_PHASES))]
            out += ['  s_mov_b32 s64, 0', f'  s_mov_b32 s50, {ids["batch"]}', '  s_memtime s[46:47]',
                    '  s_memrealtime s[66:67]', '  s_waitcnt lgkmcnt(0)', '  v_readfirstlane_b32 s65, v0',
                    '  s_lshr_b32 s65, s65, 6', f'  s_mul_i32 s44, s2, {waves}', '  s_add_u32 s65, s65, s44']
        elif line == '// @stampout':
            out += stamp(ids['batch'])
            out += ['  s_memrealtime s[68:69]', '  s_load_dwordx2 s[70:71], s[0:1], 0xa0', '  s_waitcnt lgkmcnt(0)',
                    '  s_cmp_eq_u64 s[70:71], 0', '  s_cbranch_scc1 .Lstamp_skip', '  s_mov_b64 exec, 1',
                    '  s_lshl_b32 s44, s65, 6', '  v_mov_b32_e32 v1, s44']
            for i in range(len(STAMP_PHASES)):
                out += [f'  v_mov_b32_e32 v2, s{acc0 + i}', f'  global_store_dword v1, v2, s[70:71] offset:{4 * i}']
            for i, sg in enumerate(('s64', 's66', 's68')):
                out += [f'  v_mov_b32_e32 v2, {sg}',
                        f'  global_store_dword v1, v2, s[70:71] offset:{4 * (len(STAMP_PHASES) + i)}']
            out += ['  s_waitcnt vmcnt(0)', '.Lstamp_skip:']
        else:
            out.append(line)
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--waves', type=int, default=WAVES)
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args()
    with open(a.out, 'w') as f:
        f.write(gen_nadicb('fthe_nadic_b76', a.waves))
