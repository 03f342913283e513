#!/usr/bin/env python3
"""Generator of the Paillier-2048 ciphertext-add kernel with a matrix-core Barrett reduction (gfx950 assembly):
fthe_addb_q152, out[g] = x[g] y[g] mod N for N = n^2 (4095-4096 bits), canonical 128-word rows in and out
(paillier.cpp:92-105, paillier_gmp.cpp:16-21).  tools/addb_model.py is the bit-exact model of the
arithmetic (parameters, bounds, column corrections); this file lays it out on the machine.

One quad of lanes per ciphertext (lane j of the quad owns limbs [38j, 38j+38) of 27 bits), 16 ciphertexts
per wave, 12 waves per workgroup (one workgroup per CU: its LDS holds the key's constant images once).

  1. rows -> limbs (the row I/O of gen_montprog.gen_quad); y's limbs become the wave's A column in LDS.
  2. z = x y on the VALU by one level of Karatsuba on 76-limb halves (section 2K; "nokara" keeps the plain
     152-step scan): P1 = (xL + xH)(yL + yH), P0 = xL yL, P2 = xH yH, each 76 operand-scanning steps of 19
     v_mad_u64_u32 per lane into a ring of 64-bit columns -- 4,332 MADs per lane instead of 5,776 -- the lowest
     column of lane 0 retiring as a limb (P0 / P2: into the A column row whose multiplier was consumed the step
     before; P1: into registers), then z = P0 + (P1 - P0 - P2) B^76 + P2 B^152 in signed limbs, normalised
     across lanes and blocks: 5% more adds/s (profiles/r05e_addb_kara_ab.jsonl, r05f_addb_libs_ab.jsonl).
  3. The window (z >> 4104) is normalised; z >> 4104 and z mod 2^4104 become dwords in the quad layout
     (lane j: dwords [32j, 32j+32)); q1 = z >> 4072 = [bits 4072..4103, (z >> 4104)] goes to a staging row
     per ciphertext, bytes fed as b ^ 0x80 (= b - 128, signed), padded with zero (fed 0) bytes.
  4. Product 1 (q1 mu, output byte columns 512..1039) on v_mfma_i32_16x16x64_i8: the B operand is 64 bytes x
     16 ciphertexts (lane l: ciphertext l & 15, bytes 16 (l >> 4) .. +15 of the K-block), the A operand a
     16 x 64 Toeplitz tile of mu's balanced digits (lane l: output row l & 15, the same 16 K bytes), read
     from one of 16 byte-shifted copies of mu so every read is one aligned ds_read_b128; the int32
     accumulators start from the column corrections (128 sum mu[s - k], and the -2^4121 bias).  Only the
     tiles whose constant entries are not all zero are issued (185 of 297).
  5. Each lane folds its 4 rows of a tile into an int64 group P_G = sum_i C_i 256^i (G = 4 t + (l >> 4)),
     the groups go through LDS, and quad lane j normalises the groups of chunk j (output tiles 8j .. 8j+7,
     chunk 3: 24 .. 32) into dwords with a signed carry handed on by DPP: q3 = floor(N1 / 2^4128) = the
     dwords of groups 1..128 (clamped to 0 when the sum is negative).
  6. q3 -> staging -> B; product 2 (q3 N mod 2^4104, columns 0..527, 153 tiles; q3 has 129 dwords so that
     rows >= N, which the reference reduces too, stay exact) and its fold give r2;
     r = (z - r2) mod 2^4104 (dword borrow chains, rippled across the quad) lies in [0, 3N); two
     conditional subtractions of N (dwords from the key's context) make it canonical; rows are stored.

kernarg: 0 u64 x rows, 8 u64 y rows, 16 u64 out rows, 24 u64 kctx, 32 u32 count, 36 u32 workgroups launched
(persistent: workgroup wg owns the batches of 16 ciphertexts wg, wg + workgroups, ...; its waves take them in
turn from a counter in LDS, so a wave that the SIMD's arbiter favours takes more of them and the 12 waves end
together), 40 u64 x index
list, 48 u64 y index list (0: row g is operand row g; else operand row g is row idx[g] of the operand array,
idx[g] < 0 the integer 1: the gathered products of the histogram scatter / segment sums).
kctx: the LDS image (IMG_BYTES: mu copies, N copies, corrections), then N as 128 dwords, then the row 1.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# ---- layout constants shared with the host image builder (fthe.hip addb_image) and tools/addb_model.py ----
S, Q, B = 152, 38, 27
MASK = (1 << B) - 1
WAVES = 12                       # waves per workgroup (one workgroup per CU, 3 waves per SIMD)
CT_PER_WAVE = 16
RB = 72                          # A-column row: 16 ciphertexts x 4 B + pad; 18 dwords: the window / z-limb
                                 # accesses of a 32-lane group (4 quad lanes 19 or 38 rows apart) at most 2-way
                                 # (68 B: 3-way; 76 B does not fit the LDS)
COPY = 800                       # one byte-shifted copy of a constant (== 32 mod 256: conflict-free reads)
KO1, KO2 = 64, 560               # copy offsets: y = KO + 16 (4 kb - t) + 16 h
A1_OFF = 0
A2_OFF = A1_OFF + 16 * COPY
TILES1, TILES2 = 33, 33
CORR1_OFF = A2_OFF + 16 * COPY
CORR2_OFF = CORR1_OFF + TILES1 * 64
IMG_BYTES = CORR2_OFF + TILES2 * 64          # 29,824
N_OFF = IMG_BYTES                            # N dwords in kctx (not copied to LDS)
ONE_OFF = N_OFF + 512                        # the integer 1 as a row (gathered index < 0)
KCTX_BYTES = ONE_OFF + 512
QROW = 656                                   # q staging row: 9 K-blocks of 64 bytes, stride = 4 (mod 32)
                                             # dwords: the quads' staging writes 4-way, not 16-way, per bank
GROW = 552                                   # group staging row: two chunks' 64-68 int64 groups; 138 dwords ==
                                             # 10 (mod 32): the folds' 16-lane ds_write_b64 hit 32 distinct banks
GCH = 264                                    # the pair's second chunk at byte 264 (66 dwords == 2 mod 64): with
                                             # GROW the normalisation's ds_read_b64 are conflict-free too
                                             # (tools/lds_conflicts.py; 16-byte rows for b128 reads cannot be)
WAVE_AREA = (max(S * RB, 16 * QROW, 16 * GROW) + 15) // 16 * 16   # A column (152 rows) / q staging / groups
LDS_WAVES = IMG_BYTES
LDS_CNT = LDS_WAVES + WAVES * WAVE_AREA      # the workgroup's batch counter (dword)
LDS_BYTES = LDS_CNT + 16
KB1, KB2 = 9, 9
NQ1, NQ3 = 129, 129                          # q1, q3 dwords (rows >= N: q3 < 2^4098)
MU_SHIFT = 4072 + 4128                       # mu = floor(2^(A + C) / N)
S1_BASE = 512                                # product-1 output byte columns from 512
BIAS_COL, BIAS_DIGIT = 515, -2               # -2^4121 in product 1's corrections
M_A = (0, 1, 2, 3, 12, 13, 14, 15)           # rows whose copies sit in slots 0..7 (ds_read_b128 lane groups)
M_B = (4, 5, 6, 7, 8, 9, 10, 11)             # slots 8..15
assert IMG_BYTES % 16 == 0 and WAVE_AREA % 16 == 0 and LDS_BYTES <= 160 * 1024
assert WAVE_AREA >= max(S * RB, 16 * QROW, 16 * GROW) and QROW % 16 == 0 and (QROW // 4) % 32 == 4


def layout_header():
    """gen/addb_layout.h: the constants the host image builder (addb_image.hpp) and launcher need"""
    vals = dict(kAddbMuShift=MU_SHIFT, kAddbNd1=515, kAddbNd2=513, kAddbKctxBytes=KCTX_BYTES, kAddbA1Off=A1_OFF,
                kAddbA2Off=A2_OFF, kAddbS1Base=S1_BASE, kAddbKO1=KO1, kAddbKO2=KO2, kAddbCopy=COPY,
                kAddbTiles1=TILES1, kAddbTiles2=TILES2, kAddbNq1=NQ1, kAddbNq3=NQ3, kAddbBiasCol=BIAS_COL,
                kAddbBiasDigit=BIAS_DIGIT, kAddbCorr1Off=CORR1_OFF, kAddbCorr2Off=CORR2_OFF, kAddbNOff=N_OFF, kAddbOneOff=ONE_OFF,
                kAddbImgBytes=IMG_BYTES, kAddbWaves=WAVES, kAddbPerWg=WAVES * CT_PER_WAVE, kAddbLdsBytes=LDS_BYTES)
    lines = ["// generated by fedtree_amd/build.py from gen_addb.py -- layout of fthe_addb_q152", "#pragma once"]
    lines += [f"constexpr int {k} = {v};" for k, v in vals.items()]
    return "\n".join(lines) + "\n"


def copy_slot(m):
    return M_A.index(m) if m in M_A else 8 + M_B.index(m)


def band(nd, s0, k0):
    """the A tile of output bytes [s0, s0+16) x input bytes [k0, k0+64) has a nonzero digit c[s - k]"""
    lo, hi = s0 - k0 - 63, s0 + 15 - k0
    return not (hi < 0 or lo >= nd)


# ---- the matrix-core product z = x y (section 2M, "mfz"; tools/addb_mfz_model.py is its bit-exact model) ------
# one ciphertext at a time per wave: x, y in balanced base-256 digits (513 each); z's byte columns
# c = i + 16 j + 256 u (MFMA row i, column j, block u) accumulate over tiles t the products of x digits
# a = i + 64 t + k - MZ_DELTA (row i's Toeplitz window) and y digits b = c - a (independent of i)
MZ_DELTA = -1
MZ_XOFF = 64                                 # x staging: byte MZ_XOFF + a holds digit a (zero pad below / above)


def _mz_valid(t, u):
    for i in range(16):
        for j in range(16):
            c = i + 16 * j + 256 * u
            a0 = i + 64 * t - MZ_DELTA
            if max(max(0, c - 512), a0) <= min(min(512, c), a0 + 63):
                return True
    return False


MZ_TILES = [(t, u) for t in range(-2, 10) for u in range(4) if _mz_valid(t, u)]          # 28
MZ_TS = sorted({t for t, _ in MZ_TILES})                                                 # -1 .. 7
_mz_btop = [256 * u + 16 * j - 64 * t - 16 * h + MZ_DELTA for t, u in MZ_TILES for j in range(16) for h in range(4)]
MZ_RY = max(_mz_btop) + (15 - max(_mz_btop)) % 16    # yr byte p holds y digit RY - p (RY = 15 mod 16)
MZ_YAREA = (MZ_RY - min(_mz_btop) + 31) // 16 * 16
MZ_XAREA = (MZ_XOFF + 15 + 64 * MZ_TS[-1] + 48 - MZ_DELTA + 20 + 15) // 16 * 16
# B fragments by v = 4 u - t (one 16-byte read per v serves every tile with that v): byte offset 64 (VMAX - v)
MZ_V = sorted({4 * u - t for t, u in MZ_TILES})
# wave-area layout of the product phase (it ends before the Barrett phases use the same bytes)
MZ_XS = 0
MZ_YS = MZ_XS + MZ_XAREA
MZ_GS = MZ_YS + MZ_YAREA                     # 256 int64 groups
MZ_ZS = MZ_GS + 2048                         # z: 256 dwords
MZ_WS = MZ_ZS + 1024                         # z >> 4104: 128 dwords at byte 12 + 4 w
MZ_END = MZ_WS + 528
assert MZ_RY >= 515 and (MZ_RY - MZ_DELTA) % 16 == 0 and (MZ_RY - 127) % 16 == 0 and len(MZ_TILES) == 28
assert all(x % 16 == 0 for x in (MZ_YS, MZ_GS, MZ_ZS, MZ_WS)) and MZ_YS + MZ_YAREA <= 2048

ND1, ND2 = 515, 513                          # balanced digits of mu and N
ACT1 = [[kb for kb in range(KB1) if band(ND1, 512 + 16 * t, 64 * kb)] for t in range(TILES1)]
ACT2 = [[kb for kb in range(KB2) if band(ND2, 16 * t, 64 * kb)] for t in range(TILES2)]
CHUNKS = [list(range(0, 8)), list(range(8, 16)), list(range(16, 24)), list(range(24, 33))]


def gen_addb(name: str) -> str:
    # timing-only knock-outs (wrong results; a library built elsewhere, tools/addb_lib_ab.sh): noprod (no product
    # MADs), nomfma (no MFMAs), nonorm (no group normalisation), nobarrett (no q1/q3 staging, products, folds),
    # nocanon (no conditional subtractions); stamp: per-phase s_memtime cycle sums per wave, written after the
    # launch's output rows (tools/addb_stamps.py; the stamps' lgkmcnt(0) drains cost some overlap)
    DBG = set(os.environ.get("FTHE_GEN_ADDB_DBG", "").split(","))
    # the product z = x y as one level of Karatsuba (three 76 x 76-limb products, section 2K below) instead of
    # 152 x 152 operand scanning; "nokara" keeps the latter (a correct schedule, for the A/B)
    KARA = "nokara" not in DBG
    # the product z = x y on the matrix cores, one ciphertext at a time (section 2M), switch "mfz": bit-exact,
    # 70% fewer VALU instructions per add, but 13-15% fewer adds/s than the VALU Karatsuba product (680-685M vs
    # 775-780M at 1M adds, profiles/r06x_addb_lib_ab.jsonl): its per-ciphertext loop is latency-bound, so off
    MFZ = "mfz" in DBG
    MZ_YI = 80                                    # y's dwords (quad layout), in place: balanced, then reversed
    o = []
    e = o.append
    DPP = "row_mask:0xf bank_mask:0xf"
    # ---- VGPRs ---------------------------------------------------------------------------------------
    V_TID, V_ROW, V_LDSI, V_AI, V_SH = 0, 1, 2, (3, 4), 5
    V_TMP = 6                                     # pair 6:7
    XB = 8                                        # X limbs v8..v45 (product phase), later other limbs
    TB = 46                                       # ring of NT 64-bit columns v46..v121
    NT = Q
    HO = 122                                      # hand-off pair v[122:123] (v123 = 0 in the product phase): the
                                                  # column lane j+1 retired, src2 of the next step's top MAD
    VMASK = 124                                   # 2^27 - 1 on quad lanes 0..2, 0 on lane 3
    WD = 47                                       # W dwords (after the product) v47..v78: W[i], W[i+1] of odd i
                                                  # is an even register pair (one ds_write_b64)
    ZLB = 80                                      # z mod 2^4104 dwords v80..v111, v112 = bits 4096..4103
    ZL128 = 112
    BQ = 8                                        # B operands, 9 x 4 = v8..v43
    DQ = 44                                       # fold output dwords v44..v79 (36)
    ACC = (114, 118)                              # two accumulator sets
    AOP = (122, 126, 130, 134)                    # four A-operand buffers (reads two MFMAs ahead)
    PG, FV = 162, 164                             # int64 pairs
    CR, CR2 = 166, 6                              # int32 chunk carries (CR2 = V_TMP, free in the MFMA phases)
    V_A1, V_A2, V_C, V_B, V_G, V_GR, V_Q3W, V_ZR = 138, 139, 140, 141, 142, 143, 144, 145
    GB = 146                                      # group read buffer, 8 int64 = v146..v161
    NV = 8                                        # N dwords for the canonicalisation (v8..v39, BQ dead)
    RR = 44                                       # r dwords (reuses DQ after the subtraction) v44..v75, v76
    R128 = 76
    TT, TT128 = 80, 112                           # r - N dwords v80..v111 (+ dword 128): ZL is dead by then
    NVGPR = 168

    def X(k):
        return f"v{XB + k}"

    def T(k):
        k %= NT
        return f"v[{TB + 2 * k}:{TB + 2 * k + 1}]"

    def Tlo(k):
        return f"v{TB + 2 * (k % NT)}"

    def Thi(k):
        return f"v{TB + 2 * (k % NT) + 1}"

    def pair(n):
        return f"v[{n}:{n + 1}]"

    def quad4(n):
        return f"v[{n}:{n + 3}]"

    tmp = pair(V_TMP)
    # ---- SGPRs ---------------------------------------------------------------------------------------
    # s[0:1] kernarg, s2 wg id, s[4:5] x rows, s[6:7] y rows, s[8:9] out rows, s[10:11] kctx, s12 count,
    # s13 first ciphertext of this wave, s[14:15] scratch, s[16:17] saved exec, s18 loop counter,
    # lane masks: s[20:21] quad lane 3, s[22:23] lane 0, s[24:25] lane 1, s[26:27] lane 2,
    # s[28:29] live lanes, s30 = 256, s31 = 65536, s32 = 2^24, s33 = 0x80808080, s[34:35] x index list,
    # s[36:37] y index list (0: direct rows), s[38:39] carry scratch of the gathered addresses
    LANE_MASK = {3: "s[20:21]", 0: "s[22:23]", 1: "s[24:25]", 2: "s[26:27]"}
    LIVE = "s[28:29]"
    NSGPR = 68 if "stamp" in DBG else 50 if MFZ else 42   # s[40:41]: the product steps' carry-out sink; MFZ: s42..s48

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
    e('  s_load_dword s12, s[0:1], 0x20')
    e('  s_load_dwordx2 s[34:35], s[0:1], 0x28')
    e('  s_load_dwordx2 s[36:37], s[0:1], 0x30')
    for j, pat in ((3, 0x88888888), (0, 0x11111111), (1, 0x22222222), (2, 0x44444444)):
        lo, hi = LANE_MASK[j][2:-1].split(':')
        e(f'  s_mov_b32 s{lo}, {hex(pat)}')
        e(f'  s_mov_b32 s{hi}, {hex(pat)}')
    e('  s_movk_i32 s30, 0x100')
    e('  s_mov_b32 s31, 0x10000')
    e('  s_mov_b32 s32, 0x1000000')
    e('  s_mov_b32 s33, 0x80808080')
    e('  s_waitcnt lgkmcnt(0)')
    # ---- constant image -> LDS: every thread copies 16 B per pass (768 threads x 16 B = 12,288 B) --------
    e(f'  v_lshlrev_b32_e32 v{V_ROW}, 4, v{V_TID}')
    passes = (IMG_BYTES + 64 * WAVES * 16 - 1) // (64 * WAVES * 16)
    for p in range(passes):
        off = p * 64 * WAVES * 16
        part = off + 64 * WAVES * 16 > IMG_BYTES
        if part:
            e(f'  v_cmp_gt_u32_e32 vcc, {hex(IMG_BYTES - off)}, v{V_ROW}')
            e('  s_and_saveexec_b64 s[16:17], vcc')
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(off)}, v{V_ROW}')
        e(f'  global_load_dwordx4 v[8:11], v{V_LDSI}, s[10:11]')
        e('  s_waitcnt vmcnt(0)')
        e(f'  ds_write_b128 v{V_LDSI}, v[8:11]')
        if part:
            e('  s_mov_b64 exec, s[16:17]')
    e(f'  v_cmp_eq_u32_e32 vcc, 0, v{V_TID}')                           # thread 0: batch counter = 0
    e('  s_and_saveexec_b64 s[16:17], vcc')
    e(f'  v_mov_b32_e32 v{V_TMP}, {hex(LDS_CNT)}')
    e(f'  v_mov_b32_e32 v{V_TMP + 1}, 0')
    e(f'  ds_write_b32 v{V_TMP}, v{V_TMP + 1}')
    e('  s_mov_b64 exec, s[16:17]')
    e('  s_waitcnt lgkmcnt(0)')
    e('  s_barrier')
    # ---- the wave's batches of 16 ciphertexts: the k-th batch the workgroup hands out is wg + k * nwg
    #      (kernarg 36: the launch's workgroup count) -- persistent waves, no workgroup tails --------------
    e(f'  v_lshrrev_b32_e32 v{V_SH}, 6, v{V_TID}')                     # wave
    e('  s_nop 1')                                                      # VALU write -> v_readfirstlane: 1 state
    e('  v_readfirstlane_b32 s14, v5')
    e('  s_load_dword s19, s[0:1], 0x24')                              # workgroups launched
    e('  s_waitcnt lgkmcnt(0)')
    # wave area base + 4c; lane j's A-column write base (rows 38j ..), the ciphertext's A column
    e(f'  s_mul_i32 s15, s14, {WAVE_AREA}')
    e(f'  s_add_u32 s15, s15, {LDS_WAVES}')
    e(f'  v_and_b32_e32 v{V_TMP}, 63, v{V_TID}')
    e(f'  v_lshrrev_b32_e32 v{V_TMP + 1}, 2, v{V_TMP}')                # c
    e(f'  v_lshl_add_u32 v{V_LDSI}, v{V_TMP + 1}, 2, s15')             # area + 4c
    e(f'  v_and_b32_e32 v{V_TMP + 1}, 3, v{V_TMP}')                    # j
    e(f'  v_mul_u32_u24_e32 v{V_ZR}, {Q * RB}, v{V_TMP + 1}')
    e(f'  v_add_u32_e32 v{V_ZR}, v{V_ZR}, v{V_LDSI}')                  # area + 4c + 38 j RB
    # MFMA-layout addresses: lane l, m = l & 15, h = l >> 4
    e(f'  v_and_b32_e32 v{V_TMP + 1}, 15, v{V_TMP}')                   # m (= B column v)
    e(f'  v_lshrrev_b32_e32 v{V_SH}, 4, v{V_TMP}')                     # h
    e(f'  v_lshlrev_b32_e32 v{V_SH}, 4, v{V_SH}')                      # 16 h
    # copy slot of row m: M_A -> 0..7, M_B -> 8..15: slot = m < 4 ? m : m < 12 ? m + 4 : m - 8
    e(f'  v_add_u32_e32 v{V_A1}, 4, v{V_TMP + 1}')
    e(f'  v_subrev_u32_e32 v{V_A2}, 8, v{V_TMP + 1}')
    e(f'  v_cmp_gt_u32_e32 vcc, 12, v{V_TMP + 1}')
    e(f'  v_cndmask_b32_e32 v{V_A1}, v{V_A2}, v{V_A1}, vcc')
    e(f'  v_cmp_gt_u32_e32 vcc, 4, v{V_TMP + 1}')
    e(f'  v_cndmask_b32_e32 v{V_A1}, v{V_A1}, v{V_TMP + 1}, vcc')         # slot
    e(f'  v_mul_u32_u24_e32 v{V_A1}, {COPY}, v{V_A1}')
    e(f'  v_add_u32_e32 v{V_A1}, v{V_A1}, v{V_SH}')                    # slot*COPY + 16 h
    e(f'  v_add_u32_e32 v{V_A2}, {A2_OFF}, v{V_A1}')
    if A1_OFF:
        e(f'  v_add_u32_e32 v{V_A1}, {A1_OFF}, v{V_A1}')
    e(f'  v_add_u32_e32 v{V_C}, {CORR1_OFF}, v{V_SH}')                 # corrections: + 64 t (+ CORR2-CORR1)
    e(f'  v_mul_u32_u24_e32 v{V_B}, {QROW}, v{V_TMP + 1}')
    e(f'  v_add3_u32 v{V_B}, v{V_B}, v{V_SH}, s15')                    # staging row m + 16 h
    e(f'  v_mul_u32_u24_e32 v{V_G}, {GROW}, v{V_TMP + 1}')
    e(f'  v_lshrrev_b32_e32 v{V_TMP}, 1, v{V_SH}')                     # 8 h
    e(f'  v_add3_u32 v{V_G}, v{V_G}, v{V_TMP}, s15')                   # group row m + 8 h
    e(f'  v_and_b32_e32 v{V_TMP}, 63, v{V_TID}')
    e(f'  v_lshrrev_b32_e32 v{V_TMP}, 2, v{V_TMP}')                    # c
    e(f'  v_mul_u32_u24_e32 v{V_GR}, {GROW}, v{V_TMP}')
    e(f'  v_add_u32_e32 v{V_GR}, s15, v{V_GR}')                        # group row c
    e(f'  v_and_b32_e32 v{V_TMP + 1}, 1, v{V_TID}')
    e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {GCH}, v{V_TMP + 1}')
    e(f'  v_add_u32_e32 v{V_GR}, v{V_GR}, v{V_TMP + 1}')               # quad lanes 1, 3: the pair's 2nd chunk
    e(f'  v_mul_u32_u24_e32 v{V_Q3W}, {QROW}, v{V_TMP}')
    e(f'  v_add_u32_e32 v{V_Q3W}, s15, v{V_Q3W}')                      # staging row c (+ 128 j below)
    e(f'  v_and_b32_e32 v{V_SH}, 3, v{V_TID}')                         # j
    e(f'  v_lshlrev_b32_e32 v{V_TMP}, 7, v{V_SH}')
    e(f'  v_add_u32_e32 v{V_Q3W}, v{V_Q3W}, v{V_TMP}')
    e(f'  v_subrev_u32_e32 v{V_Q3W}, 4, v{V_Q3W}')                    # + 128 j - 4 (dword 32 j - 1)
    e(f'  v_lshlrev_b32_e32 v{V_SH}, 1, v{V_SH}')                      # 2 j (the row-I/O shift)
    if "ldsfree" in DBG:
        # timing knock-out (wrong results): the staging / group addresses spread so that their LDS
        # accesses have no bank conflicts -- the same instructions (the potential of a conflict-free layout)
        e(f'  v_and_b32_e32 v{V_TMP}, 63, v{V_TID}')                   # lane
        e(f'  v_lshl_add_u32 v{V_B}, v{V_TMP}, 4, s15')                # area + 16 lane
        e(f'  v_lshl_add_u32 v{V_G}, v{V_TMP}, 3, s15')                # area + 8 lane
        e(f'  v_lshl_add_u32 v{V_GR}, v{V_TMP}, 4, s15')               # area + 16 lane
        e(f'  v_lshl_add_u32 v{V_Q3W}, v{V_TMP}, 3, s15')
        e(f'  v_add_u32_e32 v{V_Q3W}, 0x184, v{V_Q3W}')               # area + 8 lane + 388 (== 4 mod 8, >= 380)
    e(f'  v_and_b32_e32 v{V_TID}, 63, v{V_TID}')
    e(f'  v_lshlrev_b32_e32 v{V_TID}, 7, v{V_TID}')                    # v0 = lane * 128 from here on
    e('.Lbatch:')
    e('  s_mov_b64 exec, 1')                                            # lane 0 takes the next batch
    e(f'  v_mov_b32_e32 v{V_TMP}, {hex(LDS_CNT)}')
    e(f'  v_mov_b32_e32 v{V_TMP + 1}, 1')
    e(f'  ds_add_rtn_u32 v{XB}, v{V_TMP}, v{V_TMP + 1}')
    e('  s_waitcnt lgkmcnt(0)')
    e('  s_mov_b64 exec, -1')
    e('  s_nop 1')
    e(f'  v_readfirstlane_b32 s13, v{XB}')
    e('  s_mul_i32 s13, s13, s19')
    e('  s_add_u32 s13, s13, s2')
    e('  s_lshl_b32 s13, s13, 4')                                       # first ciphertext of the batch
    if "prio" in DBG:
        e('  s_setprio 3')
    if "prioinv" in DBG:
        e('  s_setprio 0')
    e('  s_cmp_ge_u32 s13, s12')
    e('  s_cbranch_scc1 .Lend')
    # ROW = g*512 + j*128 = first*512 + lane*128; live lanes: g < count
    e('  s_lshl_b32 s17, s13, 9')
    e(f'  v_add_u32_e32 v{V_ROW}, s17, v{V_TID}')
    e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')
    e(f'  v_cmp_gt_u32_e32 vcc, s12, v{V_TMP}')
    e(f'  s_mov_b64 {LIVE}, vcc')

    # ---- row I/O helpers (gen_montprog.gen_quad's LOADW / STOREW, for this register plan) ---------------
    W0 = TB                                       # 33 loaded row words (ring area, free outside the product)

    GA = 146                                      # gathered row addresses v[146:147] (x), v[148:149] (y), the
    #                                               row 1 v[150:151], t v152 (the group read buffer, free here)
    WY = TB + 40                                  # y row words v86..v118 (ring area, free outside the product)

    def issue_row(sbase, sidx, W, ga):
        """load this lane's 33 words of operand row g (or of row idx[g] when the index list sidx is not null;
        idx < 0: the integer 1 from kctx) into W(0..32); the caller waits"""
        lab = f'.Lrow{len(o)}'
        e(f'  s_mov_b64 exec, {LIVE}')
        e(f'  s_cmp_eq_u64 {sidx}, 0')
        e(f'  s_cbranch_scc1 {lab}_direct')
        t = GA + 6
        e(f'  v_lshrrev_b32_e32 v{t}, 9, v{V_ROW}')                     # g
        e(f'  v_lshlrev_b32_e32 v{t}, 3, v{t}')
        e(f'  global_load_dwordx2 v[{ga}:{ga + 1}], v{t}, {sidx}')
        e(f'  v_mov_b32_e32 v{GA + 4}, s10')
        e(f'  v_mov_b32_e32 v{GA + 5}, s11')
        e(f'  v_add_co_u32_e32 v{GA + 4}, vcc, {hex(ONE_OFF)}, v{GA + 4}')
        e(f'  v_addc_co_u32_e32 v{GA + 5}, vcc, 0, v{GA + 5}, vcc')     # kctx + ONE_OFF
        e('  s_waitcnt vmcnt(0)')
        e(f'  v_cmp_gt_i64_e64 s[38:39], 0, v[{ga}:{ga + 1}]')          # idx < 0: the row 1
        e(f'  v_lshlrev_b64 v[{ga}:{ga + 1}], 9, v[{ga}:{ga + 1}]')
        lo, hi = sbase[2:-1].split(':')
        e(f'  v_mov_b32_e32 v{t}, s{hi}')
        e(f'  v_add_co_u32_e32 v{ga}, vcc, s{lo}, v{ga}')
        e(f'  v_addc_co_u32_e32 v{ga + 1}, vcc, v{t}, v{ga + 1}, vcc')
        e(f'  v_cndmask_b32_e64 v{ga}, v{ga}, v{GA + 4}, s[38:39]')
        e(f'  v_cndmask_b32_e64 v{ga + 1}, v{ga + 1}, v{GA + 5}, s[38:39]')
        e(f'  v_and_b32_e32 v{t}, 0x180, v{V_ROW}')                    # + 128 j
        e(f'  v_add_co_u32_e32 v{ga}, vcc, v{ga}, v{t}')
        e(f'  v_addc_co_u32_e32 v{ga + 1}, vcc, 0, v{ga + 1}, vcc')
        for i in range(8):
            e(f'  global_load_dwordx4 v[{W + 4 * i}:{W + 4 * i + 3}], v[{ga}:{ga + 1}], off offset:{16 * i}')
        e(f'  s_and_b64 exec, {LIVE}, s[20:21]')
        e(f'  global_load_dword v{W + 32}, v[{ga}:{ga + 1}], off offset:0x7c')
        e(f'  s_andn2_b64 exec, {LIVE}, s[20:21]')
        e(f'  global_load_dword v{W + 32}, v[{ga}:{ga + 1}], off offset:0x80')
        e(f'  s_mov_b64 exec, {LIVE}')
        e(f'  s_branch {lab}_issued')
        e(f'{lab}_direct:')
        for i in range(8):
            e(f'  global_load_dwordx4 v[{W + 4 * i}:{W + 4 * i + 3}], v{V_ROW}, {sbase} offset:{16 * i}')
        e(f'  v_add_u32_e32 v{V_TMP}, 0x80, v{V_ROW}')
        e(f'  v_add_u32_e32 v{V_TMP + 1}, 0x7c, v{V_ROW}')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, v{V_TMP}, v{V_TMP + 1}, s[20:21]')
        e(f'  global_load_dword v{W + 32}, v{V_TMP}, {sbase}')
        e(f'{lab}_issued:')

    def convert_row(W, dst):
        """W(0..32) (this lane's words of the row, dead lanes zero) -> 38 limbs dst(k): the 2j-bit funnel
        shift of the lane's quarter, then 27-bit fields (the row I/O of gen_montprog.gen_quad)"""
        e(f'  v_cndmask_b32_e64 v{W + 32}, v{W + 32}, 0, s[20:21]')
        for i in range(32):
            e(f'  v_alignbit_b32 v{W + i}, v{W + i + 1}, v{W + i}, v{V_SH}')
        e(f'  v_lshrrev_b32_e32 v{W + 32}, v{V_SH}, v{W + 32}')
        for jj in range(Q):
            a, sh = (B * jj) >> 5, (B * jj) & 31
            if sh + B <= 32:
                e(f'  v_bfe_u32 {dst(jj)}, v{W + a}, {sh}, {B}')
            else:
                e(f'  v_alignbit_b32 {dst(jj)}, v{W + a + 1}, v{W + a}, {sh}')
                e(f'  v_and_b32_e32 {dst(jj)}, {hex(MASK)}, {dst(jj)}')

    def limbs_to_words(src, U, t1, bo):
        """this lane's 38 limbs src(k) (bits [1026 j, 1026 j + 1026) of the number) -> dwords U(i) =
        bits [32 (32 j + i), +32) of the number (lane 3: bits >= 4096 dropped); STOREW's conversion"""
        for i in range(32):
            lo, hi = 32 * i, 32 * i + 31
            j0, j1 = lo // B, min(hi // B, Q - 1)
            e(f'  v_lshrrev_b32_e32 {U(i)}, {lo - B * j0}, {src(j0)}')
            for jj in range(j0 + 1, j1 + 1):
                e(f'  v_lshl_or_b32 {U(i)}, {src(jj)}, {B * jj - lo}, {U(i)}')
        e(f'  v_sub_u32_e32 {bo}, 32, v{V_SH}')
        e(f'  v_and_b32_e32 {bo}, 31, {bo}')                          # 32 - 2j (lane 0: 0)
        for i in range(31, 0, -1):                     # (U(i) << 2j) | (U(i-1) >> 32 - 2j); lane 0 keeps U(i)
            e(f'  v_alignbit_b32 {t1}, {U(i)}, {U(i - 1)}, {bo}')
            e(f'  v_cndmask_b32_e64 {U(i)}, {t1}, {U(i)}, s[22:23]')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp {t1}, {src(Q - 1)} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_sub_u32_e32 {bo}, {B}, v{V_SH}')                     # lane 0: shift 27 -> no bits
        e(f'  v_lshrrev_b32_e32 {t1}, {bo}, {t1}')
        e(f'  v_lshl_or_b32 {U(0)}, {U(0)}, v{V_SH}, {t1}')

    def ripple_quad(lab, vals, nv, carry, signed=False, width=B, t=(V_TMP + 0, None), top=None):
        """vals(k) (k < nv) limbs of `width` bits, a pending 64-bit carry-out in `carry` (per lane): the
        carries move to the next lane's limb 0 (lane 0 gets none) and ripple until none is left.  top: a
        register that collects quad lane 3's carries-out (< 2^32; otherwise they are dropped)."""
        shr = 'v_ashrrev_i64' if signed else 'v_lshrrev_b64'
        c0, c1 = carry
        a0, a1 = V_AI
        e(f'{lab}_loop:')
        if top is not None:
            e(f'  v_cndmask_b32_e64 v{a0}, 0, v{c0}, s[20:21]')
            e(f'  v_add_u32_e32 v{top}, v{top}, v{a0}')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{a0}, v{c0} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_mov_b32_dpp v{a1}, v{c1} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{c0}, v{a0}, 0, s[22:23]')
        e(f'  v_cndmask_b32_e64 v{c1}, v{a1}, 0, s[22:23]')
        e(f'  v_or_b32_e32 v{a0}, v{c0}, v{c1}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{a0}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        for k in range(nv):
            e(f'  v_mad_u64_u32 v[{c0}:{c1}], vcc, {vals(k)}, 1, v[{c0}:{c1}]')
            e(f'  v_and_b32_e32 {vals(k)}, {hex((1 << width) - 1)}, v{c0}')
            e(f'  {shr} v[{c0}:{c1}], {width}, v[{c0}:{c1}]')
            if k == 1 and nv > 2:                # a carry absorbed by limbs 0, 1 everywhere (the usual case):
                e(f'  v_or_b32_e32 v{a0}, v{c0}, v{c1}')      # no carry-out changes, nothing left to hand on
                e(f'  v_cmp_ne_u32_e32 vcc, 0, v{a0}')
                e('  s_nop 4')
                e(f'  s_cbranch_vccz {lab}_done')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    e('// @phase load')
    # ---- 1. x -> X limbs; y -> limbs -> the wave's A column (rows 38j + k of column c) ------------------
    # both rows in flight at once (one memory latency per batch), then y's limbs (via X) to the A column
    YW = MZ_YI if MFZ else WY                     # the matrix-core product keeps y's dwords at v80 (section 2M)
    issue_row('s[4:5]', 's[34:35]', W0, GA)
    issue_row('s[6:7]', 's[36:37]', YW, GA + 2)
    e('  s_waitcnt vmcnt(0)')
    e('  s_not_b64 exec, exec')                                          # dead lanes: zero operands
    e('  s_cbranch_execz .Lrows_live')                                   # (only in a partial batch)
    for i in range(33):
        e(f'  v_mov_b32_e32 v{W0 + i}, 0')
        e(f'  v_mov_b32_e32 v{YW + i}, 0')
    e('.Lrows_live:')
    e('  s_mov_b64 exec, -1')
    if not MFZ:
        convert_row(WY, X)
        for k in range(Q):
            e(f'  ds_write_b32 v{V_ZR}, {X(k)} offset:{k * RB}')
        convert_row(W0, X)
        e('  s_waitcnt lgkmcnt(0)')

    def classic_product():
        e('// @phase product')
        e(f'  v_mov_b64_e32 {pair(HO)}, 0')
        e(f'  v_mov_b32_e32 v{VMASK}, {hex(MASK)}')
        e(f'  v_cndmask_b32_e64 v{VMASK}, v{VMASK}, 0, s[20:21]')
        if "prio" in DBG:
            e('  s_setprio 0')
        if "prioinv" in DBG:
            e('  s_setprio 3')
        # ---- 2. z = x y: 152 steps; step i reads a_i (prefetched), adds a_i X into the window, retires the
        #         lowest column: its carry stays in the lane's next column, its low 27 bits go one lane down (the
        #         top column of lane j-1: one v_and_b32 with DPP into the hand-off pair, lane 3 receiving 0, that
        #         the next step's top multiply-add takes as its addend, so the ring needs no fresh column), and
        #         lane 0's -- the product limb z_i, written unmasked and masked when read back -- into A-column
        #         row i.  Three VALU instructions per step beside the 38 multiply-adds. -------------------------
        for k in range(NT):
            e(f'  v_mov_b64_e32 {T(k)}, 0')
        e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI}')
        e('  s_waitcnt lgkmcnt(0)')

        def step(u, row, prefetch):
            ai, nai = f"v{V_AI[u % 2]}", f"v{V_AI[(u + 1) % 2]}"
            for k in range(Q):
                if "noprod" not in DBG:
                    src2 = pair(HO) if k == Q - 1 else T(u + k)   # T(u + Q - 1): the slot of the retired T(u - 1)
                    e(f'  v_mad_u64_u32 {T(u + k)}, vcc, {ai}, {X(k)}, {src2}')
                if k == 2:
                    e(f'  v_lshrrev_b64 {tmp}, {B}, {T(u)}')
                if k == 5:
                    e(f'  v_lshl_add_u64 {T(u + 1)}, {tmp}, 0, {T(u + 1)}')
                if k == 10 and prefetch is not None:
                    e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{prefetch * RB}')
                if k == 12:                              # after the read: the step's wait leaves the write out
                    e('  s_mov_b64 exec, s[22:23]')
                    e(f'  ds_write_b32 v{V_LDSI}, {Tlo(u)} offset:{row * RB}')
                    e('  s_mov_b64 exec, -1')
            e(f'  v_and_b32_dpp v{HO}, {Tlo(u)}, v{VMASK} quad_perm:[1,2,3,0] {DPP}')
            if prefetch is not None:
                e('  s_waitcnt lgkmcnt(1)')

        NTRIP, TL = S // NT, S % NT
        assert NT % 2 == 0 and TL == 0
        e(f'  s_mov_b32 s18, {NTRIP}')
        e('.Ltrip:')
        for u in range(NT):
            step(u, u, u + 1)
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(NT * RB)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_cmp_lg_u32 s18, 0')
        e('  s_cbranch_scc1 .Ltrip')
        for u in range(TL):
            step(u, u, u + 1 if u + 1 < TL else None)
        e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(NTRIP * NT * RB)}, v{V_LDSI}')

        e('// @phase window')
        if "prio" in DBG:
            e('  s_setprio 3')
        if "prioinv" in DBG:
            e('  s_setprio 0')
        # ---- 3. window -> W limbs (X), W -> dwords WD; z mod 2^4104 limbs (LDS) -> dwords ZL ---------------
        e(f'  v_mov_b64_e32 {tmp}, 0')
        for k in range(Q):                            # columns 152 + k: T(k), the top one in the hand-off pair
            e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {T(TL + k) if k < Q - 1 else pair(HO)}')
            e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
        ripple_quad('.Lrw', X, Q, (V_TMP, V_TMP + 1))

    # ---- 2K. z = x y by one level of Karatsuba on 76-limb halves (KARA): x = xL + xH B^76, y = yL + yH B^76,
    #          P1 = (xL + xH)(yL + yH), P0 = xL yL, P2 = xH yH, z = P0 + (P1 - P0 - P2) B^76 + P2 B^152.  Each is a
    #          76-step operand scan over a 76-limb window of 19 limbs per quad lane (the step of section 2 with
    #          19 instead of 38 multiply-adds): 3 x 76 x 19 = 4,332 MADs per lane against 152 x 38 = 5,776.  The
    #          multipliers come from the A column (rows 0..75 yL, 76..151 yH; P1 adds the two rows); P1 runs first
    #          and keeps its retired limbs in registers, P0 and P2 retire theirs into their consumed rows, so the
    #          A column ends as (P0 low, P2 low).  The combination is signed limb arithmetic, normalised as one
    #          228-limb number (blocks 1..3 of z; block 0 is P0 low) with carries across lanes and blocks. -----
    Q2 = Q // 2                                   # 19 window limbs per lane
    # the multiplier prefetch after the step's ninth multiply-add (timing knob pfN: after the first measured no
    # faster, profiles/r05f_addb_libs_ab.jsonl)
    KARA_PF = next((int(t[2:]) for t in DBG if t.startswith('pf') and t[2:].isdigit()), 8)
    # P1 retires lane 0's column into its quad lane's register with one v_cndmask_b32 whose src0 is the DPP
    # broadcast of lane 0 (vcc = the lanes that keep theirs: the steps' multiply-adds write their carry-outs,
    # always 0, to s[40:41] instead of vcc); "nocnd" keeps the broadcast + v_cndmask_b32_e64 pair (A/B)
    CND = "nocnd" not in DBG and "stamp" not in DBG            # (the stamp build's timers live in s[40:..])
    CSINK = "s[40:41]" if CND else "vcc"
    HALF = S // 2                                 # 76
    XW = {"L": 46, "H": 65, "S": 84}              # 19-limb windows of xL, xH, xL + xH (later P0 / P2 / P1 high)
    HO2 = 104                                     # hand-off pair v[104:105] (v105 stays 0)
    P1L, P1TOP = 146, 165                         # P1's retired limbs (lane k: limbs 19 k + p), lane 3: limb 152
    BI = (125, 126)                               # P1: the yH multiplier's double buffer
    RT = 127                                      # P1: the retired limb broadcast over the quad
    VZ = 128                                      # A-column base of lane j's 19-limb blocks: area + 4c + 19 j RB
    CB = (129, 130, 131)                          # combination: carries of blocks 1..3
    CI = (132, 133, 134)                          # their carries-in
    RO = (135, 136, 137)                          # rotated carries

    def T2(k):
        k %= Q2
        return f"v[{XB + 2 * k}:{XB + 2 * k + 1}]"

    def T2lo(k):
        return f"v{XB + 2 * (k % Q2)}"

    def W_(nm):
        return lambda k: f"v{XW[nm] + k}"

    def kara_step(mode, u, W):
        """step u (0..37 of a two-trip loop body) of pass `mode`: multiplier rows u (+76: yH); P1 adds the yL
        and yH limbs, P0 / P2 retire lane 0's column into rows u / 76 + u, P1 into register u mod 19 of the
        quad lane (2 trip + u div 19) (mask s[38:39], shifted per trip)"""
        ai, nai = f"v{V_AI[u % 2]}", f"v{V_AI[(u + 1) % 2]}"
        bi, nbi = f"v{BI[u % 2]}", f"v{BI[(u + 1) % 2]}"
        if mode == "P1":
            e(f'  v_add_u32_e32 {ai}, {ai}, {bi}')              # yL_i + yH_i (< 2^28)
        for k in range(Q2):
            if "noprod" not in DBG:
                src2 = pair(HO2) if k == Q2 - 1 else T2(u + k)
                e(f'  v_mad_u64_u32 {T2(u + k)}, {CSINK}, {ai}, {W(k)}, {src2}')
            if k == 2:
                e(f'  v_lshrrev_b64 {tmp}, {B}, {T2(u)}')
            if k == 5:
                e(f'  v_lshl_add_u64 {T2(u + 1)}, {tmp}, 0, {T2(u + 1)}')
            if k == KARA_PF:                          # prefetch the next step's multiplier(s)
                if mode in ("P1", "P0"):
                    e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(u + 1) * RB}')
                if mode == "P1":
                    e(f'  ds_read_b32 {nbi}, v{V_LDSI} offset:{(HALF + u + 1) * RB}')
                if mode == "P2":
                    e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(HALF + u + 1) * RB}')
            if k == 12 and mode in ("P0", "P2"):      # after the read: the step's wait leaves the write out
                e('  s_mov_b64 exec, s[22:23]')
                e(f'  ds_write_b32 v{V_LDSI}, {T2lo(u)} offset:{(u if mode == "P0" else HALF + u) * RB}')
                e('  s_mov_b64 exec, -1')
            if k == 13 and mode == "P1" and not CND:
                e(f'  v_mov_b32_dpp v{RT}, {T2lo(u)} quad_perm:[0,0,0,0] {DPP}')
            if k == 16 and mode == "P1":
                if CND:
                    e(f'  v_cndmask_b32_dpp v{P1L + u % Q2}, {T2lo(u)}, v{P1L + u % Q2}, vcc quad_perm:[0,0,0,0] {DPP}')
                else:
                    e(f'  v_cndmask_b32_e64 v{P1L + u % Q2}, v{P1L + u % Q2}, v{RT}, s[38:39]')
        e(f'  v_and_b32_dpp v{HO2}, {T2lo(u)}, v{VMASK} quad_perm:[1,2,3,0] {DPP}')
        if mode == "P1" and u % Q2 == Q2 - 1:
            e('  s_lshl_b64 s[38:39], s[38:39], 1')          # the next trip's quad lane
            if CND:
                e('  s_not_b64 vcc, s[38:39]')
        e(f'  s_waitcnt lgkmcnt({0 if mode == "P1" else 1})')

    def kara_pass(mode, W, out, top=None):
        """one 76 x 76 product over window W; its top 76 (+1) limbs normalised into out(k) (19 per lane)"""
        lab = f'.Lk{mode}'
        for k in range(Q2):
            e(f'  v_mov_b64_e32 {T2(k)}, 0')
        e(f'  v_mov_b64_e32 {pair(HO2)}, 0')
        if mode in ("P1", "P0"):
            e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI}')
        if mode == "P1":
            e(f'  ds_read_b32 v{BI[0]}, v{V_LDSI} offset:{HALF * RB}')
            e('  s_mov_b64 s[38:39], s[22:23]')                  # trip 0: quad lane 0
            if CND:
                e('  s_not_b64 vcc, s[38:39]')
        if mode == "P2":
            e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI} offset:{HALF * RB}')
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_mov_b32 s18, 2')
        e(f'{lab}_trip:')
        for u in range(2 * Q2):
            kara_step(mode, u, W)
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(2 * Q2 * RB)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_cmp_lg_u32 s18, 0')
        e(f'  s_cbranch_scc1 {lab}_trip')
        e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(HALF * RB)}, v{V_LDSI}')
        # the window: columns 76 + k of the lane's 19 (the top one in the hand-off pair), normalised
        e(f'  v_mov_b64_e32 {tmp}, 0')
        for k in range(Q2):
            e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {T2(k) if k < Q2 - 1 else pair(HO2)}')
            e(f'  v_and_b32_e32 {out(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
        ripple_quad(f'{lab}_rw', out, Q2, (V_TMP, V_TMP + 1), top=top)

    def kara_product():
        e('// @phase product')
        e(f'  v_mov_b32_e32 v{VMASK}, {hex(MASK)}')
        e(f'  v_cndmask_b32_e64 v{VMASK}, v{VMASK}, 0, s[20:21]')
        # the windows: lane j of xL holds limbs 19 j .. 19 j + 18, i.e. limbs 19 (j & 1) + p of quad lane j >> 1's
        # 38 (xH: of quad lane 2 + (j >> 1)); xS = xL + xH limb by limb (28 bits)
        e('  s_or_b64 s[16:17], s[24:25], s[20:21]')                # quad lanes 1, 3
        ta, tb = f"v{V_AI[0]}", f"v{V_AI[1]}"
        for p in range(Q2):
            for nm, qp in (("L", "[0,0,1,1]"), ("H", "[2,2,3,3]")):
                e(f'  v_mov_b32_dpp {ta}, {X(p)} quad_perm:{qp} {DPP}')
                e(f'  v_mov_b32_dpp {tb}, {X(Q2 + p)} quad_perm:{qp} {DPP}')
                e(f'  v_cndmask_b32_e64 v{XW[nm] + p}, {ta}, {tb}, s[16:17]')
            e(f'  v_add_u32_e32 v{XW["S"] + p}, v{XW["L"] + p}, v{XW["H"] + p}')
        e(f'  v_mov_b32_e32 v{P1TOP}, 0')
        kara_pass("P1", W_("S"), W_("S"), top=P1TOP)                # P1 high -> the xS registers
        kara_pass("P0", W_("L"), W_("L"))                           # P0 high -> xL's
        kara_pass("P2", W_("H"), W_("H"))                           # P2 high -> xH's
        e('// @phase window')
        # z1 (limbs 76 + 19 j + p) = P0H + P1L - P0L - P2L, z2 (152 + ...) = P2L + P1H - P0H - P2H,
        # z3 (228 + ...) = P2H (+ P1's limb 152 at z limb 228); P0L / P2L are A-column rows 19 j + p / 76 + 19 j + p
        e(f'  v_add_u32_e32 v{VZ}, v{V_LDSI}, v{V_ZR}')
        e(f'  v_lshrrev_b32_e32 v{VZ}, 1, v{VZ}')                    # area + 4c + 19 j RB
        R0, R2 = XB, XB + Q2                                        # the ring is dead
        for p in range(Q2):
            e(f'  ds_read_b32 v{R0 + p}, v{VZ} offset:{p * RB}')
            e(f'  ds_read_b32 v{R2 + p}, v{VZ} offset:{(HALF + p) * RB}')
        e('  s_waitcnt lgkmcnt(0)')
        P0H, P1H, P2H = XW["L"], XW["S"], XW["H"]
        for p in range(Q2):
            e(f'  v_and_b32_e32 v{R0 + p}, {hex(MASK)}, v{R0 + p}')
            e(f'  v_and_b32_e32 v{R2 + p}, {hex(MASK)}, v{R2 + p}')
            e(f'  v_and_b32_e32 v{P1L + p}, {hex(MASK)}, v{P1L + p}')
            e(f'  v_add_u32_e32 v{P1L + p}, v{P1L + p}, v{P0H + p}')
            e(f'  v_sub_u32_e32 v{P1L + p}, v{P1L + p}, v{R0 + p}')
            e(f'  v_sub_u32_e32 v{P1L + p}, v{P1L + p}, v{R2 + p}')       # z1
            e(f'  v_add_u32_e32 v{P1H + p}, v{P1H + p}, v{R2 + p}')
            e(f'  v_sub_u32_e32 v{P1H + p}, v{P1H + p}, v{P0H + p}')
            e(f'  v_sub_u32_e32 v{P1H + p}, v{P1H + p}, v{P2H + p}')       # z2
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{RT}, v{P1TOP} quad_perm:[3,3,3,3] {DPP}')   # P1's limb 152 -> z3 limb 0 of lane 0
        e(f'  v_cndmask_b32_e64 v{RT}, 0, v{RT}, s[22:23]')
        e(f'  v_add_u32_e32 v{P2H}, v{P2H}, v{RT}')
        blocks = (P1L, P1H, P2H)                                    # z1, z2, z3: signed limbs
        for b, base in enumerate(blocks):                           # each lane's segments, carries out
            for p in range(Q2):
                if p:
                    e(f'  v_add_u32_e32 v{base + p}, v{base + p}, v{CB[b]}')
                e(f'  v_ashrrev_i32_e32 v{CB[b]}, {B}, v{base + p}')
                e(f'  v_and_b32_e32 v{base + p}, {hex(MASK)}, v{base + p}')
        # carries across segments: block b, lane j -> lane j + 1; lane 3 -> block b + 1, lane 0 (z < B^304: the top
        # segment's carry is 0 at the end); repeated until no segment receives a carry
        lab = f'.Lkc{len(o)}'
        e(f'{lab}_loop:')
        e('  s_nop 1')
        for b in range(3):
            e(f'  v_mov_b32_dpp v{RO[b]}, v{CB[b]} quad_perm:[3,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{CI[0]}, v{RO[0]}, 0, s[22:23]')
        e(f'  v_cndmask_b32_e64 v{CI[1]}, v{RO[1]}, v{RO[0]}, s[22:23]')
        e(f'  v_cndmask_b32_e64 v{CI[2]}, v{RO[2]}, v{RO[1]}, s[22:23]')
        e(f'  v_or3_b32 v{RT}, v{CI[0]}, v{CI[1]}, v{CI[2]}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{RT}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        for b in range(3):
            e(f'  v_mov_b32_e32 v{CB[b]}, v{CI[b]}')
        for p in range(Q2):
            for b, base in enumerate(blocks):
                e(f'  v_add_u32_e32 v{base + p}, v{base + p}, v{CB[b]}')
                e(f'  v_ashrrev_i32_e32 v{CB[b]}, {B}, v{base + p}')
                e(f'  v_and_b32_e32 v{base + p}, {hex(MASK)}, v{base + p}')
            if p == 1:                                # absorbed by limbs 0, 1 everywhere (the usual case)
                e(f'  v_or3_b32 v{RT}, v{CB[0]}, v{CB[1]}, v{CB[2]}')
                e(f'  v_cmp_ne_u32_e32 vcc, 0, v{RT}')
                e('  s_nop 4')
                e(f'  s_cbranch_vccz {lab}_done')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')
        # z1 -> A-column rows 76 + 19 j + p (rows 0..151 = z mod 2^4104 as limbs, read below as before)
        for p in range(Q2):
            e(f'  ds_write_b32 v{VZ}, v{P1L + p} offset:{(HALF + p) * RB}')
        # z >> 4104 = (z2, z3) -> X: lane j holds limbs 38 j + k, i.e. segment 2 j + (k >= 19) of blocks 2, 3
        ta, tb = f"v{V_AI[0]}", f"v{V_AI[1]}"
        e('  s_or_b64 s[16:17], s[22:23], s[24:25]')                # quad lanes 0, 1
        for k in range(Q2):
            for half, qp in ((0, "[0,2,0,2]"), (1, "[1,3,1,3]")):
                e(f'  v_mov_b32_dpp {ta}, v{P1H + k} quad_perm:{qp} {DPP}')
                e(f'  v_mov_b32_dpp {tb}, v{P2H + k} quad_perm:{qp} {DPP}')
                e(f'  v_cndmask_b32_e64 {X(Q2 * half + k)}, {tb}, {ta}, s[16:17]')   # lanes 0, 1: block 2
        e('  s_waitcnt lgkmcnt(0)')

    # ---- 2M. z = x y on the matrix cores (MFZ; tools/addb_mfz_model.py).  Both rows become balanced base-256
    #          digits in place (x + 0x80..80, every byte XORed with 0x80; the carry out is digit 512), y's dwords
    #          are reversed and byte-swapped; then per ciphertext c of the batch (a loop of 16): its quad stages
    #          x (forward) and y (reversed) in the wave's area, every lane builds its nine A fragments (row i:
    #          digits i + 64 t + k + 1, a dword-aligned five-dword read funnel-shifted by v_alignbyte_b32), reads
    #          the 13 B fragments (one aligned 16-byte read per v = 4 u - t) and issues the 28 MFMAs into four
    #          accumulator sets (column blocks u); each lane folds its four rows into an int64 group, lane l
    #          normalises groups 4 l .. 4 l + 3 and the carries move lane to lane (DPP wave_shr) until none is left;
    #          z (256 dwords) and z >> 4104 (128) go to LDS, from where the quad reads ZL / ZL128 / WD. ---------
    def mfz_product():
        e('// @phase product')
        XI, YI = W0, MZ_YI                        # 32 dwords each (+ the digit-512 slot: v78 / v112)
        CXI, CYI = XI + 32, YI + 32
        DA = (114, 118, 122, 126)                 # accumulators of the column blocks u = 0..3
        AT = {t: 8 + 4 * n for n, t in enumerate(MZ_TS)}       # A fragments v8..v43
        R4 = (44, 45, 79)                         # the A reads' fifth dwords
        BB = (130, 134, 148)                      # B fragments (three buffers)
        V_AX, V_S, V_BY, V_GW, V_GR, V_ZA, V_WA, V_XS, V_YS, V_QZ, V_QW = \
            146, 147, 152, 153, 154, 156, 157, 158, 159, 160, 161
        V_WB = 113
        CIN, SG, C1, NXT = 164, 165, 166, 167
        CO, BIN, TT = 114, 115, 116               # conversion scratch (the accumulators are free then)
        GQ = 8                                    # the four groups of a lane (pairs v8..v15, A fragments dead)
        WW = 16                                   # its four W dwords
        assert AT[MZ_TS[-1]] + 4 <= 44 and len(MZ_TS) == 9
        # ---- balanced digits (all 16 ciphertexts at once, quad layout) ----
        VK = 117                                  # 0x80808080 (v_addc reads vcc: no SGPR beside it)
        e(f'  v_mov_b32_e32 v{VK}, s33')
        for R, cx in ((XI, CXI), (YI, CYI)):
            lab = f'.Lmzb{R}'
            e(f'  v_add_co_u32_e32 v{R}, vcc, s33, v{R}')
            for i in range(1, 32):
                e(f'  v_addc_co_u32_e32 v{R + i}, vcc, v{VK}, v{R + i}, vcc')
            e(f'  v_cndmask_b32_e64 v{CO}, 0, 1, vcc')
            e(f'  v_mov_b32_e32 v{cx}, 0')
            e(f'{lab}_loop:')
            e(f'  v_add_u32_e32 v{cx}, v{cx}, v{CO}')                 # lane 3: the carry out (digit 512)
            e('  s_nop 1')
            e(f'  v_mov_b32_dpp v{BIN}, v{CO} quad_perm:[0,0,1,2] {DPP}')
            e(f'  v_cndmask_b32_e64 v{BIN}, v{BIN}, 0, s[22:23]')     # lane 0 receives none
            e(f'  v_mov_b32_e32 v{CO}, 0')
            e(f'  v_cmp_ne_u32_e32 vcc, 0, v{BIN}')
            e('  s_nop 4')
            e(f'  s_cbranch_vccz {lab}_done')
            e(f'  v_add_co_u32_e32 v{R}, vcc, v{R}, v{BIN}')
            e('  s_nop 4')
            e(f'  s_cbranch_vccz {lab}_loop')                          # absorbed by dword 0 everywhere (usual)
            e('  s_and_saveexec_b64 s[38:39], vcc')
            for i in range(1, 32):
                e(f'  v_addc_co_u32_e32 v{R + i}, vcc, 0, v{R + i}, vcc')
            e(f'  v_cndmask_b32_e64 v{CO}, 0, 1, vcc')
            e('  s_mov_b64 exec, s[38:39]')
            e(f'  s_branch {lab}_loop')
            e(f'{lab}_done:')
            for i in range(32):
                e(f'  v_xor_b32_e32 v{R + i}, s33, v{R + i}')
        # y reversed and byte-swapped: YI[m] = bswap(y dword 31 - m of the lane)
        e('  s_mov_b32 s48, 0x10203')
        for m in range(16):
            e(f'  v_perm_b32 v{TT}, v{YI + m}, v{YI + m}, s48')
            e(f'  v_perm_b32 v{YI + m}, v{YI + 31 - m}, v{YI + 31 - m}, s48')
            e(f'  v_mov_b32_e32 v{YI + 31 - m}, v{TT}')
        # ---- per-lane addresses (l the lane, i = l & 15, h = l >> 4, q = l & 3) ----
        T0, T1, T2, T3 = 8, 9, 10, 11
        e(f'  v_lshrrev_b32_e32 v{T0}, 7, v{V_TID}')                  # l
        e(f'  v_and_b32_e32 v{T1}, 15, v{T0}')                         # i
        e(f'  v_lshrrev_b32_e32 v{T2}, 4, v{T0}')                      # h
        e(f'  v_lshl_add_u32 v{T3}, v{T2}, 4, v{T1}')                  # i + 16 h
        e(f'  v_add_u32_e32 v{T3}, {MZ_XOFF - MZ_DELTA}, v{T3}')
        e(f'  v_lshrrev_b32_e32 v{T3}, 2, v{T3}')
        e(f'  v_lshl_add_u32 v{V_AX}, v{T3}, 2, s15')
        e(f'  v_subrev_u32_e32 v{V_AX}, {64 - MZ_XS}, v{V_AX}')       # tile t at offset 64 (t + 1)
        e(f'  v_add_u32_e32 v{V_S}, {MZ_XOFF - MZ_DELTA}, v{T1}')
        e(f'  v_and_b32_e32 v{V_S}, 3, v{V_S}')                        # the byte shift
        e(f'  v_lshlrev_b32_e32 v{T3}, 4, v{T2}')
        e(f'  v_lshlrev_b32_e32 v{V_BY}, 4, v{T1}')
        e(f'  v_sub_u32_e32 v{V_BY}, v{T3}, v{V_BY}')                  # 16 h - 16 j
        e(f'  v_add_u32_e32 v{V_BY}, {MZ_YS + MZ_RY - MZ_DELTA - 64 * MZ_V[-1]}, v{V_BY}')
        e(f'  v_add_u32_e32 v{V_BY}, s15, v{V_BY}')
        e(f'  v_lshlrev_b32_e32 v{V_GW}, 3, v{T2}')
        e(f'  v_lshl_add_u32 v{V_GW}, v{T1}, 5, v{V_GW}')
        e(f'  v_add_u32_e32 v{V_GW}, {MZ_GS}, v{V_GW}')
        e(f'  v_add_u32_e32 v{V_GW}, s15, v{V_GW}')                    # group 4 j + h (+ 64 u)
        e(f'  v_mov_b32_e32 v{V_WB}, s15')
        for reg, sh, base in ((V_GR, 5, MZ_GS), (V_ZA, 4, MZ_ZS), (V_WA, 4, MZ_WS + 12 - 512)):
            e(f'  v_lshlrev_b32_e32 v{reg}, {sh}, v{T0}')
            e(f'  v_add3_u32 v{reg}, v{reg}, v{V_WB}, {base}' if 0 <= base <= 64 else
              f'  v_add_u32_e32 v{reg}, {base}, v{reg}')
            if not 0 <= base <= 64:
                e(f'  v_add_u32_e32 v{reg}, s15, v{reg}')
        e(f'  v_and_b32_e32 v{T3}, 3, v{T0}')                          # q
        e(f'  v_lshlrev_b32_e32 v{T3}, 7, v{T3}')                      # 128 q
        e(f'  v_add_u32_e32 v{V_XS}, {MZ_XS + MZ_XOFF}, v{T3}')
        e(f'  v_add_u32_e32 v{V_XS}, s15, v{V_XS}')
        e(f'  v_sub_u32_e32 v{V_YS}, v{V_WB}, v{T3}')
        e(f'  v_add_u32_e32 v{V_YS}, {MZ_YS + MZ_RY - 127 - 16}, v{V_YS}')
        e(f'  v_add_u32_e32 v{V_QZ}, {MZ_ZS}, v{T3}')
        e(f'  v_add_u32_e32 v{V_QZ}, s15, v{V_QZ}')
        e(f'  v_add_u32_e32 v{V_QW}, {MZ_WS}, v{T3}')
        e(f'  v_add_u32_e32 v{V_QW}, s15, v{V_QW}')
        # ---- zero the staging pads: [XS, YS + YAREA) ----
        for k in range(4):
            e(f'  v_mov_b32_e32 v{DA[0] + k}, 0')
        e(f'  v_lshrrev_b32_e32 v{T3}, 3, v{V_TID}')                  # 16 l
        e(f'  v_add_u32_e32 v{T3}, s15, v{T3}')
        e(f'  ds_write_b128 v{T3}, {quad4(DA[0])} offset:{MZ_XS}')
        e(f'  ds_write_b128 v{T3}, {quad4(DA[0])} offset:{MZ_XS + 1024}')
        e('  s_mov_b32 s46, 0')
        e('  s_mov_b32 s47, -1')                                       # lanes 32..63
        e('  s_mov_b64 s[44:45], 0xf')                                 # the quad of ciphertext c
        e('  s_mov_b32 s42, 16')
        e('.Lmz_ct:')
        # ---- stage ciphertext c: x forward at XS + XOFF, y reversed (digit b at YS + RY - b) ----
        e('  s_mov_b64 exec, s[44:45]')
        for k in range(8):
            e(f'  ds_write_b128 v{V_XS}, {quad4(XI + 4 * k)} offset:{16 * k}')
            e(f'  ds_write_b128 v{V_YS}, {quad4(YI + 4 * k)} offset:{16 + 16 * k}')
        e('  s_and_b64 exec, s[44:45], s[20:21]')                      # quad lane 3: the digits 512
        e(f'  ds_write_b32 v{V_XS}, v{CXI} offset:{512 - 384}')
        e(f'  v_lshlrev_b32_e32 v{TT}, 24, v{CYI}')
        e(f'  ds_write_b32 v{V_YS}, v{TT} offset:{MZ_RY - 515 - (MZ_RY - 127 - 16 - 384)}')
        e('  s_mov_b64 exec, -1')
        # ---- A fragments: three reads per tile, then the funnel shift ----
        q = []

        def issue(tag, ins):
            e(ins)
            q.append(tag)

        def wait_for(tag):
            if tag in q:
                i = len(q) - 1 - q[::-1].index(tag)
                e(f'  s_waitcnt lgkmcnt({min(len(q) - i - 1, 15)})')
                del q[:i + 1]
        for n, t in enumerate(MZ_TS):
            d = 16 * (t + 1)
            a = AT[t]
            issue(('a', t), f'  ds_read2_b32 v[{a}:{a + 1}], v{V_AX} offset0:{d} offset1:{d + 1}')
            issue(('a', t), f'  ds_read2_b32 v[{a + 2}:{a + 3}], v{V_AX} offset0:{d + 2} offset1:{d + 3}')
            issue(('a', t), f'  ds_read_b32 v{R4[n % 3]}, v{V_AX} offset:{4 * (d + 4)}')
            if n >= 2:
                tp = MZ_TS[n - 2]
                wait_for(('a', tp))
                ap, r4 = AT[tp], R4[(n - 2) % 3]
                for k in range(4):
                    hi = f"v{ap + k + 1}" if k < 3 else f"v{r4}"
                    e(f'  v_alignbyte_b32 v{ap + k}, {hi}, v{ap + k}, v{V_S}')
        for n in range(len(MZ_TS) - 2, len(MZ_TS)):
            tp = MZ_TS[n]
            wait_for(('a', tp))
            ap, r4 = AT[tp], R4[n % 3]
            for k in range(4):
                hi = f"v{ap + k + 1}" if k < 3 else f"v{r4}"
                e(f'  v_alignbyte_b32 v{ap + k}, {hi}, v{ap + k}, v{V_S}')
        # ---- B fragments and the MFMAs, by v = 4 u - t ----
        vs = MZ_V
        first = set()
        last_mfma = {}

        def read_b(n):
            issue(('b', n), f'  ds_read_b128 {quad4(BB[n % 3])}, v{V_BY} offset:{64 * (vs[-1] - vs[n])}')
        read_b(0)
        read_b(1)
        e('  s_nop 1')                                                 # VALU-written A -> MFMA operand
        last_v = {u: max(4 * uu - t for t, uu in MZ_TILES if uu == u) for u in range(4)}
        folded = []

        def fold(u):
            since = sum(1 for ln in o[last_mfma[u] + 1:] if ln.startswith('  '))
            need = 19 - since                                          # XDL -> VALU read (as XDL_WAIT)
            while need > 0:
                e(f'  s_nop {min(need, 8) - 1}')
                need -= 8
            acc = DA[u]
            e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc}, 1, 0')
            e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 1}, s30, {pair(PG)}')
            e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 2}, s31, {pair(PG)}')
            e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 3}, s32, {pair(PG)}')
            issue(('w', u), f'  ds_write_b64 v{V_GW}, {pair(PG)} offset:{512 * u}')
            folded.append(u)
        for n, v in enumerate(vs):
            wait_for(('b', n))
            for t, u in MZ_TILES:
                if 4 * u - t != v:
                    continue
                src_c = quad4(DA[u]) if u in first else '0'
                first.add(u)
                if "mzmfma" not in DBG:           # timing knock-out (wrong results): no MFMAs
                    e(f'  v_mfma_i32_16x16x64_i8 {quad4(DA[u])}, {quad4(AT[t])}, {quad4(BB[n % 3])}, {src_c}')
                last_mfma[u] = len(o) - 1
            if n + 2 < len(vs):
                read_b(n + 2)
            for u in range(4):                    # a block two v-steps past its last MFMA: fold it meanwhile
                if u not in folded and last_v[u] <= v - 2:
                    fold(u)
        # ---- fold: rows 4 h' .. 4 h' + 3 of block u -> group 4 j + h' + 64 u ----
        for u in range(4):
            if u not in folded:
                fold(u)
        if "mznorm" in DBG:                       # timing knock-out (wrong results): no normalisation / delivery
            e('  s_branch .Lmz_next')
        # ---- normalisation: lane l chains groups 4 l .. 4 l + 3 (carry-in 0) ----
        e(f'  ds_read_b128 v[{GQ}:{GQ + 3}], v{V_GR}')
        e(f'  ds_read_b128 v[{GQ + 4}:{GQ + 7}], v{V_GR} offset:16')
        e('  s_waitcnt lgkmcnt(0)')
        for k in range(1, 4):
            e(f'  v_mad_i64_i32 {pair(GQ + 2 * k)}, s[40:41], v{GQ + 2 * k - 1}, 1, {pair(GQ + 2 * k)}')
        dws = [GQ, GQ + 2, GQ + 4, GQ + 6]                             # z dwords 4 l .. 4 l + 3
        # the carries, lane to lane (slot l + 1 <- lane l; lane 0 reads slot 0 = 0), until none is left
        WSHR = f'wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0'
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{CIN}, v{GQ + 7} {WSHR}')                # lane l - 1's carry (lane 0: 0)
        e('.Lmz_cy:')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{CIN}')
        e('  s_nop 4')
        e('  s_cbranch_vccz .Lmz_cy_done')
        e(f'  v_mov_b32_e32 v{C1}, v{CIN}')
        for dd in dws:                                                 # add the signed carry, ripple its sign
            e(f'  v_add_co_u32_e32 v{dd}, vcc, v{dd}, v{C1}')
            e(f'  v_ashrrev_i32_e32 v{SG}, 31, v{C1}')
            e(f'  v_addc_co_u32_e32 v{C1}, vcc, 0, v{SG}, vcc')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{CIN}, v{C1} {WSHR}')
        e('  s_branch .Lmz_cy')
        e('.Lmz_cy_done:')
        # ---- z -> LDS; z >> 4104 (lanes 32..63) -> LDS; the quad of c reads ZL, ZL128, WD ----
        e(f'  ds_write2_b32 v{V_ZA}, v{dws[0]}, v{dws[1]} offset0:0 offset1:1')
        e(f'  ds_write2_b32 v{V_ZA}, v{dws[2]}, v{dws[3]} offset0:2 offset1:3')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{NXT}, v{dws[0]} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0')   # lane l + 1's
        for k in range(4):
            hi = f"v{dws[k + 1]}" if k < 3 else f"v{NXT}"
            e(f'  v_alignbit_b32 v{WW + k}, {hi}, v{dws[k]}, 8')
        e('  s_mov_b64 exec, s[46:47]')
        e(f'  ds_write2_b32 v{V_WA}, v{WW}, v{WW + 1} offset0:0 offset1:1')
        e(f'  ds_write2_b32 v{V_WA}, v{WW + 2}, v{WW + 3} offset0:2 offset1:3')
        e('  s_mov_b64 exec, s[44:45]')
        e('  s_waitcnt lgkmcnt(0)')
        for k in range(8):
            e(f'  ds_read_b128 {quad4(ZLB + 4 * k)}, v{V_QZ} offset:{16 * k}')
        e(f'  ds_read_b32 v{ZL128}, v{V_WB} offset:{MZ_ZS + 512}')
        e(f'  ds_read_b32 v{WD}, v{V_QW} offset:12')
        for k in range(7):
            e(f'  ds_read_b128 {quad4(WD + 1 + 4 * k)}, v{V_QW} offset:{16 + 16 * k}')
        e(f'  ds_read_b64 v[{WD + 29}:{WD + 30}], v{V_QW} offset:128')
        e(f'  ds_read_b32 v{WD + 31}, v{V_QW} offset:136')
        e('.Lmz_next:')
        e('  s_mov_b64 exec, -1')
        e('  s_lshl_b64 s[44:45], s[44:45], 4')
        e('  s_sub_u32 s42, s42, 1')
        e('  s_cmp_lg_u32 s42, 0')
        e('  s_cbranch_scc1 .Lmz_ct')
        e('  s_waitcnt lgkmcnt(0)')

    if MFZ:
        mfz_product()
    else:
        if KARA:
            kara_product()
        else:
            classic_product()
        limbs_to_words(X, lambda i: f"v{WD + i}", f"v{ZL128}", f"v{V_AI[0]}")
        for k in range(Q):
            e(f'  ds_read_b32 {X(k)}, v{V_ZR} offset:{k * RB}')
        e('  s_waitcnt lgkmcnt(0)')
        for k in range(Q):                            # the limbs were stored with their carries above bit 27
            e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, {X(k)}')
        limbs_to_words(X, lambda i: f"v{ZLB + i}", f"v{V_AI[1]}", f"v{V_AI[0]}")
        e(f'  v_lshrrev_b32_e32 v{ZL128}, 19, {X(Q - 1)}')                # lane 3: bits 4096..4103 (limb 151 >> 19)

    if "nobarrett" in DBG:
        e('  s_branch .Ldbg_sub')
    e('// @phase q1stage')
    # ---- 4. q1 staging: dword 0 = bits 4072..4103 (lane 3), dwords 1.. = W, 129..143 = 0 (fed 0) --------
    e(f'  v_lshrrev_b32_e32 v{V_TMP}, 8, v{ZLB + 31}')
    e(f'  v_lshl_or_b32 v{V_TMP}, v{ZL128}, 24, v{V_TMP}')
    e(f'  v_xor_b32_e32 v{V_TMP}, s33, v{V_TMP}')
    e(f'  v_subrev_u32_e32 v{V_TMP + 1}, {3 * 128 - 4}, v{V_Q3W}')     # lane 3: the row base
    e('  s_mov_b64 exec, s[20:21]')
    e(f'  ds_write_b32 v{V_TMP + 1}, v{V_TMP}')
    e('  s_mov_b64 exec, s[22:23]')
    e(f'  v_mov_b32_e32 v{V_TMP}, 0')
    for d in range(NQ1, 16 * KB1):                # the B reads cover 64 KB1 bytes
        e(f'  ds_write_b32 v{V_Q3W}, v{V_TMP} offset:{4 + 4 * d}')      # lane 0: row - 4
    e('  s_mov_b64 exec, -1')
    for i in range(32):
        e(f'  v_xor_b32_e32 v{WD + i}, s33, v{WD + i}')
    # W[i] at dword 1 + 32 j + i: W[0] and W[31] alone, the pairs (W[i], W[i+1]) of odd i 8-byte aligned
    e(f'  ds_write_b32 v{V_Q3W}, v{WD} offset:8')
    for i in range(1, 31, 2):
        e(f'  ds_write_b64 v{V_Q3W}, v[{WD + i}:{WD + i + 1}] offset:{8 + 4 * i}')
    e(f'  ds_write_b32 v{V_Q3W}, v{WD + 31} offset:{8 + 4 * 31}')
    e('  s_waitcnt lgkmcnt(0)')
    for kb in range(KB1):
        e(f'  ds_read_b128 {quad4(BQ + 4 * kb)}, v{V_B} offset:{64 * kb}')
    e('  s_waitcnt lgkmcnt(0)')

    # ---- 5/6. the two MFMA products, each folded chunk by chunk into DQ (quad lane j: chunk j) ----------
    # three accumulator sets (the third in GB, free outside the normalisation): the tiles of a chunk pair as one
    # stream, tile n - 2 folded right after tile n's first MFMA, so its results have long been written and the
    # fold waits only for the wait states still missing (as fthe_nadic_b76, gen_nadicb.py); "acc2" keeps two
    # sets with the fold of tile n - 1 behind fixed s_nop padding (A/B)
    ACCS = ACC + (GB,) if "acc2" not in DBG else ACC
    NACC = len(ACCS)
    XDL_WAIT = 19                                 # wait states after an MFMA before a VALU reads its result

    def mfma_product3(prod):
        A = V_A1 if prod == 1 else V_A2
        KO = KO1 if prod == 1 else KO2
        act = ACT1 if prod == 1 else ACT2
        corr = 0 if prod == 1 else CORR2_OFF - CORR1_OFF
        e(f'  v_mov_b32_e32 v{CR}, 0')
        for jp in range(0, len(CHUNKS), 2):
            t0 = CHUNKS[jp][0]
            tiles = tuple(CHUNKS[jp]) + tuple(CHUNKS[jp + 1])
            ops = [(n, t, kb) for n, t in enumerate(tiles) for kb in act[t]]
            q = []                                   # outstanding LDS ops, oldest first (tags)

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
                assert 0 <= off and off + 48 + 16 <= COPY
                issue(('a', x), f'  ds_read_b128 {quad4(AOP[x % 4])}, v{A} offset:{off}')

            def read_corr(n, t):
                issue(('c', n), f'  ds_read_b128 {quad4(ACCS[n % NACC])}, v{V_C} offset:{corr + 64 * t}')

            last_mfma = {}

            def settle(n):
                """wait states before a VALU read of tile n's accumulators: one per instruction issued since"""
                since = sum(1 for ln in o[last_mfma[n] + 1:] if ln.startswith('  '))
                need = XDL_WAIT - since
                while need > 0:
                    e(f'  s_nop {min(need, 8) - 1}')
                    need -= 8

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
                    e(f'  v_mfma_i32_16x16x64_i8 {quad4(ACCS[n % NACC])}, {quad4(AOP[x % 4])}, {quad4(BQ + 4 * kb)}, '
                      f'{quad4(ACCS[n % NACC])}')
                last_mfma[n] = len(o) - 1
                if x + 3 < len(ops):                 # the buffer MFMA x - 1 read at its issue
                    read_a(x + 3)
                if first and n >= NACC - 1:
                    m = n - (NACC - 1)
                    settle(m)
                    fold_tile(ACCS[m % NACC], 4 * (tiles[m] - t0))
                    q.append(('w', m))
                    if m + NACC < len(tiles):
                        read_corr(m + NACC, tiles[m + NACC])
            for m in range(max(0, len(tiles) - (NACC - 1)), len(tiles)):
                settle(m)
                fold_tile(ACCS[m % NACC], 4 * (tiles[m] - t0))
            e('  s_waitcnt lgkmcnt(0)')
            e('// @phase norm')
            if "nonorm" not in DBG:
                norm_pair(jp, jp + 1)
            e(f'// @phase prod{prod}')

    def mfma_product(prod):
        if NACC == 3:
            mfma_product3(prod)
            return
        """The tiles of one product chunk by chunk: every A read is issued two MFMAs ahead into one of four
        buffers, each tile's corrections (srcC) into its accumulator set right after the fold of the tile
        that used the set last, and s_waitcnt lgkmcnt(n) waits for exactly the read an MFMA needs (LDS
        returns in order); tile t-1 is folded after tile t's MFMAs are issued."""
        A = V_A1 if prod == 1 else V_A2
        KO = KO1 if prod == 1 else KO2
        act = ACT1 if prod == 1 else ACT2
        corr = 0 if prod == 1 else CORR2_OFF - CORR1_OFF
        e(f'  v_mov_b32_e32 v{CR}, 0')
        for j, tiles in enumerate(CHUNKS):
            t0 = CHUNKS[j & ~1][0]                   # groups staged from the pair's first tile
            ops = [(n, t, kb) for n, t in enumerate(tiles) for kb in act[t]]
            q = []                                   # outstanding LDS ops, oldest first (tags)

            def issue(tag, ins):
                e(ins)
                q.append(tag)

            def wait_for(tag):
                if tag not in q:                     # completed with a later op already waited for
                    return
                i = q.index(tag)
                left = len(q) - i - 1
                e(f'  s_waitcnt lgkmcnt({min(left, 15)})')
                del q[:i + 1]

            def read_a(x):
                n, t, kb = ops[x]
                off = KO + 16 * (4 * kb - t)
                assert 0 <= off and off + 48 + 16 <= COPY
                issue(('a', x), f'  ds_read_b128 {quad4(AOP[x % 4])}, v{A} offset:{off}')

            def read_corr(n, t):
                issue(('c', n), f'  ds_read_b128 {quad4(ACC[n % 2])}, v{V_C} offset:{corr + 64 * t}')

            read_corr(0, tiles[0])
            for x in range(min(2, len(ops))):
                read_a(x)
            for x, (n, t, kb) in enumerate(ops):
                first = x == 0 or ops[x - 1][0] != n
                if first:
                    wait_for(('c', n))
                wait_for(('a', x))
                if "nomfma" not in DBG:
                    e(f'  v_mfma_i32_16x16x64_i8 {quad4(ACC[n % 2])}, {quad4(AOP[x % 4])}, {quad4(BQ + 4 * kb)}, '
                      f'{quad4(ACC[n % 2])}')
                if x + 2 < len(ops):
                    read_a(x + 2)
                last = x + 1 == len(ops) or ops[x + 1][0] != n
                if last:
                    if n >= 1:                       # fold tile n-1 (its set is then free for tile n+1)
                        e('  s_nop 7')
                        e('  s_nop 7')
                        fold_tile(ACC[(n - 1) % 2], 4 * (tiles[n - 1] - t0))
                        q.append(('w', n - 1))
                    if n + 1 < len(tiles):
                        read_corr(n + 1, tiles[n + 1])
            e('  s_nop 7')
            e('  s_nop 7')
            e('  s_nop 7')
            fold_tile(ACC[(len(tiles) - 1) % 2], 4 * (tiles[-1] - t0))
            if j % 2 == 0:
                continue                             # the pair's second chunk first
            e('  s_waitcnt lgkmcnt(0)')
            e('// @phase norm')
            if "nonorm" not in DBG:
                norm_pair(j - 1, j)
            e(f'// @phase prod{prod}')

    def norm_pair(ja, jb):
        """Chunks ja, jb = ja + 1 at once: quad lane ja from its carry-in (lane ja - 1's final carry; 0 for chunk
        0), quad lane jb from 0, one v_mad_i64_i32 chain each (D_g = low dword of group g + carry, carry = its
        high dword, signed); then lane ja's carry-out is added to lane jb's lowest dword, and the signed overflow
        of that add, rare, ripples through lane jb's dwords on a slow path into its carry.  CR: the final carries
        (lane 3's: the clamp's).  Two passes per product instead of four chunk after chunk."""
        na, nb = 4 * len(CHUNKS[ja]), 4 * len(CHUNKS[jb])
        assert na == 32 and nb in (32, 36) and DQ % 2 == 0
        e(f'  s_or_b64 s[16:17], {LANE_MASK[ja]}, {LANE_MASK[jb]}')
        if ja:
            e('  s_nop 1')
            e(f'  v_mov_b32_dpp v{CR2}, v{CR} quad_perm:[0,0,1,2] {DPP}')      # lane ja: lane ja - 1's carry
        else:
            e(f'  v_mov_b32_e32 v{CR2}, 0')
        e(f'  v_cndmask_b32_e64 v{CR2}, v{CR2}, 0, {LANE_MASK[jb]}')          # lane jb: 0
        e('  s_mov_b64 exec, s[16:17]')
        cv = f"v{CR2}"
        ng = max(na, nb)
        if "norm1" not in DBG:
            cv = norm_two_chains(ja, jb, na, ng, cv)
        else:
            cv = norm_one_chain(ja, jb, na, nb, ng, cv)
        e('  s_mov_b64 exec, s[16:17]')
        e(f'  v_mov_b32_e32 v{CR}, {cv}')
        e('  s_mov_b64 exec, -1')
        lane_delivery(ja, jb, nb)

    def norm_one_chain(ja, jb, na, nb, ng, cv):
        def rd(g):
            for hh in (0, 1):                             # groups g, g + 1: two ds_read_b64 (8-byte rows)
                b = GB + 4 * ((g // 2) % 2) + 2 * hh
                e(f'  ds_read_b64 v[{b}:{b + 1}], v{V_GR} offset:{8 * (g + hh)}')
        rd(0)
        rd(2)
        for g0 in range(0, ng, 2):
            if g0 == na and nb > na:                 # lane ja's chunk ends (its carry stays in FV + 1)
                e(f'  s_mov_b64 exec, {LANE_MASK[jb]}')
            e(f'  s_waitcnt lgkmcnt({2 if g0 + 2 < ng else 0})')
            for g in (g0, g0 + 1):
                src = pair(GB + 4 * ((g0 // 2) % 2) + 2 * (g - g0))
                if g % 2 == 0:
                    e(f'  v_mad_i64_i32 {pair(DQ + g)}, vcc, {cv}, 1, {src}')
                    cv = f"v{DQ + g + 1}"
                else:
                    e(f'  v_mad_i64_i32 {pair(FV)}, vcc, {cv}, 1, {src}')
                    e(f'  v_mov_b32_e32 v{DQ + g}, v{FV}')
                    cv = f"v{FV + 1}"
            if g0 + 4 < ng:
                rd(g0 + 4)
        assert cv == f"v{FV + 1}"
        return cv

    def norm_two_chains(ja, jb, na, ng, cv):
        """each lane's chain split in two interleaved halves (half the dependent v_mad_i64_i32 latency, as
        fthe_nadic_b76's normalisation): A = groups 0..15 from the lane's carry-in, B = groups 16.. from 0; then
        A's carry-out is added to B's lowest dword, the rare signed overflow rippling through B's dwords on a slow
        path into B's carry-out, which is returned (the lane's final carry)"""
        H = 16
        q = []

        def rd(g, tag):
            b = GB + (8 if g >= H else 0) + 4 * ((g // 2) % 2)
            for hh in (0, 1):                             # groups g, g + 1: two ds_read_b64 (8-byte rows)
                e(f'  ds_read_b64 v[{b + 2 * hh}:{b + 2 * hh + 1}], v{V_GR} offset:{8 * (g + hh)}')
                q.append(tag)

        def wait_for(tag):
            if tag in q:
                i = len(q) - 1 - q[::-1].index(tag)       # the tag's last read
                e(f'  s_waitcnt lgkmcnt({min(len(q) - i - 1, 15)})')
                del q[:i + 1]

        def link(g, cvx, tmp):
            """group g into dword g: even g -> the pair (DQ g, DQ g+1), odd g through tmp; the next carry"""
            src = pair(GB + (8 if g >= H else 0) + 4 * ((g // 2) % 2) + 2 * (g % 2))
            if g % 2 == 0:
                e(f'  v_mad_i64_i32 {pair(DQ + g)}, vcc, {cvx}, 1, {src}')
                return f"v{DQ + g + 1}"
            e(f'  v_mad_i64_i32 {pair(tmp)}, vcc, {cvx}, 1, {src}')
            e(f'  v_mov_b32_e32 v{DQ + g}, v{tmp}')
            return f"v{tmp + 1}"
        for g in (0, 2, H, H + 2):
            rd(g, g)
        ca, cb = cv, "0"
        for i in range(0, max(H, ng - H), 2):
            if H + i == na and ng > na:               # only lane jb's chunk has groups here (A is done)
                e(f'  s_mov_b64 exec, {LANE_MASK[jb]}')
            if i < H:
                wait_for(i)
                ca = link(i, ca, FV)
                ca = link(i + 1, ca, FV)
                if i + 4 < H:
                    rd(i + 4, i + 4)
            if H + i < ng:
                wait_for(H + i)
                cb = link(H + i, cb, PG)
                cb = link(H + i + 1, cb, PG)
                if H + i + 4 < ng:
                    rd(H + i + 4, H + i + 4)
        assert ca == f"v{FV + 1}" and cb == f"v{PG + 1}"
        e('  s_mov_b64 exec, s[16:17]')
        # A's carry into B's lowest dword (both lanes), the overflow rippling on a slow path
        X, TP = CR + 1, V_TMP
        lab = f'.Lnc{len(o)}'
        e(f'  v_mov_b32_e32 v{TP}, v{DQ + H}')
        e(f'  v_mov_b32_e32 v{TP + 1}, 0')
        e(f'  v_mad_i64_i32 {pair(TP)}, vcc, {ca}, 1, {pair(TP)}')
        e(f'  v_mov_b32_e32 v{DQ + H}, v{TP}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{TP + 1}')
        e('  s_nop 4')
        if "slowall" in DBG:                          # test build: every lane through the slow path (carry 0: no-op)
            e('  s_mov_b64 vcc, exec')
        else:
            e(f'  s_cbranch_vccz {lab}_done')
        e('  s_and_saveexec_b64 s[38:39], vcc')                              # the overflowing lanes
        e(f'  v_mov_b32_e32 v{X}, v{TP + 1}')

        def ripple(lo, hi):
            for i in range(lo, hi):
                e(f'  v_mov_b32_e32 v{TP}, v{DQ + i}')
                e(f'  v_mov_b32_e32 v{TP + 1}, 0')
                e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{X}, 1, {pair(TP)}')
                e(f'  v_mov_b32_e32 v{DQ + i}, v{TP}')
                e(f'  v_mov_b32_e32 v{X}, v{TP + 1}')
        ripple(H + 1, na)
        if ng > na:                                   # lane jb's dwords na.. (lane ja's carry goes in first)
            e(f'  s_and_b64 s[40:41], exec, {LANE_MASK[ja]}')
            e(f'  s_andn2_b64 exec, exec, {LANE_MASK[ja]}')
            ripple(na, ng)
            e('  s_or_b64 exec, exec, s[40:41]')
        e(f'  v_add_u32_e32 {cb}, v{X}, {cb}')
        e('  s_mov_b64 exec, s[38:39]')
        e(f'{lab}_done:')
        return cb

    def lane_delivery(ja, jb, nb):
        # lane ja's carry-out into lane jb's lowest dword
        X, TP = CR + 1, V_TMP
        lab = f'.Lnp{len(o)}'
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{X}, v{CR} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{X}, 0, v{X}, {LANE_MASK[jb]}')              # lane jb only
        e(f'  v_mov_b32_e32 v{TP}, v{DQ}')
        e(f'  v_mov_b32_e32 v{TP + 1}, 0')
        e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{X}, 1, {pair(TP)}')
        e(f'  v_mov_b32_e32 v{DQ}, v{TP}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{TP + 1}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        e('  s_and_saveexec_b64 s[16:17], vcc')                              # slow path: the overflowing lanes
        e(f'  v_mov_b32_e32 v{X}, v{TP + 1}')
        for i in range(1, nb):
            e(f'  v_mov_b32_e32 v{TP}, v{DQ + i}')
            e(f'  v_mov_b32_e32 v{TP + 1}, 0')
            e(f'  v_mad_i64_i32 {pair(TP)}, vcc, v{X}, 1, {pair(TP)}')
            e(f'  v_mov_b32_e32 v{DQ + i}, v{TP}')
            e(f'  v_mov_b32_e32 v{X}, v{TP + 1}')
        e(f'  v_add_u32_e32 v{CR}, v{X}, v{CR}')
        e('  s_mov_b64 exec, s[16:17]')
        e(f'{lab}_done:')

    def fold_tile(acc, gl):
        """acc's 4 int32 rows (output bytes 4h..4h+3 of the tile) -> int64 group -> LDS (group 4 (t - t0) + h, t0
        the first tile of the chunk pair)"""
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc}, 1, 0')                # sign-extended row 0
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 1}, s30, {pair(PG)}')
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 2}, s31, {pair(PG)}')
        e(f'  v_mad_i64_i32 {pair(PG)}, vcc, v{acc + 3}, s32, {pair(PG)}')
        e(f'  ds_write_b64 v{V_G}, {pair(PG)} offset:{8 * gl + (GCH - 256 if gl >= 32 else 0)}')

    e('// @phase prod1')
    mfma_product(1)
    e('// @phase q3stage')
    # clamp: a negative N1 (lane 3's final carry) -> q3 = 0
    e('  s_nop 4')                                                      # EXEC written by SALU -> DPP
    e(f'  v_mov_b32_dpp v{CR2}, v{CR} quad_perm:[3,3,3,3] {DPP}')
    e(f'  v_cmp_gt_i32_e32 vcc, 0, v{CR2}')
    e('  s_and_saveexec_b64 s[16:17], vcc')
    e('  s_cbranch_execz .Lnoclamp')                                   # (q1 = 0: z < 2^4072 only)
    for g in range(36):
        e(f'  v_mov_b32_e32 v{DQ + g}, 0')
    e('.Lnoclamp:')
    e('  s_mov_b64 exec, s[16:17]')
    # q3 dword i = D_{i+1}: lane j writes its D_{32j+k} (k = 0..31; lane 3 also k = 32, 33) at dword 32j + k - 1
    for k in range(34):
        e(f'  v_xor_b32_e32 v{DQ + k}, s33, v{DQ + k}')
    e(f'  s_mov_b64 exec, {LANE_MASK[0]}')
    e('  s_not_b64 exec, exec')                                          # lanes 1..3: D_{32j} at dword 32j - 1
    e(f'  ds_write_b32 v{V_Q3W}, v{DQ}')
    e('  s_mov_b64 exec, -1')
    for k in range(1, 32):
        e(f'  ds_write_b32 v{V_Q3W}, v{DQ + k} offset:{4 * k}')
    e(f'  s_mov_b64 exec, {LANE_MASK[3]}')
    e(f'  ds_write_b32 v{V_Q3W}, v{DQ + 32} offset:128')
    e(f'  ds_write_b32 v{V_Q3W}, v{DQ + 33} offset:132')                   # q3 dword 128 (rows >= N only)
    e('  s_mov_b64 exec, -1')
    e('  s_waitcnt lgkmcnt(0)')
    for kb in range(KB2):
        e(f'  ds_read_b128 {quad4(BQ + 4 * kb)}, v{V_B} offset:{64 * kb}')
    e('  s_waitcnt lgkmcnt(0)')
    e('// @phase prod2')
    mfma_product(2)
    # lane 3 keeps D2_128's low 8 bits (r2 mod 2^4104)

    e('.Ldbg_sub:')
    e('// @phase sub')
    # ---- 7. r = (z - r2) mod 2^4104: borrow chains per lane, rippled across the quad --------------------
    def borrow_ripple(lab, R, R128_, bo, bin_):
        """lane k (k < 3) hands its borrow bo (0/1) to lane k+1, which subtracts it from its dwords R(0..31)
        and (lane 3) its dword 128; repeated until no lane receives a borrow (lane 3's own is dropped: the
        arithmetic is mod 2^4128 on the quad, the caller keeps the bits it needs)"""
        e(f'{lab}_loop:')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{bin_}, v{bo} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{bin_}, v{bin_}, 0, s[22:23]')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{bin_}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        e(f'  v_sub_co_u32_e32 v{R}, vcc, v{R}, v{bin_}')
        e(f'  v_mov_b32_e32 v{bo}, 0')                                   # the borrows handed on are delivered
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')                               # absorbed by dword 0 everywhere (usual)
        e('  s_and_saveexec_b64 s[38:39], vcc')                         # the lanes whose dword 0 borrowed
        for i in range(1, 32):
            e(f'  v_subb_co_u32_e64 v{R + i}, vcc, v{R + i}, 0, vcc')
        e(f'  v_cndmask_b32_e64 v{bo}, 0, 1, vcc')
        e(f'  v_subb_co_u32_e64 v{R128_}, vcc, v{R128_}, 0, vcc')
        e('  s_mov_b64 exec, s[38:39]')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    e(f'  v_sub_co_u32_e32 v{RR}, vcc, v{ZLB}, v{DQ}')
    for i in range(1, 32):
        e(f'  v_subb_co_u32_e32 v{RR + i}, vcc, v{ZLB + i}, v{DQ + i}, vcc')
    e(f'  v_cndmask_b32_e64 v{V_AI[0]}, 0, 1, vcc')                     # borrow out of dword 31
    e(f'  v_subb_co_u32_e32 v{R128}, vcc, v{ZL128}, v{DQ + 32}, vcc')    # lane 3: dword 128 (others: unused)
    borrow_ripple('.Lrb', RR, R128, V_AI[0], V_AI[1])
    e(f'  v_and_b32_e32 v{R128}, 0xff, v{R128}')                        # r = (z - r2) mod 2^4104, < 3N

    e('// @phase canon')
    if "nocanon" in DBG:
        e('  s_branch .Ldbg_store')
    # ---- 8. two conditional subtractions of N, then the canonical row ------------------------------------
    e(f'  v_bfe_u32 v{V_TMP}, v{V_ROW}, 7, 2')
    e(f'  v_lshlrev_b32_e32 v{V_TMP}, 7, v{V_TMP}')                     # 128 j
    e(f'  v_add_u32_e32 v{V_TMP}, {hex(N_OFF)}, v{V_TMP}')
    for i in range(8):
        e(f'  global_load_dwordx4 {quad4(NV + 4 * i)}, v{V_TMP}, s[10:11] offset:{16 * i}')
    e('  s_waitcnt vmcnt(0)')
    for rnd in range(2):
        e(f'  v_sub_co_u32_e32 v{TT}, vcc, v{RR}, v{NV}')
        for i in range(1, 32):
            e(f'  v_subb_co_u32_e32 v{TT + i}, vcc, v{RR + i}, v{NV + i}, vcc')
        e(f'  v_cndmask_b32_e64 v{V_AI[0]}, 0, 1, vcc')
        e(f'  v_subb_co_u32_e64 v{TT128}, vcc, v{R128}, 0, vcc')
        borrow_ripple(f'.Lcn{rnd}', TT, TT128, V_AI[0], V_AI[1])
        # r < N  <=>  r - N < 0  <=>  lane 3's dword 128 of r - N is negative
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{V_AI[0]}, v{TT128} quad_perm:[3,3,3,3] {DPP}')
        e(f'  v_cmp_le_i32_e32 vcc, 0, v{V_AI[0]}')                      # r >= N: take r - N
        for i in range(32):
            e(f'  v_cndmask_b32_e32 v{RR + i}, v{RR + i}, v{TT + i}, vcc')
        e(f'  v_cndmask_b32_e32 v{R128}, v{R128}, v{TT128}, vcc')
    e('.Ldbg_store:')
    e('// @phase store')
    e(f'  s_mov_b64 exec, {LIVE}')
    for i in range(8):
        e(f'  global_store_dwordx4 v{V_ROW}, {quad4(RR + 4 * i)}, s[8:9] offset:{16 * i}')
    e('  s_mov_b64 exec, -1')
    e('// @phase loop')
    e('  s_branch .Lbatch')
    e('.Lend:')
    e('// @stampout')
    e('  s_waitcnt vmcnt(0)')
    e('  s_endpgm')
    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    if "stamp" in DBG:
        o = stamp_pass(o)
    return "\n".join(o) + "\n" + descriptor(name, LDS_BYTES, NVGPR, NSGPR)


STAMP_PHASES = ['entry', 'load', 'product', 'window', 'q1stage', 'prod1', 'norm', 'q3stage', 'prod2', 'sub',
                'canon', 'store', 'loop']


def stamp_pass(o):
    """the stamp build: every '// @phase X' marker adds the cycles since the last stamp to the accumulator of the
    phase the marker ends (the textually previous one; the loop head is ended by 'load'), s[40:41] the last
    stamp, s45 + p the sums, s58 the wave's global index, s59 the batches; after the last batch lane 0 stores
    16 dwords per wave at out + 512 count + 64 wave: the 13 sums, the batches, the s_memtime and s_memrealtime
    (100 MHz) ticks from the first batch to the end (the clock: their ratio x 100 MHz)"""
    acc = {ph: 45 + i for i, ph in enumerate(STAMP_PHASES)}
    out, cur = [], 'entry'

    def stamp(ended):
        return ['  s_memtime s[42:43]', '  s_waitcnt lgkmcnt(0)', '  s_sub_u32 s44, s42, s40',
                f'  s_add_u32 s{acc[ended]}, s{acc[ended]}, s44', '  s_mov_b64 s[40:41], s[42:43]']
    for line in o:
        if line.startswith('// @phase'):
            ph = line.split()[2]
            ended = 'loop' if ph == 'load' else cur
            out += stamp(ended)
            if ph == 'load':
                out.append('  s_add_u32 s59, s59, 1')
            cur = ph
            out.append(line)
        elif line == '// @stampout':
            out += ['  s_memtime s[42:43]', '  s_memrealtime s[64:65]', '  s_waitcnt lgkmcnt(0)',
                    '  s_sub_u32 s62, s42, s62', '  s_sub_u32 s63, s64, s60']
            out += ['  s_mov_b64 exec, 1', '  s_lshl_b32 s44, s12, 9', '  s_lshl_b32 s42, s58, 6',
                    '  s_add_u32 s44, s44, s42', '  v_mov_b32_e32 v1, s44']
            for i, ph in enumerate(STAMP_PHASES):        # 'entry' (never stamped): the first batch's realtime
                out += [f'  v_mov_b32_e32 v2, s{acc[ph] if ph != "entry" else 60}',
                        f'  global_store_dword v1, v2, s[8:9] offset:{4 * i}']
            out += ['  v_mov_b32_e32 v2, s59', f'  global_store_dword v1, v2, s[8:9] offset:{4 * len(STAMP_PHASES)}']
            out += ['  v_mov_b32_e32 v2, s62', f'  global_store_dword v1, v2, s[8:9] offset:{4 * len(STAMP_PHASES) + 4}']
            out += ['  v_mov_b32_e32 v2, s63', f'  global_store_dword v1, v2, s[8:9] offset:{4 * len(STAMP_PHASES) + 8}']
        elif line == '.Lbatch:':
            # first pass: zero the sums, the wave's index, the first stamp
            out += [f'  s_mov_b32 s{45 + i}, 0' for i in range(len(STAMP_PHASES))]
            out += ['  s_mov_b32 s59, 0', f'  s_mul_i32 s58, s2, {WAVES}', '  s_add_u32 s58, s58, s14', '  s_memtime s[40:41]', '  s_memrealtime s[60:61]',
                    '  s_waitcnt lgkmcnt(0)', '  s_mov_b32 s62, s40', '.Lbatch:']
        else:
            out.append(line)
    return out


def descriptor(name, lds_bytes, nvgpr, nsgpr):
    o = []
    e = o.append
    e('.rodata')
    e('.p2align 6')
    e(f'.amdhsa_kernel {name}')
    e(f'  .amdhsa_group_segment_fixed_size {lds_bytes}')
    e('  .amdhsa_private_segment_fixed_size 0')
    e('  .amdhsa_kernarg_size 56')
    e('  .amdhsa_user_sgpr_count 2')
    e('  .amdhsa_user_sgpr_kernarg_segment_ptr 1')
    e('  .amdhsa_system_sgpr_workgroup_id_x 1')
    e('  .amdhsa_system_vgpr_workitem_id 0')
    e(f'  .amdhsa_next_free_vgpr {nvgpr}')
    e(f'  .amdhsa_next_free_sgpr {nsgpr}')
    e(f'  .amdhsa_accum_offset {((nvgpr + 3) // 4) * 4}')
    e('  .amdhsa_reserve_vcc 1')
    e('  .amdhsa_ieee_mode 0')
    e('  .amdhsa_dx10_clamp 0')
    e('.end_amdhsa_kernel')
    e('')
    e('.amdgpu_metadata')
    e('---')
    e('amdhsa.kernels:')
    e('  - .args:')
    for off_, sz, kind in ((0, 8, 'global_buffer'), (8, 8, 'global_buffer'), (16, 8, 'global_buffer'),
                           (24, 8, 'global_buffer'), (32, 4, 'by_value'), (36, 4, 'by_value'),
                           (40, 8, 'global_buffer'), (48, 8, 'global_buffer')):
        e(f'      - .offset: {off_}')
        e(f'        .size: {sz}')
        e(f'        .value_kind: {kind}')
        if kind == 'global_buffer':
            e('        .address_space: global')
    e(f'    .group_segment_fixed_size: {lds_bytes}')
    e('    .kernarg_segment_align: 8')
    e('    .kernarg_segment_size: 56')
    e(f'    .max_flat_workgroup_size: {64 * WAVES}')
    e(f'    .name: {name}')
    e('    .private_segment_fixed_size: 0')
    e(f'    .sgpr_count: {nsgpr + 2}')
    e(f'    .symbol: {name}.kd')
    e(f'    .vgpr_count: {nvgpr}')
    e('    .wavefront_size: 64')
    e('amdhsa.target: amdgcn-amd-amdhsa--gfx950')
    e('amdhsa.version:')
    e('  - 1')
    e('  - 2')
    e('...')
    e('.end_amdgpu_metadata')
    return "\n".join(o) + "\n"
