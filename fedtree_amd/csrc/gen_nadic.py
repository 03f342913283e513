#!/usr/bin/env python3
"""Generator of the n-adic four-lane kernel (gfx950 assembly): the public-key encrypt's r^n mod n^2 with
X = x0 + x1 n kept as two base-n digits of 2048 bits, one ciphertext per quad of lanes.

    X Y == x0 y0 + (x0 y1 + x1 y0) n   (mod n^2)
    x0 y0 = u1 n + u0                  classical product mod n (u1: the sum of its quotient digits)
    Z = u0 + ((x0 y1 + x1 y0 + u1) mod n) n

Each product is two classical MSB-first products mod the 2048-bit n run in lockstep over the
multiplier limbs (the MULWC scheme of gen_montprog.py gen_quad at 76 limbs instead of 152):
window 1 accumulates y0_i X0, window 2 y0_i X1 + y1_i X0 (a squaring: (2 x0_i) X1) plus, in its
lowest column, window 1's quotient digit of the same step -- u1 is never stored.  Per step and lane:
19 + 19 (+ 19 + 19) multiply-adds over 76 steps, against 38 + 38 over 152 steps for the Montgomery
product mod the 4096-bit n^2 -- a squaring is ~1.6x fewer instructions, a general product ~1.35x.
tools/nadic_model.py is the bit-exact model (column order, 64-bit wrap, estimate, bounds).

Layout: lane k of a quad owns limbs [19k, 19k + 19) of x0, x1 and n (VGPRs) and of both column
windows (register rings of 22 pairs: offset o at step t in pair (o - t) mod 22, one 64-bit DPP
hand-off per lane and window per step).  Multiplier limbs stream from LDS (rows 0..75: y0 or x0,
rows 76..151: y1), one broadcast read per quad and step.  Slots are the s152 slots of the key
(limb-major [k][g]): limbs 0..75 hold x0, 76..151 x1.  168 VGPRs -> 3 waves/SIMD.

Ops (uint32 pairs, bn_host.hpp Prog):
    0 END
    1 LOADX  slot   digits <- slot
    2 STOREX slot   slot <- digits
    3 SQR    count  X <- X^2, count times
    4 MUL    slot   X <- X * (digits of slot)   (y0, y1 any limbs < 2^27: only X must be reduced)
   20 CANON  -      x0 (< 2n) -> x0 mod n with its carry into x1, then x1 -> x1 mod n (x1 <= n + 1)
   14 / 16 LOADGD(16) j   digits <- fixed-base table entry (j << W) | digit j of the ciphertext (W = 8 / 16)
   15 / 17 MULGD(16) j    X <- X * that entry  (tables in digit form: y0 then y1, each as four lane quarters
                          of 19 limbs + 1 pad word: 160 words per entry)
Products leave x0 in [0, n) and x1 in [0, n]; CANON makes both canonical (before the output and after
a LOADX of a raw r < 2n).

Kernel arguments: those of gen_montprog.py; ctx = MontMod(n, 76 x 27-bit, four lanes).ctx: n limbs,
nprime (unused), the quotient-estimate doubles -k1, -k2, -k3, bias at words 77..84 (bn_host.hpp).
n of 2042..2050 bits (the estimate's ignored columns; 2n below 2^2052); the s152 slots of n^2 stop at 2048.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_montprog import QUAD_ROWB, _descriptor  # noqa: E402


def gen_nadic(S: int, B: int, name: str, mont: bool = False) -> str:
    """mont: the Montgomery form (fthe_nadic_m76, tools/nadic_mont_model.py) -- each product
    Mont(X, Y) = X Y R^-1 mod n^2 (R = 2^(B S)) as two interleaved LSB-first Montgomery reductions mod n,
    q = col0 n' mod 2^B on lane 0 instead of the classical form's f64 quotient estimates and overflow
    folds; digits stay in [0, 2n) between products (no conditional subtraction), CANON reduces them."""
    assert S % 4 == 0
    Q = S // 4
    MASK = (1 << B) - 1
    NTC = Q + 3                                  # ring pairs per window (offsets 0..Q + free; even: the
    #                                              a_i double buffer keeps its parity across trips)
    # ---- VGPR plan -----------------------------------------------------------
    V_LDSW = 0                                   # the lane's A-write base (v0 = tid at entry)
    V_TID = 0
    V_ROW, V_LDSI = 1, 2                         # (g, k) encoding; A read cursor (column base)
    V_AI = (3, 4)                                # y0_i / x0_i, double-buffered
    V_Q = 5                                      # -q1 (window 1), also the slot offset of LOADX / STOREX
    V_TMP = 6                                    # v[6:7] 64-bit temp
    V_BI = (8, 9)                                # y1_i, double-buffered (MUL)
    V_Q2 = 10                                    # -q2 (window 2)
    V_A2 = 11                                    # 2 x0_i (SQR)
    V_L0N = 12                                   # -1 on lane 0 of the quad, else 0
    DF0, DACC1, DACC2, DBIAS = 14, 16, 18, 20    # estimate doubles
    X0B = 22
    X1B = X0B + Q
    NB = X1B + Q
    TB1 = (NB + Q + 1) & ~1
    TB2 = TB1 + 2 * NTC
    NVGPR = TB2 + 2 * NTC
    assert NVGPR <= 168, NVGPR                   # 3 waves per SIMD
    NSGPR = 48
    RB_ = QUAD_ROWB
    ROWS = 2 * S                                 # LDS rows per wave: y0 then y1
    lds_per_wave = ROWS * RB_
    lds_bytes = 4 * lds_per_wave
    DPP = "row_mask:0xf bank_mask:0xf"
    tmp = f"v[{V_TMP}:{V_TMP + 1}]"

    def X0(k):
        return f"v{X0B + k}"

    def X1(k):
        return f"v{X1B + k}"

    def NV(k):
        return f"v{NB + k}"

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
    # lane masks: k == 3 -> s[20:21], k == 0 -> s[22:23]
    e('  s_mov_b32 s20, 0x88888888')
    e('  s_mov_b32 s21, 0x88888888')
    e('  s_mov_b32 s22, 0x11111111')
    e('  s_mov_b32 s23, 0x11111111')
    e('  s_waitcnt lgkmcnt(0)')
    e(f'  s_load_dwordx8 s[36:43], s[8:9], {hex(4 * (S + 1))}')   # -k1, -k2, -k3, bias (doubles)
    if mont:
        e(f'  s_load_dword s44, s[8:9], {hex(4 * S)}')                # n' = -n^-1 mod 2^B
    # ROW = g*512 + k*128 = wg*32768 + tid*128 (g = wg*64 + tid>>2, k = tid & 3)
    e('  s_lshl_b32 s14, s2, 15')
    e(f'  v_lshlrev_b32_e32 v{V_ROW}, 7, v{V_TID}')
    e(f'  v_add_u32_e32 v{V_ROW}, s14, v{V_ROW}')
    e(f'  v_and_b32_e32 v{V_TMP}, 3, v{V_TID}')                   # k
    e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {Q}, v{V_TMP}')         # k*Q
    e(f'  v_lshlrev_b32_e32 v{V_Q}, 2, v{V_TMP + 1}')             # k*Q*4
    for j in range(Q):
        e(f'  global_load_dword {NV(j)}, v{V_Q}, s[8:9] offset:{4 * j}')
    # A column of ciphertext c = (tid>>2)&15 in wave w = tid>>6
    e(f'  v_lshrrev_b32_e32 v{V_LDSI}, 6, v{V_TID}')
    e(f'  v_mul_u32_u24_e32 v{V_LDSI}, {hex(lds_per_wave)}, v{V_LDSI}')
    e(f'  v_lshrrev_b32_e32 v{V_Q}, 2, v{V_TID}')
    e(f'  v_and_b32_e32 v{V_Q}, 15, v{V_Q}')
    e(f'  v_lshl_add_u32 v{V_LDSI}, v{V_Q}, 2, v{V_LDSI}')
    e(f'  v_mul_u32_u24_e32 v{V_LDSW}, {Q * RB_}, v{V_TMP}')        # k*Q*row (tid dies here)
    e(f'  v_add_u32_e32 v{V_LDSW}, v{V_LDSW}, v{V_LDSI}')
    e(f'  v_cndmask_b32_e64 v{V_L0N}, 0, -1, s[22:23]')
    e(f'  v_mov_b32_e32 v{DBIAS}, 0')
    e(f'  v_mov_b32_e32 v{DBIAS + 1}, 0x3f900000')                 # +2^-6
    e('  s_waitcnt vmcnt(0) lgkmcnt(0)')

    e('.Lprog:')
    e('  s_load_dwordx2 s[14:15], s[6:7], 0x0')
    e('  s_add_u32 s6, s6, 8')
    e('  s_addc_u32 s7, s7, 0')
    e('  s_waitcnt lgkmcnt(0)')
    for code, lab in ((1, '.Lloadx'), (2, '.Lstorex'), (3, '.Lsqr'), (4, '.Lmul'), (20, '.Lcanon'),
                      (14, '.Lloadgd'), (15, '.Lmulgd'), (16, '.Lloadgd16'), (17, '.Lmulgd16')):
        e(f'  s_cmp_eq_u32 s14, {code}')
        e(f'  s_cbranch_scc1 {lab}')
    e('  s_branch .Lend')

    # ---- slot access: limb j of this lane's quarter of digit d at slot limb d*S + k*Q + j
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

    def goff():
        e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')            # g
        e(f'  v_lshlrev_b32_e32 v{V_TMP}, 2, v{V_TMP}')            # g*4
        e(f'  v_bfe_u32 v{V_TMP + 1}, v{V_ROW}, 7, 2')             # k
        e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {Q}, v{V_TMP + 1}')  # k*Q
        e(f'  v_mul_lo_u32 v{V_TMP + 1}, v{V_TMP + 1}, s10')       # k*Q*L*4
        e(f'  v_add_u32_e32 v{V_Q}, v{V_TMP}, v{V_TMP + 1}')

    def digits_io(d0, d1, store):
        goff()
        slot_addr()
        for dig, f in enumerate((d0, d1)):
            for j in range(Q):
                if store:
                    e(f'  global_store_dword v{V_Q}, {f(j)}, s[16:17]')
                else:
                    e(f'  global_load_dword {f(j)}, v{V_Q}, s[16:17]')
                if j != Q - 1:
                    step_addr()
            if dig == 0:
                step_addr(S - Q + 1)                                 # limb k*Q + Q - 1 -> S + k*Q
        e('  s_waitcnt vmcnt(0)')

    # ---- quad helpers (carry ripple, conditional subtraction) -----------------
    def ripple_quad(X, signed=False):
        """X limbs + this lane's pending 64-bit carry-out in tmp -> carries move to the next lane's
        limb 0 (DPP quad_perm [0,0,1,2]; lane 0 gets none) and ripple until no lane has one (at most
        3 passes); lane 3's carry out of the number is dropped (it is 0: values below 2^(B S))."""
        shr = 'v_ashrrev_i64' if signed else 'v_lshrrev_b64'
        lab = f'.Lrq{len(o)}'
        e(f'{lab}_loop:')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp v{V_AI[0]}, v{V_TMP} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_mov_b32_dpp v{V_AI[1]}, v{V_TMP + 1} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, v{V_AI[0]}, 0, s[22:23]')     # lane 0: no carry in
        e(f'  v_cndmask_b32_e64 v{V_TMP + 1}, v{V_AI[1]}, 0, s[22:23]')
        e(f'  v_or_b32_e32 v{V_Q}, v{V_TMP}, v{V_TMP + 1}')
        e(f'  v_cmp_ne_u32_e32 vcc, 0, v{V_Q}')
        e('  s_nop 4')                                           # VALU vcc -> vccz read
        e(f'  s_cbranch_vccz {lab}_done')
        for k in range(Q):
            e(f'  v_mad_u64_u32 {tmp}, vcc, {X(k)}, 1, {tmp}')
            e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  {shr} {tmp}, {B}, {tmp}')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')

    D0 = TB1                                     # canon scratch: window 1's ring (free by then)

    def canon_once(X, tag):
        """X (normalised, < 2N) -> X mod N across the quad; leaves vcc = (X was >= N) on every lane"""
        bo, fin, t1 = f"v{V_AI[0]}", f"v{V_AI[1]}", f"v{V_TMP}"
        for j in range(Q):                         # D = X - N (this quarter), borrow-out bo in {0,-1}
            e(f'  v_sub_u32_e32 v{D0 + j}, {X(j)}, {NV(j)}')
            if j:
                e(f'  v_add_u32_e32 v{D0 + j}, v{D0 + j}, {bo}')
            e(f'  v_ashrrev_i32_e32 {bo}, 31, v{D0 + j}')
            e(f'  v_and_b32_e32 v{D0 + j}, {hex(MASK)}, v{D0 + j}')
        e(f'  v_mov_b32_e32 {fin}, 0')
        lab = f'.L{tag}_borrow'
        e(f'{lab}_loop:')
        e(f'  v_cndmask_b32_e64 {t1}, 0, {bo}, s[20:21]')            # lane 3: borrow out of the number
        e(f'  v_or_b32_e32 {fin}, {fin}, {t1}')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp {t1}, {bo} quad_perm:[0,0,1,2] {DPP}')
        e(f'  v_cndmask_b32_e64 {bo}, {t1}, 0, s[22:23]')            # borrow into lane k from lane k-1
        e(f'  v_cmp_ne_u32_e32 vcc, 0, {bo}')
        e('  s_nop 4')
        e(f'  s_cbranch_vccz {lab}_done')
        for j in range(Q):
            e(f'  v_add_u32_e32 v{D0 + j}, v{D0 + j}, {bo}')
            e(f'  v_ashrrev_i32_e32 {bo}, 31, v{D0 + j}')
            e(f'  v_and_b32_e32 v{D0 + j}, {hex(MASK)}, v{D0 + j}')
        e(f'  s_branch {lab}_loop')
        e(f'{lab}_done:')
        e('  s_nop 1')
        e(f'  v_mov_b32_dpp {t1}, {fin} quad_perm:[3,3,3,3] {DPP}')
        e(f'  v_cmp_eq_u32_e32 vcc, 0, {t1}')                      # no borrow: X >= N -> X - N
        for j in range(Q):
            e(f'  v_cndmask_b32_e32 {X(j)}, {X(j)}, v{D0 + j}, vcc')

    def carry_into_x1_col(add_to):
        """vcc (digit 0 was reduced) -> +1 at position 0 of digit 1: add_to(tmp) adds the 64-bit tmp
        (1 on lane 0 when vcc, else 0)"""
        e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, 1, vcc')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, v{V_TMP}, s[22:23]')    # lane 0 only
        e(f'  v_mov_b32_e32 v{V_TMP + 1}, 0')
        add_to(tmp)

    # ---- LOADX / STOREX / CANON -------------------------------------------------
    e('.Lloadx:')
    digits_io(X0, X1, False)
    e('  s_branch .Lprog')

    e('.Lstorex:')
    digits_io(X0, X1, True)
    e('  s_branch .Lprog')

    e('.Lcanon:')
    canon_once(X0, 'cx0')

    def add_x1_limb0(t):
        e(f'  v_mov_b32_e32 v{V_TMP + 1}, 0')
        e(f'  v_add_u32_e32 {X1(0)}, {X1(0)}, v{V_TMP}')
        e(f'  v_mov_b64_e32 {tmp}, 0')
        for k in range(Q):                       # limb 0 may reach 2^B: normalise the quarter
            e(f'  v_mad_u64_u32 {tmp}, vcc, {X1(k)}, 1, {tmp}')
            e(f'  v_and_b32_e32 {X1(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
        ripple_quad(X1)
    carry_into_x1_col(add_x1_limb0)
    canon_once(X1, 'cx1')
    if mont:                                     # x1 < 2n + 1 after the carry: a second round
        canon_once(X1, 'cx1b')
    e('  s_branch .Lprog')

    # ---- A operand -> LDS ------------------------------------------------------------
    def write_rows(src, row0):
        for k in range(Q):
            e(f'  ds_write_b32 v{V_LDSW}, {src(k)} offset:{(row0 + k) * RB_}')
            if k % 8 == 7:
                e('  s_waitcnt lgkmcnt(0)')
        e('  s_waitcnt lgkmcnt(0)')

    e('.Lmul:')
    digits_io(lambda j: f"v{TB1 + j}", lambda j: f"v{TB1 + Q + j}", False)
    write_rows(lambda j: f"v{TB1 + j}", 0)
    write_rows(lambda j: f"v{TB1 + Q + j}", S)
    e('  s_mov_b32 s19, 0')
    e('  s_branch .Lprod_mul')

    # ---- gathered fixed-base table entries (digit form) ------------------------------------
    # entry (j << W) | dig[j][g] of the table at rows[0]: EW = 8 QP words, y0 then y1, each as four lane
    # quarters of QP = Q + 1 words (Q limbs and a pad word: 16-byte aligned, so lane k reads its quarters
    # with dwordx4 loads); the digit array (u8, or u16 when W = 16) [window][L] at rows[1]
    QP = Q + 1
    assert QP % 4 == 0
    EW = 8 * QP

    def gather_entry(wide):
        """the entry's quarters of y0, y1 -> v[TB1 .. TB1 + QP), v[TB1 + QP .. TB1 + 2 QP)"""
        vt, vt2, vk = f"v{V_Q}", f"v{V_Q2}", f"v{V_A2}"
        addr = f"v[{V_TMP}:{V_TMP + 1}]"
        e('  s_load_dwordx2 s[16:17], s[0:1], 0x30')        # digit array
        e('  s_lshr_b32 s14, s10, 2')                        # L
        e('  s_mul_i32 s14, s14, s15')                       # j * L
        if wide:
            e('  s_lshl_b32 s14, s14, 1')                    # u16 digits
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_add_u32 s16, s16, s14')
        e('  s_addc_u32 s17, s17, 0')
        e(f'  v_lshrrev_b32_e32 {vt}, 9, v{V_ROW}')          # g
        if wide:
            e(f'  v_lshlrev_b32_e32 {vt}, 1, {vt}')
        e(f'  global_load_{"ushort" if wide else "ubyte"} {vt}, {vt}, s[16:17]')
        e('  s_load_dwordx2 s[16:17], s[0:1], 0x28')        # table
        e(f'  s_lshl_b32 s14, s15, {16 if wide else 8}')     # j << W
        e(f'  v_mov_b32_e32 {vt2}, {4 * EW}')
        e(f'  v_bfe_u32 {vk}, v{V_ROW}, 7, 2')               # k
        e(f'  v_mul_u32_u24_e32 {vk}, {4 * QP}, {vk}')       # this lane's quarter
        e('  s_waitcnt vmcnt(0) lgkmcnt(0)')
        e(f'  v_or_b32_e32 {vt}, s14, {vt}')
        e(f'  v_mad_u64_u32 {addr}, vcc, {vt}, {vt2}, s[16:17]')     # 64-bit entry address (tables > 4 GiB)
        e(f'  v_add_co_u32_e32 v{V_TMP}, vcc, v{V_TMP}, {vk}')
        e(f'  v_addc_co_u32_e32 v{V_TMP + 1}, vcc, 0, v{V_TMP + 1}, vcc')
        for dig in range(2):
            for i in range(QP // 4):
                r0 = TB1 + dig * QP + 4 * i
                e(f'  global_load_dwordx4 v[{r0}:{r0 + 3}], {addr}, off offset:{4 * (dig * 4 * QP + 4 * i)}')
        e('  s_waitcnt vmcnt(0)')

    for wide in (False, True):
        sfx = "16" if wide else ""
        e(f'.Lloadgd{sfx}:')
        gather_entry(wide)
        for j in range(Q):
            e(f'  v_mov_b32_e32 {X0(j)}, v{TB1 + j}')
            e(f'  v_mov_b32_e32 {X1(j)}, v{TB1 + QP + j}')
        e('  s_branch .Lprog')
        e(f'.Lmulgd{sfx}:')
        gather_entry(wide)
        write_rows(lambda j: f"v{TB1 + j}", 0)
        write_rows(lambda j: f"v{TB1 + QP + j}", S)
        e('  s_mov_b32 s19, 0')
        e('  s_branch .Lprod_mul')

    # FTHE_GEN_NADIC_AB=dbl (Montgomery form): a squaring also writes 2 x0 into rows S.. and window 2 reads its
    # multiplier limb from there (one LDS read per step instead of a VALU doubling)
    dbl = mont and "dbl" in os.environ.get("FTHE_GEN_NADIC_AB", "").split(",")
    e('.Lsqr:')
    e('  s_mov_b32 s19, s15')
    e('.Lsqr_loop:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    write_rows(X0, 0)
    if dbl:
        for j in range(Q):                       # the rings are free between products
            e(f'  v_lshlrev_b32_e32 v{TB1 + j}, 1, {X0(j)}')
        write_rows(lambda j: f"v{TB1 + j}", S)
    e('  s_branch .Lprod_sq')

    # ---- the fused product ------------------------------------------------------------
    def emit_product(sq):
        lab = '.Lprod_sq' if sq else '.Lprod_mul'

        def R(tb, off, u):
            k = (off - u) % NTC
            return f"v[{tb + 2 * k}:{tb + 2 * k + 1}]"

        def Rlo(tb, off, u):
            return f"v{tb + 2 * ((off - u) % NTC)}"

        def Rhi(tb, off, u):
            return f"v{tb + 2 * ((off - u) % NTC) + 1}"

        STEPC = NTC
        NTRIPC, TLC = S // STEPC, S % STEPC
        assert TLC > 0 and STEPC % 2 == 0
        d0 = f"v[{DF0}:{DF0 + 1}]"
        bias = f"v[{DBIAS}:{DBIAS + 1}]"
        cur = [0]

        def move_cursor(to_row):
            dlt = (to_row - cur[0]) * RB_
            if dlt > 0:
                e(f'  v_add_u32_e32 v{V_LDSI}, {hex(dlt)}, v{V_LDSI}')
            elif dlt < 0:
                e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(-dlt)}, v{V_LDSI}')
            cur[0] = to_row

        def est_list(tb, u, qreg, dacc):
            acc = f"v[{dacc}:{dacc + 1}]"
            ab = os.environ.get("FTHE_GEN_NADIC_AB", "")
            if "noest" in ab.split(","):                             # timing only: q = 0 (wrong results)
                return [f'  v_mov_b32_e32 v{qreg}, 0', None, None,
                        f'  v_mov_b32_dpp v{qreg}, v{qreg} quad_perm:[3,3,3,3] {DPP}']
            if "fold" in ab.split(","):
                # y = col[Q-1] + (col[Q-2] >> 27) with two 64-bit integer instructions (v[6:7] is free inside
                # the product), then -q = trunc(bias - y 2^27 invN) through a two-term fma chain: one
                # conversion and one fma fewer than the chain over col[Q-1] and hi32(col[Q-2]).  Bit-exact
                # (tools/nadic_model.py, the GPU tests) but 1.2% slower: 453k vs 459k public-key encrypts/s
                # (profiles/r03zh_nadic_fold_ab.jsonl) -- the chain becomes serial; so opt-in, not the default
                return [
                    f'  v_ashrrev_i64 {tmp}, {B}, {R(tb, Q - 2, u)}',
                    f'  v_lshl_add_u64 {tmp}, {R(tb, Q - 1, u)}, 0, {tmp}',
                    f'  v_cvt_f64_i32_e32 {d0}, v{V_TMP + 1}',
                    f'  v_fma_f64 {acc}, {d0}, s[40:41], {bias}',
                    f'  v_cvt_f64_u32_e32 {d0}, v{V_TMP}',
                    f'  v_fma_f64 {acc}, {d0}, s[38:39], {acc}',
                    f'  v_cvt_i32_f64_e32 v{qreg}, {acc}',
                    None, None,                                   # DPP read-after-VALU-write spacing
                    f'  v_mov_b32_dpp v{qreg}, v{qreg} quad_perm:[3,3,3,3] {DPP}',
                ]
            return [
                # -q = trunc(bias - V invN) with the constants negated on the host (as MULWC)
                f'  v_cvt_f64_i32_e32 {d0}, {Rhi(tb, Q - 2, u)}',
                f'  v_fma_f64 {acc}, {d0}, s[36:37], {bias}',
                f'  v_cvt_f64_u32_e32 {d0}, {Rlo(tb, Q - 1, u)}',
                f'  v_fma_f64 {acc}, {d0}, s[38:39], {acc}',
                f'  v_cvt_f64_i32_e32 {d0}, {Rhi(tb, Q - 1, u)}',
                f'  v_fma_f64 {acc}, {d0}, s[40:41], {acc}',
                f'  v_cvt_i32_f64_e32 v{qreg}, {acc}',
                None, None,                                   # DPP read-after-VALU-write spacing
                f'  v_mov_b32_dpp v{qreg}, v{qreg} quad_perm:[3,3,3,3] {DPP}',
            ]

        def hand(tb, u):
            return [f'  v_mov_b32_dpp {Rlo(tb, 0, u)}, {Rlo(tb, Q, u)} quad_perm:[3,0,1,2] {DPP}',
                    f'  v_mov_b32_dpp {Rhi(tb, 0, u)}, {Rhi(tb, Q, u)} quad_perm:[3,0,1,2] {DPP}']

        def window_phase(tb, terms, qreg, dacc, est_start, extra_after=None, prefetch=None):
            """terms: list of (column offset, a register, X register) in issue order, the top two
            columns first (complete after MAD est_start); after the second MAD the hand-off, from
            MAD est_start on one estimate item per MAD"""
            est = est_list(tb, u_cur[0], qreg, dacc)
            ei = 0
            for n, (j, a, x) in enumerate(terms):
                e(f'  v_mad_u64_u32 {R(tb, j, u_cur[0])}, vcc, {a}, {x}, {R(tb, j, u_cur[0])}')
                if n == 1:
                    for ins in hand(tb, u_cur[0]):
                        e(ins)
                if n >= est_start and ei < len(est):
                    ins = est[ei]
                    ei += 1
                    if ins is not None:
                        e(ins)
                if prefetch is not None and n == 12:
                    prefetch()
            for ins in est[ei:]:
                e(ins if ins is not None else '  s_nop 0')
            if extra_after:
                extra_after()
            for j in range(Q - 1, -1, -1):
                e(f'  v_mad_i64_i32 {R(tb, j, u_cur[0])}, vcc, v{qreg}, {NV(j)}, {R(tb, j, u_cur[0])}')

        u_cur = [0]

        def step(u, i, pref):
            u_cur[0] = u
            ai = f"v{V_AI[u % 2]}"
            nai = f"v{V_AI[(u + 1) % 2]}"
            bi = f"v{V_BI[u % 2]}"
            nbi = f"v{V_BI[(u + 1) % 2]}"
            # 1. shift (lane 3): fold TT into offset Q-1 and clear it, both windows
            e('  s_mov_b64 exec, s[20:21]')
            for tb in (TB1, TB2):
                e(f'  v_lshlrev_b64 {d0}, {B}, {R(tb, Q, u)}')
                e(f'  v_lshl_add_u64 {R(tb, Q - 1, u)}, {d0}, 0, {R(tb, Q - 1, u)}')
                e(f'  v_mov_b64_e32 {R(tb, Q, u)}, 0')
            e('  s_mov_b64 exec, -1')
            if sq:
                e(f'  v_lshlrev_b32_e32 v{V_A2}, 1, {ai}')

            def prefetch():
                if pref is None:
                    return
                e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(pref - cur[0]) * RB_}')
                if not sq:
                    e(f'  ds_read_b32 {nbi}, v{V_LDSI} offset:{(S + pref - cur[0]) * RB_}')

            order = [Q - 1, Q - 2] + list(range(Q - 3, -1, -1))
            # 2. window 1: + a_i X0, estimate q1, - q1 N
            window_phase(TB1, [(j, ai, X0(j)) for j in order], V_Q, DACC1, 1, prefetch=prefetch)
            # 3. window 2: + 2 a_i X1 (SQR) / a_i X1 + b_i X0 (MUL), + q1 at position 0, estimate, - q2 N
            if sq:
                terms = [(j, f"v{V_A2}", X1(j)) for j in order]
            else:
                terms = []
                for j in order:
                    terms += [(j, ai, X1(j)), (j, bi, X0(j))]

            def add_q1():
                # lane 0's offset 0 is position 0: += q1 = (-q1)(-1); the other lanes add 0
                e(f'  v_mad_i64_i32 {R(TB2, 0, u)}, vcc, v{V_Q}, v{V_L0N}, {R(TB2, 0, u)}')
            window_phase(TB2, terms, V_Q2, DACC2, 1 if sq else 3, extra_after=add_q1)
            e('  s_waitcnt lgkmcnt(0)')

        e(f'{lab}:')
        for k in range(NTC):
            e(f'  v_mov_b64_e32 v[{TB1 + 2 * k}:{TB1 + 2 * k + 1}], 0')
            e(f'  v_mov_b64_e32 v[{TB2 + 2 * k}:{TB2 + 2 * k + 1}], 0')
        first = S - 1
        move_cursor(first - STEPC)                                # row below trip 0's lowest limb
        e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI} offset:{(first - cur[0]) * RB_}')
        if not sq:
            e(f'  ds_read_b32 v{V_BI[0]}, v{V_LDSI} offset:{(S + first - cur[0]) * RB_}')
        e('  s_waitcnt lgkmcnt(0)')
        # NTRIPC full trips, then the first TLC steps of one more (as gen_montprog's MSB product)
        e(f'  s_mov_b32 s18, {NTRIPC + 1}')
        e(f'{lab}_trip:')
        base = cur[0]
        for u in range(STEPC):
            i = base + STEPC - u
            step(u, i, i - 1)
            if u == TLC - 1:
                e('  s_cmp_eq_u32 s18, 1')
                e(f'  s_cbranch_scc1 {lab}_done')
        e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(STEPC * RB_)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e(f'  s_branch {lab}_trip')
        e(f'{lab}_done:')
        cur[0] -= NTRIPC * STEPC
        move_cursor(0)
        ue = TLC - 1

        def normalise(tb, X):
            e(f'  v_mov_b64_e32 {tmp}, 0')
            for k in range(Q):
                e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {R(tb, k, ue)}')
                e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
                e(f'  v_ashrrev_i64 {tmp}, {B}, {tmp}')
            ripple_quad(X, signed=True)

        normalise(TB1, X0)
        canon_once(X0, f'{lab[2:]}0')
        carry_into_x1_col(lambda t: e(f'  v_lshl_add_u64 {R(TB2, 0, ue)}, {t}, 0, {R(TB2, 0, ue)}'))
        normalise(TB2, X1)
        canon_once(X1, f'{lab[2:]}1')
        e('  s_cmp_eq_u32 s19, 0')
        e('  s_cbranch_scc1 .Lprog')
        e('  s_sub_u32 s19, s19, 1')
        e('  s_branch .Lsqr_loop')

    # ---- the Montgomery fused product (mont) -------------------------------------------------
    def emit_product_mont(sq):
        """LSB-first: step i takes multiplier limb i (rows i, S + i), per window 19 + 19 multiply-adds per
        lane, q from lane 0's lowest column (v_mul_lo_u32 by n', mask, DPP broadcast), then every lane
        splits its lowest column, keeps hi in its next column and hands lo to the lane below as that
        lane's new top column (gen_montprog.py gen_quad's step; lane 0's lo is 0).  Window 2 takes -q1
        into its lowest column (lane 0) and its columns are signed (arithmetic split).  Rings of NTC
        pairs per window: position k at step u in pair (u + k) mod NTC.  The hand-off is one v_and_b32 with
        DPP into a fixed pair per window whose high dword stays 0, the next step's first multiply-add into
        that column takes the pair as its addend (no fresh column to clear), and q is masked and broadcast
        by one v_and_b32 with DPP: 88 VALU instructions per step, 76 of them multiply-adds."""
        lab = '.Lprod_sq' if sq else '.Lprod_mul'
        NT = NTC
        assert NT % 2 == 0 and NT >= Q + 1

        def T(tb, k):
            k %= NT
            return f"v[{tb + 2 * k}:{tb + 2 * k + 1}]"

        def Tlo(tb, k):
            return f"v{tb + 2 * (k % NT)}"

        def Thi(tb, k):
            return f"v{tb + 2 * (k % NT) + 1}"

        tmp2 = f"v[{DF0}:{DF0 + 1}]"
        HO = {TB1: DACC1, TB2: DACC2}            # hand-off pairs (the estimate registers of the classical form)
        VMK = DBIAS                              # 2^27 - 1

        def reduce_split(tb, qreg, t, shr):
            for j in range(Q):
                e(f'  v_mad_u64_u32 {T(tb, u_[0] + j)}, vcc, v{qreg}, {NV(j)}, {T(tb, u_[0] + j)}')
                if j == 3:
                    e(f'  {shr} {t}, {B}, {T(tb, u_[0])}')
                if j == 9:
                    e(f'  v_lshl_add_u64 {T(tb, u_[0] + 1)}, {t}, 0, {T(tb, u_[0] + 1)}')
            e(f'  v_and_b32_dpp v{HO[tb]}, {Tlo(tb, u_[0])}, v{VMK} quad_perm:[1,2,3,0] {DPP}')

        def qstep(j, tb, qreg):
            if j == 3:
                e(f'  v_mul_lo_u32 v{qreg}, {Tlo(tb, u_[0])}, s44')
            if j == 9:
                e(f'  v_and_b32_dpp v{qreg}, v{qreg}, v{VMK} quad_perm:[0,0,0,0] {DPP}')

        def top(tb, u, j):
            """the addend of the multiply-add that first touches position u + j: the hand-off pair for the top
            column (j = Q - 1), else the ring"""
            return f"v[{HO[tb]}:{HO[tb] + 1}]" if j == Q - 1 else T(tb, u + j)

        u_ = [0]

        def step(u, last):
            u_[0] = u
            ai = f"v{V_AI[u % 2]}"
            nai = f"v{V_AI[(u + 1) % 2]}"
            bi = f"v{V_BI[u % 2]}"
            nbi = f"v{V_BI[(u + 1) % 2]}"
            if sq and not dbl:
                e(f'  v_lshlrev_b32_e32 v{V_A2}, 1, {ai}')
            a2 = bi if dbl else f"v{V_A2}"
            # window 1: + a_i X0, q1, + q1 N, split
            for j in range(Q):
                e(f'  v_mad_u64_u32 {T(TB1, u + j)}, vcc, {ai}, {X0(j)}, {top(TB1, u, j)}')
                qstep(j, TB1, V_Q)
                if j == 11 and not last:
                    e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(u + 1) * RB_}')
                    if not sq or dbl:
                        e(f'  ds_read_b32 {nbi}, v{V_LDSI} offset:{(S + u + 1) * RB_}')
            reduce_split(TB1, V_Q, tmp, 'v_lshrrev_b64')
            # window 2: + 2 a_i X1 (SQR) / a_i X1 + b_i X0 (MUL), - q1 at position 0, q2, + q2 N, split
            for j in range(Q):
                if sq:
                    e(f'  v_mad_u64_u32 {T(TB2, u + j)}, vcc, {a2}, {X1(j)}, {top(TB2, u, j)}')
                else:
                    e(f'  v_mad_u64_u32 {T(TB2, u + j)}, vcc, {ai}, {X1(j)}, {top(TB2, u, j)}')
                    e(f'  v_mad_u64_u32 {T(TB2, u + j)}, vcc, {bi}, {X0(j)}, {T(TB2, u + j)}')
                if j == 0:       # lane 0: += q1 (-1); the other lanes add 0
                    e(f'  v_mad_i64_i32 {T(TB2, u)}, vcc, v{V_Q}, v{V_L0N}, {T(TB2, u)}')
                qstep(j, TB2, V_Q2)
            reduce_split(TB2, V_Q2, tmp2, 'v_ashrrev_i64')
            e('  s_waitcnt lgkmcnt(0)')

        e(f'{lab}:')
        for k in range(NT):
            e(f'  v_mov_b64_e32 v[{TB1 + 2 * k}:{TB1 + 2 * k + 1}], 0')
            e(f'  v_mov_b64_e32 v[{TB2 + 2 * k}:{TB2 + 2 * k + 1}], 0')
        e(f'  v_mov_b64_e32 v[{HO[TB1]}:{HO[TB1] + 1}], 0')
        e(f'  v_mov_b64_e32 v[{HO[TB2]}:{HO[TB2] + 1}], 0')
        e(f'  v_mov_b32_e32 v{VMK}, {hex(MASK)}')

        e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI}')
        if not sq or dbl:
            e(f'  ds_read_b32 v{V_BI[0]}, v{V_LDSI} offset:{S * RB_}')
        e('  s_waitcnt lgkmcnt(0)')
        NTRIP, TL = S // NT, S % NT
        assert NTRIP > 0 and TL > 0
        e(f'  s_mov_b32 s18, {NTRIP}')
        e(f'{lab}_trip:')
        for u in range(NT):
            step(u, False)
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(NT * RB_)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_cmp_lg_u32 s18, 0')
        e(f'  s_cbranch_scc1 {lab}_trip')
        for u in range(TL):
            step(u, u == TL - 1)
        e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(NTRIP * NT * RB_)}, v{V_LDSI}')   # back to the column base

        def normalise(tb, X):
            e(f'  v_mov_b64_e32 {tmp}, 0')
            for k in range(Q):                   # the top column is in the hand-off pair
                e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {T(tb, TL + k) if k < Q - 1 else f"v[{HO[tb]}:{HO[tb] + 1}]"}')
                e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
                e(f'  v_ashrrev_i64 {tmp}, {B}, {tmp}')
            ripple_quad(X, signed=True)

        normalise(TB1, X0)                       # digits in [0, 2n): no conditional subtraction
        normalise(TB2, X1)
        e('  s_cmp_eq_u32 s19, 0')
        e('  s_cbranch_scc1 .Lprog')
        e('  s_sub_u32 s19, s19, 1')
        e('  s_branch .Lsqr_loop')

    for sq in (True, False):
        (emit_product_mont if mont else emit_product)(sq)
    e('.Lend:')
    e('  s_endpgm')
    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    o.extend(_descriptor(name, lds_bytes, NVGPR, NSGPR).splitlines())
    return "\n".join(o) + "\n"


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--limbs', type=int, default=76)
    ap.add_argument('--name', default='fthe_nadic_q76')
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args()
    with open(a.out, 'w') as f:
        f.write(gen_nadic(a.limbs, 27, a.name))
