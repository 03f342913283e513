#!/usr/bin/env python3
"""Generator for the hand-scheduled gfx950 Montgomery "program" kernel.

The kernel runs one big-integer modular computation per LANE (64 independent
ciphertexts per wavefront).  Every lane executes the same uniform op program
(an exponent schedule produced on the host), so all control flow is
wave-uniform.  The hot loop is a radix-2^B CIOS Montgomery product

    X <- A * X * R^-1 mod N,      R = 2^(B*S)

with the S limbs of X in VGPRs, the A operand streamed one limb per outer
iteration from LDS (lane-interleaved, one column per lane, conflict-free),
the modulus N in SGPRs (it is the same for the whole launch) and a window of
64-bit column accumulators T[] in VGPRs.  B < 32 leaves headroom in the 64-bit
accumulators, so every 32x32 partial product is exactly ONE v_mad_u64_u32
(half-rate on gfx950, measured 3.45e13/s chip-wide) -- no add-with-carry
chains.  R > 4N ("almost Montgomery"), so no conditional subtraction is ever
needed inside an exponentiation; results stay < 2N.

Why hand-written assembly: the CIOS state is ~250 VGPRs per lane.  hipcc's
scheduler hoists the LDS reads and spills hundreds of registers at this size
(measured: 116-913 spilled VGPRs across formulations), so the register
allocation is done here, explicitly.

Ops (uint32 pairs, read with s_load from the program buffer):
    0 END
    1 LOADX  slot   X <- slot
    2 STOREX slot   slot <- X
    3 SQR    count  repeat count times: A <- X ; X <- MontMul(A, X)
    4 MUL    slot   A <- slot ; X <- MontMul(A, X)
    5 ADDSLOT slot  X <- X + slot          (integer add, limbs renormalised)
    6 ADDSMALL k    X <- X + k             (k < 2^B)
   12 PREFA  slot   LDS A buffer <- slot, asynchronously (LDS-DMA)
   13 MULA   -      X <- MontMul(A buffer, X) after the PREFA landed
   14 LOADXGD j     X <- table entry j*256 + dig[j][g]       (fixed-base tables:
   15 MULGD   j     X <- MontMul(table entry j*256 + dig[j][g], X)  rows[0] = table
                    of entries of EW = 4*ceil(S/4) radix-2^B words, rows[1] = u8
                    digit array [window][L])
   16/17            the same with 16-bit windows: u16 digits, entry j*65536 + dig

Slot memory: slot s, limb k, lane g at  slots + s*slot_stride + k*L*4 + g*4
(limb-major, lane-interleaved: every global access is fully coalesced).

Kernel arguments (kernarg segment):
    0  u64 slots         8  u64 prog        16 u64 ctx (N[S] u32, nprime u32)
    24 u32 limb_stride (=L*4 bytes)          28 u32 slot_stride (=S*L*4 bytes)
    32 u32 live ciphertexts in this launch   36 u32 reserved
    40 u64 rows[16]: row-array pointers of the row I/O ops (four-lane kernel only)
"""
import argparse
import os
import sys

# q = T0 n' mod 2^B from the low word of a v_mad_u64_u32 (full rate) instead of
# v_mul_lo_u32 (quarter rate); FTHE_GEN_QLO=1 restores the latter (A/B builds)
Q_VIA_MAD = not os.environ.get("FTHE_GEN_QLO")
# four-lane kernel: accumulator window as a register ring (no window moves);
# FTHE_GEN_NORING=1 restores the sliding window (A/B builds)
QUAD_RING = not os.environ.get("FTHE_GEN_NORING")
# four-lane kernel: every lane keeps the carry of its retiring column and hands
# down only the low B bits (one DPP, no masks); FTHE_GEN_HANDOFF64=1 restores the
# 64-bit hand-off with lane masks (A/B builds)
QUAD_LOW_HANDOFF = not os.environ.get("FTHE_GEN_HANDOFF64")
# four-lane kernel: A-operand rows of 17 words (16 ciphertexts + 1 pad) so that the
# four lanes of a quad, which write rows 38 apart, land in different LDS banks;
# FTHE_GEN_LDS64=1 restores the unpadded 16-word rows (A/B builds)
QUAD_ROWB = 64 if os.environ.get("FTHE_GEN_LDS64") else 68


def gen(S: int, B: int, U: int, name: str, sqr_unrolled: bool = True) -> str:
    assert U % 2 == 0 and U >= 2
    MASK = (1 << B) - 1
    NTRIPS = S // U
    TAIL = S % U
    # ---- VGPR plan -------------------------------------------------------
    V_TID, V_GOFF, V_LDSA = 0, 1, 2
    V_AI = (3, 4)          # double-buffered a_i
    V_Q = 5
    V_LDSI = 6
    V_TMP = 8              # v[8:9] 64-bit temp (even aligned)
    XB = 10                # X limbs v[10 .. 10+S-1]
    TB = XB + S
    if TB % 2:
        TB += 1
    NT = S + U              # T window entries (64-bit)
    NVGPR = TB + 2 * NT
    assert NVGPR <= 256, f"VGPR budget exceeded: {NVGPR}"
    # ---- SGPR plan -------------------------------------------------------
    # s[0:1] kernarg, s2 wg id, s[4:5] slots, s[6:7] prog, s[8:9] ctx,
    # s10 limb stride, s11 slot stride, s12 nprime, s[14:15] op/arg,
    # s[16:17] addr, s18 trip counter, s19 sqr counter, s20.. N limbs
    SN = 20
    NSGPR = SN + S
    assert NSGPR <= 100, f"SGPR budget exceeded: {NSGPR}"

    def T(k):
        return f"v[{TB + 2 * k}:{TB + 2 * k + 1}]"

    def Tlo(k):
        return f"v{TB + 2 * k}"

    def X(k):
        return f"v{XB + k}"

    o = []
    e = o.append
    lds_per_wave = S * 256
    lds_bytes = 4 * lds_per_wave
    e('.amdgcn_target "amdgcn-amd-amdhsa--gfx950"')
    e('.amdhsa_code_object_version 5')
    e('.text')
    e(f'.globl {name}')
    e('.p2align 8')
    e(f'.type {name},@function')
    e(f'{name}:')
    # -- prologue: kernel args
    e('  s_load_dwordx2 s[4:5], s[0:1], 0x0')
    e('  s_load_dwordx2 s[6:7], s[0:1], 0x8')
    e('  s_load_dwordx2 s[8:9], s[0:1], 0x10')
    e('  s_load_dwordx2 s[10:11], s[0:1], 0x18')
    e('  s_waitcnt lgkmcnt(0)')
    # -- modulus limbs into SGPRs
    off = 0
    sreg = SN
    rem = S
    for width in (16, 8, 4, 2, 1):
        while rem >= width:
            assert sreg % min(width, 4) == 0
            suffix = f"x{width}" if width > 1 else ""
            dst = f"s[{sreg}:{sreg + width - 1}]" if width > 1 else f"s{sreg}"
            e(f'  s_load_dword{suffix} {dst}, s[8:9], {hex(off)}')
            off += 4 * width
            sreg += width
            rem -= width
    e(f'  s_load_dword s12, s[8:9], {hex(4 * S)}')
    # -- per-lane addresses
    e('  s_lshl_b32 s14, s2, 10')                 # wg*256*4
    e(f'  v_lshlrev_b32_e32 v{V_GOFF}, 2, v{V_TID}')
    e(f'  v_add_u32_e32 v{V_GOFF}, s14, v{V_GOFF}')
    e(f'  v_lshrrev_b32_e32 v{V_LDSA}, 6, v{V_TID}')
    e(f'  v_mul_u32_u24_e32 v{V_LDSA}, {hex(lds_per_wave)}, v{V_LDSA}')
    e(f'  v_and_b32_e32 v{V_Q}, 63, v{V_TID}')
    e(f'  v_lshl_add_u32 v{V_LDSA}, v{V_Q}, 2, v{V_LDSA}')
    e(f'  v_readfirstlane_b32 s13, v{V_LDSA}')       # this wave's A buffer (LDS-DMA base)
    e('  s_waitcnt lgkmcnt(0)')

    # -- op dispatcher
    e('.Lprog:')
    e('  s_load_dwordx2 s[14:15], s[6:7], 0x0')
    e('  s_add_u32 s6, s6, 8')
    e('  s_addc_u32 s7, s7, 0')
    e('  s_waitcnt lgkmcnt(0)')
    for code, lab in ((1, '.Lloadx'), (2, '.Lstorex'), (3, '.Lsqr'), (4, '.Lmul'),
                      (5, '.Laddslot'), (6, '.Laddsmall'), (12, '.Lprefa'), (13, '.Lmula'),
                      (14, '.Lloadxgd'), (15, '.Lmulgd'),
                      (16, '.Lloadxgd16'), (17, '.Lmulgd16')):
        e(f'  s_cmp_eq_u32 s14, {code}')
        e(f'  s_cbranch_scc1 {lab}')
    e('  s_branch .Lend')

    def slot_addr():
        # s[16:17] = slots + arg*slot_stride   (64-bit: slot regions exceed 4 GiB)
        e('  s_mul_i32 s16, s15, s11')
        e('  s_mul_hi_u32 s17, s15, s11')
        e('  s_add_u32 s16, s4, s16')
        e('  s_addc_u32 s17, s5, s17')

    def step_addr():
        e('  s_add_u32 s16, s16, s10')
        e('  s_addc_u32 s17, s17, 0')

    def emit_square():
        """X <- X^2 R^-1 mod N, fully unrolled (S(S+1)/2 + S^2 v_mad_u64_u32)."""
        touched = set()

        def R(c):                       # register pair of column c
            k = c % S
            return f"v[{TB + 2 * k}:{TB + 2 * k + 1}]"

        def Rlo(c):
            return f"v{TB + 2 * (c % S)}"

        def mad(c, a, b):
            src2 = R(c) if c in touched else "0"
            touched.add(c)
            e(f'  v_mad_u64_u32 {R(c)}, vcc, {a}, {b}, {src2}')

        q = f"v{V_Q}"
        d = f"v{V_AI[0]}"
        tmp = f"v[{V_TMP}:{V_TMP + 1}]"
        for i in range(S):
            if i == 0:
                mad(0, X(0), X(0))
            # q = T_i n' mod 2^B: the low word of a (full-rate) 32x32->64 multiply-add
            if Q_VIA_MAD:
                e(f'  v_mad_u64_u32 {tmp}, vcc, {Rlo(i)}, s12, 0')
            else:
                e(f'  v_mul_lo_u32 v{V_TMP}, {Rlo(i)}, s12')
            e(f'  v_lshlrev_b32_e32 {d}, 1, {X(i)}')
            cnt = 0
            if i > 0:
                mad(2 * i, X(i), X(i))
                cnt += 1
            for j in range(i + 1, S):
                mad(i + j, d, X(j))
                cnt += 1
                if cnt == 2:
                    e(f'  v_and_b32_e32 {q}, {hex(MASK)}, v{V_TMP}')
            if cnt < 2:
                e(f'  v_and_b32_e32 {q}, {hex(MASK)}, v{V_TMP}')
            for j in range(S):
                mad(i + j, q, f"s{SN + j}")
                if j == 3:
                    e(f'  v_lshrrev_b64 {tmp}, {B}, {R(i)}')
                if j == 7 or (j == S - 1 and S <= 7):
                    pass
                if j == 7:
                    e(f'  v_lshl_add_u64 {R(i + 1)}, {tmp}, 0, {R(i + 1)}')
            touched.discard(i)          # column i retired: its pair is reused for column i + S
        # result columns S .. 2S-1 -> X
        e(f'  v_and_b32_e32 {X(0)}, {hex(MASK)}, {Rlo(S)}')
        e(f'  v_lshrrev_b64 {tmp}, {B}, {R(S)}')
        for k in range(1, S):
            e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {R(S + k)}')
            e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
            if k != S - 1:
                e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')

    # LOADX
    e('.Lloadx:')
    slot_addr()
    for k in range(S):
        e(f'  global_load_dword {X(k)}, v{V_GOFF}, s[16:17]')
        if k != S - 1:
            step_addr()
        if k % 32 == 31:
            e('  s_waitcnt vmcnt(0)')
    e('  s_waitcnt vmcnt(0)')
    e('  s_branch .Lprog')

    # STOREX
    e('.Lstorex:')
    slot_addr()
    for k in range(S):
        e(f'  global_store_dword v{V_GOFF}, {X(k)}, s[16:17]')
        if k != S - 1:
            step_addr()
        if k % 32 == 31:
            e('  s_waitcnt vmcnt(0)')
    e('  s_waitcnt vmcnt(0)')
    e('  s_branch .Lprog')

    def normalise32():
        # X limbs < 2^31 -> radix-2^B limbs (sequential carry; value < R)
        c = f"v{V_TMP}"
        e(f'  v_lshrrev_b32_e32 {c}, {B}, {X(0)}')
        e(f'  v_and_b32_e32 {X(0)}, {hex(MASK)}, {X(0)}')
        for k in range(1, S):
            e(f'  v_add_u32_e32 {X(k)}, {X(k)}, {c}')
            if k != S - 1:
                e(f'  v_lshrrev_b32_e32 {c}, {B}, {X(k)}')
                e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, {X(k)}')

    # ADDSLOT: X <- X + slot (plain integer add, value must stay < R)
    e('.Laddslot:')
    slot_addr()
    for k in range(S):
        e(f'  global_load_dword v{TB + k}, v{V_GOFF}, s[16:17]')
        if k != S - 1:
            step_addr()
        if k % 32 == 31:
            e('  s_waitcnt vmcnt(0)')
    e('  s_waitcnt vmcnt(0)')
    for k in range(S):
        e(f'  v_add_u32_e32 {X(k)}, {X(k)}, v{TB + k}')
    normalise32()
    e('  s_branch .Lprog')

    # ADDSMALL: X <- X + arg (arg < 2^B)
    e('.Laddsmall:')
    e(f'  v_add_u32_e32 {X(0)}, s15, {X(0)}')
    normalise32()
    e('  s_branch .Lprog')

    # MUL: A <- slot (through the free T registers), then MontMul
    e('.Lmul:')
    slot_addr()
    for k in range(S):
        e(f'  global_load_dword v{TB + k}, v{V_GOFF}, s[16:17]')
        if k != S - 1:
            step_addr()
        if k % 32 == 31:
            e('  s_waitcnt vmcnt(0)')
    e('  s_waitcnt vmcnt(0)')
    for k in range(S):
        e(f'  ds_write_b32 v{V_LDSA}, v{TB + k} offset:{k * 256}')
        if k % 8 == 7:
            e('  s_waitcnt lgkmcnt(0)')
    e('  s_waitcnt lgkmcnt(0)')
    e('  s_mov_b32 s19, 0')      # after the product: back to the dispatcher
    e('  s_branch .Lmontmul')

    # PREFA slot: the A operand of the next MULA goes slot -> LDS A buffer by
    # LDS-DMA (global_load_lds: wave base in M0 + 4*lane, no VGPRs) and is left
    # in flight across the squarings that precede the multiply (they never touch
    # LDS).  MULA: wait for it, multiply; the buffer keeps A for further MULAs.
    e('.Lprefa:')
    slot_addr()
    e('  s_mov_b32 m0, s13')
    e('  s_nop 0')
    for k in range(S):
        e(f'  global_load_lds_dword v{V_GOFF}, s[16:17]')
        if k != S - 1:
            step_addr()
            e('  s_add_u32 m0, m0, 0x100')
            e('  s_nop 0')
    e('  s_branch .Lprog')

    e('.Lmula:')
    e('  s_waitcnt vmcnt(0)')
    e('  s_mov_b32 s19, 0')
    e('  s_branch .Lmontmul')

    # Fixed-base tables (gathered by a per-lane digit): entry j*256 + dig[j][g] of
    # rows[0], EW words each; the digit byte array rows[1] is [window][L].  The
    # entry lands in the free T registers (dwordx4 loads), then X or the LDS A column.
    EW = 4 * ((S + 3) // 4)
    assert 2 * NT >= EW + 2 and TB % 2 == 0

    def gather_entry(wide):
        """Entry (j << W) | dig[j][g] of the table at rows[0] (W = 8, or 16 when
        wide: u16 digits) -> v[TB+2 ..]; 64-bit entry address (tables > 4 GiB)."""
        e('  s_load_dwordx2 s[16:17], s[0:1], 0x30')        # digit array
        e('  s_lshr_b32 s14, s10, 2')                        # L
        e('  s_mul_i32 s14, s14, s15')                       # j*L
        if wide:
            e('  s_lshl_b32 s14, s14, 1')                    # u16 digits
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_add_u32 s16, s16, s14')
        e('  s_addc_u32 s17, s17, 0')
        e(f'  v_lshrrev_b32_e32 v{V_TMP}, {1 if wide else 2}, v{V_GOFF}')   # g (bytes: g * digit size)
        e(f'  global_load_{"ushort" if wide else "ubyte"} v{V_TMP}, v{V_TMP}, s[16:17]')
        e('  s_load_dwordx2 s[16:17], s[0:1], 0x28')        # table
        e(f'  s_lshl_b32 s14, s15, {16 if wide else 8}')     # j << W
        e(f'  v_mov_b32_e32 v{V_TMP + 1}, {4 * EW}')
        e('  s_waitcnt vmcnt(0) lgkmcnt(0)')
        e(f'  v_or_b32_e32 v{V_TMP}, s14, v{V_TMP}')
        e(f'  v_mad_u64_u32 v[{TB}:{TB + 1}], vcc, v{V_TMP}, v{V_TMP + 1}, s[16:17]')
        for i in range(EW // 4):
            e(f'  global_load_dwordx4 v[{TB + 2 + 4 * i}:{TB + 5 + 4 * i}], v[{TB}:{TB + 1}], off offset:{16 * i}')
        e('  s_waitcnt vmcnt(0)')

    for wide in (False, True):
        sfx = "16" if wide else ""
        e(f'.Lloadxgd{sfx}:')
        gather_entry(wide)
        for k in range(S):
            e(f'  v_mov_b32_e32 {X(k)}, v{TB + 2 + k}')
        e('  s_branch .Lprog')
        e(f'.Lmulgd{sfx}:')
        gather_entry(wide)
        for k in range(S):
            e(f'  ds_write_b32 v{V_LDSA}, v{TB + 2 + k} offset:{k * 256}')
            if k % 8 == 7:
                e('  s_waitcnt lgkmcnt(0)')
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_mov_b32 s19, 0')
        e('  s_branch .Lmontmul')


    # SQR: count in s15.  Fully unrolled Montgomery squaring: a = X is in
    # registers (no LDS), only the j >= i half of the a*X products is formed
    # (2 a_i folded into one operand), columns live in S register pairs used
    # as a ring (column c -> pair c mod S), so there is no window move.
    e('.Lsqr:')
    e('  s_mov_b32 s19, s15')
    e('.Lsqr_loop:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    if sqr_unrolled:
        emit_square()
        e('  s_sub_u32 s19, s19, 1')
        e('  s_branch .Lsqr_loop')
    else:
        for k in range(S):
            e(f'  ds_write_b32 v{V_LDSA}, {X(k)} offset:{k * 256}')
            if k % 8 == 7:
                e('  s_waitcnt lgkmcnt(0)')
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_branch .Lmontmul')

    # ---------------- Montgomery product ---------------------------------
    def iteration(u, last_in_block):
        ai = f"v{V_AI[u % 2]}"
        nai = f"v{V_AI[(u + 1) % 2]}"
        q = f"v{V_Q}"
        # a_i * X into T[u..u+S-1]; q computed off the first column
        for j in range(S):
            e(f'  v_mad_u64_u32 {T(u + j)}, vcc, {ai}, {X(j)}, {T(u + j)}')
            if j == 3:
                if Q_VIA_MAD:
                    e(f'  v_mad_u64_u32 v[{V_TMP}:{V_TMP + 1}], vcc, {Tlo(u)}, s12, 0')
                else:
                    e(f'  v_mul_lo_u32 v{V_TMP}, {Tlo(u)}, s12')
            if j == 6:
                e(f'  v_and_b32_e32 {q}, {hex(MASK)}, v{V_TMP}')
            if j == 8:
                # prefetch next a limb (next iteration / next trip / tail)
                e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(u + 1) * 256}')
        # q * N into T[u..u+S-1]; carry out of column u into column u+1
        for j in range(S):
            e(f'  v_mad_u64_u32 {T(u + j)}, vcc, {q}, s{SN + j}, {T(u + j)}')
            if j == 3:
                e(f'  v_lshrrev_b64 v[{V_TMP}:{V_TMP + 1}], {B}, {T(u)}')
            if j == 7:
                e(f'  v_lshl_add_u64 {T(u + 1)}, v[{V_TMP}:{V_TMP + 1}], 0, {T(u + 1)}')
        e('  s_waitcnt lgkmcnt(0)')

    e('.Lmontmul:')
    for k in range(NT):
        e(f'  v_mov_b64_e32 {T(k)}, 0')
    e(f'  v_mov_b32_e32 v{V_LDSI}, v{V_LDSA}')
    e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI}')
    e('  s_waitcnt lgkmcnt(0)')
    if NTRIPS > 0:
        e(f'  s_mov_b32 s18, {NTRIPS}')
        e('.Ltrip:')
        for u in range(U):
            iteration(u, u == U - 1)
        # slide the window by U columns
        for k in range(S):
            e(f'  v_mov_b64_e32 {T(k)}, {T(k + U)}')
        for k in range(S, S + U):
            e(f'  v_mov_b64_e32 {T(k)}, 0')
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(U * 256)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_cmp_lg_u32 s18, 0')
        e('  s_cbranch_scc1 .Ltrip')
    for u in range(TAIL):
        iteration(u, u == TAIL - 1)
    # normalise T[TAIL .. TAIL+S-1] into S radix-2^B limbs of X
    tmp = f"v[{V_TMP}:{V_TMP + 1}]"
    e(f'  v_and_b32_e32 {X(0)}, {hex(MASK)}, {Tlo(TAIL)}')
    e(f'  v_lshrrev_b64 {tmp}, {B}, {T(TAIL)}')
    for k in range(1, S):
        e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {T(TAIL + k)}')
        e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
        if k != S - 1:
            e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
    # return: s19 == 0 -> dispatcher, else one more squaring
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    e('  s_sub_u32 s19, s19, 1')
    e('  s_branch .Lsqr_loop')

    e('.Lend:')
    e('  s_endpgm')
    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    o.extend(_descriptor(name, lds_bytes, NVGPR, NSGPR).splitlines())
    return "\n".join(o) + "\n"



def _descriptor(name, lds_bytes, NVGPR, NSGPR, max_wg=256):
    o = []
    e = o.append
    # ---- kernel descriptor ------------------------------------------------
    e('.rodata')
    e('.p2align 6')
    e(f'.amdhsa_kernel {name}')
    e(f'  .amdhsa_group_segment_fixed_size {lds_bytes}')
    e('  .amdhsa_private_segment_fixed_size 0')
    e('  .amdhsa_kernarg_size 168')
    e('  .amdhsa_user_sgpr_count 2')
    e('  .amdhsa_user_sgpr_kernarg_segment_ptr 1')
    e('  .amdhsa_system_sgpr_workgroup_id_x 1')
    e('  .amdhsa_system_vgpr_workitem_id 0')
    e(f'  .amdhsa_next_free_vgpr {NVGPR}')
    e(f'  .amdhsa_next_free_sgpr {NSGPR}')
    e(f'  .amdhsa_accum_offset {((NVGPR + 3) // 4) * 4}')
    e('  .amdhsa_reserve_vcc 1')
    e('  .amdhsa_ieee_mode 0')
    e('  .amdhsa_dx10_clamp 0')
    e('.end_amdhsa_kernel')
    e('')
    # ---- metadata -----------------------------------------------------
    e('.amdgpu_metadata')
    e('---')
    e('amdhsa.kernels:')
    e('  - .args:')
    kargs = ((0, 8, 'global_buffer'), (8, 8, 'global_buffer'), (16, 8, 'global_buffer'),
             (24, 4, 'by_value'), (28, 4, 'by_value'), (32, 4, 'by_value'), (36, 4, 'by_value'))
    kargs += tuple((40 + 8 * t, 8, 'global_buffer') for t in range(16))
    for off_, sz, kind in kargs:
        e(f'      - .offset: {off_}')
        e(f'        .size: {sz}')
        e(f'        .value_kind: {kind}')
        if kind == 'global_buffer':
            e('        .address_space: global')
    e(f'    .group_segment_fixed_size: {lds_bytes}')
    e('    .kernarg_segment_align: 8')
    e('    .kernarg_segment_size: 168')
    e(f'    .max_flat_workgroup_size: {max_wg}')
    e(f'    .name: {name}')
    e('    .private_segment_fixed_size: 0')
    e(f'    .sgpr_count: {NSGPR + 2}')
    e(f'    .symbol: {name}.kd')
    e(f'    .vgpr_count: {NVGPR}')
    e('    .wavefront_size: 64')
    e('amdhsa.target: amdgcn-amd-amdhsa--gfx950')
    e('amdhsa.version:')
    e('  - 1')
    e('  - 2')
    e('...')
    e('.end_amdgpu_metadata')
    return "\n".join(o) + "\n"


def gen_quad(S: int, B: int, U: int, name: str) -> str:
    """Four lanes per ciphertext, for moduli up to B*S - 8 bits (n^2 of
    Paillier-2048: S = 152 limbs of B = 27 bits; 2*152 products of < 2^54 keep
    every 64-bit column below 2^63).  Lane k of a quad owns limbs [kQ, (k+1)Q)
    of X, of the modulus N (held in VGPRs: it differs per lane) and of the
    accumulator window.  Per outer iteration q is computed on lane 0 and
    broadcast inside the quad (DPP quad_perm), the carry of the retired column
    stays on lane 0, and every lane hands its lowest column to the lane below
    (DPP) -- one 64-bit hand-off per lane per iteration.  16 ciphertexts per
    wavefront, 168 VGPRs -> 3 waves/SIMD.

    Slot layout is the limb-major [k][g] layout of gen(), g the ciphertext
    index; kernarg limb_stride = L*4 for L ciphertexts."""
    assert S % 4 == 0 and U % 2 == 0
    Q = S // 4
    # row I/O (LOADW/MULW/STOREW and the gathers) is laid out for 152 limbs of 27 bits
    # (4096-bit rows of n^2); other shapes (the 80-limb mod-p^2 latency kernel) dispatch
    # the slot ops only and end the program on any other opcode
    rowio = Q == 38 and B == 27
    MASK = (1 << B) - 1
    NTRIPS, TAIL = S // U, S % U
    # VGPRs: v0 tid (set-up) then the lane's A-write base, v1 lane offset in a
    # slot row, v2 A read cursor (rests at the ciphertext's A column), v3/v4 a_i,
    # v5 q, v[6:7] 64-bit temp, then X, N quarter, T window.
    V_TID = V_LDSW = 0
    V_ROW, V_LDSI = 1, 2
    V_AI = (3, 4)
    V_Q = 5
    V_TMP = 6
    XB = 8
    NB = XB + Q
    TB = NB + Q
    if TB % 2:
        TB += 1
    NT = Q + U
    NVGPR = TB + 2 * NT
    assert NVGPR <= 256, NVGPR
    NSGPR = 48
    # MULWC (classical MSB-first product, row I/O shape only): its ring of NTC pairs, the
    # estimate's double temporaries and the -bias constant in the VGPRs past the ring
    NTC = Q + 2
    DF0, DACC, DBIAS = V_TMP, TB + 2 * NTC, TB + 2 * NTC + 2
    assert DBIAS + 2 <= NVGPR, (DBIAS, NVGPR)

    # window position k -> register pair k mod NT (a ring in the ring form)
    def T(k):
        k %= NT
        return f"v[{TB + 2 * k}:{TB + 2 * k + 1}]"

    def Tlo(k):
        return f"v{TB + 2 * (k % NT)}"

    def Thi(k):
        return f"v{TB + 2 * (k % NT) + 1}"

    def X(k):
        return f"v{XB + k}"

    def NV(k):
        return f"v{NB + k}"

    o = []
    e = o.append
    RB_ = QUAD_ROWB
    lds_per_wave = S * RB_         # A[i][c]: 16 ciphertexts x 4 B per row (+ pad)
    lds_bytes = 4 * lds_per_wave
    DPP = "row_mask:0xf bank_mask:0xf"
    tmp = f"v[{V_TMP}:{V_TMP + 1}]"
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
    e('  s_load_dword s28, s[0:1], 0x20')                        # live ciphertexts
    # lane masks: k == 3 -> s[20:21], k == 0 -> s[22:23]
    e('  s_mov_b32 s20, 0x88888888')
    e('  s_mov_b32 s21, 0x88888888')
    e('  s_mov_b32 s22, 0x11111111')
    e('  s_mov_b32 s23, 0x11111111')
    e('  s_waitcnt lgkmcnt(0)')
    e(f'  s_load_dword s12, s[8:9], {hex(4 * S)}')
    # MULWC quotient-estimate constants (doubles k1, k2, k3, -bias at ctx[S+1 .. S+8])
    e(f'  s_load_dwordx8 s[36:43], s[8:9], {hex(4 * (S + 1))}')
    # ROW = g*512 + k*128 = wg*32768 + tid*128 (g = wg*64 + tid>>2, k = tid & 3):
    # the lane's quarter of a 128-word row, and an encoding of (g, k) for the slot ops
    e('  s_lshl_b32 s14, s2, 15')
    e(f'  v_lshlrev_b32_e32 v{V_ROW}, 7, v{V_TID}')
    e(f'  v_add_u32_e32 v{V_ROW}, s14, v{V_ROW}')
    e(f'  v_and_b32_e32 v{V_TMP}, 3, v{V_TID}')                 # k
    e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {Q}, v{V_TMP}')       # k*Q
    e(f'  v_lshlrev_b32_e32 v{V_Q}, 2, v{V_TMP + 1}')            # k*Q*4
    for j in range(Q):
        e(f'  global_load_dword {NV(j)}, v{V_Q}, s[8:9] offset:{4 * j}')
    # A column of ciphertext c = (tid>>2)&15 in wave w = tid>>6
    e(f'  v_lshrrev_b32_e32 v{V_LDSI}, 6, v{V_TID}')
    e(f'  v_mul_u32_u24_e32 v{V_LDSI}, {hex(lds_per_wave)}, v{V_LDSI}')
    e(f'  v_lshrrev_b32_e32 v{V_Q}, 2, v{V_TID}')
    e(f'  v_and_b32_e32 v{V_Q}, 15, v{V_Q}')
    e(f'  v_lshl_add_u32 v{V_LDSI}, v{V_Q}, 2, v{V_LDSI}')
    e(f'  v_mul_u32_u24_e32 v{V_LDSW}, {Q * RB_}, v{V_TMP}')       # k*Q*row (tid dies here)
    e(f'  v_add_u32_e32 v{V_LDSW}, v{V_LDSW}, v{V_LDSI}')
    e('  s_waitcnt vmcnt(0) lgkmcnt(0)')

    e('.Lprog:')
    e('  s_load_dwordx2 s[14:15], s[6:7], 0x0')
    e('  s_add_u32 s6, s6, 8')
    e('  s_addc_u32 s7, s7, 0')
    e('  s_waitcnt lgkmcnt(0)')
    ops = ((1, '.Lloadx'), (2, '.Lstorex'), (3, '.Lsqr'), (4, '.Lmul'), (5, '.Laddslot'), (6, '.Laddsmall'))
    if rowio:
        ops += ((7, '.Lloadw'), (8, '.Lmulw'), (9, '.Lstorew'), (10, '.Lloadwg'), (11, '.Lmulwg'),
                (14, '.Lloadwd'), (15, '.Lmulwd'), (16, '.Lloadwd16'), (17, '.Lmulwd16'), (18, '.Lmulwc'), (19, '.Lmulwgc'),
                (20, '.Lcanon'))
    for code, lab in ops:
        e(f'  s_cmp_eq_u32 s14, {code}')
        e(f'  s_cbranch_scc1 {lab}')
    e('  s_branch .Lend')

    def slot_addr():
        e('  s_mul_i32 s16, s15, s11')
        e('  s_mul_hi_u32 s17, s15, s11')
        e('  s_add_u32 s16, s4, s16')
        e('  s_addc_u32 s17, s5, s17')

    def step_addr():
        e('  s_add_u32 s16, s16, s10')
        e('  s_addc_u32 s17, s17, 0')

    V_GOFF = V_Q          # slot offset g*4 + k*Q*L*4, recomputed from ROW when needed

    def goff():
        e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')            # g
        e(f'  v_lshlrev_b32_e32 v{V_TMP}, 2, v{V_TMP}')            # g*4
        e(f'  v_bfe_u32 v{V_TMP + 1}, v{V_ROW}, 7, 2')             # k
        e(f'  v_mul_u32_u24_e32 v{V_TMP + 1}, {Q}, v{V_TMP + 1}')  # k*Q
        e(f'  v_mul_lo_u32 v{V_TMP + 1}, v{V_TMP + 1}, s10')       # k*Q*L*4
        e(f'  v_add_u32_e32 v{V_GOFF}, v{V_TMP}, v{V_TMP + 1}')

    def load_quarter(dst):
        goff()
        slot_addr()
        for k in range(Q):
            e(f'  global_load_dword {dst(k)}, v{V_GOFF}, s[16:17]')
            if k != Q - 1:
                step_addr()
        e('  s_waitcnt vmcnt(0)')

    def ripple_quad(signed=False):
        """X limbs + a pending 64-bit carry-out in tmp (of this lane) -> carries
        move to the next lane's limb 0 (DPP quad_perm [0,0,1,2]; lane 0 gets
        none) and ripple until no lane has one (at most 3 passes).  signed: the
        carries are two's-complement (MULWC's columns), shifted arithmetically."""
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

    def normalise_quad32():
        """X limbs (small sums) -> radix 2^B, across the quad."""
        e(f'  v_mov_b64_e32 {tmp}, 0')
        for k in range(Q):
            e(f'  v_mad_u64_u32 {tmp}, vcc, {X(k)}, 1, {tmp}')
            e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
        ripple_quad()

    def canon_once(tag):
        """X (normalised, < 2N) -> X mod N: D = X - N across the quad (DPP borrow ripple), then
        select; uses the T registers from TB (free outside a product) and V_AI / V_TMP."""
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

    e('.Lloadx:')
    load_quarter(X)
    e('  s_branch .Lprog')

    e('.Lstorex:')
    goff()
    slot_addr()
    for k in range(Q):
        e(f'  global_store_dword v{V_GOFF}, {X(k)}, s[16:17]')
        if k != Q - 1:
            step_addr()
    e('  s_waitcnt vmcnt(0)')
    e('  s_branch .Lprog')

    e('.Laddslot:')
    load_quarter(lambda k: f"v{TB + k}")
    for k in range(Q):
        e(f'  v_add_u32_e32 {X(k)}, {X(k)}, v{TB + k}')
    normalise_quad32()
    e('  s_branch .Lprog')

    e('.Laddsmall:')
    e(f'  v_mov_b32_e32 v{V_TMP}, s15')
    e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, v{V_TMP}, s[22:23]')     # only lane 0 of the quad
    e(f'  v_add_u32_e32 {X(0)}, {X(0)}, v{V_TMP}')
    normalise_quad32()
    e('  s_branch .Lprog')

    def write_a(src):
        for k in range(Q):
            e(f'  ds_write_b32 v{V_LDSW}, {src(k)} offset:{k * RB_}')
            if k % 8 == 7:
                e('  s_waitcnt lgkmcnt(0)')
        e('  s_waitcnt lgkmcnt(0)')

    e('.Lmul:')
    load_quarter(lambda k: f"v{TB + k}")
    write_a(lambda k: f"v{TB + k}")
    e('  s_mov_b32 s19, 0')
    e('  s_branch .Lmontmul')

    e('.Lsqr:')
    e('  s_mov_b32 s19, s15')
    e('.Lsqr_loop:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    write_a(X)
    e('  s_branch .Lmontmul')

    # ---- row I/O: canonical 128-word rows (n^2 of Paillier-2048) read and
    # written in place of the layout-conversion kernels.  Row table entry t
    # (kernarg 32) points at row 0 of this launch; ciphertext g's lane k owns
    # words [32k, 32k+32) and the radix-2^B limbs [kQ, kQ+Q) = bits [1026k, 1026k+1026).
    # (row I/O is emitted only for this shape; other quad shapes run slot programs alone)
    W0 = TB               # 33 row words (T window is free outside a product)
    A0 = TB + 34          # 38 limbs of a MULW operand
    D0 = TB               # STOREW: X - N
    U0 = TB + 40          # STOREW: 32 output words (4-aligned for dwordx4)
    SH = V_Q              # 2k

    def row_ptr():         # row pointer t lives in the kernarg segment at 40 + 8t
        e('  s_lshl_b32 s16, s15, 3')
        e('  s_add_u32 s16, s16, 40')
        e('  s_load_dwordx2 s[30:31], s[0:1], s16')
        e('  s_waitcnt lgkmcnt(0)')

    def live_mask():       # lanes of ciphertexts g >= live: off for the row access
        e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')
        e(f'  v_cmp_gt_u32_e32 vcc, s28, v{V_TMP}')
        e('  s_and_saveexec_b64 s[24:25], vcc')

    def restore_exec():
        e('  s_mov_b64 exec, s[24:25]')

    def load_row_limbs(dst):
        """row words -> Q radix-2^B limbs of this lane's quarter, into dst(j)"""
        for i in range(8):
            e(f'  global_load_dwordx4 v[{W0 + 4 * i}:{W0 + 4 * i + 3}], v{V_ROW}, s[30:31] offset:{16 * i}')
        # word 32k+32 (lane 3: none -- load word 127 and clear it)
        e(f'  v_add_u32_e32 v{V_TMP}, 0x80, v{V_ROW}')
        e(f'  v_add_u32_e32 v{V_TMP + 1}, 0x7c, v{V_ROW}')
        e(f'  v_cndmask_b32_e64 v{V_TMP}, v{V_TMP}, v{V_TMP + 1}, s[20:21]')
        e(f'  global_load_dword v{W0 + 32}, v{V_TMP}, s[30:31]')
        e('  s_waitcnt vmcnt(0)')
        words_to_limbs(dst)

    def words_to_limbs(dst):
        """W0 .. W0+32 (row words 32k .. 32k+32) -> this lane's Q limbs"""
        e(f'  v_bfe_u32 v{SH}, v{V_ROW}, 6, 3')
        e(f'  v_and_b32_e32 v{SH}, 6, v{SH}')                    # 2k
        e(f'  v_cndmask_b32_e64 v{W0 + 32}, v{W0 + 32}, 0, s[20:21]')
        # funnel the stream down by 2k bits: bit 1026k of the row becomes bit 0
        for i in range(32):
            e(f'  v_alignbit_b32 v{W0 + i}, v{W0 + i + 1}, v{W0 + i}, v{SH}')
        e(f'  v_lshrrev_b32_e32 v{W0 + 32}, v{SH}, v{W0 + 32}')
        for j in range(Q):
            a, sh = (B * j) >> 5, (B * j) & 31
            if sh + B <= 32:
                e(f'  v_bfe_u32 {dst(j)}, v{W0 + a}, {sh}, {B}')
            else:
                e(f'  v_alignbit_b32 {dst(j)}, v{W0 + a + 1}, v{W0 + a}, {sh}')
                e(f'  v_and_b32_e32 {dst(j)}, {hex(MASK)}, {dst(j)}')

    mark = len(o)
    e('.Lloadw:')
    row_ptr()
    live_mask()
    load_row_limbs(X)
    restore_exec()
    e('  s_branch .Lprog')

    e('.Lmulw:')
    row_ptr()
    live_mask()
    load_row_limbs(lambda j: f"v{A0 + j}")
    restore_exec()
    write_a(lambda j: f"v{A0 + j}")
    e('  s_mov_b32 s19, 0')
    e('  s_branch .Lmontmul')

    # Gathered rows: LOADWG / MULWG t read row idx[g] of the array at rows[0], idx an
    # int64 array at rows[t] (one entry per ciphertext of the launch); idx < 0 -> 1.
    def load_gather_limbs(dst, digits=False, wide=False):
        if digits:
            # fixed-base table: row (j << W) | dig[j][g] of rows[0]; digit array
            # [window][L] (u8, or u16 when wide: W = 16) at rows[1]; arg = window j
            e('  s_load_dwordx2 s[32:33], s[0:1], 0x30')           # digit array
            e('  s_load_dwordx2 s[30:31], s[0:1], 0x28')           # table rows
            e('  s_lshr_b32 s16, s10, 2')                           # L
            e('  s_mul_i32 s16, s16, s15')                          # j*L
            if wide:
                e('  s_lshl_b32 s16, s16, 1')
            e('  s_waitcnt lgkmcnt(0)')
            e('  s_add_u32 s32, s32, s16')
            e('  s_addc_u32 s33, s33, 0')
            live_mask()
            e('  s_mov_b64 s[34:35], exec')
            e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')          # g
            if wide:
                e(f'  v_lshlrev_b32_e32 v{V_TMP}, 1, v{V_TMP}')
            e(f'  global_load_{"ushort" if wide else "ubyte"} v{V_TMP}, v{V_TMP}, s[32:33]')
            e(f'  s_lshl_b32 s16, s15, {16 if wide else 8}')        # j << W
            e('  s_waitcnt vmcnt(0)')
            e(f'  v_or_b32_e32 v{V_TMP}, s16, v{V_TMP}')
            e(f'  v_mov_b32_e32 v{V_TMP + 1}, 0')
        else:
            e('  s_lshl_b32 s16, s15, 3')
            e('  s_add_u32 s16, s16, 40')
            e('  s_load_dwordx2 s[32:33], s[0:1], s16')                # idx array
            e('  s_load_dwordx2 s[30:31], s[0:1], 40')                 # row base
            e('  s_waitcnt lgkmcnt(0)')
            live_mask()
            e(f'  v_lshrrev_b32_e32 v{V_TMP}, 9, v{V_ROW}')
            e(f'  v_lshlrev_b32_e32 v{V_TMP}, 3, v{V_TMP}')
            e(f'  global_load_dwordx2 v[{V_TMP}:{V_TMP + 1}], v{V_TMP}, s[32:33]')
            e('  s_waitcnt vmcnt(0)')
            e(f'  v_cmp_gt_i32_e32 vcc, 0, v{V_TMP + 1}')               # idx < 0
            e('  s_and_saveexec_b64 s[34:35], vcc')
            for j in range(Q):
                e(f'  v_mov_b32_e32 {dst(j)}, 0')
            e(f'  v_cndmask_b32_e64 {dst(0)}, 0, 1, s[22:23]')        # the integer 1
            e('  s_andn2_b64 exec, s[34:35], exec')                     # live lanes with idx >= 0
        e(f'  v_lshlrev_b64 v[{V_TMP}:{V_TMP + 1}], 9, v[{V_TMP}:{V_TMP + 1}]')
        e(f'  v_and_b32_e32 v{V_AI[0]}, 0x180, v{V_ROW}')           # 128k
        e(f'  v_add_co_u32_e32 v{V_TMP}, vcc, v{V_TMP}, v{V_AI[0]}')
        e(f'  v_addc_co_u32_e32 v{V_TMP + 1}, vcc, 0, v{V_TMP + 1}, vcc')
        e(f'  v_mov_b32_e32 v{V_AI[0]}, s31')
        e(f'  v_add_co_u32_e32 v{V_TMP}, vcc, s30, v{V_TMP}')
        e(f'  v_addc_co_u32_e32 v{V_TMP + 1}, vcc, v{V_AI[0]}, v{V_TMP + 1}, vcc')
        for i in range(8):
            e(f'  global_load_dwordx4 v[{W0 + 4 * i}:{W0 + 4 * i + 3}], v[{V_TMP}:{V_TMP + 1}], off offset:{16 * i}')
        e(f'  v_mov_b32_e32 v{V_AI[0]}, 0x80')
        e(f'  v_mov_b32_e32 v{V_AI[1]}, 0x7c')
        e(f'  v_cndmask_b32_e64 v{V_AI[0]}, v{V_AI[0]}, v{V_AI[1]}, s[20:21]')
        e(f'  v_add_co_u32_e32 v{V_AI[1]}, vcc, v{V_TMP}, v{V_AI[0]}')
        e(f'  v_addc_co_u32_e32 v{V_AI[1] + 1}, vcc, 0, v{V_TMP + 1}, vcc')
        e(f'  global_load_dword v{W0 + 32}, v[{V_AI[1]}:{V_AI[1] + 1}], off')
        e('  s_waitcnt vmcnt(0)')
        words_to_limbs(dst)
        e('  s_mov_b64 exec, s[34:35]')

    e('.Lloadwg:')
    load_gather_limbs(X)
    restore_exec()
    e('  s_branch .Lprog')

    e('.Lmulwg:')
    load_gather_limbs(lambda j: f"v{A0 + j}")
    restore_exec()
    write_a(lambda j: f"v{A0 + j}")
    e('  s_mov_b32 s19, 0')
    e('  s_branch .Lmontmul')

    # MULWC t: X <- row_t * X mod N, classical (no Montgomery factor): the pairwise add of two
    # canonical ciphertexts in one product.  Needs X < N (canonical) and N >= 2^(B S - 10).
    e('.Lmulwc:')
    e('  s_lshr_b32 s19, s15, 8')                # arg bit 8: canonical output (chained products)
    e('  s_and_b32 s15, s15, 0xff')
    row_ptr()
    live_mask()
    load_row_limbs(lambda j: f"v{A0 + j}")
    restore_exec()
    write_a(lambda j: f"v{A0 + j}")
    e('  s_branch .Lmontmul_msb')

    # MULWGC t: the same with the gathered row of MULWG t (idx list at rows[t], idx < 0 -> 1)
    e('.Lmulwgc:')
    e('  s_lshr_b32 s19, s15, 8')
    e('  s_and_b32 s15, s15, 0xff')
    load_gather_limbs(lambda j: f"v{A0 + j}")
    restore_exec()
    write_a(lambda j: f"v{A0 + j}")
    e('  s_branch .Lmontmul_msb')

    # CANON: X (normalised limbs, < 4N: any 4096-bit row) -> X mod N, the precondition of MULWC
    e('.Lcanon:')
    for r in range(3):
        # skip the remaining rounds once every quad's top limb is below N's (then X < N):
        # the case of every ciphertext (< n^2 <= N) after at most one round
        e(f'  v_cmp_lt_u32_e32 vcc, {X(Q - 1)}, {NV(Q - 1)}')
        e('  s_nop 4')
        e('  s_and_b64 s[26:27], vcc, s[20:21]')
        e('  s_cmp_eq_u64 s[26:27], s[20:21]')
        e('  s_cbranch_scc1 .Lcanon_done')
        canon_once(f'cn{r}')
    e('.Lcanon_done:')
    e('  s_branch .Lprog')

    for wide in (False, True):
        sfx = "16" if wide else ""
        e(f'.Lloadwd{sfx}:')
        load_gather_limbs(X, digits=True, wide=wide)
        restore_exec()
        e('  s_branch .Lprog')
        e(f'.Lmulwd{sfx}:')
        load_gather_limbs(lambda j: f"v{A0 + j}", digits=True, wide=wide)
        restore_exec()
        write_a(lambda j: f"v{A0 + j}")
        e('  s_mov_b32 s19, 0')
        e('  s_branch .Lmontmul')

    # STOREW: X (< 2N) -> X mod N -> row words.
    e('.Lstorew:')
    row_ptr()
    live_mask()
    canon_once('sw')
    bo, t1 = f"v{V_AI[0]}", f"v{V_TMP}"
    # own bit stream -> words U_i (bits [32i, 32i+32) of this quarter)
    for i in range(32):
        lo, hi = 32 * i, 32 * i + 31
        j0, j1 = lo // B, min(hi // B, Q - 1)
        e(f'  v_lshrrev_b32_e32 v{U0 + i}, {lo - B * j0}, {X(j0)}')
        for j in range(j0 + 1, j1 + 1):
            e(f'  v_lshl_or_b32 v{U0 + i}, {X(j)}, {B * j - lo}, v{U0 + i}')
    # shift up by 2k and take the low 2k bits from the top of lane k-1's quarter
    e(f'  v_bfe_u32 v{SH}, v{V_ROW}, 6, 3')
    e(f'  v_and_b32_e32 v{SH}, 6, v{SH}')                        # 2k
    e(f'  v_sub_u32_e32 {bo}, 31, v{SH}')                        # 31 - 2k
    for i in range(31, 0, -1):
        e(f'  v_lshrrev_b32_e32 {t1}, {bo}, v{U0 + i - 1}')
        e(f'  v_lshrrev_b32_e32 {t1}, 1, {t1}')
        e(f'  v_lshl_or_b32 v{U0 + i}, v{U0 + i}, v{SH}, {t1}')
    e(f'  v_mov_b32_dpp {t1}, {X(Q - 1)} quad_perm:[0,0,1,2] {DPP}')
    e(f'  v_sub_u32_e32 {bo}, {B}, v{SH}')                       # lane 0: shift 27 -> no bits
    e(f'  v_lshrrev_b32_e32 {t1}, {bo}, {t1}')
    e(f'  v_lshl_or_b32 v{U0}, v{U0}, v{SH}, {t1}')
    for i in range(8):
        e(f'  global_store_dwordx4 v{V_ROW}, v[{U0 + 4 * i}:{U0 + 4 * i + 3}], s[30:31] offset:{16 * i}')
    e('  s_waitcnt vmcnt(0)')
    restore_exec()
    e('  s_branch .Lprog')

    if not rowio:
        del o[mark:]

    def iteration(u):
        ai = f"v{V_AI[u % 2]}"
        nai = f"v{V_AI[(u + 1) % 2]}"
        q = f"v{V_Q}"
        for j in range(Q):
            e(f'  v_mad_u64_u32 {T(u + j)}, vcc, {ai}, {X(j)}, {T(u + j)}')
            if j == 3:
                if Q_VIA_MAD:
                    e(f'  v_mad_u64_u32 {tmp}, vcc, {Tlo(u)}, s12, 0')
                else:
                    e(f'  v_mul_lo_u32 v{V_TMP}, {Tlo(u)}, s12')
            if j == 6:
                e(f'  v_and_b32_e32 {q}, {hex(MASK)}, v{V_TMP}')
            if j == 9:
                e(f'  v_mov_b32_dpp {q}, {q} quad_perm:[0,0,0,0] {DPP}')
            if j == 11:
                e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(u + 1) * RB_}')
        if QUAD_LOW_HANDOFF:
            # Every lane splits its lowest column c = lo + 2^B hi: hi stays in the lane's
            # next column (absolute column c + 1 is the same lane's), lo moves to lane k-1
            # as its new top column.  Lane 0's lo is 0 (the Montgomery step zeroed it), so
            # the rotation [1,2,3,0] also hands lane 3 the zero its fresh column needs.
            for j in range(Q):
                e(f'  v_mad_u64_u32 {T(u + j)}, vcc, {q}, {NV(j)}, {T(u + j)}')
                if j == 3:
                    e(f'  v_lshrrev_b64 {tmp}, {B}, {T(u)}')
                if j == 9:
                    e(f'  v_lshl_add_u64 {T(u + 1)}, {tmp}, 0, {T(u + 1)}')
                if j == 12:
                    e(f'  v_and_b32_e32 {Tlo(u)}, {hex(MASK)}, {Tlo(u)}')
            e(f'  v_mov_b32_dpp {Tlo(u + Q)}, {Tlo(u)} quad_perm:[1,2,3,0] {DPP}')
            e(f'  v_mov_b32_e32 {Thi(u + Q)}, 0')
            e('  s_waitcnt lgkmcnt(0)')
            return
        for j in range(Q):
            e(f'  v_mad_u64_u32 {T(u + j)}, vcc, {q}, {NV(j)}, {T(u + j)}')
            if j == 3:
                e(f'  v_lshrrev_b64 {tmp}, {B}, {T(u)}')
            if j == 6:
                e(f'  v_cndmask_b32_e64 v{V_TMP}, 0, v{V_TMP}, s[22:23]')
                e(f'  v_cndmask_b32_e64 v{V_TMP + 1}, 0, v{V_TMP + 1}, s[22:23]')
            if j == 9:
                e(f'  v_lshl_add_u64 {T(u + 1)}, {tmp}, 0, {T(u + 1)}')
        # hand the lowest column to the lane below; lane 3 starts a fresh column
        e(f'  v_mov_b32_dpp {Tlo(u + Q)}, {Tlo(u)} quad_perm:[1,2,3,3] {DPP}')
        e(f'  v_mov_b32_dpp {Thi(u + Q)}, {Thi(u)} quad_perm:[1,2,3,3] {DPP}')
        e(f'  v_cndmask_b32_e64 {Tlo(u + Q)}, {Tlo(u + Q)}, 0, s[20:21]')
        e(f'  v_cndmask_b32_e64 {Thi(u + Q)}, {Thi(u + Q)}, 0, s[20:21]')
        e('  s_waitcnt lgkmcnt(0)')

    def emit_montmul_msb():
        """X <- A X mod N, MSB first (tools/msb_model.py is the bit-exact model).  Window positions
        0..S-1 of signed 64-bit columns + the top TT (position S), lane k owning [kQ, kQ+Q) and lane 3
        also TT; offset o of a lane at step t lives in ring pair (o - t) mod NTC, so the shift up by
        one position per step is a relabelling plus one 64-bit DPP hand-off per lane.  Per step
        (i = S-1-t): hand off; + a_i X; fold W = TT 2^B + col[S-1]; q = trunc(W_hi k3 + W_lo k2 +
        col[S-2]_hi k1 - bias) in double (lane 3, broadcast); - q N (v_mad_i64_i32).  Then the
        columns are normalised with signed carries: X in [0, 2N), canonicalised by STOREW."""
        def R(o, u):
            k = (o - u) % NTC
            return f"v[{TB + 2 * k}:{TB + 2 * k + 1}]"

        def Rlo(o, u):
            return f"v{TB + 2 * ((o - u) % NTC)}"

        def Rhi(o, u):
            return f"v{TB + 2 * ((o - u) % NTC) + 1}"

        STEPC = NTC
        assert STEPC % 2 == 0
        NTRIPC, TLC = S // STEPC, S % STEPC
        q = f"v{V_Q}"
        d0 = f"v[{DF0}:{DF0 + 1}]"
        acc = f"v[{DACC}:{DACC + 1}]"
        bias = f"v[{DBIAS}:{DBIAS + 1}]"
        cur = [0]                       # V_LDSI - column base, in LDS rows

        def move_cursor(to_row):
            d = (to_row - cur[0]) * RB_
            if d > 0:
                e(f'  v_add_u32_e32 v{V_LDSI}, {hex(d)}, v{V_LDSI}')
            elif d < 0:
                e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(-d)}, v{V_LDSI}')
            cur[0] = to_row

        def step(u, i, prefetch):
            """one MSB step at ring phase u reading a_i (already in V_AI[u % 2])"""
            ai = f"v{V_AI[u % 2]}"
            nai = f"v{V_AI[(u + 1) % 2]}"
            # 1. shift.  Lane 3 (exec = lane 3 alone): fold TT (offset Q, the old position S-1) into
            #    its new offset Q-1 as TT 2^B (the estimate's W; the a_i X term is added below, the
            #    order is immaterial) and clear it.  Then one rotation hands every lane's offset Q to
            #    lane k+1's new offset 0 -- lane 0 receives lane 3's cleared TT, i.e. 0.  (DPP must not
            #    run under a partial exec: a disabled source lane would not be read.)
            e('  s_mov_b64 exec, s[20:21]')
            e(f'  v_lshlrev_b64 {d0}, {B}, {R(Q, u)}')
            e(f'  v_lshl_add_u64 {R(Q - 1, u)}, {d0}, 0, {R(Q - 1, u)}')      # (shift field: 0-4 only)
            e(f'  v_mov_b64_e32 {R(Q, u)}, 0')
            e('  s_mov_b64 exec, -1')
            # 2. + a_i X, the top two columns first (lane 3's estimate)
            order = [Q - 1, Q - 2] + list(range(Q - 3, -1, -1))
            hand = [                                     # after two MADs: the DPP source was just written
                f'  v_mov_b32_dpp {Rlo(0, u)}, {Rlo(Q, u)} quad_perm:[3,0,1,2] {DPP}',
                f'  v_mov_b32_dpp {Rhi(0, u)}, {Rhi(Q, u)} quad_perm:[3,0,1,2] {DPP}',
            ]
            est = [
                # -q = trunc(bias - V invN) with the constants negated on the host: trunc toward
                # zero of a value in (-2^29, 2^-6] is -floor(V invN - bias), or 0 when that is < 0
                f'  v_cvt_f64_i32_e32 {d0}, {Rhi(Q - 2, u)}',
                f'  v_fma_f64 {acc}, {d0}, s[36:37], {bias}',
                f'  v_cvt_f64_u32_e32 {d0}, {Rlo(Q - 1, u)}',
                f'  v_fma_f64 {acc}, {d0}, s[38:39], {acc}',
                f'  v_cvt_f64_i32_e32 {d0}, {Rhi(Q - 1, u)}',
                f'  v_fma_f64 {acc}, {d0}, s[40:41], {acc}',
                f'  v_cvt_i32_f64_e32 {q}, {acc}',
                None, None,                                   # DPP read-after-VALU-write spacing
                f'  v_mov_b32_dpp {q}, {q} quad_perm:[3,3,3,3] {DPP}',
            ]
            ei = 0
            for n, j in enumerate(order):
                e(f'  v_mad_u64_u32 {R(j, u)}, vcc, {ai}, {X(j)}, {R(j, u)}')
                if n == 1:
                    for ins in hand:
                        e(ins)
                if n >= 1:
                    while ei < len(est):
                        ins = est[ei]
                        ei += 1
                        if ins is not None:
                            e(ins)
                            break
                        else:
                            break
                if n == 12 and prefetch is not None:
                    e(f'  ds_read_b32 {nai}, v{V_LDSI} offset:{(prefetch - cur[0]) * RB_}')
            for ins in est[ei:]:
                if ins is not None:
                    e(ins)
                else:
                    e('  s_nop 0')
            # 3. - q N
            for j in range(Q - 1, -1, -1):
                e(f'  v_mad_i64_i32 {R(j, u)}, vcc, {q}, {NV(j)}, {R(j, u)}')
            e('  s_waitcnt lgkmcnt(0)')

        e('.Lmontmul_msb:')
        for k in range(NTC):
            e(f'  v_mov_b64_e32 v[{TB + 2 * k}:{TB + 2 * k + 1}], 0')
        e(f'  v_mov_b32_e32 v{DBIAS}, 0')
        e(f'  v_mov_b32_e32 v{DBIAS + 1}, 0x3f900000')            # +2^-6
        # trips of STEPC steps from the top limb down; the cursor sits one row below the trip's
        # lowest limb so every read (and the next step's prefetch) has a non-negative offset
        first = S - 1
        move_cursor(first - STEPC)                                # row below trip 0's lowest limb
        e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI} offset:{(first - cur[0]) * RB_}')
        e('  s_waitcnt lgkmcnt(0)')
        # NTRIPC full trips, then the first TLC steps of one more (the same code: after NTRIPC trips
        # the cursor row is TLC - 1 - STEPC, so step u reads limb TLC - 1 - u); the last trip leaves
        # after step TLC - 1 (its prefetch of "limb -1" lands outside the wave's rows and is unused)
        assert TLC > 0
        e(f'  s_mov_b32 s18, {NTRIPC + 1}')
        e('.Ltripc:')
        base = cur[0]
        for u in range(STEPC):
            i = base + STEPC - u                                  # limb read at this step (trip 0)
            step(u, i, i - 1)
            if u == TLC - 1:
                e('  s_cmp_eq_u32 s18, 1')
                e('  s_cbranch_scc1 .Ltripc_done')
        e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(STEPC * RB_)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_branch .Ltripc')
        e('.Ltripc_done:')
        cur[0] -= NTRIPC * STEPC
        move_cursor(0)
        # normalise the signed columns (window phase u = TLC - 1) into X, then across lanes
        ue = TLC - 1 if TLC else STEPC - 1
        e(f'  v_mov_b64_e32 {tmp}, 0')
        for k in range(Q):
            e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {R(k, ue)}')
            e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
            e(f'  v_ashrrev_i64 {tmp}, {B}, {tmp}')
        ripple_quad(signed=True)
        e('  s_cmp_eq_u32 s19, 0')                                # [0, 2N) -> canonical when chained
        e('  s_cbranch_scc1 .Lprog')
        canon_once('mc')
        e('  s_branch .Lprog')

    e('.Lmontmul:')
    for k in range(Q):
        e(f'  v_mov_b64_e32 {T(k)}, 0')
    e(f'  ds_read_b32 v{V_AI[0]}, v{V_LDSI}')
    e('  s_waitcnt lgkmcnt(0)')
    # trips of STEP iterations: ring form = one full turn of the NT-pair ring
    # (window positions wrap onto the same registers, nothing moves); sliding
    # form = U iterations then a Q-pair window move
    STEP = NT if QUAD_RING else U
    assert STEP % 2 == 0                       # a_i double-buffer parity across trips
    NTRIP, TL = S // STEP, S % STEP
    if NTRIP > 0:
        e(f'  s_mov_b32 s18, {NTRIP}')
        e('.Ltrip:')
        for u in range(STEP):
            iteration(u)
        if not QUAD_RING:
            for k in range(Q):
                e(f'  v_mov_b64_e32 {T(k)}, {T(k + U)}')
        e(f'  v_add_u32_e32 v{V_LDSI}, {hex(STEP * RB_)}, v{V_LDSI}')
        e('  s_sub_u32 s18, s18, 1')
        e('  s_cmp_lg_u32 s18, 0')
        e('  s_cbranch_scc1 .Ltrip')
    for u in range(TL):
        iteration(u)
    TAIL = TL
    e(f'  v_subrev_u32_e32 v{V_LDSI}, {hex(NTRIP * STEP * RB_)}, v{V_LDSI}')   # back to the column base
    # normalise T[TAIL .. TAIL+Q-1] (64-bit columns) into X, then across lanes
    e(f'  v_mov_b64_e32 {tmp}, 0')
    for k in range(Q):
        e(f'  v_lshl_add_u64 {tmp}, {tmp}, 0, {T(TAIL + k)}')
        e(f'  v_and_b32_e32 {X(k)}, {hex(MASK)}, v{V_TMP}')
        e(f'  v_lshrrev_b64 {tmp}, {B}, {tmp}')
    ripple_quad()
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    e('  s_sub_u32 s19, s19, 1')
    e('  s_branch .Lsqr_loop')
    if rowio:
        emit_montmul_msb()
    e('.Lend:')
    e('  s_endpgm')
    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    o.extend(_descriptor(name, lds_bytes, NVGPR, NSGPR).splitlines())
    return "\n".join(o) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--limbs', type=int, required=True)
    ap.add_argument('--bits', type=int, default=28)
    ap.add_argument('--unroll', type=int, default=12)
    ap.add_argument('--name', required=True)
    ap.add_argument('--quad', action='store_true', help='four lanes per ciphertext')
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args()
    src = (gen_quad if a.quad else gen)(a.limbs, a.bits, a.unroll, a.name)
    with open(a.out, 'w') as f:
        f.write(src)


if __name__ == '__main__':
    sys.exit(main())
