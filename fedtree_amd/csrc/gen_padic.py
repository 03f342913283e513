#!/usr/bin/env python3
"""Generator of the P-adic exponentiation kernel (gfx950 assembly): X^e mod P^2 with X kept as two
base-P digits, X = x0 + x1 P, one ciphertext half per lane.

    X Y == x0 y0 + (x0 y1 + x1 y0) P   (mod P^2)          x1 y1 P^2 vanishes
    x0 y0 = u1 P + u0                                     Barrett: quotient and remainder
    Z = u0 + ((x0 y1 + x1 y0 + u1) mod P) P               second Barrett, remainder only

A product mod P^2 is then three (squaring: two) products of 1024-bit digits plus two Barrett
reductions by the 1024-bit P: ~5,030 v_mad per squaring and ~7,030 per general product, against
8,251 and 10,952 for the Montgomery product mod the 2048-bit P^2 of the s74 kernel (gen_montprog.py).
The CRT encrypt's y^P mod P^2 and the decrypt's c^(P-1) mod P^2 are these exponentiations.

Digits are K = 37 radix-2^28 limbs, never reduced below P: with the quotient truncated Barrett
leaves them in [0, 5P), and the bounds hold for inputs in that range (P of 1009..1030 bits), so
there is no correction loop.  tools/padic_model.py is the bit-exact model of this arithmetic
(column order, 64-bit wrap, truncation, bounds).

Products are column-wise (product scanning) into normalised limbs: column c's terms accumulate in
NCH independent 64-bit chains (v_mad_u64_u32 / v_mad_i64_i32), which are summed, given the carry of
column c-1 and split into the limb and the next carry.  That tail is interleaved with the next
column's multiply-adds so that its dependent steps do not stall the wave.

Ops (uint32 pairs from the program buffer; the host's Prog of bn_host.hpp):
    0 END
    1 LOADX  slot   digits <- slot (raw: limbs 0..K-1 = x0, K..2K-1 = x1)
   14 / 16 LOADXGD(16) j   digits <- fixed-base table entry (j << 8 | 16) | digit j of the lane
   15 / 17 MULGD(16) j     X <- X * that entry (tables in digit form, the register-bank layout)
    2 STOREX slot   slot <- digits (raw)
    3 SQR    count  X <- X^2, count times
    4 MUL    slot   X <- X * (digits of slot)
   22 LOADP  slot   digits <- plain X of the slot (2K limbs, X < 50 P^2): one Barrett
   23 STOREP slot   slot <- x0 + x1 P as 2K normalised limbs (< 6 P^2, not reduced mod P^2)

Kernel arguments: those of gen_montprog.py; ctx = [-P limbs (K, int32), zero words up to SGPR 20 + K
rounded up to a multiple of 4, mu limbs (K+1)] with mu = floor(2^(56 K) / P).  K = 37 (Paillier-2048,
P of 1009..1030 bits) and K = 19 (Paillier-1024, P of 505..516 bits; the key's
s37 CRT shape admits 505..514).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_montprog import _descriptor  # noqa: E402

NCH = int(os.environ.get("FTHE_GEN_PADIC_CHAINS", "2"))     # accumulator chains per column (PAIR off)
PAIR = not os.environ.get("FTHE_GEN_PADIC_NOPAIR")             # adjacent columns side by side, one chain each
GROUP = int(os.environ.get("FTHE_GEN_PADIC_GROUP", "2"))       # columns side by side (PAIR)


def gen_padic(K: int, B: int, name: str) -> str:
    MASK = (1 << B) - 1
    assert 2 <= NCH <= 4
    # ---- VGPR plan ---------------------------------------------------------
    V_TID, V_GOFF = 0, 1                        # v2..v9 unused
    NACC = max(NCH, GROUP) if PAIR else NCH     # accumulators per column set
    ACC0 = 10                                   # 2 column sets x NACC accumulators, 64-bit each
    CARRY = ACC0 + 4 * NACC                     # v[CARRY:CARRY+1]
    BK = (CARRY + 2 + 1) & ~1                   # banks start even
    KB = K + (K & 1)                            # bank size (even)
    BANK = [BK + KB * i for i in range(4)]
    VR = BANK[3] + KB                           # 2K limbs
    NVGPR = VR + 2 * K
    assert NVGPR <= 256, f"VGPR budget exceeded: {NVGPR}"
    # ---- SGPR plan ---------------------------------------------------------
    # s[0:1] kernarg, s2 wg id, s[4:5] slots, s[6:7] prog, s[8:9] ctx, s10 limb stride,
    # s11 slot stride, s[12:13] return address, s[14:15] op/arg, s[16:17] addr, s19 counter,
    # s[2:3] call target (after the prologue); -P limbs from s20, mu limbs from s20 + K + 3
    SNP = 20
    SMU = (SNP + K + 3) & ~3                    # mu from a 4-aligned SGPR (s_load_dwordx4+ alignment)
    NSGPR = SMU + K + 1
    assert SMU % 4 == 0 and NSGPR <= 102, (SMU, NSGPR)

    def bank(b, i):
        return f"v{BANK[b] + i}"

    def vr(i):
        return f"v{VR + i}"

    def pair(r):
        n = int(r[1:])
        return f"v[{n}:{n + 1}]"

    def acc(s, ch):
        n = ACC0 + 2 * (NACC * s + ch)
        return f"v[{n}:{n + 1}]"

    def acclo(s, ch):
        return f"v{ACC0 + 2 * (NACC * s + ch)}"

    carry = f"v[{CARRY}:{CARRY + 1}]"
    NP = lambda j: f"s{SNP + j}"                # -P_j
    MU = lambda j: f"s{SMU + j}"

    o = []
    e = o.append

    # ---- column engine -----------------------------------------------------
    def columns(cols, signed=False):
        """cols: list of dicts with keys
             terms: [(a, b)] multiply-adds of the column (a VGPR, b VGPR or SGPR; b may be '1')
             dbl:   double the column's term sum before adding the carry (cross terms)
             sq:    register x: add x*x after the doubling
             out:   register for the limb (None: carry only)
             last:  keep the whole accumulator (low word) as the limb, no carry out
             nocarry: the limb is masked but no carry leaves the column (mod b^n)
        The carry of the first column is 0.  PAIR: two adjacent columns accumulate side by side, one
        chain each (no chain-combining instruction); else NCH chains per column."""
        mad = 'v_mad_i64_i32' if signed else 'v_mad_u64_u32'
        shr = 'v_ashrrev_i64' if signed else 'v_lshrrev_b64'
        pending = []                             # tail instructions of the previous group

        def flush(n):
            for _ in range(min(n, len(pending))):
                e(pending.pop(0))

        def tail_of(ci, col, chains):
            """tail of column ci whose term sum is in chains[0] (+ the other used chains)"""
            t = []
            a0 = chains[0][0]
            lo0 = chains[0][1]
            used = [c for c in chains if c[2]]
            for c in used[1:]:
                t.append(f'  v_lshl_add_u64 {a0}, {c[0]}, 0, {a0}')
            first = ci == 0
            if not used:
                if col.get('sq'):
                    raise AssertionError("square term without cross terms")
                t.append(f'  v_mov_b64_e32 {a0}, {"0" if first else carry}')
            elif col.get('dbl'):
                t.append(f'  v_lshl_add_u64 {a0}, {a0}, 1, {"0" if first else carry}')
            elif not first:
                t.append(f'  v_lshl_add_u64 {a0}, {a0}, 0, {carry}')
            if col.get('sq'):
                x = col['sq']
                t.append(f'  {mad} {a0}, vcc, {x}, {x}, {a0}')
            if col.get('out') is not None:
                if col.get('last'):
                    t.append(f'  v_mov_b32_e32 {col["out"]}, {lo0}')
                else:
                    t.append(f'  v_and_b32_e32 {col["out"]}, {hex(MASK)}, {lo0}')
            if not col.get('last') and not col.get('nocarry'):
                t.append(f'  {shr} {carry}, {B}, {a0}')
            return t

        group = GROUP if PAIR else 1
        for gi in range(0, len(cols), group):
            s = (gi // group) % 2
            members = list(range(gi, min(gi + group, len(cols))))
            if PAIR:
                # member m accumulates in chain m of set s
                streams = [[(acc(s, m), cols[ci]['terms'])] for m, ci in enumerate(members)]
            else:
                ci = members[0]
                streams = [[(acc(s, ch), cols[ci]['terms'][ch::NCH])] for ch in range(NCH)]
            # interleave the multiply-adds of all streams
            seqs = [st[0] for st in streams]
            used = [False] * len(seqs)
            n = 0
            for t in range(max(len(q[1]) for q in seqs) if seqs else 0):
                for k, (ac, terms) in enumerate(seqs):
                    if t < len(terms):
                        a_, b_ = terms[t]
                        e(f'  {mad} {ac}, vcc, {a_}, {b_}, {ac if used[k] else "0"}')
                        used[k] = True
                        n += 1
                        if n % 2 == 0:
                            flush(1)
            flush(len(pending))
            tail = []
            if PAIR:
                for m, ci in enumerate(members):
                    a_ = acc(s, m)
                    tail += tail_of(ci, cols[ci], [(a_, acclo(s, m), used[m])])
            else:
                ci = members[0]
                tail += tail_of(ci, cols[ci], [(acc(s, ch), acclo(s, ch), used[ch]) for ch in range(NCH)])
            pending = tail
        flush(len(pending))

    def product_cols(a, b, n_out, outs, a2=None, b2=None):
        """a x b (+ a2 x b2) over digit limb lists -> n_out columns (last keeps the carry)"""
        cols = []
        for c in range(n_out):
            terms = []
            for i in range(len(a)):
                j = c - i
                if 0 <= j < len(b):
                    terms.append((a[i], b[j]))
                    if a2 is not None:
                        terms.append((a2[i], b2[j]))
            cols.append({'terms': terms, 'out': outs[c], 'last': c == n_out - 1})
        return cols

    # ---- Barrett: T (2K limbs) -> q3 (K limbs), r = (T - q3 P) mod b^K in place of T[0..K-1]
    def barrett(T, q3, rout=None):
        """q3 = the truncated-Barrett quotient of T by P, r = (T - q3 P) mod b^K into rout (default:
        in place of T[0..K-1]; rout may not alias q3)"""
        rout = rout or T[:K]
        q1 = T[K - 1:2 * K]                      # K + 1 limbs
        cols = []
        for c in range(K - 1, 2 * K + 1):
            terms = []
            for i in range(K + 1):
                j = c - i
                if 0 <= j < K + 1:
                    terms.append((q1[i], MU(j)))
            out = q3[c - K - 1] if c >= K + 1 else None
            cols.append({'terms': terms, 'out': out, 'last': c == 2 * K})
        columns(cols)
        cols = []
        for c in range(K):
            terms = [(T[c], '1')]
            for i in range(K):
                j = c - i
                if 0 <= j < K:
                    terms.append((q3[i], NP(j)))
            cols.append({'terms': terms, 'out': rout[c], 'last': False})
        cols[-1]['nocarry'] = True
        columns(cols, signed=True)

    X0 = [bank(0, i) for i in range(K)]
    X1 = [bank(1, i) for i in range(K)]
    Y0 = [bank(2, i) for i in range(K)]
    Y1 = [bank(3, i) for i in range(K)]
    VV = [vr(i) for i in range(2 * K)]
    TT = X1 + Y1                                 # T of both products and of LOADP: banks 1 and 3

    def move_digit(dst, src):
        for i in range(0, K - 1, 2):
            e(f'  v_pk_mov_b32 {pair(dst[i])}, {pair(src[i])}, {pair(src[i])} op_sel:[0,1]')
        if K % 2:
            e(f'  v_mov_b32_e32 {dst[K - 1]}, {src[K - 1]}')

    # ---- prologue ------------------------------------------------------------
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
    e('  s_waitcnt lgkmcnt(0)')
    off, sreg, rem = 0, SNP, NSGPR - SNP
    for width in (16, 8, 4, 2, 1):
        while rem >= width:
            assert sreg % min(width, 4) == 0
            suffix = f"x{width}" if width > 1 else ""
            dst = f"s[{sreg}:{sreg + width - 1}]" if width > 1 else f"s{sreg}"
            e(f'  s_load_dword{suffix} {dst}, s[8:9], {hex(off)}')
            off += 4 * width
            sreg += width
            rem -= width
    e('  s_lshl_b32 s14, s2, 10')                  # wg * 256 * 4
    e(f'  v_lshlrev_b32_e32 v{V_GOFF}, 2, v{V_TID}')
    e(f'  v_add_u32_e32 v{V_GOFF}, s14, v{V_GOFF}')
    e('  s_waitcnt lgkmcnt(0)')

    e('.Lprog:')
    e('  s_load_dwordx2 s[14:15], s[6:7], 0x0')
    e('  s_add_u32 s6, s6, 8')
    e('  s_addc_u32 s7, s7, 0')
    e('  s_waitcnt lgkmcnt(0)')
    for code, lab in ((1, '.Lloadx'), (2, '.Lstorex'), (3, '.Lsqr'), (4, '.Lmul'), (22, '.Lloadp'), (23, '.Lstorep'),
                      (14, '.Lloadxgd'), (15, '.Lmulgd'), (16, '.Lloadxgd16'), (17, '.Lmulgd16')):
        e(f'  s_cmp_eq_u32 s14, {code}')
        e(f'  s_cbranch_scc1 {lab}')
    e('  s_branch .Lend')

    def slot_addr():
        e('  s_mul_i32 s16, s15, s11')
        e('  s_mul_hi_u32 s17, s15, s11')
        e('  s_add_u32 s16, s4, s16')
        e('  s_addc_u32 s17, s5, s17')

    def load_limbs(regs):
        slot_addr()
        for k, r in enumerate(regs):
            e(f'  global_load_dword {r}, v{V_GOFF}, s[16:17]')
            if k != len(regs) - 1:
                e('  s_add_u32 s16, s16, s10')
                e('  s_addc_u32 s17, s17, 0')
        e('  s_waitcnt vmcnt(0)')

    def store_limbs(regs):
        slot_addr()
        for k, r in enumerate(regs):
            e(f'  global_store_dword v{V_GOFF}, {r}, s[16:17]')
            if k != len(regs) - 1:
                e('  s_add_u32 s16, s16, s10')
                e('  s_addc_u32 s17, s17, 0')
        e('  s_waitcnt vmcnt(0)')

    ncall = [0]

    def call(label):
        n = ncall[0]
        ncall[0] += 1
        e('  s_getpc_b64 s[2:3]')
        e(f'.Lpc{n}:')
        e(f'  s_add_u32 s2, s2, {label}-.Lpc{n}')
        e('  s_addc_u32 s3, s3, 0')
        e('  s_swappc_b64 s[12:13], s[2:3]')

    # LOADX / STOREX: raw digits
    e('.Lloadx:')
    load_limbs(X0 + X1)
    e('  s_branch .Lprog')
    e('.Lstorex:')
    store_limbs(X0 + X1)
    e('  s_branch .Lprog')

    # SQR: V = 2 x0 x1 (x1 dead), T = x0^2 into banks 1, 3 (x0 dead), Barretts
    e('.Lsqr:')
    e('  s_mov_b32 s19, s15')
    e('.Lsqr_loop:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    cols = []
    for c in range(2 * K):
        terms = [(X0[i], X1[c - i]) for i in range(K) if 0 <= c - i < K]
        cols.append({'terms': terms, 'dbl': True, 'out': VV[c], 'last': c == 2 * K - 1})
    columns(cols)
    cols = []
    for c in range(2 * K):
        terms = [(X0[i], X0[c - i]) for i in range(K) if i < c - i < K]
        sq = X0[c // 2] if c % 2 == 0 and c // 2 < K else None
        col = {'terms': terms, 'out': TT[c], 'last': c == 2 * K - 1}
        if terms:
            col['dbl'] = True
            if sq:
                col['sq'] = sq
        elif sq:                                 # c == 0 or the top square: x*x alone
            col['terms'] = [(sq, sq)]
        cols.append(col)
    columns(cols)
    call('.Lreduce')
    e('  s_sub_u32 s19, s19, 1')
    e('  s_branch .Lsqr_loop')

    # MUL slot: y -> banks 2, 3; W = x0 y1 + x1 y0 (x1, y1 dead), T = x0 y0 into banks 1, 3
    e('.Lmul:')
    load_limbs(Y0 + Y1)
    e('.Lmul_body:')
    columns(product_cols(X0, Y1, 2 * K, VV, a2=X1, b2=Y0))
    columns(product_cols(X0, Y0, 2 * K, TT))
    call('.Lreduce')
    e('  s_branch .Lprog')

    # Fixed-base tables in digit form (the exact randomizer's gathered products): entry
    # (j << W) | dig[j][g] of the table at rows[0], EW = 2 KB words laid out like the register banks
    # (x0 limbs, pad, x1 limbs, pad), so it loads with dwordx4 straight into banks 0, 1 (LOADXGD) or
    # 2, 3 (MULGD, then the product); rows[1] = the u8 / u16 digit array [window][L].
    EW = 2 * KB
    assert EW % 4 == 0 and BANK[1] == BANK[0] + KB and BANK[3] == BANK[2] + KB

    def gather_entry(wide, dst0):
        e('  s_load_dwordx2 s[16:17], s[0:1], 0x30')        # digit array
        e('  s_lshr_b32 s14, s10, 2')                        # L
        e('  s_mul_i32 s14, s14, s15')                       # j * L
        if wide:
            e('  s_lshl_b32 s14, s14, 1')                    # u16 digits
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_add_u32 s16, s16, s14')
        e('  s_addc_u32 s17, s17, 0')
        e(f'  v_lshrrev_b32_e32 v4, {1 if wide else 2}, v{V_GOFF}')   # g x digit size
        e(f'  global_load_{"ushort" if wide else "ubyte"} v4, v4, s[16:17]')
        e('  s_load_dwordx2 s[16:17], s[0:1], 0x28')        # table
        e(f'  s_lshl_b32 s14, s15, {16 if wide else 8}')     # j << W
        e(f'  v_mov_b32_e32 v5, {4 * EW}')
        e('  s_waitcnt vmcnt(0) lgkmcnt(0)')
        e('  v_or_b32_e32 v4, s14, v4')
        e('  v_mad_u64_u32 v[2:3], vcc, v4, v5, s[16:17]')  # 64-bit entry address (tables > 4 GiB)
        for i in range(EW // 4):
            e(f'  global_load_dwordx4 v[{dst0 + 4 * i}:{dst0 + 4 * i + 3}], v[2:3], off offset:{16 * i}')
        e('  s_waitcnt vmcnt(0)')

    for wide in (False, True):
        sfx = "16" if wide else ""
        e(f'.Lloadxgd{sfx}:')
        gather_entry(wide, BANK[0])
        e('  s_branch .Lprog')
        e(f'.Lmulgd{sfx}:')
        gather_entry(wide, BANK[2])
        e('  s_branch .Lmul_body')

    # LOADP slot: plain X -> T -> (q3, r) -> x0 = r, x1 = q3
    e('.Lloadp:')
    load_limbs(TT)
    barrett(TT, Y0, X0)                          # q3 -> bank 2, r -> bank 0 (x0)
    move_digit(X1, Y0)                           # x1 = q3
    e('  s_branch .Lprog')

    # STOREP slot: x0 + x1 P = x0 - (-x1)(... ) with -P in SGPRs: (-x1_i)(-P_j)
    e('.Lstorep:')
    for i in range(K):
        e(f'  v_sub_u32_e32 {Y0[i]}, 0, {X1[i]}')
    cols = []
    for c in range(2 * K):
        terms = [(X0[c], '1')] if c < K else []
        terms += [(Y0[i], NP(c - i)) for i in range(K) if 0 <= c - i < K]
        cols.append({'terms': terms, 'out': VV[c], 'last': c == 2 * K - 1})
    columns(cols, signed=True)
    store_limbs(VV)
    e('  s_branch .Lprog')

    e('.Lend:')
    e('  s_endpgm')

    # shared reduction of SQR and MUL: T (banks 1, 3) -> q3 = u1 (bank 2), r = u0 into bank 0;
    # V += u1; V -> q3' (bank 3), r' into bank 1: the digits land where the next op reads them
    e('.Lreduce:')
    barrett(TT, Y0, X0)                          # u1 -> bank 2 (y0 / unused), u0 -> bank 0 (x0 is dead)
    e('.Lreduce_v:')
    for i in range(K):
        e(f'  v_add_u32_e32 {VV[i]}, {VV[i]}, {Y0[i]}')
    barrett(VV, Y1, X1)                          # q3' -> bank 3 (T's top, consumed), r' -> bank 1 (x1)
    e('  s_setpc_b64 s[12:13]')

    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    o.extend(_descriptor(name, 0, NVGPR, NSGPR).splitlines())
    return "\n".join(o) + "\n"


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--digit-limbs', type=int, default=37)
    ap.add_argument('--name', default='fthe_padic_k37')
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args()
    with open(a.out, 'w') as f:
        f.write(gen_padic(a.digit_limbs, 28, a.name))
