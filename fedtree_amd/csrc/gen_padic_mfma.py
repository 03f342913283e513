#!/usr/bin/env python3
"""Generator of the P-adic exponentiation kernel with matrix-core Barrett reductions (gfx950 assembly):
fthe_padic_m37, X^e mod P^2 with X = x0 + x1 P kept as two base-P digits of K = 37 radix-2^28 limbs,
one ciphertext half per lane -- the arithmetic of gen_padic.py (see its docstring), except where the
work goes.

The products of a squaring (2 x0 x1, x0^2) are variable x variable and stay on the VALU (product
scanning, v_mad_u64_u32).  The two Barrett reductions that follow every product are 60% of the
multiply-adds of fthe_padic_k37, and both of their products have a constant operand (mu, P): over the
64 lanes of a wave they are matrix products, so they run on v_mfma_i32_32x32x32_i8:

  * each lane packs its operand (q1 = T >> 28 (K-1), or q3) into base-256 digits fed as b ^ 0x80 = b - 128
    (40 dwords, region XB), and v_permlane32_swap turns them into the B operands of two 32-lane groups
    (lanes 0-31 / 32-63 of the wave);
  * the A operand is a 32 x 32 tile of the constant's Toeplitz matrix in balanced base-256 digits, read
    from LDS (19 tiles, 19 KB, filled once per workgroup from the key's context; the correction for the
    -128 offset and the truncation bias ride in one extra digit column, tools/padic_mfma_model.py);
  * each M-tile (32 output columns) accumulates its K-tiles in int32 (16 VGPRs per group); adjacent rows are
    paired in 32-bit, the two groups' accumulators exchanged with v_permlane32_swap (only the registers the
    fold reads) so that every lane holds its own 32 column sums, and the lane folds them into 28-bit limbs:
    one v_mad_i64_i32 per (paired) column (x 2^sh), one mask and one arithmetic shift per limb, the carry
    entering the next limb's first multiply-add;
  * the limbs that only feed the matrix cores (the upper product halves, q3) are produced with their operand
    bytes already XORed with 0x80 (v_bitop3_b32), so packing them costs no XOR.

Product 1 forms columns 112..271 of q1 mu and yields q3 = Barrett's quotient estimate or one less (q3 is
clamped to 0 when q1 = 0); product 2 forms columns 0..129 of q3 P (as matrix columns 1..130, the constant
digit leading) and r = (T - q3 P) mod b^K exactly.
The digits stay within [0, 5P) as in fthe_padic_k37 (the bounds are asserted by the model).

Ops: those of gen_padic.py except the fixed-base table ops (LOADXGD / MULGD), which the host keeps on
fthe_padic_k37:  0 END, 1 LOADX, 2 STOREX, 3 SQR, 4 MUL, 22 LOADP, 23 STOREP.
ctx: [-P limbs (K, int32) ...] as for fthe_padic_k37, and the LDS tile image at byte 512 (20 KB).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_montprog import _descriptor  # noqa: E402

# A/B variants for tools/build_m37_ab.sh only (fedtree_amd/build.py clears the switch): the timing-only ones
# give wrong results (noswap, nonop, nomfma); the others are correct schedules: nodbuf, nointerleave, nopair,
# noprepair, nodesync, spill, pingpong[,ppodd], col3 / col4, marginN, prioN / noprio, noprexor, nocmerge,
# ldsx[,ldsxa]
AB = os.environ.get("FTHE_GEN_M37_AB", "")
TILE_OFF = 512                  # byte offset of the tile image in ctx
TILE_BYTES = 20 * 1024          # 19 tiles of 1 KB, padded to 5 dwordx4 per thread
SPILL_BYTES = 10 * 1024         # per wave: V[37..73] while Barrett 1 runs (9 x dwordx4 + 1 dword per lane)
SPILL = "spill" in AB           # measured: no gain (profiles/r02zzi_spill_ab.jsonl), so off
# ping-pong halves in 512-thread workgroups (s_barrier between products and reduction): no gain
# (profiles/r03t_m37_pingpong_ab.jsonl), so off
PP = "pingpong" in AB
# VALU instructions kept between a tile's last MFMA and the lane exchange that reads its results (>= 24: the
# 8-pass XDL -> VALU hazard then needs no s_nop); A/B knob marginN (24..90 within noise,
# profiles/r03zj_m37_margin_ab.jsonl)
MARGIN = next((int(t[6:]) for t in AB.split(',') if t.startswith('margin') and t[6:].isdigit()), 30)
assert MARGIN >= 24
# the limbs that only ever reach the matrix cores (the upper product halves and q3) leave the column tails /
# chunk folds with bit 7 of every byte already flipped (v_bitop3_b32 (x & mask) ^ pattern in place of the
# mask), so packing them into the b ^ 0x80 operand bytes needs no v_xor per dword: 128 fewer VALU per
# squaring, 71.7-72.2 vs 73.0-73.5 ms (profiles/r03y_m37_prexor_ab.jsonl)
PREXOR = "noprexor" not in AB
# a chunk's carry enters the next chunk's first multiply-add (no carry add in its tail): 162 fewer VALU per
# squaring, 69.8-70.5 vs 71.7-72.9 ms (profiles/r03za_m37_cmerge_ab.jsonl)
CMERGE = "nocmerge" not in AB
# ldsx: the B operands' lane-half exchange through LDS (each half writes the 4 dwords per K-block the other half
# needs under a half EXEC mask and reads the partner's back) instead of 20 v_permlane32_swap per product, which
# cost 8 issue cycles each (profiles/r03zr_mfma_hold_probe.jsonl).  Measured slower: 72.1-72.4 vs 70.9-71.0 ms,
# with ldsxa 74.6-75.3 (profiles/r03zs_m37_ldsx_ab.jsonl): the stores' VGPR transfer and the round trip the
# wave waits out cost more than the swaps, so off
LDSX = "ldsx" in AB
# ldsxa (with ldsx): also the accumulator exchange of every fully paired M-tile (8 of a Barrett's 10): the 8
# pairs packed into the tile's first 8 accumulator registers, 2 dwordx4 per half through LDS for 8 swaps
LDSXA = LDSX and "ldsxa" in AB
LDSX_BYTES = 5 * 1024           # per wave: 5 K-blocks x 64 lanes x 16 B
# kara: a squaring's cross term V = 2 x0 x1 by one level of Karatsuba on the halves x = xL + xH b^19 (19 / 18
# limbs): 2 P0 = 2 xL yL and 2 P2 = 2 xH yH normalised first (P0 into V[0..18] and C, P2 complemented into
# V[38..73]), then the middle columns of (x0L + x0H)(2 x1L + 2 x1H) - 2 P0 - 2 P2 added at b^19 with a biased
# carry, and the carry rippled through V[57..73] beside x0^2's multiply-adds: 1,046 instead of 1,369
# multiply-adds per squaring, 4,076 instead of 4,102 VALU (see kara_cross below).  Measured +0.5%: 133.8-134.1 vs
# 134.5-134.9 ms per 786,432 lanes, 67.8-68.4 vs 68.0-68.5 per 393,216 (profiles/r05i_m37_kara_ab.jsonl) -- the
# MAD cycles saved mostly reappear as exposed latency of the matrix phases; nokara keeps the plain product (A/B)
KARA = "nokara" not in AB
assert not (KARA and LDSX)
assert not (LDSX and (PP or SPILL))
LDS_BYTES = TILE_BYTES + (4 * SPILL_BYTES if SPILL else 0) + (4 * LDSX_BYTES if LDSX else 0)
S1_LO = 112                     # product-1 columns S1_LO .. S1_LO + 159
QBIT = 28 * 38                  # q3 = floor(N / 2^1064)
TILE_D1 = (-3, -2, -1, 0, 1)    # product-1 Toeplitz tiles (k <= 3) by m - k; then k = 4 for m = 0..4
TILE_D2 = (0, 1, 2, 3)          # product-2: k = 0 for m = 0..4 (tiles 10..14), then Toeplitz (k >= 1) by m - k


def tile_index(prod, m, k):
    if prod == 1:
        return TILE_D1.index(m - k) if k <= 3 else 5 + m
    return 10 + m if k == 0 else 15 + TILE_D2.index(m - k)


def gen_padic_mfma(name: str) -> str:
    K, B = 37, 28
    MASK = (1 << B) - 1
    # ---- VGPR plan ---------------------------------------------------------
    V_TID, V_GOFF = 0, 1
    VA = (2, 6, 10)                              # A-tile buffers v[2:5], v[6:9], v[10:13] (ACC is free)
    # product columns: NCOL adjacent columns side by side (one 64-bit accumulator chain each), two column
    # sets (the tails of one set run inside the next set's multiply-adds)
    NCOL = next((int(t[3:]) for t in AB.split(',') if t in ('col3', 'col4')), 2)
    assert NCOL == 2 or not KARA, "col3 / col4 predate the Karatsuba cross term (wrong results, r06s): add nokara"
    ACC0 = 10 if NCOL == 2 else 2                # v[ACC0 .. ACC0 + 4 NCOL); below v20 either way
    CARRY = ACC0 + 4 * NCOL
    XA = 20                                      # x0 digit (v20..v56); Barrett: accumulators v20..v51
    G0, G1 = XA, XA + 16
    # Barrett scratch in XA above the accumulators: chunk sums v[52:55], clamp mask v56, chunk carry v[58:59]
    XB = 60                                      # x1 digit (v60..v96); Barrett: operand dwords D0..D39
    TT = 100                                     # T limbs v100..v173
    VV = 174                                     # V limbs v174..v247
    V_LDS = 248                                  # (lane & 63) * 16
    V_SPILL = 249                                # this wave's spill area + (lane & 63) * 16 (SPILL only)
    PATV = (249, 250)                            # PREXOR: byte-flip patterns of even / odd limbs
    assert not (SPILL and PREXOR)
    NVGPR = 250 if SPILL else 251 if PREXOR else 249
    V_XW, V_XR = NVGPR, NVGPR + 1                # LDSX: this wave's exchange area + lane * 16, and ^ 512
    if LDSX:
        NVGPR += 2

    def pat(t):
        """flip pattern of limb t of a packed number (limb t at bit 28 t): bits j with 28 t + j = 7 mod 8"""
        return f"v{PATV[t % 2]}"
    PATVAL = (0x00808080, 0x08080808)
    X0 = [f"v{XA + i}" for i in range(K)]
    X1 = [f"v{XB + i}" for i in range(K)]
    T = [f"v{TT + i}" for i in range(2 * K)]
    V = [f"v{VV + i}" for i in range(2 * K)]
    D = [f"v{XB + i}" for i in range(40)]
    # ---- SGPR plan ---------------------------------------------------------
    # s[0:1] kernarg, s2 wg id, s[2:3] call target, s[4:5] slots, s[6:7] prog, s[8:9] ctx, s10 limb
    # stride, s11 slot stride, s[12:13] return address, s[14:15] op/arg, s[16:17] addr, s18 half (PP), s19 counter;
    # s20..s27 = 2^0, 2^4, .., 2^28; s28..s34 = -2^0, .., -2^24; -P limbs from s36
    SPOW, SNEG, SNP = 20, 28, 36                   # s35 = 0x0fffffff
    NSGPR = SNP + K
    SLO, SHI = 74, 76                            # LDSX: EXEC masks of lanes 0-31 / 32-63
    if LDSX:
        NSGPR = SHI + 2
    if KARA:                                     # s76..s78: 2, 3, 4 x mask
        NSGPR = 79
    POW = lambda sh: f"s{SPOW + sh // 4}"
    NEG = lambda sh: f"s{SNEG + sh // 4}"
    NP = lambda j: f"s{SNP + j}"

    def pair(n):
        return f"v[{n}:{n + 1}]"

    def acc(s, ch):
        n = ACC0 + 2 * (NCOL * s + ch)
        return f"v[{n}:{n + 1}]"

    def acclo(s, ch):
        return f"v{ACC0 + 2 * (NCOL * s + ch)}"

    carry = pair(CARRY)
    o = []
    sink = [o]                                   # capture() redirects the emitter into a side list

    def e(line):
        sink[-1].append(line)

    def phase():
        if PP:
            e('  s_barrier')

    def capture(fn):
        sink.append([])
        try:
            fn()
        finally:
            out = sink.pop()
        return out

    # ---- column engine (product scanning, two adjacent columns side by side) --------------------
    def columns(cols, signed=False, carry_in=False, bg=()):
        """product scanning over cols (dicts): 'terms' [(a, b)] multiply-adds, 'dbl' (column x 2), 'sq' (one
        more x*x after the doubling), 'out' (the limb register), 'px' (flip pattern of a pre-XORed limb), 'cpl'
        (store mask - limb), 'last' (no mask, no carry), 'addend' (a register pair with a zero high dword: the
        first multiply-add's addend), 'pre' (instructions that must precede the column's first multiply-add:
        emitted during the previous group's multiply-adds).  carry_in: the carry register holds column 0's
        carry.  bg: independent instructions spread over the multiply-adds (one per two while no tail is
        pending), the rest emitted at the end."""
        mad = 'v_mad_i64_i32' if signed else 'v_mad_u64_u32'
        shr = 'v_ashrrev_i64' if signed else 'v_lshrrev_b64'
        pending = []
        bgq = list(bg)

        def flush(n):
            for _ in range(min(n, len(pending))):
                e(pending.pop(0))

        def tick():
            if pending:
                flush(1)
            elif bgq:
                e(bgq.pop(0))

        def tail_of(ci, col, a0, lo0, used):
            t = []
            first = ci == 0 and not carry_in
            if not used:
                if col.get('addend'):
                    t.append(f'  v_lshl_add_u64 {a0}, {col["addend"]}, 0, {"0" if first else carry}')
                else:
                    t.append(f'  v_mov_b64_e32 {a0}, {"0" if first else carry}')
            elif col.get('dbl'):
                t.append(f'  v_lshl_add_u64 {a0}, {a0}, 1, {"0" if first else carry}')
            elif not first:
                t.append(f'  v_lshl_add_u64 {a0}, {a0}, 0, {carry}')
            if col.get('sq'):
                x = col['sq']
                t.append(f'  {mad} {a0}, vcc, {x}, {x}, {a0}')
            if col.get('out') is not None:
                px = col.get('px')
                if col.get('cpl'):                           # mask - limb (the top limb: < 2^28 asserted by
                    assert not px                            # the model, so the XOR is the same)
                    if col.get('last'):
                        t.append(f'  v_xor_b32_e32 {col["out"]}, {SMASK}, {lo0}')
                    else:
                        t.append(f'  v_bitop3_b32 {col["out"]}, {lo0}, {SMASK}, {lo0} bitop3:0xc')
                elif col.get('last'):
                    if px:
                        t.append(f'  v_xor_b32_e32 {col["out"]}, {px}, {lo0}')
                    else:
                        t.append(f'  v_mov_b32_e32 {col["out"]}, {lo0}')
                elif px:                                     # (lo & mask) ^ pattern
                    t.append(f'  v_bitop3_b32 {col["out"]}, {lo0}, {SMASK}, {px} bitop3:0x6a')
                else:
                    t.append(f'  v_and_b32_e32 {col["out"]}, {hex(MASK)}, {lo0}')
            if not col.get('last') and not col.get('nocarry'):
                t.append(f'  {shr} {carry}, {B}, {a0}')
            return t

        for ci in range(min(NCOL, len(cols))):
            for ins in cols[ci].get('pre', ()):
                e(ins)
        for gi in range(0, len(cols), NCOL):
            s = (gi // NCOL) % 2
            members = list(range(gi, min(gi + NCOL, len(cols))))
            seqs = [(acc(s, m), cols[ci]['terms'], cols[ci].get('addend')) for m, ci in enumerate(members)]
            used = [False] * len(seqs)
            for ci in range(gi + NCOL, min(gi + 2 * NCOL, len(cols))):
                pending += list(cols[ci].get('pre', ()))
            n = 0
            for t in range(max(len(q[1]) for q in seqs)):
                for k, (ac, terms, add) in enumerate(seqs):
                    if t < len(terms):
                        a_, b_ = terms[t]
                        e(f'  {mad} {ac}, vcc, {a_}, {b_}, {ac if used[k] else (add or "0")}')
                        used[k] = True
                        n += 1
                        if n % 2 == 0:
                            tick()
            flush(len(pending))
            tail = []
            for m, ci in enumerate(members):
                tail += tail_of(ci, cols[ci], acc(s, m), acclo(s, m), used[m])
            pending = tail
        flush(len(pending))
        for ins in bgq:
            e(ins)

    def product_cols(a, b, n_out, outs, a2=None, b2=None):
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
            if PREXOR and c >= K:                      # the upper half only feeds Barrett's q1 bytes
                cols[-1]['px'] = pat(c - (K - 1))
        return cols

    def move(dst, src):
        n = len(src)
        for i in range(0, n - 1, 2):
            if int(dst[i][1:]) % 2 == 0 and int(src[i][1:]) % 2 == 0:
                e(f'  v_pk_mov_b32 {pair(int(dst[i][1:]))}, {pair(int(src[i][1:]))}, {pair(int(src[i][1:]))} op_sel:[0,1]')
            else:
                e(f'  v_mov_b32_e32 {dst[i]}, {src[i]}')
                e(f'  v_mov_b32_e32 {dst[i + 1]}, {src[i + 1]}')
        if n % 2:
            e(f'  v_mov_b32_e32 {dst[n - 1]}, {src[n - 1]}')

    # ---- matrix-core Barrett -------------------------------------------------
    CACC2 = (pair(XA + 32), pair(XA + 34))      # chunk sums, alternating by chunk parity: v[52:53], v[54:55]
    CCARRY = pair(XA + 38)                      # chunk carry v[58:59]
    SMASK = "s35"                               # 0x0fffffff (v_bfi_b32 operand)
    S2MASK, S3MASK, S4MASK = "s76", "s77", "s78"  # KARA: 2, 3, 4 x 0x0fffffff

    def orpack(limbs, shift_bits, ndw, xor_masks, lead_one=False, norm0=False, pre=()):
        """normalised 28-bit limbs (limb t at bit 28 t + shift_bits) -> dwords D[0..ndw-1] XOR xor_masks[w],
        each dword from the (at most two) limbs it overlaps: no carry chain.  lead_one: byte 0 is the
        constant digit 1 (shift_bits = 8).  norm0: limb 0 may hold a bit 28 (masked off here).  pre: the
        limbs already XORed with pat(t) (PREXOR); only the flips they do not carry are applied here."""
        n = len(limbs)
        pre = set(pre)

        def carried(w):
            """bits of dword w already flipped by pre-XORed limbs"""
            m = 0
            for b in range(32):
                q = 32 * w - shift_bits + b                   # bit of the packed number
                if q < 0 or (lead_one and w == 0 and b < 8):
                    continue
                t, j = q // B, q % B
                if t in pre and t < n and (PATVAL[t % 2] >> j) & 1:
                    m |= 1 << b
            return m
        xor_masks = [xor_masks[w] ^ carried(w) for w in range(ndw)]
        for w in range(ndw):
            d = D[w]
            if lead_one and w == 0:
                e(f'  v_lshl_or_b32 {d}, {limbs[0]}, 8, 1')
            else:
                lo = (32 * w - shift_bits) // B
                off = 32 * w - shift_bits - B * lo
                hi_ok = lo + 1 < n
                if norm0 and lo == 0:
                    assert off == 0 and hi_ok
                    e(f'  v_lshlrev_b32_e32 {d}, 28, {limbs[1]}')
                    e(f'  v_bfi_b32 {d}, {SMASK}, {limbs[0]}, {d}')
                elif not hi_ok:
                    e(f'  v_lshrrev_b32_e32 {d}, {off}, {limbs[lo]}')
                elif off == 0:
                    e(f'  v_lshl_or_b32 {d}, {limbs[lo + 1]}, 28, {limbs[lo]}')
                else:
                    e(f'  v_lshrrev_b32_e32 {d}, {off}, {limbs[lo]}')
                    e(f'  v_lshl_or_b32 {d}, {limbs[lo + 1]}, {B - off}, {d}')
            if xor_masks[w]:
                e(f'  v_xor_b32_e32 {d}, {hex(xor_masks[w])}, {d}')

    def swap_operands():
        if LDSX:
            # lane r + 32's D[8k + j] <-> lane r's D[8k + 4 + j], as the swaps below; LDS executes one wave's
            # operations in order, and the last one (K-block 4) is never the first tile's first K-block, which
            # issue_tile's lgkmcnt counts then leave the only exchange operation possibly still in flight
            lo, hi = f"s[{SLO}:{SLO + 1}]", f"s[{SHI}:{SHI + 1}]"
            e(f'  s_mov_b64 exec, {lo}')
            for k in range(5):
                e(f'  ds_write_b128 v{V_XW}, v[{XB + 8 * k + 4}:{XB + 8 * k + 7}] offset:{1024 * k}')
            e(f'  s_mov_b64 exec, {hi}')
            for k in range(5):
                e(f'  ds_write_b128 v{V_XW}, v[{XB + 8 * k}:{XB + 8 * k + 3}] offset:{1024 * k}')
            for k in range(5):
                e(f'  ds_read_b128 v[{XB + 8 * k}:{XB + 8 * k + 3}], v{V_XR} offset:{1024 * k}')
            e(f'  s_mov_b64 exec, {lo}')
            for k in range(5):
                e(f'  ds_read_b128 v[{XB + 8 * k + 4}:{XB + 8 * k + 7}], v{V_XR} offset:{1024 * k}')
            e('  s_mov_b64 exec, -1')
            return
        e('  s_nop 1')
        for k in range(5):
            for j in range(4):
                e(f'  v_permlane32_swap_b32_e32 {D[8 * k + j]}, {D[8 * k + 4 + j]}')
        e('  s_nop 4')

    def rd(prod, m, k, n):
        b_ = VA[n % 3]
        e(f'  ds_read_b128 v[{b_}:{b_ + 3}], v{V_LDS} offset:{1024 * tile_index(prod, m, k)}')

    def prefetch(prod, m, ks):
        """the first two A-tile reads of M-tile m (issued while the lane still has VALU work)"""
        for n in range(min(2, len(ks))):
            rd(prod, m, ks[n], n)

    GB0, GB1 = TT + 38, TT + 54                  # second accumulator set v[138:153], v[154:169] (T[38..69])
    GV0, GV1 = VV + 38, VV + 54                  # or v[212:227], v[228:243] (V[38..69], spilled to LDS)

    def issue_tile(prod, m, ks, G0x, G1x, prefetched=True):
        """the MFMAs of M-tile m over K-tiles ks (both lane groups) into accumulators G0x, G1x; with
        prefetched its first two A-tile reads are already in flight, the rest rotate through three
        buffers one step ahead"""
        L = len(ks)
        if not prefetched:
            prefetch(prod, m, ks)
        for n, k in enumerate(ks):
            if n + 2 < L:
                rd(prod, m, ks[n + 2], n + 2)
            e(f'  s_waitcnt lgkmcnt({min(L, n + 3) - n - 1})')
            buf = VA[n % 3]
            for g, G in ((0, G0x), (1, G1x)):
                src_c = "0" if n == 0 else f"v[{G}:{G + 15}]"
                bo = 8 * k + 4 * g
                if "nomfma" not in AB:
                    e(f'  v_mfma_i32_32x32x32_i8 v[{G}:{G + 15}], v[{buf}:{buf + 3}], v[{XB + bo}:{XB + bo + 3}], {src_c}')

    def consumed(prod, m):
        """the rows (output columns rho of M-tile m) the fold reads: all of product 1; product 2 drops matrix
        column 0 (the constant digit's) and the columns above 130"""
        if prod == 1:
            return set(range(32))
        return {rho for rho in range(32) if 1 <= 32 * m + rho <= 130}

    def plan(C):
        """accumulator register rr holds row 8 (rr >> 2) + 4 h + (rr & 3) of the lane half h, i.e. output
        column rho_a = 8 (rr >> 2) + (rr & 3) or rho_a + 4 after the exchange.  Even rr whose two rows are both
        read (or both unread) in both halves are paired before the exchange, c_rho + 256 c_(rho+1) in 32-bit
        arithmetic (|c| < 2^21.2: exact), so the odd register need not move; returns (paired even rr, the rr
        to exchange)"""
        paired, swaps = set(), []
        for rr in range(0, 16, 2):
            ra = 8 * (rr >> 2) + (rr & 3)
            rhos = (ra, ra + 4)
            if "noprepair" not in AB and all((r in C) == (r + 1 in C) for r in rhos) \
                    and any(r in C for r in rhos):
                paired.add(rr)
        for rr in range(16):
            ra = 8 * (rr >> 2) + (rr & 3)
            if (ra in C or ra + 4 in C) and not (rr % 2 and rr - 1 in paired):
                swaps.append(rr)
        return paired, swaps

    def compact(tile):
        """LDSXA: all 8 even rr paired, the pairs then sit in rr / 2 and move through LDS"""
        return LDSXA and plan(consumed(*tile))[0] == set(range(0, 16, 2))

    def exchange(G0x, G1x, waited=False, tile=None):
        """results -> VALU: wait out the last MFMA writing them (8-pass XDL: 11 wait states on gfx950), pair
        adjacent rows (plan), then exchange the halves of the registers still needed; waited: at least 30
        VALU instructions already separate that MFMA from here"""
        if "nonop" not in AB and not waited:
            e('  s_nop 7')
            e('  s_nop 7')
            e('  s_nop 7')
        paired, swaps = plan(consumed(*tile))
        if compact(tile):
            for rr in range(0, 16, 2):
                for G in (G0x, G1x):
                    e(f'  v_lshl_add_u32 v{G + rr // 2}, v{G + rr + 1}, 8, v{G + rr}')
            # lanes 0-31 send the group-1 pairs and receive the partner's group-0 pairs into them, lanes
            # 32-63 the other way round (the permlane32_swap of every pair register, as below)
            lo, hi = f"s[{SLO}:{SLO + 1}]", f"s[{SHI}:{SHI + 1}]"
            e(f'  s_mov_b64 exec, {lo}')
            for j in range(2):
                e(f'  ds_write_b128 v{V_XW}, v[{G1x + 4 * j}:{G1x + 4 * j + 3}] offset:{1024 * j}')
            e(f'  s_mov_b64 exec, {hi}')
            for j in range(2):
                e(f'  ds_write_b128 v{V_XW}, v[{G0x + 4 * j}:{G0x + 4 * j + 3}] offset:{1024 * j}')
            for j in range(2):
                e(f'  ds_read_b128 v[{G0x + 4 * j}:{G0x + 4 * j + 3}], v{V_XR} offset:{1024 * j}')
            e(f'  s_mov_b64 exec, {lo}')
            for j in range(2):
                e(f'  ds_read_b128 v[{G1x + 4 * j}:{G1x + 4 * j + 3}], v{V_XR} offset:{1024 * j}')
            e('  s_mov_b64 exec, -1')
            e('  s_waitcnt lgkmcnt(0)')
            return
        for rr in sorted(paired):
            for G in (G0x, G1x):
                e(f'  v_lshl_add_u32 v{G + rr}, v{G + rr + 1}, 8, v{G + rr}')
        if paired:
            e('  s_nop 1')
        for rr in (swaps if "noswap" not in AB else []):
            e(f'  v_permlane32_swap_b32_e32 v{G0x + rr}, v{G1x + rr}')
        e('  s_nop 1')

    def tile_cols(prod, m, s_of, creg):
        """(output column, register, pre-paired) of M-tile m in column order, after exchange()"""
        C = consumed(prod, m)
        paired, _ = plan(C)
        cp = compact((prod, m))
        out = []
        for rho in sorted(C):
            rr = (rho & 3) + 4 * (rho >> 3)
            if rho % 2 and rr - 1 in paired:
                continue                              # folded into rho - 1 before the exchange
            src = rho
            if cp:                                    # the pair of rr sits in rr / 2 of the same group
                src = (rr // 2 & 3) + 8 * (rr // 2 >> 2) + 4 * (rho >> 2 & 1)
            out.append((s_of(rho), creg(src), rho % 2 == 0 and rr in paired))
        return out

    def mtile_mfmas(prod, m, ks, nxt=None):
        """one M-tile, issued and then waited for (single accumulator set)"""
        issue_tile(prod, m, ks, G0, G1)
        if nxt is not None:
            prefetch(*nxt)
        exchange(G0, G1, tile=(prod, m))

    def col_reg(rho, G0x=G0, G1x=G1):
        """register of column rho (0..31) of the M-tile after the exchange"""
        rr = (rho & 3) + 4 * (rho >> 3)
        return f"v{(G1x if (rho >> 2) & 1 else G0x) + rr}"

    def run_tiles(tiles, consume, nxt, dbuf, after_issue0=None, setb=None):
        """all M-tiles of a product: consume(m, col_reg_of_the_tile) after each; dbuf: two accumulator sets,
        tile m+1's MFMAs issued before tile m's results are folded, so the matrix core works while the
        lane does (needs T[38..69] free); tile 0's first A tiles are prefetched by the caller"""
        if not dbuf:
            for m in range(5):
                mtile_mfmas(*tiles[m], nxt=tiles[m + 1] if m < 4 else nxt)
                consume(m, col_reg)
            return
        sets = ((G0, G1), setb or (GB0, GB1))
        issue_tile(*tiles[0], *sets[0])
        separated = False                        # >= 30 VALU instructions after this tile's last MFMA
        if after_issue0 is not None:             # independent VALU work while tile 0 runs
            work = capture(after_issue0)
            for ins in work:
                e(ins)
            separated = len(work) >= MARGIN
        for m in range(5):
            if m < 4:
                nxt_issue = capture(lambda: issue_tile(*tiles[m + 1], *sets[(m + 1) % 2], prefetched=False))
            else:
                nxt_issue = capture(lambda: prefetch(*nxt)) if nxt is not None else []
            ga, gb = sets[m % 2]
            # tiles after the first were issued inside the previous fold, whose last 40% has no MFMA
            exchange(ga, gb, waited=separated, tile=tuple(tiles[m][:2]))
            fold = capture(lambda: consume(m, lambda rho, ga=ga, gb=gb: col_reg(rho, ga, gb)))
            if "nointerleave" in AB:
                for ins in nxt_issue + fold:
                    e(ins)
                separated = False
                continue
            # the next tile's reads and MFMAs spread through this tile's fold: an in-order wave waiting to
            # issue its next MFMA issues nothing else, so the MFMAs go out between VALU instructions
            items, grp = [], []
            for ins in nxt_issue:
                grp.append(ins)
                if "v_mfma" in ins or "ds_read" in ins:
                    items.append(grp)
                    grp = []
            if grp:
                items.append(grp)
            room = len(fold) - MARGIN              # the MFMAs go before the last MARGIN instructions of the fold
            gap = max(1, room // (len(items) + 1)) if items else 0
            separated = items != [] and len(fold) - gap * len(items) >= MARGIN
            k = 0
            for i, ins in enumerate(fold):
                if items and k < len(items) and i % gap == 0:
                    for x in items[k]:
                        e(x)
                    k += 1
                e(ins)
            for grp in items[k:]:
                for x in grp:
                    e(x)

    class Chunks:
        """column sums -> 28-bit limbs.  Chunk t (bits [base + 28 t, +28)) sums its columns (x 2^sh) into its
        own accumulator (two, alternating), independent of the carry; its tail (+ carry, mask, carry out)
        is deferred into the next chunk's multiply-adds, so the carry chain never stalls the wave."""

        def __init__(self, base_bits, t0, t_last, outs, neg, inits=None, nocarry_last=False, px=False):
            self.base, self.t, self.t0, self.t_last, self.outs, self.neg = base_bits, t0, t0, t_last, outs, neg
            self.inits, self.nocarry_last, self.px = inits, nocarry_last, px
            self.pending = []
            self.fresh = True
            self.begun = False

        def acc(self):
            return CACC2[(self.t - self.t0) & 1]

        def emit(self, ins):
            e(ins)
            if self.pending:
                e(self.pending.pop(0))

        def addend0(self):
            """addend of a chunk's first multiply-add: the previous chunk's carry under CMERGE"""
            return CCARRY if CMERGE and self.t != self.t0 else "0"

        def start(self):
            if self.inits is not None and 0 <= self.t < len(self.inits):
                self.emit(f'  v_mad_u64_u32 {self.acc()}, vcc, {self.inits[self.t]}, 1, {self.addend0()}')
                self.fresh = False

        def close(self):
            for ins in self.pending:
                e(ins)
            a = self.acc()
            tail = []
            if self.t != self.t0 and not CMERGE:
                tail.append(f'  v_lshl_add_u64 {a}, {a}, 0, {CCARRY}')
            if 0 <= self.t < len(self.outs):
                if self.px:                              # q3 limbs leave pre-flipped (PREXOR)
                    tail.append(f'  v_bitop3_b32 {self.outs[self.t]}, v{a[2:a.index(":")]}, {SMASK}, '
                                f'{pat(self.t)} bitop3:0x6a')
                else:
                    tail.append(f'  v_and_b32_e32 {self.outs[self.t]}, {hex(MASK)}, v{a[2:a.index(":")]}')
            if not (self.nocarry_last and self.t == self.t_last):
                if CMERGE:                               # the next chunk's first multiply-add reads it
                    e(f'  v_ashrrev_i64 {CCARRY}, {B}, {a}')
                else:
                    tail.append(f'  v_ashrrev_i64 {CCARRY}, {B}, {a}')
            self.pending = tail
            self.t += 1
            self.fresh = True
            if self.t <= self.t_last:
                self.start()

        def column(self, s, reg):
            t = (8 * s - self.base) // B
            while t > self.t:
                self.close()
            if not self.begun:
                self.begun = True
                self.start()
            sh = 8 * s - self.base - B * t
            mul = NEG(sh) if self.neg else POW(sh)
            a = self.acc()
            self.emit(f'  v_mad_i64_i32 {a}, vcc, {reg}, {mul}, {self.addend0() if self.fresh else a}')
            self.fresh = False

        def finish(self):
            while self.t <= self.t_last:
                self.close()
            for ins in self.pending:
                e(ins)
            self.pending = []

    def fold_columns(ch, cols):
        """cols: [(s, reg, paired)] of one tile in column order (paired: reg already holds c_s + 256 c_(s+1),
        formed before the exchange).  Two adjacent unpaired columns of the same chunk whose shifts are sh
        and sh + 8 <= 24 are combined first, c_s + 256 c_(s+1) in 32-bit arithmetic (|c| < 2^21.2, so |sum| <
        2^29.3: exact), and enter the chunk as one v_mad_i64_i32: ~2 instead of 3.5 64-bit multiply-adds per
        28-bit chunk.  A pair whose second column lies in the next chunk enters this chunk at shift sh <= 24:
        its bits above 28 leave through the chunk's carry, exactly."""
        i = 0
        while i < len(cols):
            s_, r_, pr_ = cols[i]
            if not pr_ and i + 1 < len(cols) and "nopair" not in AB:
                s2_, r2_, pr2_ = cols[i + 1]
                t1, t2 = (8 * s_ - ch.base) // B, (8 * s2_ - ch.base) // B
                if not pr2_ and s2_ == s_ + 1 and t1 == t2 and 8 * s_ - ch.base - B * t1 <= 16:
                    e(f'  v_lshl_add_u32 {r_}, {r2_}, 8, {r_}')
                    ch.column(s_, r_)
                    i += 2
                    continue
            ch.column(s_, r_)
            i += 1

    P1_TILES = [(1, m, [k for k in range(5) if m - k <= 1]) for m in range(5)]
    P2_TILES = [(2, m, [k for k in range(5) if m >= k]) for m in range(5)]
    assert P1_TILES[0][2][0] != 4 and P2_TILES[0][2][0] != 4      # LDSX: see swap_operands

    def mfma_barrett(Tl, q3out, clamp, prefetched=False, dbuf=False, setb=None, pre_in=None):
        """product 1: q3 = Barrett's quotient of T (Tl: 2K limbs, Tl[K-1] < 2^29 allowed) -> q3out (K regs,
        may be Tl[K:]); clamp: q3 = -1 (q1 = 0) -> 0; prefetched: its first A-tile reads are in flight;
        dbuf: double-buffered accumulators (T[38..69] free); pre_in: Tl[K..2K-1] arrive pre-flipped
        (PREXOR, default); q3out leaves pre-flipped under PREXOR"""
        if pre_in is None:
            pre_in = PREXOR
        if not prefetched:
            prefetch(*P1_TILES[0])
        orpack(Tl[K - 1:2 * K], 0, 34, [0x80808080] * 34, norm0=True, pre=range(1, K + 1) if pre_in else ())
        e(f'  v_bfe_u32 {D[34]}, {Tl[K - 1]}, 28, 1')              # c = bit 28 of q1[0] -> digit 16 c at byte 137
        e(f'  v_lshl_or_b32 {D[34]}, {D[34]}, 12, 1')               # and the constant digit 1 at byte 136
        for w in range(35, 40):
            e(f'  v_mov_b32_e32 {D[w]}, 0')
        swap_operands()
        ch = Chunks(QBIT, (8 * S1_LO - QBIT) // B, 39, q3out, neg=False, px=PREXOR)

        def consume(m, creg):
            fold_columns(ch, tile_cols(1, m, lambda rho: S1_LO + 32 * m + rho, creg))
        run_tiles(P1_TILES, consume, P2_TILES[0], dbuf, setb=setb)
        ch.finish()
        if clamp:                                  # final carry = 0, or -1 when q1 = 0 (q3 = -1 -> 0)
            e(f'  v_not_b32_e32 v{XA + 36}, v{XA + 38}')
            for t, r in enumerate(q3out):
                if PREXOR:                         # ((r ^ pat) & m) ^ pat
                    e(f'  v_bitop3_b32 {r}, {r}, v{XA + 36}, {pat(t)} bitop3:0xe2')
                else:
                    e(f'  v_and_b32_e32 {r}, {r}, v{XA + 36}')
        return q3out

    def mfma_remainder(Tl, q3, rout, nxt_p1, dbuf=False, after_pack=None):
        """product 2: r = (T - q3 P) mod b^K -> rout (may be Tl[:K]); the product-2 tile-0 reads are already
        in flight; nxt_p1: prefetch product 1's first tiles at the end (the next Barrett); after_pack: the
        caller's last use of the q3 limbs (dbuf may then take their registers)"""
        orpack(q3, 8, 33, [0x80808000] + [0x80808080] * 32, lead_one=True, pre=range(K) if PREXOR else ())
        if after_pack and not dbuf:
            after_pack()
        e(f'  v_mov_b32_e32 {D[33]}, 0x80')          # q3 byte 131 (zero, offset) at byte 132; pads 0
        for w in range(34, 40):
            e(f'  v_mov_b32_e32 {D[w]}, 0')
        swap_operands()
        # matrix column s holds column s - 1 of q3 P (bits 8 s - 8): P'[s - i] is a plain Toeplitz band
        ch = Chunks(8, 0, K - 1, rout, neg=True, inits=Tl[:K], nocarry_last=True)

        def consume(m, creg):
            fold_columns(ch, tile_cols(2, m, lambda rho: 32 * m + rho, creg))
        # dbuf: the caller's last use of q3 runs while tile 0 (first accumulator set) is in the matrix core;
        # the second set (q3's registers) is first written by tile 1
        run_tiles(P2_TILES, consume, P1_TILES[0] if nxt_p1 else None, dbuf,
                  after_issue0=after_pack if dbuf else None)
        ch.finish()

    # ---- prologue ------------------------------------------------------------
    e('.amdgcn_target "amdgcn-amd-amdhsa--gfx950"')
    e('.amdhsa_code_object_version 5')
    e('.text')
    e(f'.globl {name}')
    e('.p2align 8')
    e(f'.type {name},@function')
    e(f'{name}:')
    # DYN: persistent waves with dynamic jobs -- the launch holds at most the resident workgroups; job j = the
    # lanes [64 j, 64 j + 64); a wave's first job is 4 wg + wave (the static mapping), the next ones come from a
    # device counter (kernarg rows[14], zeroed by the launcher) offset by the waves launched (kernarg 0x24), so
    # a wave the SIMD's arbiter favours runs more jobs and the launch has no workgroup-granular tail
    DYN = "dyn" in AB and not PP
    STAMP = "stamp" in AB                        # timing build: each wave's start / end realtime (100 MHz) and
    if STAMP:                                    # where it ran, 16 B at kernarg rows[15] + 16 (4 wg + wave)
        e('  s_memrealtime s[80:81]')
        e('  s_mov_b32 s85, s2')
    e('  s_load_dwordx2 s[4:5], s[0:1], 0x0')
    e('  s_load_dwordx2 s[6:7], s[0:1], 0x8')
    e('  s_load_dwordx2 s[8:9], s[0:1], 0x10')
    e('  s_load_dwordx2 s[10:11], s[0:1], 0x18')
    if DYN:
        e('  s_load_dwordx2 s[92:93], s[0:1], 0x20')                  # live lanes, waves launched
        e('  s_load_dwordx2 s[94:95], s[0:1], 0x98')                  # job counter
    e('  s_waitcnt lgkmcnt(0)')
    if DYN:
        e('  s_mov_b64 s[90:91], s[6:7]')                             # the program's first op
        e('  s_add_u32 s92, s92, 63')
        e('  s_lshr_b32 s92, s92, 6')                                 # jobs
    off, sreg, rem = 0, SNP, K
    for width in (16, 8, 4, 2, 1):
        while rem >= width:
            suffix = f"x{width}" if width > 1 else ""
            dst = f"s[{sreg}:{sreg + width - 1}]" if width > 1 else f"s{sreg}"
            e(f'  s_load_dword{suffix} {dst}, s[8:9], {hex(off)}')
            off += 4 * width
            sreg += width
            rem -= width
    for i in range(8):
        e(f'  s_mov_b32 s{SPOW + i}, {hex(1 << (4 * i))}')
    for i in range(7):
        e(f'  s_mov_b32 s{SNEG + i}, {hex((-(1 << (4 * i))) & 0xFFFFFFFF)}')
    e(f'  s_mov_b32 s35, {hex(MASK)}')
    if KARA:
        for r_, m_ in ((S2MASK, 2), (S3MASK, 3), (S4MASK, 4)):
            e(f'  s_mov_b32 {r_}, {hex(m_ * MASK)}')
    if PREXOR:
        for v_, val in zip(PATV, PATVAL):
            e(f'  v_mov_b32_e32 v{v_}, {hex(val)}')
    # PP (ping-pong): 512-thread workgroups, the two waves of a SIMD are waves w and w + 4 of one workgroup;
    # half 1 runs one phase behind half 0 (s_barrier between the products and the reduction of every
    # SQR / MUL / LOADP), so one wave's matrix phases meet the other wave's product phase
    e(f'  s_lshl_b32 s14, s2, {11 if PP else 10}')
    if PP:
        e(f'  v_readfirstlane_b32 s18, v{V_TID}')
        if "ppodd" in AB:                          # s18 = half (odd waves: 1)
            e('  s_bfe_u32 s18, s18, 0x10006')
        else:                                      # s18 = half (waves 0-3: 0, waves 4-7: 1)
            e('  s_lshr_b32 s18, s18, 8')
    e(f'  v_lshlrev_b32_e32 v{V_GOFF}, 2, v{V_TID}')
    e(f'  v_add_u32_e32 v{V_GOFF}, s14, v{V_GOFF}')
    # LDS tile image: 5 x 4 KB, each thread one dwordx4 per 4 KB
    if PP:                                       # threads t and t + 256 write the same image words
        e(f'  v_and_b32_e32 v10, 0xff, v{V_TID}')
        e('  v_lshlrev_b32_e32 v10, 4, v10')
    else:
        e(f'  v_lshlrev_b32_e32 v10, 4, v{V_TID}')
    for it in range(TILE_BYTES // 4096):
        e(f'  global_load_dwordx4 v[2:5], v10, s[8:9] offset:{TILE_OFF}')
        e('  s_waitcnt vmcnt(0)')
        e('  ds_write_b128 v10, v[2:5]')
        if it != TILE_BYTES // 4096 - 1:
            e('  v_add_u32_e32 v10, 0x1000, v10')
    e(f'  v_and_b32_e32 v{V_LDS}, 63, v{V_TID}')
    e(f'  v_lshlrev_b32_e32 v{V_LDS}, 4, v{V_LDS}')
    if SPILL:
        e(f'  v_lshrrev_b32_e32 v{V_SPILL}, 6, v{V_TID}')             # wave in the workgroup
        e(f'  v_mul_u32_u24_e32 v{V_SPILL}, {hex(SPILL_BYTES)}, v{V_SPILL}')
        e(f'  v_add_u32_e32 v{V_SPILL}, {hex(TILE_BYTES)}, v{V_SPILL}')
        e(f'  v_add_u32_e32 v{V_SPILL}, v{V_SPILL}, v{V_LDS}')
    if LDSX:
        e(f'  v_lshrrev_b32_e32 v{V_XW}, 6, v{V_TID}')                # wave in the workgroup
        e(f'  v_mul_u32_u24_e32 v{V_XW}, {hex(LDSX_BYTES)}, v{V_XW}')
        e(f'  v_add_u32_e32 v{V_XW}, {hex(TILE_BYTES)}, v{V_XW}')
        e(f'  v_add_u32_e32 v{V_XW}, v{V_XW}, v{V_LDS}')
        e(f'  v_xor_b32_e32 v{V_XR}, 0x200, v{V_XW}')                # lane ^ 32
        e(f'  s_mov_b32 s{SLO}, -1')
        e(f'  s_mov_b32 s{SLO + 1}, 0')
        e(f'  s_mov_b32 s{SHI}, 0')
        e(f'  s_mov_b32 s{SHI + 1}, -1')
    e('  s_waitcnt lgkmcnt(0)')
    e('  s_barrier')
    if PP:
        e('  s_cmp_eq_u32 s18, 1')                  # half 1: one barrier ahead = one phase behind
        e('  s_cbranch_scc0 .Lpp_start')
        e('  s_barrier')
        e('.Lpp_start:')
    elif "nodesync" not in AB:
        # odd workgroups start ~8K cycles late: the two waves of a SIMD then reach their matrix-core
        # phases at different times (s_sleep spends no issue slots); 1.5% (profiles/r02zt_desync_ab.jsonl)
        e('  s_bitcmp1_b32 s2, 0')
        e('  s_cbranch_scc0 .Ldesync_done')
        nsl = int(os.environ.get("FTHE_GEN_M37_SLEEPS", "1"))
        for _ in range(nsl):
            e('  s_sleep 127')
        e('.Ldesync_done:')

    e('.Lprog:')
    e('  s_load_dwordx2 s[14:15], s[6:7], 0x0')
    e('  s_add_u32 s6, s6, 8')
    e('  s_addc_u32 s7, s7, 0')
    e('  s_waitcnt lgkmcnt(0)')
    for code, lab in ((1, '.Lloadx'), (2, '.Lstorex'), (3, '.Lsqr'), (4, '.Lmul'), (22, '.Lloadp'), (23, '.Lstorep')):
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

    e('.Lloadx:')
    load_limbs(X0 + X1)
    e('  s_branch .Lprog')
    e('.Lstorex:')
    store_limbs(X0 + X1)
    e('  s_branch .Lprog')

    def kara_cross():
        """V = 2 x0 x1 (74 limbs, the upper 37 pre-XORed) by one level of Karatsuba; returns the ripple of the
        final carry through V[57..73] as independent instructions for x0^2's column pass.  Halves: x = xL + xH
        b^19, xL = limbs 0..18, xH = limbs 19..36.  Temporaries in T (free until x0^2): S0 = x0L + x0H (T[0..17],
        S0_18 = x0_18), S1 = 2 (x1L + x1H) (T[18..36]), C = limbs 19..37 of 2 P0 (T[37..55]); the middle
        columns' addends in v2 / v4 over permanently zero v3 / v5.
          1. 2 P0 = 2 x0L x1L: limbs 0..18 -> V[0..18], 19..37 -> C (limb 37 < 2^29, unmasked);
          2. 2 P2 = 2 x0H x1H: limbs 0..35 -> V[38..73] as mask - limb (complemented);
          3. column k = 0..37 of S0 S1 (at most 2^63.1: unsigned) plus t'_k = L_k - P0_k - P2_k + 3 mask, where
             L_k is the limb of 2 P0 + 2 P2 b^38 at position k + 19 and P0_k, P2_k the limbs subtracted (t'_k in
             [0, 2^30): the first multiply-add's addend), plus the carry, which starts at 3: with t' biased by
             3 mask = 3 (2^28 - 1) every column value is the true one plus 3 2^28 >= 0 (the true one >= -2^29 - 2),
             so its limb is exact and its carry the true one plus 3; limb -> V[k + 19];
          4. V[57..73] += the final carry (>= 0, minus the bias 3), complemented limbs restored."""
        S0 = T[:18] + [X0[18]]
        S1 = T[18:37]
        C = T[37:56]
        TPL, TPH = ("v2", "v4"), ("v3", "v5")
        bg = []
        for i in range(18):
            bg.append(f'  v_add_u32_e32 {S0[i]}, {X0[i]}, {X0[19 + i]}')
            bg.append(f'  v_add_lshl_u32 {S1[i]}, {X1[i]}, {X1[19 + i]}, 1')
        bg.append(f'  v_lshlrev_b32_e32 {S1[18]}, 1, {X1[18]}')
        bg += [f'  v_mov_b32_e32 {h}, 0' for h in TPH]
        cols = []
        for c in range(38):                                     # 2 P0
            terms = [(X0[i], X1[c - i]) for i in range(19) if 0 <= c - i < 19]
            cols.append({'terms': terms, 'dbl': True, 'out': V[c] if c < 19 else C[c - 19], 'last': c == 37})
        columns(cols, bg=bg)
        cols = []
        for c in range(36):                                     # 2 P2, complemented
            terms = [(X0[19 + i], X1[19 + c - i]) for i in range(18) if 0 <= c - i < 18]
            cols.append({'terms': terms, 'dbl': True, 'out': V[38 + c], 'cpl': True, 'last': c == 35})
        columns(cols)
        e(f'  v_mov_b64_e32 {carry}, 3')
        cols = []
        for k in range(38):                                     # middle columns at b^19
            tl = TPL[k % 2]
            if k <= 18:                                         # C_k - P0_k + (mask - P2_k) + 2 mask
                pre = [f'  v_sub_u32_e32 {tl}, {C[k]}, {V[k]}',
                       f'  v_add3_u32 {tl}, {tl}, {V[38 + k]}, {S2MASK}']
            elif k <= 35:                                       # P2c_k - P2c_(k-19) - C_(k-19) + 3 mask
                pre = [f'  v_sub_u32_e32 {tl}, {V[38 + k]}, {V[k + 19]}',
                       f'  v_sub_u32_e32 {tl}, {tl}, {C[k - 19]}',
                       f'  v_add_u32_e32 {tl}, {S3MASK}, {tl}']
            else:                                               # P2_36 = P2_37 = 0: 4 mask - P2c - C
                pre = [f'  v_sub_u32_e32 {tl}, {S4MASK}, {V[k + 19]}',
                       f'  v_sub_u32_e32 {tl}, {tl}, {C[k - 19]}']
            terms = [(S0[i], S1[k - i]) for i in range(19) if 0 <= k - i < 19]
            col = {'terms': terms, 'out': V[k + 19], 'addend': f'v[{tl[1:]}:{int(tl[1:]) + 1}]', 'pre': pre}
            if PREXOR and k + 19 >= K:
                col['px'] = pat(k + 19 - (K - 1))
            cols.append(col)
        columns(cols, carry_in=True)
        # 4. ripple: v = (mask ^ P2c_19) + carry - 3, then limb / carry through V[73] (v2 value, v3 carry)
        e(f'  v_xad_u32 v2, {V[57]}, {SMASK}, v{CARRY}')
        rip = ['  v_add_u32_e32 v2, -3, v2']
        for j in range(57, 2 * K):
            px = pat(j - (K - 1)) if PREXOR else None
            if j == 2 * K - 1:
                rip.append(f'  v_xor_b32_e32 {V[j]}, {px}, v2' if px else f'  v_mov_b32_e32 {V[j]}, v2')
                break
            rip.append(f'  v_bitop3_b32 {V[j]}, v2, {SMASK}, {px} bitop3:0x6a' if px
                       else f'  v_and_b32_e32 {V[j]}, {hex(MASK)}, v2')
            rip.append('  v_lshrrev_b32_e32 v3, 28, v2')
            rip.append(f'  v_xad_u32 v2, {V[j + 1]}, {SMASK}, v3')
        return rip

    # SQR: V = 2 x0 x1, T = x0^2, reduce
    e('.Lsqr:')
    e('  s_mov_b32 s19, s15')
    e('.Lsqr_loop:')
    e('  s_cmp_eq_u32 s19, 0')
    e('  s_cbranch_scc1 .Lprog')
    rip = []
    if KARA:
        rip = kara_cross()
    else:
        cols = []
        for c in range(2 * K):
            terms = [(X0[i], X1[c - i]) for i in range(K) if 0 <= c - i < K]
            cols.append({'terms': terms, 'dbl': True, 'out': V[c], 'last': c == 2 * K - 1})
            if PREXOR and c >= K:
                cols[-1]['px'] = pat(c - (K - 1))
        columns(cols)
    cols = []
    for c in range(2 * K):
        terms = [(X0[i], X0[c - i]) for i in range(K) if i < c - i < K]
        sq = X0[c // 2] if c % 2 == 0 and c // 2 < K else None
        col = {'terms': terms, 'out': T[c], 'last': c == 2 * K - 1}
        if PREXOR and c >= K:
            col['px'] = pat(c - (K - 1))
        if terms:
            col['dbl'] = True
            if sq:
                col['sq'] = sq
        elif sq:
            col['terms'] = [(sq, sq)]
        cols.append(col)
    columns(cols, bg=rip)
    phase()
    call('.Lreduce')
    phase()
    e('  s_sub_u32 s19, s19, 1')
    e('  s_branch .Lsqr_loop')

    # MUL slot: y0 -> T[0..K-1], y1 -> T[K..]; W = x0 y1 + x1 y0 -> V; T = x0 y0 -> (XB, T[K..]); move
    e('.Lmul:')
    Y0, Y1 = T[:K], T[K:]
    load_limbs(Y0 + Y1)
    columns(product_cols(X0, Y1, 2 * K, V, a2=X1, b2=Y0))
    TM = X1 + T[K:]                              # x1, y1 dead
    columns(product_cols(X0, Y0, 2 * K, TM))
    move(T[:K], X1)
    phase()
    call('.Lreduce')
    phase()
    e('  s_branch .Lprog')

    # LOADP slot: plain X -> T -> (q3 = x1, r = x0)
    e('.Lloadp:')
    load_limbs(T)
    phase()
    q3 = mfma_barrett(T, T[K:], clamp=True, pre_in=False)
    mfma_remainder(T, q3, T[:K], nxt_p1=False)
    phase()
    move(X0, T[:K])
    if PREXOR:
        for i in range(K):
            e(f'  v_xor_b32_e32 {X1[i]}, {pat(i)}, {T[K + i]}')
    else:
        move(X1, T[K:2 * K])
    e('  s_branch .Lprog')

    # STOREP slot: x0 + x1 P with -P in SGPRs (scratch -x1 in T[0..K-1]; out V)
    e('.Lstorep:')
    NX1 = T[:K]
    for i in range(K):
        e(f'  v_sub_u32_e32 {NX1[i]}, 0, {X1[i]}')
    cols = []
    for c in range(2 * K):
        terms = [(X0[c], '1')] if c < K else []
        terms += [(NX1[i], NP(c - i)) for i in range(K) if 0 <= c - i < K]
        cols.append({'terms': terms, 'out': V[c], 'last': c == 2 * K - 1})
    columns(cols, signed=True)
    store_limbs(V)
    e('  s_branch .Lprog')

    e('.Lend:')
    if DYN:
        e('  s_mov_b64 exec, 1')
        e('  v_mov_b32_e32 v2, 0')
        e('  v_mov_b32_e32 v3, 1')
        e('  global_atomic_add v4, v2, v3, s[94:95] sc0')
        e('  s_waitcnt vmcnt(0)')
        e('  s_mov_b64 exec, -1')
        e('  v_readfirstlane_b32 s96, v4')
        e('  s_add_u32 s96, s96, s93')                                # job = waves launched + draw
        e('  s_cmp_ge_u32 s96, s92')
        e('  s_cbranch_scc1 .Ljobs_done')
        e('  s_lshl_b32 s96, s96, 8')
        e(f'  v_and_b32_e32 v2, 63, v{V_TID}')
        e('  v_lshlrev_b32_e32 v2, 2, v2')
        e(f'  v_add_u32_e32 v{V_GOFF}, s96, v2')
        e('  s_mov_b64 s[6:7], s[90:91]')
        e('  s_branch .Lprog')
        e('.Ljobs_done:')
    if PP:                                       # half 0 pays back half 1's extra barrier
        e('  s_cmp_eq_u32 s18, 0')
        e('  s_cbranch_scc0 .Lpp_end')
        e('  s_barrier')
        e('.Lpp_end:')
    if STAMP:
        e('  s_waitcnt vmcnt(0)')
        e('  s_memrealtime s[82:83]')
        e('  s_getreg_b32 s84, hwreg(HW_REG_HW_ID)')
        e('  s_getreg_b32 s86, hwreg(HW_REG_XCC_ID)')
        e('  s_load_dwordx2 s[88:89], s[0:1], 0xa0')
        e('  s_waitcnt lgkmcnt(0)')
        e('  s_cmp_eq_u64 s[88:89], 0')
        e('  s_cbranch_scc1 .Lstamp_done')
        e('  s_mov_b64 exec, 1')
        e(f'  v_lshrrev_b32_e32 v2, 6, v{V_TID}')
        e(f'  v_lshl_add_u32 v2, s85, {3 if PP else 2}, v2')             # wave index in the launch
        e('  v_lshlrev_b32_e32 v7, 4, v2')
        e('  v_mov_b32_e32 v2, s80')
        e('  v_mov_b32_e32 v3, s82')
        e('  v_mov_b32_e32 v4, s84')
        e('  v_mov_b32_e32 v5, s86')
        e('  global_store_dwordx4 v7, v[2:5], s[88:89]')
        e('  s_waitcnt vmcnt(0)')
        e('.Lstamp_done:')
    e('  s_endpgm')

    # reduce (SQR, MUL): T (x0^2 or x0 y0), V (cross terms) -> x0 = T mod P, x1 = (V + T div P) mod P
    e('.Lreduce:')
    # default s_setprio 3 over the reduction (noprio: none): -0.5..1% (profiles/r03s_m37_prio_ab.jsonl)
    PRIO = next((int(t[4:]) for t in AB.split(',') if t.startswith('prio') and t[4:].isdigit()),
                0 if "noprio" in AB else 3)
    if PRIO:
        e(f'  s_setprio {PRIO}')                # the latency-bound matrix phases win the SIMD's VALU issue
    dbuf = "nodbuf" not in AB
    spill = dbuf and SPILL
    if spill:
        # V[37..73] waits in LDS while Barrett 1 runs, so its product 1 gets a second accumulator set too
        for j in range(9):
            e(f'  ds_write_b128 v{V_SPILL}, v[{VV + 38 + 4 * j}:{VV + 41 + 4 * j}] offset:{1024 * j}')
        e(f'  ds_write_b32 v{V_SPILL}, {V[K]} offset:{9 * 1024}')
    q3 = mfma_barrett(T, T[K:], clamp=True, dbuf=spill, setb=(GV0, GV1))    # u1 -> T[K..2K-1]

    def add_u1():
        for i in range(K):
            if PREXOR:                                      # V += u1 ^ pat (u1 arrives pre-flipped)
                e(f'  v_xad_u32 {V[i]}, {q3[i]}, {pat(i)}, {V[i]}')
            else:
                e(f'  v_add_u32_e32 {V[i]}, {V[i]}, {q3[i]}')  # V += u1 (limbs < 2^29); u1 dies here
        if spill:                                           # V[37..73] back (older than every tile read)
            for j in range(9):
                e(f'  ds_read_b128 v[{VV + 38 + 4 * j}:{VV + 41 + 4 * j}], v{V_SPILL} offset:{1024 * j}')
            e(f'  ds_read_b32 {V[K]}, v{V_SPILL} offset:{9 * 1024}')
    mfma_remainder(T, q3, T[:K], nxt_p1=True, dbuf=dbuf, after_pack=add_u1)      # u0 -> T[0..K-1]
    q3b = mfma_barrett(V, V[K:], clamp=False, prefetched=True, dbuf=dbuf)        # T[K..] is free
    mfma_remainder(V, q3b, V[:K], nxt_p1=False, dbuf=dbuf)
    move(X0, T[:K])
    move(X1, V[:K])
    if PRIO:
        e('  s_setprio 0')
    e('  s_setpc_b64 s[12:13]')

    e(f'.Lfunc_end_{name}:')
    e(f'  .size {name}, .Lfunc_end_{name}-{name}')
    e('')
    o.extend(_descriptor(name, LDS_BYTES, NVGPR, 98 if DYN else 90 if STAMP else NSGPR,
                         max_wg=512 if PP else 256).splitlines())
    return "\n".join(o) + "\n"


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--name', default='fthe_padic_m37')
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args()
    with open(a.out, 'w') as f:
        f.write(gen_padic_mfma(a.name))
