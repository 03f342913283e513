#!/usr/bin/env python3
"""Emulator of one quad (lanes 0..3 of wave 0, workgroup 0) for the instruction subset of the n-adic
four-lane kernel (fedtree_amd/csrc/gen_nadic.py): per-lane VGPRs, EXEC / VCC lane masks, DPP
quad_perm, LDS, the f64 quotient estimate (exact fma) -- to check register allocation, ring
relabelling, hand-offs and control flow on the CPU before the kernel runs on the GPU.

  python tools/quad_emu.py      (self-test: r^e (1 + m n) mod n^2 through the kernel vs pow())
"""
import random
import re
import struct
import sys
from fractions import Fraction

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1
NL = 4                                       # lanes emulated


def s32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def f2b(x):
    return struct.unpack('<Q', struct.pack('<d', x))[0]


def b2f(b):
    return struct.unpack('<d', struct.pack('<Q', b & M64))[0]


class QuadEmu:
    def __init__(self, asm_text, lds_bytes):
        self.lines, self.labels = [], {}
        for raw in asm_text.splitlines():
            line = raw.split('//')[0].rstrip()
            s = line.strip()
            if not s:
                continue
            if s.startswith('.amdhsa_kernel') or s.startswith('.rodata'):
                break
            if s.endswith(':'):
                self.labels[s[:-1]] = len(self.lines)
                continue
            if s.startswith('.'):
                continue
            self.lines.append(s)
        self.v = [dict() for _ in range(NL)]
        self.s = {}
        self.mem = {}
        self.lds = {}
        self.lds_bytes = lds_bytes
        self.exec = (1 << NL) - 1
        self.vcc = 0
        self.scc = 0
        self.count = {}

    # ---- operands ------------------------------------------------------------
    @staticmethod
    def rr(tok):
        m = re.fullmatch(r'([vs])\[(\d+):(\d+)\]', tok)
        if m:
            return m.group(1), int(m.group(2)), int(m.group(3)) - int(m.group(2)) + 1
        m = re.fullmatch(r'([vs])(\d+)', tok)
        if m:
            return m.group(1), int(m.group(2)), 1
        return None

    def sread(self, tok):
        if tok == 'vcc':
            return self.vcc
        if tok == 'exec':
            return self.exec
        r = self.rr(tok)
        if r is None:
            return int(tok, 0) & M64
        kind, b, n = r
        assert kind == 's', tok
        out = 0
        for i in range(n):
            out |= (self.s.get(b + i, 0) & M32) << (32 * i)
        return out

    def swrite(self, tok, val):
        if tok == 'exec':
            self.exec = val & ((1 << NL) - 1)
            return
        if tok == 'vcc':
            self.vcc = val & ((1 << NL) - 1)
            return
        kind, b, n = self.rr(tok)
        assert kind == 's'
        for i in range(n):
            self.s[b + i] = (val >> (32 * i)) & M32

    def lane_mask(self, tok):
        """a 64-bit SGPR pair / vcc used as a lane mask -> bits of lanes 0..3"""
        return self.sread(tok) & ((1 << NL) - 1)

    def vread(self, lane, tok, width=1):
        r = self.rr(tok)
        if r is None:
            val = int(tok, 0)
            return val & (M32 if width == 1 else M64)
        kind, b, n = r
        if kind == 's':
            v = self.sread(tok)
            return v
        f = self.v[lane]
        out = 0
        for i in range(n):
            out |= (f.get(b + i, 0) & M32) << (32 * i)
        return out

    def vwrite(self, lane, tok, val):
        kind, b, n = self.rr(tok)
        assert kind == 'v', tok
        for i in range(n):
            self.v[lane][b + i] = (val >> (32 * i)) & M32

    def active(self):
        return [ln for ln in range(NL) if self.exec >> ln & 1]

    def label_value(self, expr):
        m = re.fullmatch(r'(\.L\w+)-(\.L\w+)', expr)
        if m:
            return (self.labels[m.group(1)] - self.labels[m.group(2)]) * 8
        return int(expr, 0)

    # ---- execution --------------------------------------------------------------
    def run(self, entry, max_steps=200_000_000):
        pc = self.labels[entry]
        steps = 0
        while True:
            steps += 1
            if steps > max_steps:
                raise RuntimeError('step limit')
            ins = self.lines[pc]
            pc += 1
            op, _, rest = ins.partition(' ')
            args = [a.strip() for a in rest.split(',')] if rest else []
            self.count[op] = self.count.get(op, 0) + 1
            if op == 's_endpgm':
                return
            if op in ('s_waitcnt', 's_nop'):
                continue
            if op == 's_branch':
                pc = self.labels[args[0]]
                continue
            if op in ('s_cbranch_scc1', 's_cbranch_scc0'):
                if self.scc == (1 if op.endswith('1') else 0):
                    pc = self.labels[args[0]]
                continue
            if op == 's_cbranch_vccz':
                if self.vcc == 0:
                    pc = self.labels[args[0]]
                continue
            if op.startswith('s_load_dword'):
                dst, base, off = args
                _, b0, n = self.rr(dst)
                addr = self.sread(base) + (self.sread(off) if off.startswith('s') else int(off, 0))
                for i in range(n):
                    self.s[b0 + i] = self.mem.get(addr + 4 * i, 0)
                continue
            if op == 's_add_u32':
                a = self.sread(args[1]) & M32
                b = (self.label_value(args[2]) if args[2].startswith('.L') else self.sread(args[2])) & M32
                r = a + b
                self.scc = r >> 32
                self.swrite(args[0], r & M32)
                continue
            if op == 's_addc_u32':
                r = (self.sread(args[1]) & M32) + (self.sread(args[2]) & M32) + self.scc
                self.scc = r >> 32
                self.swrite(args[0], r & M32)
                continue
            if op == 's_sub_u32':
                a, b = self.sread(args[1]) & M32, self.sread(args[2]) & M32
                self.scc = 1 if b > a else 0
                self.swrite(args[0], (a - b) & M32)
                continue
            if op == 's_mul_i32':
                self.swrite(args[0], (self.sread(args[1]) * self.sread(args[2])) & M32)
                continue
            if op == 's_mul_hi_u32':
                self.swrite(args[0], ((self.sread(args[1]) & M32) * (self.sread(args[2]) & M32)) >> 32)
                continue
            if op in ('s_mov_b32', 's_mov_b64'):
                val = self.sread(args[1])
                if args[1] == '-1':
                    val = M64
                self.swrite(args[0], val)
                continue
            if op == 's_lshl_b32':
                r = (self.sread(args[1]) << self.sread(args[2])) & M32
                self.scc = int(r != 0)
                self.swrite(args[0], r)
                continue
            if op == 's_lshr_b32':
                r = (self.sread(args[1]) & M32) >> (self.sread(args[2]) & 31)
                self.scc = int(r != 0)
                self.swrite(args[0], r)
                continue
            if op in ('global_load_ubyte', 'global_load_ushort'):
                dst, voff, sbase = args
                for ln in self.active():
                    addr = self.sread(sbase) + (self.vread(ln, voff) & M32)
                    w = self.mem.get(addr & ~3, 0) >> (8 * (addr & 3))
                    self.vwrite(ln, dst, w & (0xff if op.endswith('ubyte') else 0xffff))
                continue
            if op == 'global_load_dwordx4':
                dst, vaddr = args[0], args[1]
                m = re.search(r'offset:(\d+)', ins)
                off = int(m.group(1)) if m else 0
                _, b0, n = self.rr(dst)
                for ln in self.active():
                    addr = self.vread(ln, vaddr, 2) + off
                    assert addr % 16 == 0, addr
                    for i in range(n):
                        self.v[ln][b0 + i] = self.mem.get(addr + 4 * i, 0)
                continue
            if op == 'global_load_dword' and args[2].split()[0] == 'off':
                dst, vaddr = args[0], args[1]
                m = re.search(r'offset:(\d+)', ins)
                off = int(m.group(1)) if m else 0
                for ln in self.active():
                    addr = self.vread(ln, vaddr, 2) + off
                    assert addr % 4 == 0
                    self.vwrite(ln, dst, self.mem.get(addr, 0))
                continue
            if op == 's_cmp_eq_u32':
                self.scc = int((self.sread(args[0]) & M32) == (self.sread(args[1]) & M32))
                continue
            if op == 's_cmp_lg_u32':
                self.scc = int((self.sread(args[0]) & M32) != (self.sread(args[1]) & M32))
                continue
            # ---- vector (per active lane) ----
            if op == 'v_and_b32_dpp':                 # dst = dpp(src0) & src1
                m = re.search(r'quad_perm:\[(\d),(\d),(\d),(\d)\]', ins)
                perm = [int(m.group(i)) for i in range(1, 5)]
                dst, src, msk = args[0], args[1], args[2].split()[0]
                vals = [self.vread(ln, src) for ln in range(NL)]
                for ln in self.active():
                    q = ln & ~3
                    self.vwrite(ln, dst, vals[q + perm[ln & 3]] & self.vread(ln, msk))
                continue
            if op == 'v_mov_b32_dpp':
                m = re.search(r'quad_perm:\[(\d),(\d),(\d),(\d)\]', ins)
                perm = [int(m.group(i)) for i in range(1, 5)]
                dst, src = args[0], args[1].split()[0]
                vals = [self.vread(ln, src) for ln in range(NL)]
                for ln in self.active():
                    q = ln & ~3
                    self.vwrite(ln, dst, vals[q + perm[ln & 3]])
                continue
            if op.startswith('v_cmp_'):
                cond = op.split('_')[2]
                a_, b_ = args[1], args[2]
                mask = 0
                for ln in self.active():
                    a, b = self.vread(ln, a_), self.vread(ln, b_)
                    if cond == 'ne':
                        t = a != b
                    elif cond == 'eq':
                        t = a == b
                    else:
                        raise NotImplementedError(ins)
                    mask |= int(t) << ln
                self.vcc = mask
                continue
            if op == 'ds_read_b32':
                dst, vaddr = args[0], args[1].split()[0]
                m = re.search(r'offset:(\d+)', ins)
                off = int(m.group(1)) if m else 0
                for ln in self.active():
                    addr = (self.vread(ln, vaddr) + off) & M32
                    val = self.lds.get(addr, 0) if addr + 4 <= self.lds_bytes else 0
                    self.vwrite(ln, dst, val)
                continue
            if op == 'ds_write_b32':
                vaddr, src = args[0], args[1].split()[0]
                m = re.search(r'offset:(\d+)', ins)
                off = int(m.group(1)) if m else 0
                for ln in self.active():
                    addr = (self.vread(ln, vaddr) + off) & M32
                    assert addr + 4 <= self.lds_bytes and addr % 4 == 0, addr
                    self.lds[addr] = self.vread(ln, src)
                continue
            if op in ('global_load_dword', 'global_store_dword'):
                if op == 'global_load_dword':
                    dst, voff, rest2 = args[0], args[1], args[2]
                else:
                    voff, src, rest2 = args[0], args[1], args[2]
                parts = rest2.split()
                sbase = parts[0]
                off = int(parts[1].split(':')[1]) if len(parts) > 1 else 0
                for ln in self.active():
                    addr = self.sread(sbase) + (self.vread(ln, voff) & M32) + off
                    assert addr % 4 == 0
                    if op == 'global_load_dword':
                        self.vwrite(ln, dst, self.mem.get(addr, 0))
                    else:
                        self.mem[addr] = self.vread(ln, src) & M32
                continue
            self.valu(op, args, ins)

    def valu(self, op, args, ins):
        lanes = self.active()
        newvcc = self.vcc
        for ln in lanes:
            R = lambda t, w=1: self.vread(ln, t, w)
            W = lambda t, x: self.vwrite(ln, t, x)
            if op == 'v_lshlrev_b32_e32':
                W(args[0], (R(args[2]) << (R(args[1]) & 31)) & M32)
            elif op == 'v_lshrrev_b32_e32':
                W(args[0], (R(args[2]) & M32) >> (R(args[1]) & 31))
            elif op == 'v_ashrrev_i32_e32':
                W(args[0], (s32(R(args[2])) >> (R(args[1]) & 31)) & M32)
            elif op == 'v_or_b32_e32':
                W(args[0], R(args[1]) | R(args[2]))
            elif op == 'v_and_b32_e32':
                W(args[0], R(args[1]) & R(args[2]))
            elif op == 'v_add_u32_e32':
                W(args[0], (R(args[1]) + R(args[2])) & M32)
            elif op == 'v_sub_u32_e32':
                W(args[0], (R(args[1]) - R(args[2])) & M32)
            elif op == 'v_subrev_u32_e32':
                W(args[0], (R(args[2]) - R(args[1])) & M32)
            elif op == 'v_mov_b32_e32':
                W(args[0], R(args[1]))
            elif op == 'v_mov_b64_e32':
                W(args[0], R(args[1], 2))
            elif op == 'v_mul_u32_u24_e32':
                W(args[0], ((R(args[1]) & 0xffffff) * (R(args[2]) & 0xffffff)) & M32)
            elif op == 'v_add_co_u32_e32':
                r = (R(args[2]) & M32) + (R(args[3]) & M32)
                W(args[0], r & M32)
                newvcc = (newvcc & ~(1 << ln)) | ((r >> 32) << ln)
            elif op == 'v_addc_co_u32_e32':
                r = (R(args[2]) & M32) + (R(args[3]) & M32) + (self.vcc >> ln & 1)
                W(args[0], r & M32)
                newvcc = (newvcc & ~(1 << ln)) | ((r >> 32) << ln)
            elif op == 'v_mul_lo_u32':
                W(args[0], (R(args[1]) * R(args[2])) & M32)
            elif op == 'v_lshl_add_u32':
                W(args[0], ((R(args[1]) << R(args[2])) + R(args[3])) & M32)
            elif op == 'v_bfe_u32':
                W(args[0], (R(args[1]) >> int(args[2])) & ((1 << int(args[3])) - 1))
            elif op in ('v_mad_u64_u32', 'v_mad_i64_i32'):
                dst, _, a, b, c = args
                va, vb = R(a) & M32, R(b) & M32
                vc = R(c, 2) & M64
                if op == 'v_mad_i64_i32':
                    va, vb = s32(va), s32(vb)
                    vc = vc - (1 << 64) if vc >> 63 else vc
                    full = va * vb + vc
                    ovf = not (-(1 << 63) <= full < (1 << 63))
                else:
                    full = va * vb + vc
                    ovf = full >> 64 != 0
                W(dst, full & M64)
                newvcc = (newvcc & ~(1 << ln)) | (int(ovf) << ln)
            elif op == 'v_lshl_add_u64':
                dst, a, sh, c = args
                W(dst, ((R(a, 2) << int(sh)) + R(c, 2)) & M64)
            elif op == 'v_lshrrev_b64':
                W(args[0], (R(args[2], 2) & M64) >> int(args[1]))
            elif op == 'v_lshlrev_b64':
                W(args[0], (R(args[2], 2) << int(args[1])) & M64)
            elif op == 'v_ashrrev_i64':
                x = R(args[2], 2) & M64
                if x >> 63:
                    x -= 1 << 64
                W(args[0], (x >> int(args[1])) & M64)
            elif op == 'v_cndmask_b32_e64':
                m = self.lane_mask(args[3])
                W(args[0], R(args[2]) if m >> ln & 1 else R(args[1]))
            elif op == 'v_cndmask_b32_e32':
                W(args[0], R(args[2]) if self.vcc >> ln & 1 else R(args[1]))
            elif op == 'v_cvt_f64_i32_e32':
                W(args[0], f2b(float(s32(R(args[1])))))
            elif op == 'v_cvt_f64_u32_e32':
                W(args[0], f2b(float(R(args[1]) & M32)))
            elif op == 'v_fma_f64':
                a, b, c = (b2f(R(t, 2)) for t in args[1:4])
                W(args[0], f2b(float(Fraction(a) * Fraction(b) + Fraction(c))))
            elif op == 'v_cvt_i32_f64_e32':
                x = b2f(R(args[1], 2))
                q = int(x)
                q = max(min(q, (1 << 31) - 1), -(1 << 31))
                W(args[0], q & M32)
            else:
                raise NotImplementedError(ins)
        self.vcc = newvcc


def pow_ops(e, tbl0, sq_slot, w, op):
    """bn_host.hpp Prog::pow as (op, arg) pairs (sliding window; not the all-ones chain)"""
    nb = e.bit_length()
    if nb == 1:
        return
    ntab = 1 << (w - 1)
    op(2, tbl0)
    op(3, 1)
    op(2, sq_slot)
    op(1, tbl0)
    for k in range(1, ntab):
        op(4, sq_slot)
        op(2, tbl0 + k)
    bit = lambda b: (e >> b) & 1

    def window(top):
        low = max(top - w + 1, 0)
        while not bit(low):
            low += 1
        val = 0
        for b in range(top, low - 1, -1):
            val = (val << 1) | bit(b)
        return low, val
    low, v = window(nb - 1)
    op(1, tbl0 + (v - 1) // 2)
    i = low - 1
    pend = 0
    while i >= 0:
        if not bit(i):
            pend += 1
            i -= 1
            continue
        low, v = window(i)
        pend += i - low + 1
        if pend:
            op(3, pend)
        op(4, tbl0 + (v - 1) // 2)
        pend = 0
        i = low - 1
    if pend:
        op(3, pend)


def selftest(trials=2, ebits=24, mont=False):
    """mont: the Montgomery form fthe_nadic_m76 (tools/nadic_mont_model.py) and its encrypt program
    LOADX, CANON, pow(e), MUL (1, m), MUL K (K = R^(e+1) mod n^2), CANON, STOREX"""
    sys.path.insert(0, 'fedtree_amd/csrc')
    sys.path.insert(0, 'tools')
    from gen_nadic import gen_nadic
    import nadic_model as nm
    S, B, SS = 76, 27, 152
    kname = 'fthe_nadic_m76' if mont else 'fthe_nadic_q76'
    asm = gen_nadic(S, B, kname, mont=mont)
    lds_bytes = 4 * 2 * S * 68
    rng = random.Random(11)
    for trial in range(trials):
        n = rng.getrandbits(2048) | (1 << 2047) | 1
        n2 = n * n
        em = QuadEmu(asm, lds_bytes)
        L = 256
        KA, CTX, PROG, SLOTS = 0x100, 0x1000, 0x2000, 0x100000
        for i, v in enumerate([SLOTS & M32, SLOTS >> 32, PROG, 0, CTX, 0, L * 4, SS * L * 4, L, 0]):
            em.mem[KA + 4 * i] = v
        k1, k2, k3, bias = nm.consts(n)
        ctxw = nm.limbs(n) + [(-pow(n, -1, 1 << B)) % (1 << B)]
        for d in (k1, k2, k3, bias):
            b_ = f2b(d)
            ctxw += [b_ & M32, b_ >> 32]
        for i, w in enumerate(ctxw):
            em.mem[CTX + 4 * i] = w
        r = n + rng.randrange(1, n) if trial == 0 else n - 1          # a raw r in [n, 2n): CANON
        r %= 1 << 2048
        m = rng.getrandbits(64)
        e = rng.getrandbits(ebits) | (1 << (ebits - 1))
        prog = []
        op = lambda o, a: prog.extend([o, a])
        op(1, 0)
        op(20, 0)
        pow_ops(e, 16, 9, 3, op)
        op(4, 3)
        if mont:
            op(4, 4)
        op(20, 0)
        op(2, 6)
        op(0, 0)
        for i, w_ in enumerate(prog):
            em.mem[PROG + 4 * i] = w_

        def put_slot(s, limbs):
            for k_, limb in enumerate(limbs):
                em.mem[SLOTS + s * SS * L * 4 + k_ * L * 4] = limb          # ciphertext 0
        put_slot(0, [(r >> (B * k_)) & ((1 << B) - 1) for k_ in range(SS)])
        put_slot(3, nm.limbs(1) + nm.limbs(m))
        if mont:
            K = pow(1 << (B * S), e + 1, n2)
            put_slot(4, nm.limbs(K % n) + nm.limbs(K // n))
        em.s[0], em.s[1], em.s[2] = KA, 0, 0
        for ln in range(NL):
            em.v[ln][0] = ln                                  # tid
        em.run(kname)
        out = [em.mem.get(SLOTS + 6 * SS * L * 4 + k_ * L * 4, 0) for k_ in range(SS)]
        x0 = sum(out[k_] << (B * k_) for k_ in range(S))
        x1 = sum(out[S + k_] << (B * k_) for k_ in range(S))
        want = pow(r, e, n2) * (1 + m * n) % n2
        assert x0 < n and x1 < n, (x0 < n, x1 < n)
        assert x0 + x1 * n == want, f'trial {trial}: mismatch'
        mads = em.count.get('v_mad_u64_u32', 0) + em.count.get('v_mad_i64_i32', 0)
        print(f'trial {trial}: ok ({ebits}-bit exponent, {mads} MAD instructions)')
    print('quad_emu selftest ok')


def nadic_entry(v, n, S=76, B=27):
    """digit-form table entry of v (gen_nadic.py): y0 = v mod n, y1 = v div n, each as four lane quarters
    of S/4 limbs and a pad word"""
    import nadic_model as nm
    Q = S // 4
    out = []
    for y in (v % n, v // n):
        lim = nm.limbs(y)
        for k in range(4):
            out += lim[k * Q:(k + 1) * Q] + [0]
    return out


def selftest_gather(wide=False):
    """LOADGD(16) / MULGD(16) from a digit-form table: X = e0 e1 (1 + m n) mod n^2 for entries e0, e1 at
    windows 0 and 1 selected by per-ciphertext digits, against Python integers"""
    sys.path.insert(0, 'fedtree_amd/csrc')
    sys.path.insert(0, 'tools')
    from gen_nadic import gen_nadic
    import nadic_model as nm
    S, B, SS = 76, 27, 152
    asm = gen_nadic(S, B, 'fthe_nadic_q76')
    rng = random.Random(13)
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    n2 = n * n
    em = QuadEmu(asm, 4 * 2 * S * 68)
    L = 256
    KA, CTX, PROG, SLOTS, TAB, DIG = 0x100, 0x1000, 0x2000, 0x100000, 0x10000000, 0x8000000
    W = 16 if wide else 8
    kargs = [SLOTS & M32, SLOTS >> 32, PROG, 0, CTX, 0, L * 4, SS * L * 4, L, 0]
    kargs += [TAB & M32, TAB >> 32, DIG & M32, DIG >> 32]            # rows[0] (offset 40), rows[1] (48)
    for i, v in enumerate(kargs):
        em.mem[KA + 4 * i] = v
    k1, k2, k3, bias = nm.consts(n)
    ctxw = nm.limbs(n) + [0]
    for d in (k1, k2, k3, bias):
        b_ = f2b(d)
        ctxw += [b_ & M32, b_ >> 32]
    for i, w in enumerate(ctxw):
        em.mem[CTX + 4 * i] = w
    dg = [rng.randrange(1 << W), rng.randrange(1 << W)]
    vals = {}
    for j, d in enumerate(dg):
        v = rng.randrange(n2) if j == 0 else n2 - 1 - rng.randrange(1 << 64)
        vals[j] = v
        ent = (j << W) | d
        words = nadic_entry(v, n)
        for i_, w_ in enumerate(words):
            em.mem[TAB + ent * 4 * len(words) + 4 * i_] = w_
        # digit of ciphertext 0 in window j (u8 / u16 array [window][L])
        a = DIG + (j * L) * (2 if wide else 1)
        w0 = em.mem.get(a & ~3, 0)
        sh = 8 * (a & 3)
        w0 |= d << sh
        em.mem[a & ~3] = w0
    m = rng.getrandbits(64)
    prog = []
    op = lambda o, a_: prog.extend([o, a_])
    op(16 if wide else 14, 0)
    op(17 if wide else 15, 1)
    op(4, 3)
    op(20, 0)
    op(2, 6)
    op(0, 0)
    for i, w_ in enumerate(prog):
        em.mem[PROG + 4 * i] = w_
    for k_, limb in enumerate(nm.limbs(1) + nm.limbs(m)):
        em.mem[SLOTS + 3 * SS * L * 4 + k_ * L * 4] = limb
    em.s[0], em.s[1], em.s[2] = KA, 0, 0
    for ln in range(NL):
        em.v[ln][0] = ln
    em.run('fthe_nadic_q76')
    out = [em.mem.get(SLOTS + 6 * SS * L * 4 + k_ * L * 4, 0) for k_ in range(SS)]
    x0 = sum(out[k_] << (B * k_) for k_ in range(S))
    x1 = sum(out[S + k_] << (B * k_) for k_ in range(S))
    assert x0 < n and x1 < n
    assert x0 + x1 * n == vals[0] * vals[1] * (1 + m * n) % n2
    print(f'gather ({W}-bit windows): ok')


if __name__ == '__main__':
    selftest(int(sys.argv[1]) if len(sys.argv) > 1 else 2, int(sys.argv[2]) if len(sys.argv) > 2 else 24)
    selftest_gather(False)
    selftest_gather(True)
