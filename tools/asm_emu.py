#!/usr/bin/env python3
"""Single-lane emulator for the instruction subset of the generated one-lane kernels
(fedtree_amd/csrc/gen_padic.py), for checking register allocation and control flow on the CPU before
a kernel ever runs on the GPU.  Lane 0 of workgroup 0; memory is a sparse dict of 32-bit words.

  python tools/asm_emu.py      (self-test: y^e mod P^2 through the P-adic kernel vs pow())
"""
import random
import re
import sys

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


def s32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


class Emu:
    def __init__(self, asm_text):
        self.lines = []
        self.labels = {}
        for raw in asm_text.splitlines():
            line = raw.split('//')[0].rstrip()
            if not line.strip() or line.startswith('.') and not line.endswith(':'):
                if line.startswith('.amdhsa_kernel') or line.startswith('.rodata'):
                    break
                continue
            s = line.strip()
            if s.endswith(':'):
                self.labels[s[:-1]] = len(self.lines)
                continue
            self.lines.append(s)
        self.v = {}
        self.s = {}
        self.mem = {}
        self.count = {}

    # ---- operands -------------------------------------------------------
    def reg_range(self, tok):
        m = re.fullmatch(r'([vs])\[(\d+):(\d+)\]', tok)
        if m:
            return m.group(1), int(m.group(2)), int(m.group(3)) - int(m.group(2)) + 1
        m = re.fullmatch(r'([vs])(\d+)', tok)
        if m:
            return m.group(1), int(m.group(2)), 1
        return None

    def read(self, tok, width=1):
        if tok == 'vcc':
            return self.s.get('vcc', 0)
        if tok == 'exec':
            return M64
        if tok == 'm0':
            return self.s.get('m0', 0)
        r = self.reg_range(tok)
        if r is None:
            val = int(tok, 0)
            if val < 0:
                val &= (1 << (32 * width)) - 1 if width == 1 else M64
            return val
        kind, base, n = r
        f = self.v if kind == 'v' else self.s
        out = 0
        for i in range(n):
            out |= (f.get(base + i, 0) & M32) << (32 * i)
        return out

    def write(self, tok, val):
        if tok == 'vcc':
            self.s['vcc'] = val & M64
            return
        if tok == 'm0':
            self.s['m0'] = val & M32
            return
        kind, base, n = self.reg_range(tok)
        f = self.v if kind == 'v' else self.s
        for i in range(n):
            f[base + i] = (val >> (32 * i)) & M32

    def label_value(self, expr):
        m = re.fullmatch(r'(\.L\w+)-(\.L\w+)', expr)
        if m:
            return (self.labels[m.group(1)] - self.labels[m.group(2)]) * 8
        return int(expr, 0)

    # ---- execution --------------------------------------------------------
    def run(self, entry, max_steps=50_000_000, stop=None):
        pc = self.labels[entry]
        steps = 0
        stop_pc = self.labels[stop] if stop else -1
        while True:
            if pc == stop_pc:
                return
            steps += 1
            if steps > max_steps:
                raise RuntimeError("step limit")
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
                if self.s.get('scc', 0) == (1 if op.endswith('1') else 0):
                    pc = self.labels[args[0]]
                continue
            if op == 's_getpc_b64':
                self.write(args[0], pc * 8)
                continue
            if op == 's_swappc_b64':
                tgt = self.read(args[1])
                self.write(args[0], pc * 8)
                assert tgt % 8 == 0
                pc = tgt // 8
                continue
            if op == 's_setpc_b64':
                pc = self.read(args[0]) // 8
                continue
            if op.startswith('s_load_dword'):
                dst, base, off = args
                kind, b0, n = self.reg_range(dst)
                addr = self.read(base) + (self.read(off) if off.startswith('s') else int(off, 0))
                for i in range(n):
                    self.s[b0 + i] = self.mem.get(addr + 4 * i, 0)
                continue
            if op == 's_add_u32':
                a, b = self.read(args[1]), (self.label_value(args[2]) if args[2].startswith('.L') else self.read(args[2]))
                r = (a & M32) + (b & M32)
                self.s['scc'] = r >> 32
                self.write(args[0], r)
                continue
            if op == 's_addc_u32':
                r = (self.read(args[1]) & M32) + (self.read(args[2]) & M32) + self.s.get('scc', 0)
                self.s['scc'] = r >> 32
                self.write(args[0], r)
                continue
            if op == 's_sub_u32':
                a, b = self.read(args[1]) & M32, self.read(args[2]) & M32
                self.s['scc'] = 1 if b > a else 0
                self.write(args[0], a - b)
                continue
            if op == 's_mul_i32':
                self.write(args[0], self.read(args[1]) * self.read(args[2]))
                continue
            if op == 's_mul_hi_u32':
                self.write(args[0], ((self.read(args[1]) & M32) * (self.read(args[2]) & M32)) >> 32)
                continue
            if op == 's_mov_b32':
                self.write(args[0], self.read(args[1]))
                continue
            if op == 's_lshl_b32':
                r = (self.read(args[1]) << self.read(args[2])) & M32
                self.s['scc'] = int(r != 0)
                self.write(args[0], r)
                continue
            if op == 's_lshr_b32':
                r = (self.read(args[1]) & M32) >> self.read(args[2])
                self.s['scc'] = int(r != 0)
                self.write(args[0], r)
                continue
            if op == 's_cmp_eq_u32':
                self.s['scc'] = int((self.read(args[0]) & M32) == (self.read(args[1]) & M32))
                continue
            # ---- vector ----
            if op == 'v_lshlrev_b32_e32':
                self.write(args[0], self.read(args[2]) << self.read(args[1]))
                continue
            if op == 'v_lshrrev_b32_e32':
                self.write(args[0], (self.read(args[2]) & M32) >> self.read(args[1]))
                continue
            if op == 'v_or_b32_e32':
                self.write(args[0], self.read(args[1]) | self.read(args[2]))
                continue
            if op == 'v_add_u32_e32':
                self.write(args[0], self.read(args[1]) + self.read(args[2]))
                continue
            if op == 'v_sub_u32_e32':
                self.write(args[0], self.read(args[1]) - self.read(args[2]))
                continue
            if op == 'v_and_b32_e32':
                self.write(args[0], self.read(args[1]) & self.read(args[2]))
                continue
            if op == 'v_mov_b32_e32':
                self.write(args[0], self.read(args[1]))
                continue
            if op == 'v_mov_b64_e32':
                self.write(args[0], self.read(args[1], 2))
                continue
            if op == 'v_pk_mov_b32':
                # v_pk_mov_b32 dst[2], src0[2], src1[2] op_sel:[0,1]: dst.x = src0.x, dst.y = src1.y
                dst, a, b = args[0], args[1], args[2].split()[0]
                lo = self.read(a) & M32
                hi = (self.read(b) >> 32) & M32
                assert 'op_sel:[0,1]' in ins
                self.write(dst, lo | (hi << 32))
                continue
            if op in ('v_mad_u64_u32', 'v_mad_i64_i32'):
                dst, _, a, b, c = args
                va, vb = self.read(a) & M32, self.read(b) & M32
                vc = self.read(c, 2) & M64
                if op == 'v_mad_i64_i32':
                    va, vb = s32(va), s32(vb)
                self.write(dst, (va * vb + vc) & M64)
                continue
            if op == 'v_lshl_add_u64':
                dst, a, sh, c = args
                self.write(dst, ((self.read(a, 2) << int(sh)) + self.read(c, 2)) & M64)
                continue
            if op == 'v_lshrrev_b64':
                self.write(args[0], (self.read(args[2], 2) & M64) >> int(args[1]))
                continue
            if op == 'v_ashrrev_i64':
                x = self.read(args[2], 2) & M64
                if x >> 63:
                    x -= 1 << 64
                self.write(args[0], (x >> int(args[1])) & M64)
                continue
            if op in ('global_load_ubyte', 'global_load_ushort'):
                dst, voff, sbase = args
                addr = self.read(sbase) + (self.read(voff) & M32)
                w = self.mem.get(addr & ~3, 0) >> (8 * (addr & 3))
                self.write(dst, w & (0xff if op.endswith('ubyte') else 0xffff))
                continue
            if op == 'global_load_dwordx4':
                # global_load_dwordx4 v[a:a+3], v[addr:addr+1], off offset:N
                dst, vaddr = args[0], args[1]
                rest_ = args[2].split()
                off = int(rest_[1].split(':')[1]) if len(rest_) > 1 else 0
                addr = self.read(vaddr) + off
                kind, b0, n = self.reg_range(dst)
                for i in range(n):
                    self.v[b0 + i] = self.mem.get(addr + 4 * i, 0)
                continue
            if op == 'global_load_dword':
                dst, voff, sbase = args
                addr = self.read(sbase) + (self.read(voff) & M32)
                self.write(dst, self.mem.get(addr, 0))
                continue
            if op == 'global_store_dword':
                voff, src, sbase = args
                addr = self.read(sbase) + (self.read(voff) & M32)
                self.mem[addr] = self.read(src) & M32
                continue
            raise NotImplementedError(ins)


def selftest():
    sys.path.insert(0, 'fedtree_amd/csrc')
    sys.path.insert(0, 'tools')
    from gen_padic import gen_padic
    import padic_model as pm
    K, B = 37, 28
    asm = gen_padic(K, B, 'fthe_padic_k37')
    rng = random.Random(7)
    for trial in range(3):
        P = rng.getrandbits(1024) | (3 << 1022) | 1
        P2 = P * P
        key = pm.PadicKey(P, K)
        em = Emu(asm)
        # memory: kernarg at 0x100, ctx at 0x1000, prog at 0x2000, slots at 0x100000 (L = 256 lanes)
        L = 256
        S = 2 * K
        KA, CTX, PROG, SLOTS = 0x100, 0x1000, 0x2000, 0x100000
        for i, (v) in enumerate([SLOTS & M32, SLOTS >> 32, PROG, 0, CTX, 0, L * 4, S * L * 4, L, 0]):
            em.mem[KA + 4 * i] = v
        ctxw = [(-x) & M32 for x in pm.limbs(P, K)] + [0, 0, 0] + key.mu
        for i, w in enumerate(ctxw):
            em.mem[CTX + 4 * i] = w
        X = rng.randrange(P2) if trial else rng.randrange(P)
        e = P if trial != 1 else P - 1
        # program: LOADP 0; pow; STOREP 40
        prog = []
        op = lambda o, a: prog.extend([o, a])
        tbl0, sq, w = 2, 1, 4
        bits = bin(e)[2:]
        ntab = 1 << (w - 1)
        op(22, 0)
        op(2, tbl0); op(3, 1); op(2, sq); op(1, tbl0)
        for k in range(1, ntab):
            op(4, sq); op(2, tbl0 + k)
        i = 0
        started = False
        pend = 0
        while i < len(bits):
            if bits[i] == '0':
                pend += 1
                i += 1
                continue
            j = min(len(bits), i + w)
            while bits[j - 1] == '0':
                j -= 1
            v = int(bits[i:j], 2)
            if not started:
                op(1, tbl0 + (v - 1) // 2)
                started = True
            else:
                pend += j - i
                op(3, pend); pend = 0
                op(4, tbl0 + (v - 1) // 2)
            i = j
        if pend:
            op(3, pend)
        op(23, 40)
        op(0, 0)
        for i, w_ in enumerate(prog):
            em.mem[PROG + 4 * i] = w_
        for k, limb in enumerate(pm.limbs(X, S)):
            em.mem[SLOTS + k * L * 4] = limb                   # lane 0 of slot 0
        em.s[0], em.s[1], em.s[2] = KA, 0, 0
        em.v[0] = 0
        em.run('fthe_padic_k37')
        out = [em.mem.get(SLOTS + 40 * S * L * 4 + k * L * 4, 0) for k in range(S)]
        got = pm.value(out)
        assert got % P2 == pow(X, e, P2), f"trial {trial}: mismatch"
        assert got < 6 * P2
        mads = em.count.get('v_mad_u64_u32', 0) + em.count.get('v_mad_i64_i32', 0)
        print(f"trial {trial}: ok ({len(bits)}-bit exponent, {mads} MADs executed)")
    print("asm_emu selftest ok")


if __name__ == "__main__":
    selftest()
