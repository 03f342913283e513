#!/usr/bin/env python3
"""Emulator of whole wavefronts (64 lanes) for the instruction subsets of the matrix-core kernels: the
Barrett add (fedtree_amd/csrc/gen_addb.py) and the P-adic exponentiation fthe_padic_m37 (gen_padic_mfma.py):
per-lane VGPRs, SGPRs, EXEC / VCC / SCC, DPP quad_perm, LDS, global memory, v_mfma_i32_16x16x64_i8 and
v_mfma_i32_32x32x32_i8 and v_permlane32_swap (lane maps measured on the GPU: profiles/r03c_mfma16_probe.txt,
profiles/r02zh_mfma_probe.txt), the s_getpc / s_swappc call of m37's shared reduction -- so that register
plans, lane layouts, LDS offsets and control flow are checked on the CPU before the kernel runs on a GPU.  A
workgroup is emulated wave by wave: every wave up to its s_barrier, then each wave to its end (the kernels'
waves share only what they wrote before the barrier).

  python tools/wave_emu.py         (self-test: 16 random adds mod n^2 and edge cases vs Python integers)
  python tools/wave_emu.py m37     (one wave of fthe_padic_m37: LOADP, STOREX, SQR, MUL, STOREP = x^3 mod P^2)
"""
import os
import random
import re
import sys

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1
ALL = (1 << 64) - 1


def s32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


class Mem:
    """flat global memory: buffers at fixed bases"""

    def __init__(self):
        self.bufs = []            # (base, bytearray)

    def alloc(self, data, base):
        self.bufs.append((base, bytearray(data)))
        return base

    def find(self, addr, n):
        for b, ba in self.bufs:
            if b <= addr and addr + n <= b + len(ba):
                return ba, addr - b
        raise IndexError(f"global access out of bounds: {addr:#x} +{n}")

    def read(self, addr, n):
        ba, o = self.find(addr, n)
        return int.from_bytes(ba[o:o + n], 'little')

    def write(self, addr, n, v):
        ba, o = self.find(addr, n)
        ba[o:o + n] = (v & ((1 << (8 * n)) - 1)).to_bytes(n, 'little')


class Wave:
    def __init__(self, prog, labels, lds, mem, sgpr_init, tid0, nvgpr):
        self.prog, self.labels, self.lds, self.mem = prog, labels, lds, mem
        self.v = [[0] * 64 for _ in range(nvgpr)]      # v[reg][lane]
        for lane in range(64):
            self.v[0][lane] = tid0 + lane
        self.s = [0] * 128
        for k, val in sgpr_init.items():
            self.s[k] = val & M32
        self.exec = ALL
        self.vcc = 0
        self.scc = 0
        self.pc = 0
        self.done = False
        self.at_barrier = False
        self.count = 0

    # ---- operand helpers ----------------------------------------------------------------------------
    @staticmethod
    def rr(tok):
        m = re.fullmatch(r'([vs])\[(\d+):(\d+)\]', tok)
        if m:
            return m.group(1), int(m.group(2)), int(m.group(3)) - int(m.group(2)) + 1
        m = re.fullmatch(r'([vs])(\d+)', tok)
        if m:
            return m.group(1), int(m.group(2)), 1
        return None

    def sget(self, tok, width=1):
        if tok == 'vcc':
            return self.vcc
        if tok == 'exec':
            return self.exec
        r = self.rr(tok)
        if r is None:
            m = re.fullmatch(r'(\.L\w+)-(\.L\w+)', tok)          # label difference (s_getpc-relative call)
            if m:
                return (self.labels[m.group(1)] - self.labels[m.group(2)]) & M32
            return int(tok, 0) & (M64 if width == 2 else M32)
        kind, b, n = r
        assert kind == 's', tok
        val = 0
        for i in range(n):
            val |= self.s[b + i] << (32 * i)
        return val

    def sset(self, tok, val):
        if tok == 'vcc':
            self.vcc = val & M64
            return
        if tok == 'exec':
            self.exec = val & M64
            return
        kind, b, n = self.rr(tok)
        assert kind == 's'
        for i in range(n):
            self.s[b + i] = (val >> (32 * i)) & M32

    def vget(self, lane, tok, width=1):
        """operand of a lane: a VGPR / VGPR range (all its registers), an SGPR / SGPR range, vcc or a literal
        (masked to 32 bits, or 64 when width == 2)"""
        r = self.rr(tok)
        if r is None:
            if tok == 'vcc':
                return self.vcc
            return int(tok, 0) & (M64 if width == 2 else M32)
        kind, b, n = r
        val = 0
        for i in range(n):
            val |= (self.s[b + i] if kind == 's' else self.v[b + i][lane]) << (32 * i)
        return val

    def vset(self, lane, tok, val):
        kind, b, n = self.rr(tok)
        assert kind == 'v', tok
        for i in range(n):
            self.v[b + i][lane] = (val >> (32 * i)) & M32

    def lanes(self):
        ex = self.exec
        return [l for l in range(64) if ex >> l & 1]

    # ---- execution ----------------------------------------------------------------------------------
    def run(self, max_steps=5_000_000):
        while not self.done and not self.at_barrier:
            assert self.count < max_steps, "runaway"
            op, args = self.prog[self.pc]
            self.pc += 1
            self.count += 1
            self.step(op, args)

    def step(self, op, a):
        if op == 's_endpgm':
            self.done = True
            return
        if op == 's_barrier':
            self.at_barrier = True
            return
        if op in ('s_nop', 's_waitcnt', 's_setprio', 's_sleep'):
            return
        if op == 's_cbranch_scc0':
            if not self.scc:
                self.pc = self.labels[a[0]]
            return
        if op == 's_getpc_b64':                    # pc = index of the next instruction
            self.sset(a[0], self.pc)
            return
        if op == 's_swappc_b64':
            ret = self.pc
            self.pc = self.sget(a[1], 2)
            self.sset(a[0], ret)
            return
        if op == 's_setpc_b64':
            self.pc = self.sget(a[0], 2)
            return
        if op == 'v_mfma_i32_32x32x32_i8':
            return self.mfma32(a)
        if op == 'v_permlane32_swap_b32_e32':      # the upper half of vdst <-> the lower half of vsrc
            x, y = self.rr(a[0])[1], self.rr(a[1])[1]
            for l in range(32):
                self.v[x][l + 32], self.v[y][l] = self.v[y][l], self.v[x][l + 32]
            return
        if op == 's_branch':
            self.pc = self.labels[a[0]]
            return
        if op == 's_cbranch_scc1':
            if self.scc:
                self.pc = self.labels[a[0]]
            return
        if op == 's_cbranch_execz':
            if self.exec == 0:
                self.pc = self.labels[a[0]]
            return
        if op == 's_cbranch_vccz':
            if (self.vcc & self.exec) == 0:
                self.pc = self.labels[a[0]]
            return
        if op.startswith('s_'):
            return self.salu(op, a)
        if op.startswith('ds_'):
            return self.ds(op, a)
        if op.startswith('global_'):
            return self.glob(op, a)
        if op == 'v_mfma_i32_16x16x64_i8':
            return self.mfma(a)
        if op == 'v_readfirstlane_b32':
            ln = self.lanes()
            self.sset(a[0], self.vget(ln[0] if ln else 0, a[1]))
            return
        if op == 'v_and_b32_dpp':                  # dst = dpp(src0) & src1
            perm = [int(x) for x in re.search(r'quad_perm:\[([0-9,]+)\]', ' '.join(a)).group(1).split(',')]
            src, msk, dst = self.rr(a[1])[1], self.rr(a[2])[1], self.rr(a[0])[1]
            old, om = list(self.v[src]), list(self.v[msk])
            for l in self.lanes():
                sl = (l & ~3) + perm[l & 3]
                assert self.exec >> sl & 1, "DPP source lane disabled"
                self.v[dst][l] = old[sl] & om[l]
            return
        if op == 'v_cndmask_b32_dpp':              # dst = vcc ? src1 : dpp(src0)
            perm = [int(x) for x in re.search(r'quad_perm:\[([0-9,]+)\]', ' '.join(a)).group(1).split(',')]
            assert a[3] == 'vcc'
            src, s1, dst = self.rr(a[1])[1], self.rr(a[2])[1], self.rr(a[0])[1]
            old, o1 = list(self.v[src]), list(self.v[s1])
            for l in self.lanes():
                sl = (l & ~3) + perm[l & 3]
                assert self.exec >> sl & 1, "DPP source lane disabled"
                self.v[dst][l] = o1[l] if (self.vcc >> l) & 1 else old[sl]
            return
        if op == 'v_mov_b32_dpp' and ('wave_shr:1' in a or 'wave_shl:1' in a):
            # whole-wave shift by one lane; bound_ctrl:0 (the BC bit): the lane without a source gets 0
            assert 'bound_ctrl:0' in a and self.exec == ALL, "wave shift: full EXEC and bound_ctrl:0"
            src, dst = self.rr(a[1])[1], self.rr(a[0])[1]
            old = list(self.v[src])
            d = -1 if 'wave_shr:1' in a else 1
            for l in range(64):
                self.v[dst][l] = old[l + d] if 0 <= l + d < 64 else 0
            return
        if op == 'v_mov_b32_dpp':
            perm = [int(x) for x in re.search(r'quad_perm:\[([0-9,]+)\]', ' '.join(a)).group(1).split(',')]
            src = self.rr(a[1])[1]
            dst = self.rr(a[0])[1]
            old = list(self.v[src])
            for l in self.lanes():
                sl = (l & ~3) + perm[l & 3]
                assert self.exec >> sl & 1, "DPP source lane disabled"
                self.v[dst][l] = old[sl]
            return
        return self.valu(op, a)

    def salu(self, op, a):
        g = self.sget
        if op in ('s_load_dwordx2', 's_load_dwordx4', 's_load_dwordx8', 's_load_dwordx16'):
            n = int(op[len('s_load_dwordx'):])
            addr = g(a[1], 2) + int(a[2], 0)
            self.sset(a[0], self.mem.read(addr, 4 * n))
        elif op == 's_bitcmp1_b32':
            self.scc = (g(a[0]) >> (g(a[1]) & 31)) & 1
        elif op == 's_mul_hi_u32':
            self.sset(a[0], (g(a[1]) * g(a[2])) >> 32)
        elif op == 's_addc_u32':
            r = g(a[1]) + g(a[2]) + self.scc
            self.sset(a[0], r)
            self.scc = r >> 32
        elif op == 's_load_dword':
            addr = g(a[1], 2) + int(a[2], 0)
            self.sset(a[0], self.mem.read(addr, 4))
        elif op in ('s_mov_b32', 's_movk_i32'):
            self.sset(a[0], g(a[1]))
        elif op == 's_mov_b64':
            self.sset(a[0], g(a[1], 2) if a[1] != '-1' else ALL)
        elif op == 's_not_b64':
            self.sset(a[0], ~g(a[1], 2) & M64)
            self.scc = int(self.sget(a[0], 2) != 0)
        elif op == 's_and_saveexec_b64':
            self.sset(a[0], self.exec)
            self.exec = self.exec & g(a[1], 2)
            self.scc = int(self.exec != 0)
        elif op == 's_mul_i32':
            self.sset(a[0], g(a[1]) * g(a[2]))
        elif op == 's_or_b64':
            r = g(a[1], 2) | g(a[2], 2)
            self.sset(a[0], r)
            self.scc = int(r != 0)
        elif op == 's_lshr_b32':
            r = (g(a[1]) & M32) >> (g(a[2]) & 31)
            self.sset(a[0], r)
            self.scc = int(r != 0)
        elif op == 's_lshl_b64':
            r = (g(a[1], 2) << (g(a[2]) & 63)) & M64
            self.sset(a[0], r)
            self.scc = int(r != 0)
        elif op == 's_lshl_b32':
            r = (g(a[1]) << g(a[2])) & M32
            self.sset(a[0], r)
            self.scc = int(r != 0)
        elif op == 's_add_u32':
            r = g(a[1]) + g(a[2])
            self.sset(a[0], r)
            self.scc = r >> 32
        elif op == 's_sub_u32':
            r = g(a[1]) - g(a[2])
            self.sset(a[0], r)
            self.scc = int(r < 0)
        elif op == 's_cmp_ge_u32':
            self.scc = int(g(a[0]) >= g(a[1]))
        elif op == 's_cmp_lg_u32':
            self.scc = int(g(a[0]) != g(a[1]))
        elif op == 's_cmp_eq_u32':
            self.scc = int(g(a[0]) == g(a[1]))
        elif op == 's_cmp_eq_u64':
            self.scc = int(g(a[0], 2) == g(a[1], 2))
        elif op == 's_and_b64':
            self.sset(a[0], g(a[1], 2) & g(a[2], 2))
            self.scc = int(self.sget(a[0], 2) != 0)
        elif op == 's_andn2_b64':
            self.sset(a[0], g(a[1], 2) & ~g(a[2], 2) & M64)
            self.scc = int(self.sget(a[0], 2) != 0)
        else:
            raise NotImplementedError(op)

    def ds(self, op, a):
        if op == 'ds_add_rtn_u32':                 # vdst = old; LDS[vaddr + offset] += vdata (lanes in order)
            off = next((int(t[7:], 0) for t in a[3:] if t.startswith('offset:')), 0)
            for l in self.lanes():
                addr = self.vget(l, a[1]) + off
                assert 0 <= addr and addr + 4 <= len(self.lds) and addr % 4 == 0, f"LDS atomic at {addr}"
                old = int.from_bytes(self.lds[addr:addr + 4], 'little')
                self.lds[addr:addr + 4] = ((old + self.vget(l, a[2])) & 0xffffffff).to_bytes(4, 'little')
                self.vset(l, a[0], old)
            return
        if op == 'ds_read2_b32':                   # vdst pair <- dwords at vaddr + 4 offset0 / + 4 offset1
            o0 = o1 = 0
            for t in a[2:]:
                if t.startswith('offset0:'):
                    o0 = int(t[8:], 0)
                elif t.startswith('offset1:'):
                    o1 = int(t[8:], 0)
            for l in self.lanes():
                base = self.vget(l, a[1])
                vals = []
                for oo in (o0, o1):
                    addr = base + 4 * oo
                    assert 0 <= addr and addr + 4 <= len(self.lds) and addr % 4 == 0, f"LDS read2 at {addr}"
                    vals.append(int.from_bytes(self.lds[addr:addr + 4], 'little'))
                self.vset(l, a[0], vals[0] | vals[1] << 32)
            return
        if op == 'ds_write2_b32':                  # two dwords at vaddr + 4 offset0 / + 4 offset1
            o0 = o1 = 0
            for t in a[3:]:
                if t.startswith('offset0:'):
                    o0 = int(t[8:], 0)
                elif t.startswith('offset1:'):
                    o1 = int(t[8:], 0)
            for l in self.lanes():
                base = self.vget(l, a[0])
                for tok, oo in ((a[1], o0), (a[2], o1)):
                    addr = base + 4 * oo
                    assert 0 <= addr and addr + 4 <= len(self.lds) and addr % 4 == 0, f"LDS write2 at {addr}"
                    self.lds[addr:addr + 4] = self.vget(l, tok).to_bytes(4, 'little')
            return
        width = {'ds_read_b32': 4, 'ds_read_b64': 8, 'ds_read_b128': 16, 'ds_write_b32': 4, 'ds_write_b64': 8,
                 'ds_write_b128': 16}[op]
        off = 0
        for t in a[2:]:
            if t.startswith('offset:'):
                off = int(t[7:], 0)
        write = op.startswith('ds_write')
        addr_tok = a[0] if write else a[1]
        data_tok = a[1] if write else a[0]
        for l in self.lanes():
            addr = self.vget(l, addr_tok) + off
            assert 0 <= addr and addr + width <= len(self.lds), f"LDS out of range {addr}"
            assert addr % width == 0, f"misaligned LDS b{8 * width} at {addr}"
            if write:
                self.lds[addr:addr + width] = self.vget(l, data_tok, 2 if width >= 8 else 1).to_bytes(
                    8 if width >= 8 else 4, 'little')[:width] if width <= 8 else self.vq(l, data_tok)
            else:
                self.vset(l, data_tok, int.from_bytes(self.lds[addr:addr + width], 'little'))

    def vq(self, lane, tok):
        kind, b, n = self.rr(tok)
        val = 0
        for i in range(n):
            val |= self.v[b + i][lane] << (32 * i)
        return val.to_bytes(4 * n, 'little')

    def glob(self, op, a):
        width = {'global_load_dword': 4, 'global_load_dwordx2': 8, 'global_load_dwordx4': 16,
                 'global_store_dword': 4, 'global_store_dwordx4': 16}[op]
        off = 0
        for t in a[3:]:
            if t.startswith('offset:'):
                off = int(t[7:], 0)
        store = op.startswith('global_store')
        vaddr, sbase = a[1] if not store else a[0], a[2]
        data_tok = a[0] if not store else a[1]
        flat = sbase == 'off'                  # 64-bit VGPR address, no SGPR base
        base = 0 if flat else self.sget(sbase, 2)
        for l in self.lanes():
            addr = (self.vget(l, vaddr) if flat else base + self.vget(l, vaddr)) + off
            if store:
                self.mem.write(addr, width, int.from_bytes(self.vq(l, data_tok), 'little'))
            else:
                self.vset(l, data_tok, self.mem.read(addr, width))

    def mfma(self, a):
        D, A, Bt, C = (self.rr(t) for t in a)      # C None: the inline constant 0
        Am = [[0] * 64 for _ in range(16)]
        Bm = [[0] * 16 for _ in range(64)]
        for l in range(64):
            r, h = l & 15, l >> 4
            abytes = b''.join(self.v[A[1] + i][l].to_bytes(4, 'little') for i in range(4))
            bbytes = b''.join(self.v[Bt[1] + i][l].to_bytes(4, 'little') for i in range(4))
            for j in range(16):
                Am[r][16 * h + j] = abytes[j] - 256 if abytes[j] > 127 else abytes[j]
                Bm[16 * h + j][r] = bbytes[j] - 256 if bbytes[j] > 127 else bbytes[j]
        out = [[0] * 16 for _ in range(16)]
        for i in range(16):
            for n in range(16):
                out[i][n] = sum(Am[i][k] * Bm[k][n] for k in range(64))
        newd = {}
        for l in range(64):
            h, col = l >> 4, l & 15
            for g in range(4):
                c = s32(self.v[C[1] + g][l]) if C is not None else 0
                newd[(g, l)] = (out[4 * h + g][col] + c) & M32
        for (g, l), val in newd.items():
            self.v[D[1] + g][l] = val

    def mfma32(self, a):
        """v_mfma_i32_32x32x32_i8 D, A, B, C (C may be 0): lane l (r = l & 31, h = l >> 5) holds A[r][16h + j]
        and B[16h + j][r] in byte j of its 16-byte fragment; register g of D / C is row (g & 3) + 8 (g >> 2) + 4h,
        column r (profiles/r02zh_mfma_probe.txt)"""
        D, A, Bt = (self.rr(t) for t in a[:3])
        C = self.rr(a[3])
        Am = [[0] * 32 for _ in range(32)]
        Bm = [[0] * 32 for _ in range(32)]
        for l in range(64):
            r, h = l & 31, l >> 5
            ab = b''.join(self.v[A[1] + i][l].to_bytes(4, 'little') for i in range(4))
            bb = b''.join(self.v[Bt[1] + i][l].to_bytes(4, 'little') for i in range(4))
            for j in range(16):
                Am[r][16 * h + j] = ab[j] - 256 if ab[j] > 127 else ab[j]
                Bm[16 * h + j][r] = bb[j] - 256 if bb[j] > 127 else bb[j]
        cols = [[sum(Am[i][k] * Bm[k][n] for k in range(32)) for n in range(32)] for i in range(32)]
        newd = {}
        for l in range(64):
            h, col = l >> 5, l & 31
            for gi in range(16):
                row = (gi & 3) + 8 * (gi >> 2) + 4 * h
                c = s32(self.v[C[1] + gi][l]) if C is not None else 0
                newd[(gi, l)] = (cols[row][col] + c) & M32
        for (gi, l), val in newd.items():
            self.v[D[1] + gi][l] = val

    def valu(self, op, a):
        lanes = self.lanes()
        g = self.vget
        if op == 'v_pk_mov_b32':                   # op_sel:[a,b]: lo from src0's half a, hi from src1's half b
            sel = [int(x) for x in re.search(r'op_sel:\[([01]),([01])\]', ' '.join(a)).groups()]
            for l in lanes:
                s0, s1 = g(l, a[1]), g(l, a[2])
                lo = (s0 >> (32 * sel[0])) & M32
                hi = (s1 >> (32 * sel[1])) & M32
                self.vset(l, a[0], lo | hi << 32)
            return
        if op == 'v_or3_b32':
            for l in lanes:
                self.vset(l, a[0], (g(l, a[1]) | g(l, a[2]) | g(l, a[3])) & M32)
            return
        if op == 'v_bitop3_b32':                   # bit i = table[src0_i << 2 | src1_i << 1 | src2_i]
            tbl = int(a[4].split(':')[1], 0)
            for l in lanes:
                x, y, z = g(l, a[1]), g(l, a[2]), g(l, a[3])
                r = 0
                for i in range(32):
                    r |= ((tbl >> ((x >> i & 1) << 2 | (y >> i & 1) << 1 | (z >> i & 1))) & 1) << i
                self.vset(l, a[0], r)
            return
        if op in ('v_mad_u64_u32', 'v_mad_i64_i32'):
            cmask = 0                                   # the carry-out / overflow mask written to sdst (a[1])
            for l in lanes:
                x, y = g(l, a[2]), g(l, a[3])
                c = g(l, a[4], 2)
                if op == 'v_mad_i64_i32':
                    r = s32(x) * s32(y) + s64(c)
                    ov = not (-(1 << 63) <= r < (1 << 63))
                else:
                    r = x * y + c
                    ov = r >> 64 != 0
                cmask |= int(ov) << l
                self.vset(l, a[0], r & M64)
            self.sset(a[1], cmask)
            return
        if op in ('v_sub_co_u32_e32', 'v_subb_co_u32_e32', 'v_subb_co_u32_e64'):
            nv = self.vcc
            for l in lanes:
                x, y = g(l, a[2]), g(l, a[3])
                bi = (self.vcc >> l) & 1 if op != 'v_sub_co_u32_e32' else 0
                r = x - y - bi
                self.vset(l, a[0], r & M32)
                nv = (nv | (1 << l)) if r < 0 else (nv & ~(1 << l))
            self.vcc = nv
            return
        if op in ('v_add_co_u32_e32', 'v_addc_co_u32_e32'):
            nv = self.vcc
            for l in lanes:
                ci = (self.vcc >> l) & 1 if op == 'v_addc_co_u32_e32' else 0
                r = g(l, a[2]) + g(l, a[3]) + ci
                self.vset(l, a[0], r & M32)
                nv = (nv | (1 << l)) if r >> 32 else (nv & ~(1 << l))
            self.vcc = nv
            return
        if op == 'v_cmp_gt_i64_e64':
            nv = 0
            for l in lanes:
                nv |= int(s64(g(l, a[1], 2)) > s64(g(l, a[2], 2))) << l
            self.sset(a[0], nv)
            return
        if op == 'v_cmp_gt_u32_e32':
            nv = 0
            for l in lanes:
                nv |= int(g(l, a[1]) > g(l, a[2])) << l
            self.vcc = nv
            return
        if op == 'v_cmp_eq_u32_e32':
            nv = 0
            for l in lanes:
                nv |= int(g(l, a[1]) == g(l, a[2])) << l
            self.vcc = nv
            return
        if op == 'v_cmp_ne_u32_e32':
            nv = 0
            for l in lanes:
                nv |= int(g(l, a[1]) != g(l, a[2])) << l
            self.vcc = nv
            return
        if op == 'v_cmp_gt_i32_e32':
            nv = 0
            for l in lanes:
                nv |= int(s32(g(l, a[1])) > s32(g(l, a[2]))) << l
            self.vcc = nv
            return
        if op == 'v_cmp_le_i32_e32':
            nv = 0
            for l in lanes:
                nv |= int(s32(g(l, a[1])) <= s32(g(l, a[2]))) << l
            self.vcc = nv
            return
        for l in lanes:
            if op == 'v_mov_b32_e32':
                r = g(l, a[1])
            elif op == 'v_mov_b64_e32':
                r = g(l, a[1], 2)
            elif op == 'v_lshlrev_b32_e32':
                r = g(l, a[2]) << (g(l, a[1]) & 31)
            elif op == 'v_lshrrev_b32_e32':
                r = g(l, a[2]) >> (g(l, a[1]) & 31)
            elif op == 'v_ashrrev_i32_e32':
                r = s32(g(l, a[2])) >> (g(l, a[1]) & 31)
            elif op == 'v_and_b32_e32':
                r = g(l, a[1]) & g(l, a[2])
            elif op == 'v_or_b32_e32':
                r = g(l, a[1]) | g(l, a[2])
            elif op == 'v_xor_b32_e32':
                r = g(l, a[1]) ^ g(l, a[2])
            elif op == 'v_add_u32_e32':
                r = g(l, a[1]) + g(l, a[2])
            elif op == 'v_sub_u32_e32':
                r = g(l, a[1]) - g(l, a[2])
            elif op == 'v_subrev_u32_e32':
                r = g(l, a[2]) - g(l, a[1])
            elif op == 'v_mul_lo_u32':
                r = g(l, a[1]) * g(l, a[2])
            elif op == 'v_mul_u32_u24_e32':
                r = (g(l, a[1]) & 0xFFFFFF) * (g(l, a[2]) & 0xFFFFFF)
            elif op == 'v_mad_u32_u24':
                r = (g(l, a[1]) & 0xFFFFFF) * (g(l, a[2]) & 0xFFFFFF) + g(l, a[3])
            elif op == 'v_add3_u32':
                r = g(l, a[1]) + g(l, a[2]) + g(l, a[3])
            elif op == 'v_lshl_add_u32':
                r = (g(l, a[1]) << (g(l, a[2]) & 31)) + g(l, a[3])
            elif op == 'v_lshl_or_b32':
                r = ((g(l, a[1]) << (g(l, a[2]) & 31)) | g(l, a[3]))
            elif op == 'v_add_lshl_u32':
                r = ((g(l, a[1]) + g(l, a[2])) & M32) << (g(l, a[3]) & 31)
            elif op == 'v_bfe_u32':
                off, w = g(l, a[2]) & 31, g(l, a[3]) & 31
                r = (g(l, a[1]) >> off) & ((1 << w) - 1)
            elif op == 'v_alignbyte_b32':
                r = (((g(l, a[1]) << 32) | g(l, a[2])) >> (8 * (g(l, a[3]) & 3)))
            elif op == 'v_perm_b32':                 # byte k = selector byte k of {src0, src1} (0..3: src1)
                both, sel, r = (g(l, a[1]) << 32) | g(l, a[2]), g(l, a[3]), 0
                for k in range(4):
                    sb = (sel >> (8 * k)) & 0xff
                    assert sb < 8, "v_perm_b32 selector"
                    r |= ((both >> (8 * sb)) & 0xff) << (8 * k)
            elif op == 'v_alignbit_b32':
                r = (((g(l, a[1]) << 32) | g(l, a[2])) >> (g(l, a[3]) & 31))
            elif op == 'v_lshl_add_u64':
                r = (g(l, a[1], 2) << (g(l, a[2]) & 63)) + g(l, a[3], 2)
            elif op == 'v_lshlrev_b64':
                r = g(l, a[2], 2) << (g(l, a[1]) & 63)
            elif op == 'v_lshrrev_b64':
                r = g(l, a[2], 2) >> (g(l, a[1]) & 63)
            elif op == 'v_ashrrev_i64':
                r = s64(g(l, a[2], 2)) >> (g(l, a[1]) & 63)
            elif op == 'v_cndmask_b32_e64':
                r = g(l, a[2]) if (self.sget(a[3], 2) >> l) & 1 else g(l, a[1])
            elif op == 'v_cndmask_b32_e32':
                r = g(l, a[2]) if (self.vcc >> l) & 1 else g(l, a[1])
            elif op == 'v_bfi_b32':
                r = (g(l, a[1]) & g(l, a[2])) | (~g(l, a[1]) & g(l, a[3]))
            elif op == 'v_xad_u32':
                r = (g(l, a[1]) ^ g(l, a[2])) + g(l, a[3])
            elif op == 'v_not_b32_e32':
                r = ~g(l, a[1])
            else:
                raise NotImplementedError(op)
            self.vset(l, a[0], r & (M64 if self.rr(a[0])[2] == 2 else M32))


def parse(asm):
    prog, labels = [], {}
    for raw in asm.splitlines():
        s = raw.split('//')[0].strip()
        if not s:
            continue
        if s.startswith('.amdhsa_kernel') or s.startswith('.rodata'):
            break
        if s.endswith(':'):
            labels[s[:-1]] = len(prog)
            continue
        if s.startswith('.'):
            continue
        parts = s.split(None, 1)
        op = parts[0]
        args = []
        if len(parts) > 1:
            rest = parts[1]
            # split on commas, then keep modifiers (offset:, quad_perm:...) as separate tokens
            toks = [t.strip() for t in re.split(r',(?![^\[]*\])', rest)]
            for t in toks:
                args.extend(t.split())
        prog.append((op, args))
    return prog, labels


def run_workgroup(asm, lds_bytes, waves, mem, kernarg_addr, wg, nvgpr, finish=None):
    """finish: the waves to run past their first barrier (default all)"""
    prog, labels = parse(asm)
    lds = bytearray(lds_bytes)
    ws = [Wave(prog, labels, lds, mem, {0: kernarg_addr & M32, 1: kernarg_addr >> 32, 2: wg}, 64 * w, nvgpr)
          for w in range(waves)]
    for w in ws:
        w.run()
    for i, w in enumerate(ws):
        if finish is None or i in finish:
            w.at_barrier = False
            w.run()
    return sum(w.count for w in ws)


def addb_run(n, xs, ys, asm=None):
    """one workgroup of fthe_addb_q152 (12 waves, wave 0 runs) on the rows xs, ys (len <= 16) under n: the output
    rows as integers"""
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, '..', 'fedtree_amd', 'csrc'))
    sys.path.insert(0, here)
    import gen_addb as ga
    import addb_model as am
    asm = asm or ga.gen_addb('fthe_addb_q152')
    N = n * n
    img = am.addb_image(N)
    count = len(xs)
    mem = Mem()
    XB, YB, OB, KB, KA = 0x10000000, 0x20000000, 0x30000000, 0x40000000, 0x50000000
    mem.alloc(b''.join(x.to_bytes(512, 'little') for x in xs), XB)
    mem.alloc(b''.join(y.to_bytes(512, 'little') for y in ys), YB)
    mem.alloc(bytes(512 * 16), OB)
    mem.alloc(img, KB)
    karg = XB.to_bytes(8, 'little') + YB.to_bytes(8, 'little') + OB.to_bytes(8, 'little') + \
        KB.to_bytes(8, 'little') + count.to_bytes(4, 'little') + (1).to_bytes(4, 'little') + bytes(16)
    mem.alloc(karg, KA)
    run_workgroup(asm, ga.LDS_BYTES, ga.WAVES, mem, KA, 0, 168)
    return [mem.read(OB + 512 * i, 512) for i in range(count)]


def selftest(ntests=16, count0=None):
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, '..', 'fedtree_amd', 'csrc'))
    sys.path.insert(0, here)
    import gen_addb as ga
    import addb_model as am
    rng = random.Random(5)
    asm = ga.gen_addb('fthe_addb_q152')
    for trial, n in enumerate((am.rand_n(rng), (1 << 2047) + 1, am.rand_n(rng))):
        gather = trial == 2                           # operand rows through index lists (-1: the integer 1)
        N = n * n
        img = am.addb_image(N)
        assert len(img) == ga.KCTX_BYTES
        xs = [rng.randrange(N) for _ in range(ntests)]
        ys = [rng.randrange(N) for _ in range(ntests)]
        xs[0], ys[0] = N - 1, N - 1
        xs[1], ys[1] = 0, N - 1
        xs[2], ys[2] = 1, 1
        xs[3], ys[3] = (1 << 4096) - 1, (1 << 4096) - 1          # rows >= N (reduced all the same)
        xs[4], ys[4] = N, N + 5
        count = ntests - (3 if trial else 0)         # a partly live wave on the second key
        if count0 is not None:
            count = count0 - (3 if trial else 0)
        mem = Mem()
        XB, YB, OB, KB, KA = 0x10000000, 0x20000000, 0x30000000, 0x40000000, 0x50000000
        XI, YI = 0x60000000, 0x70000000
        if gather:                                    # out[g] = xs[xi[g]] ys[yi[g]], index < 0 -> 1
            xi = [rng.randrange(-1, ntests) for _ in range(ntests)]
            yi = [rng.randrange(-1, ntests) for _ in range(ntests)]
            xi[0], yi[1] = -1, -1
            mem.alloc(b''.join(v.to_bytes(8, 'little', signed=True) for v in xi), XI)
            mem.alloc(b''.join(v.to_bytes(8, 'little', signed=True) for v in yi), YI)
        mem.alloc(b''.join(x.to_bytes(512, 'little') for x in xs), XB)
        mem.alloc(b''.join(y.to_bytes(512, 'little') for y in ys), YB)
        mem.alloc(bytes(512 * ntests), OB)
        mem.alloc(img, KB)
        karg = XB.to_bytes(8, 'little') + YB.to_bytes(8, 'little') + OB.to_bytes(8, 'little') + \
            KB.to_bytes(8, 'little') + count.to_bytes(4, 'little') + (1).to_bytes(4, 'little') + \
            ((XI.to_bytes(8, 'little') + YI.to_bytes(8, 'little')) if gather else bytes(16))
        mem.alloc(karg, KA)
        steps = run_workgroup(asm, ga.LDS_BYTES, ga.WAVES, mem, KA, 0, 168)
        bad = 0
        for i in range(ntests):
            got = mem.read(OB + 512 * i, 512)
            if gather:
                xv = xs[xi[i]] if xi[i] >= 0 else 1
                yv = ys[yi[i]] if yi[i] >= 0 else 1
            else:
                xv, yv = xs[i], ys[i]
            want = xv * yv % N if i < count else 0
            if got != want:
                bad += 1
                print(f"  ciphertext {i}: mismatch")
        print(f"key {trial}: {count} adds, {bad} mismatches, {steps} wave-instructions emulated")
        assert bad == 0
    print("wave_emu selftest OK")


def nadicb_selftest(seed=1, bits=2048, count=16, waves=1, batches=1):
    """one wave of fthe_nadic_b76 (a workgroup generated with one wave: 16 ciphertexts): LOADX r; CANON;
    STOREX T; SQR 1; STOREX U (digits up to 3n); SQR 1; MUL U; MUL T; CANON; STOREX OUT -> r^7 mod n^2 as
    canonical digits, against Python integers (r: 0, 1, n - 1, random)"""
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, '..', 'fedtree_amd', 'csrc'))
    sys.path.insert(0, here)
    import gen_nadicb as gb
    import nadicb_model as nm
    rng = random.Random(seed)
    n = nm.rand_n(rng, bits)
    N2 = n * n
    S, L, B = 152, 16 * waves * batches, 27       # batches > 1: the waves draw several (the emulator runs the
    #                                              first wave to its end, so wave 0 takes them all)
    count = max(count, L) if waves > 1 or batches > 1 else count
    asm = gb.gen_nadicb('fthe_nadic_b76', waves=waves)
    nv = int(re.search(r'\.amdhsa_next_free_vgpr (\d+)', asm).group(1))
    lds_bytes = int(re.search(r'\.amdhsa_group_segment_fixed_size (\d+)', asm).group(1))
    ctx = bytearray(gb.CTX_BYTES)
    img = nm.nadicb_image(n)
    ctx[:len(img)] = img
    for j in range(76):
        ctx[gb.N_OFF + 4 * j:gb.N_OFF + 4 * j + 4] = ((n >> (B * j)) & ((1 << B) - 1)).to_bytes(4, 'little')
    rs = [rng.randrange(n) for _ in range(L)]
    rs[:3] = [0, 1, n - 1]
    IN, T, U, OUT = 0, 1, 2, 3
    slots = bytearray(4 * S * L * 4)
    for g_, r in enumerate(rs):
        for k in range(76):
            off = (IN * S + k) * L * 4 + 4 * g_
            slots[off:off + 4] = ((r >> (B * k)) & ((1 << B) - 1)).to_bytes(4, 'little')
    prog = [1, IN, 20, 0, 2, T, 3, 1, 2, U, 3, 1, 4, U, 4, T, 20, 0, 2, OUT, 0, 0]
    mem = Mem()
    SB, PB, CB, KA = 0x10000000, 0x20000000, 0x30000000, 0x40000000
    mem.alloc(slots, SB)
    mem.alloc(b''.join(w.to_bytes(4, 'little') for w in prog), PB)
    mem.alloc(bytes(ctx), CB)
    karg = SB.to_bytes(8, 'little') + PB.to_bytes(8, 'little') + CB.to_bytes(8, 'little') + \
        (L * 4).to_bytes(4, 'little') + (S * L * 4).to_bytes(4, 'little') + L.to_bytes(4, 'little') + \
        (1).to_bytes(4, 'little') + bytes(128)
    mem.alloc(karg, KA)
    steps = run_workgroup(asm, lds_bytes, waves, mem, KA, 0, nv)
    bad = 0
    for g_ in range(count):
        x0 = x1 = 0
        for k in reversed(range(76)):
            x0 = (x0 << B) + mem.read(SB + (OUT * S + k) * L * 4 + 4 * g_, 4)
            x1 = (x1 << B) + mem.read(SB + (OUT * S + 76 + k) * L * 4 + 4 * g_, 4)
        want = pow(rs[g_], 7, N2)
        if not (x0 < n and x1 < n and x0 + x1 * n == want):
            bad += 1
            if bad <= 3:
                print(f"  ciphertext {g_}: x0 {x0:#x}\n  x1 {x1:#x}\n  want {want:#x}")
    print(f"nadic_b76: {count} ciphertexts, {bad} mismatches, {steps} wave-instructions emulated")
    return bad


def m37_selftest(seed=1, ab=None, bits=1024):
    """wave 0 of fthe_padic_m37 (one workgroup of 256 lanes, 4 waves fill the LDS tile image, wave 0 runs on):
    LOADP x; STOREX t; SQR 1; MUL t; STOREP -> x^3 mod P^2 (< 6 P^2), against Python integers on its 64 lanes
    (x < P^2: 0, 1, P - 1, P, P^2 - 1 and random).  ab: a generator switch string (FTHE_GEN_M37_AB)."""
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, '..', 'fedtree_amd', 'csrc'))
    sys.path.insert(0, here)
    if ab is not None:
        os.environ["FTHE_GEN_M37_AB"] = ab
    import importlib
    import gen_padic_mfma as gm
    gm = importlib.reload(gm)
    import padic_mfma_model as mm
    rng = random.Random(seed)
    P = rng.getrandbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
    P2 = P * P
    K, S, L, B = 37, 74, 256, 28
    asm = gm.gen_padic_mfma('fthe_padic_m37')
    nv = int(re.search(r'\.amdhsa_next_free_vgpr (\d+)', asm).group(1))
    lds_bytes = int(re.search(r'\.amdhsa_group_segment_fixed_size (\d+)', asm).group(1))
    ctx = bytearray(gm.TILE_OFF + gm.TILE_BYTES)
    for j in range(K):                                           # -P limbs (int32)
        ctx[4 * j:4 * j + 4] = ((-((P >> (B * j)) & ((1 << B) - 1))) & M32).to_bytes(4, 'little')
    img = mm.MfmaKey(P).tile_image()
    ctx[gm.TILE_OFF:gm.TILE_OFF + len(img)] = img
    xs = [rng.randrange(P2) for _ in range(L)]
    xs[:5] = [0, 1, P - 1, P, P2 - 1]
    IN, TAB, OUT = 0, 1, 2
    slots = bytearray(3 * S * L * 4)
    for g_, x in enumerate(xs):
        for k in range(S):
            off = (IN * S + k) * L * 4 + 4 * g_
            slots[off:off + 4] = ((x >> (B * k)) & ((1 << B) - 1)).to_bytes(4, 'little')
    prog = [22, IN, 2, TAB, 3, 1, 4, TAB, 23, OUT, 0, 0]
    mem = Mem()
    SB, PB, CB, KA = 0x10000000, 0x20000000, 0x30000000, 0x40000000
    mem.alloc(slots, SB)
    mem.alloc(b''.join(w.to_bytes(4, 'little') for w in prog), PB)
    mem.alloc(bytes(ctx), CB)
    karg = SB.to_bytes(8, 'little') + PB.to_bytes(8, 'little') + CB.to_bytes(8, 'little') + \
        (L * 4).to_bytes(4, 'little') + (S * L * 4).to_bytes(4, 'little') + L.to_bytes(4, 'little') + \
        (1).to_bytes(4, 'little') + bytes(128)
    mem.alloc(karg, KA)
    steps = run_workgroup(asm, lds_bytes, 4, mem, KA, 0, nv, finish=(0,))
    bad = 0
    for g_ in range(64):
        got = 0
        for k in reversed(range(S)):
            got = (got << B) + mem.read(SB + (OUT * S + k) * L * 4 + 4 * g_, 4)
        if not (got < 6 * P2 and got % P2 == pow(xs[g_], 3, P2)):
            bad += 1
            if bad <= 3:
                print(f"  lane {g_}: got {got:#x}\n   want {pow(xs[g_], 3, P2):#x}")
    print(f"m37 ({ab or 'default'}): 64 lanes, {bad} mismatches, {steps} wave-instructions emulated")
    return bad


def m37_digits_selftest(seed=1, ab=None, bits=1030):
    """wave 0 of fthe_padic_m37 on crafted digit pairs (LOADX raw digits; SQR 1; SQR 1; STOREP): the squaring's
    cross term at the extremes the kernel admits -- every limb < 2^28 and each digit < 5P, incl. digits whose
    low 36 limbs are all 2^28 - 1 (the largest Karatsuba half sums and column sums), zero halves, one-limb
    digits and random ones -- against (x0 + x1 P)^4 mod P^2 in Python integers"""
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, '..', 'fedtree_amd', 'csrc'))
    sys.path.insert(0, here)
    import importlib
    import gen_padic_mfma as gm
    saved = os.environ.get("FTHE_GEN_M37_AB")
    if ab is not None:
        os.environ["FTHE_GEN_M37_AB"] = ab
    try:
        gm = importlib.reload(gm)
        asm = gm.gen_padic_mfma('fthe_padic_m37')
    finally:
        if saved is None:
            os.environ.pop("FTHE_GEN_M37_AB", None)
        else:
            os.environ["FTHE_GEN_M37_AB"] = saved
        importlib.reload(gm)
    import padic_mfma_model as mm
    rng = random.Random(seed)
    P = rng.getrandbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
    P2 = P * P
    K, S, L, B = 37, 74, 256, 28
    MASK = (1 << B) - 1
    top = 5 * P - 1                                              # the largest digit
    allones = (1 << (B * (K - 1))) - 1                           # limbs 0..35 = 2^28 - 1
    big = allones + (((top - allones) >> (B * (K - 1))) << (B * (K - 1)))
    assert big <= top
    low19 = (1 << (B * 19)) - 1                                  # xL all ones, xH 0
    high18 = big - (big & low19)                                 # xL 0, xH max
    special = [big, 0, 1, low19, high18, top, P - 1, (1 << (B * 19)), MASK, big ^ (MASK << (B * 18))]
    pairs = [(a, b) for a in special for b in special][:40]
    while len(pairs) < 64:
        pairs.append((rng.randrange(5 * P), rng.randrange(5 * P)))
    nv = int(re.search(r'\.amdhsa_next_free_vgpr (\d+)', asm).group(1))
    lds_bytes = int(re.search(r'\.amdhsa_group_segment_fixed_size (\d+)', asm).group(1))
    ctx = bytearray(gm.TILE_OFF + gm.TILE_BYTES)
    for j in range(K):
        ctx[4 * j:4 * j + 4] = ((-((P >> (B * j)) & MASK)) & M32).to_bytes(4, 'little')
    img = mm.MfmaKey(P).tile_image()
    ctx[gm.TILE_OFF:gm.TILE_OFF + len(img)] = img
    IN, OUT = 0, 1
    slots = bytearray(2 * S * L * 4)
    for g_, (x0, x1) in enumerate(pairs):
        for k in range(K):
            for d, x in ((0, x0), (K, x1)):
                off = (IN * S + d + k) * L * 4 + 4 * g_
                slots[off:off + 4] = ((x >> (B * k)) & MASK).to_bytes(4, 'little')
    prog = [1, IN, 3, 2, 23, OUT, 0, 0]
    mem = Mem()
    SB, PB, CB, KA = 0x10000000, 0x20000000, 0x30000000, 0x40000000
    mem.alloc(slots, SB)
    mem.alloc(b''.join(w.to_bytes(4, 'little') for w in prog), PB)
    mem.alloc(bytes(ctx), CB)
    karg = SB.to_bytes(8, 'little') + PB.to_bytes(8, 'little') + CB.to_bytes(8, 'little') + \
        (L * 4).to_bytes(4, 'little') + (S * L * 4).to_bytes(4, 'little') + L.to_bytes(4, 'little') + \
        (1).to_bytes(4, 'little') + bytes(128)
    mem.alloc(karg, KA)
    steps = run_workgroup(asm, lds_bytes, 4, mem, KA, 0, nv, finish=(0,))
    bad = 0
    for g_, (x0, x1) in enumerate(pairs):
        got = 0
        for k in reversed(range(S)):
            got = (got << B) + mem.read(SB + (OUT * S + k) * L * 4 + 4 * g_, 4)
        want = pow(x0 + x1 * P, 4, P2)
        if not (got < 6 * P2 and got % P2 == want):
            bad += 1
            if bad <= 3:
                print(f"  lane {g_}: got {got:#x}\n   want {want:#x}")
    print(f"m37 digits ({ab or 'default'}): 64 lanes, {bad} mismatches, {steps} wave-instructions emulated")
    return bad


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'nadicb':
        sys.exit(1 if nadicb_selftest(waves=int(sys.argv[2]) if len(sys.argv) > 2 else 1) else 0)
    if len(sys.argv) > 1 and sys.argv[1] == 'm37':
        sys.exit(1 if m37_selftest(ab=sys.argv[2] if len(sys.argv) > 2 else None) else 0)
    elif len(sys.argv) > 1:                   # e.g. 211: wave 0 takes a second batch (the grid-stride loop)
        selftest(ntests=int(sys.argv[1]), count0=int(sys.argv[1]))
    else:
        selftest()
