#!/usr/bin/env python3
"""Dynamic instruction counts of fthe_addb_q152 by phase (the generator's `// @phase` markers), from one
emulated workgroup of tools/wave_emu.py: where a batch of 16 adds spends its wave-instructions."""
import collections
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'fedtree_amd', 'csrc'))
sys.path.insert(0, HERE)
import gen_addb as ga  # noqa: E402
import wave_emu  # noqa: E402


def phase_map(asm):
    phase, pcs, n = 'entry', [], 0
    for raw in asm.splitlines():
        if raw.startswith('// @phase'):
            phase = raw.split()[2]
        s = raw.split('//')[0].strip()
        if not s or s.startswith('.amdhsa_kernel') or s.startswith('.rodata'):
            if s:
                break
            continue
        if s.endswith(':') or s.startswith('.'):
            continue
        pcs.append(phase)
    return pcs


def main():
    asm = ga.gen_addb('fthe_addb_q152')
    pm = phase_map(asm)
    cnt = collections.defaultdict(collections.Counter)
    orig = wave_emu.Wave.step

    def step(self, op, a):
        kind = 'mfma' if 'mfma' in op else 'valu' if op.startswith('v_') else 'lds' if op.startswith('ds_') \
            else 'vmem' if op.startswith('global_') else 'salu'
        cnt[pm[self.pc - 1]][kind] += 1
        return orig(self, op, a)
    wave_emu.Wave.step = step
    wave_emu.selftest(ntests=16, count0=16)
    tot = collections.Counter()
    for c in cnt.values():
        tot.update(c)
    print(f"{'phase':10s} {'valu':>7s} {'mfma':>6s} {'lds':>6s} {'salu':>6s} {'vmem':>5s}   (2 batches)")
    for ph, c in cnt.items():
        print(f"{ph:10s} {c['valu']:7d} {c['mfma']:6d} {c['lds']:6d} {c['salu']:6d} {c['vmem']:5d}")
    print(f"{'total':10s} {tot['valu']:7d} {tot['mfma']:6d} {tot['lds']:6d} {tot['salu']:6d} {tot['vmem']:5d}")


if __name__ == '__main__':
    main()
