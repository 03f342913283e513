#!/usr/bin/env python3
"""Dynamic instruction counts of fthe_nadic_b76 by phase (the generator's `// @phase` markers), from one emulated
wave (tools/wave_emu.py nadicb_selftest: LOADX; CANON; 2 SQR; 2 MUL; CANON; STOREX on 16 ciphertexts): where a
product's wave-instructions go."""
import collections
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'fedtree_amd', 'csrc'))
sys.path.insert(0, HERE)
import gen_nadicb as gb  # noqa: E402
import wave_emu  # noqa: E402
from addb_phases import phase_map  # noqa: E402


def main():
    pm = phase_map(gb.gen_nadicb('fthe_nadic_b76', waves=1))
    cnt = collections.defaultdict(collections.Counter)
    orig = wave_emu.Wave.step

    def step(self, op, a):
        kind = 'mfma' if 'mfma' in op else 'valu' if op.startswith('v_') else 'lds' if op.startswith("ds_") \
            else 'vmem' if op.startswith('global_') else 'salu'
        cnt[pm[self.pc - 1]][kind] += 1
        return orig(self, op, a)
    wave_emu.Wave.step = step
    wave_emu.nadicb_selftest(seed=3, waves=1, batches=1)
    tot = collections.Counter()
    for c in cnt.values():
        tot.update(c)
    print(f"{'phase':10s} {'valu':>7s} {'mfma':>6s} {'lds':>6s} {'salu':>6s} {'vmem':>5s}   (4 products: 2 SQR, 2 MUL)")
    for ph, c in cnt.items():
        print(f"{ph:10s} {c['valu']:7d} {c['mfma']:6d} {c['lds']:6d} {c['salu']:6d} {c['vmem']:5d}")
    print(f"{'total':10s} {tot['valu']:7d} {tot['mfma']:6d} {tot['lds']:6d} {tot['salu']:6d} {tot['vmem']:5d}")


if __name__ == '__main__':
    main()
