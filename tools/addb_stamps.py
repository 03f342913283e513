"""Per-phase wall cycles of fthe_addb_q152 from its stamp build (FTHE_GEN_ADDB_DBG=stamp, a library built
elsewhere; wrong results are not expected but not checked): each wave sums s_memtime deltas per phase and writes
them after the output rows.  Prints one JSON line: mean cycles per batch of 16 adds per wave and phase, the
launch's kernel time and the implied shader clock (wave cycles x batches per wave / time).
  FTHE_LIB=tools/bin/libfthe_a_stamp.so python tools/addb_stamps.py [n_adds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fedtree_amd", "csrc"))

PHASES = ['entry', 'load', 'product', 'window', 'q1stage', 'prod1', 'norm', 'q3stage', 'prod2', 'sub', 'canon',
          'store', 'loop']


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    import numpy as np
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    cw = 2 * pl.n_words
    m = torch.randint(0, 2**62, (2 * n,), dtype=torch.int64, device="cuda")
    c = torch.empty((2 * n, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    extra = (256 * 12 * 64 + 4 * cw - 1) // (4 * cw) + 1
    big = torch.zeros((n + extra, cw), dtype=torch.int32, device="cuda")
    out = big[:n]
    for _ in range(3):
        pl.add_dev(c[:n], c[n:], out)
    dev.sync()
    big[n:].zero_()
    pl.add_dev(c[:n], c[n:], out)
    dev.sync()
    ms = dev.last_kernel_ms()
    rec = big[n:].cpu().numpy().view(np.uint32).reshape(-1)[:256 * 12 * 16].reshape(-1, 16).astype(np.float64)
    live = rec[rec[:, 13] > 0]
    batches = live[:, 13]
    per = {ph: round(float(np.mean(live[:, i] / batches)), 1) for i, ph in enumerate(PHASES) if ph != 'entry'}
    start = live[:, 0] - live[:, 0].min()                      # realtime ticks (10 ns), first batch
    end = start + live[:, 15]
    q = [0, 0.01, 0.1, 0.5, 0.9, 0.99, 1]
    dist = {"start_us": [round(float(x) * 0.01, 2) for x in np.quantile(start, q)],
            "end_us": [round(float(x) * 0.01, 2) for x in np.quantile(end, q)],
            "batches": [int(x) for x in np.quantile(batches, q)],
            "us_per_batch": [round(float(x) * 0.01, 2) for x in np.quantile(live[:, 15] / batches, q)]}
    wave_cycles = live[:, 1:13].sum(axis=1)
    res = {"adds": n, "waves": int(len(live)), "batches_per_wave_mean": round(float(batches.mean()), 2),
           "kernel_ms": round(ms, 4), "cycles_per_batch_per_wave": per,
           "wave_cycles_per_batch": round(float(np.mean(wave_cycles / batches)), 1), "quantiles": q, **dist,
           "implied_clock_ghz": round(float(np.median(wave_cycles)) / (ms * 1e-3) / 1e9, 3),
           "memtime_over_realtime_ghz": round(float(np.median(live[:, 14] / live[:, 15])) * 0.1, 3),
           "wave_realtime_ms_max": round(float(live[:, 15].max()) * 1e-5, 4)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
