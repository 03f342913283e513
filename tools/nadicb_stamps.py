"""Per-phase wall cycles of fthe_nadic_b76 from its stamp build (FTHE_GEN_NADICB_DBG=stamp, a library built
elsewhere): each wave sums s_memtime deltas per phase (attributed at run time) over its batches of 16 public-key
encrypts and writes them through kernarg rows[15] (FTHE_STAMP_PTR, first launch only).  Prints one JSON line:
the mean cycles per batch per wave and phase, the clock, the spread of the waves' end times.
  FTHE_LIB=tools/bin/libfthe_nb_stamp.so python tools/nadicb_stamps.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fedtree_amd", "csrc"))
from gen_nadicb import STAMP_PHASES  # noqa: E402


def main():
    import numpy as np
    import torch
    buf = torch.zeros((1 << 18,), dtype=torch.int32, device="cuda")
    os.environ["FTHE_STAMP_PTR"] = hex(buf.data_ptr())
    os.environ["FTHE_STAMP_LAUNCHES"] = "1"
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=7)
    cnt = 98304
    m = torch.arange(cnt, dtype=torch.int64, device="cuda:0")
    c = torch.empty((cnt, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.encrypt_u64_dev(m, c, seed=1, public=True)
    dev.sync()
    ms = dev.last_kernel_ms()
    rec = buf.cpu().numpy().view(np.uint32)[:3072 * 16].reshape(-1, 16).astype(np.float64)
    npd = len(STAMP_PHASES)
    live = rec[rec[:, npd] > 0]
    b = live[:, npd]
    per = {ph: round(float(np.mean(live[:, i] / b)), 0) for i, ph in enumerate(STAMP_PHASES)}
    tot = live[:, :npd].sum(axis=1)
    rt0, rt1 = live[:, npd + 1], live[:, npd + 2]
    span = rt1 - rt0
    q = [0, 0.1, 0.5, 0.9, 1]
    out = {"ciphertexts": cnt, "call_ms": round(ms, 2), "waves": int(len(live)),
           "batches_per_wave_q": [int(x) for x in np.quantile(b, q)],
           "cycles_per_batch_per_wave": per, "total_per_batch": round(float(np.mean(tot / b)), 0),
           "clock_ghz": round(float(np.median(tot / span)) * 0.1, 3),
           "wave_span_ms_q": [round(float(x) * 1e-5, 2) for x in np.quantile(span, q)]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
