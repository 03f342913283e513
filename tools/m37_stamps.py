"""Wave timeline of fthe_padic_m37 launches from its stamp build (FTHE_GEN_M37_AB=stamp, a library built
elsewhere): each wave writes its start / end realtime (100 MHz ticks), HW_ID and XCC_ID (FTHE_STAMP_PTR, one
128 KiB area per launch).  For each full launch: its span, the wave lifetimes, and how well the SIMDs stayed
occupied (mean resident waves per SIMD over the span, against the 2 that 249 VGPRs allow; the tail after the
first SIMD ran dry).
  FTHE_LIB=tools/bin/libfthe_m37_stamp.so python tools/m37_stamps.py [pairs]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NL = 48


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    import numpy as np
    import torch
    buf = torch.zeros((NL, 32768), dtype=torch.int32, device="cuda")
    os.environ["FTHE_STAMP_PTR"] = hex(buf.data_ptr())
    os.environ["FTHE_STAMP_LAUNCHES"] = str(NL)
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    cw = 2 * pl.n_words
    m = torch.randint(0, 2**62, (2 * pairs,), dtype=torch.int64, device="cuda")
    c = torch.empty((2 * pairs, cw), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m, c, seed=1)
    dev.sync()
    rec = buf.cpu().numpy().view(np.uint32).reshape(NL, -1, 4)
    out = []
    for li in range(NL):
        r = rec[li]
        r = r[(r[:, 0] != 0) | (r[:, 1] != 0)]
        if len(r) < 1024:
            continue
        st = r[:, 0].astype(np.int64)
        en = r[:, 1].astype(np.int64)
        en = np.where(en < st, en + (1 << 32), en)
        t0 = st.min()
        st, en = st - t0, en - t0
        hw, xcc = r[:, 2], r[:, 3]
        simd = (xcc.astype(np.int64) << 16) | ((hw >> 8) & 0xff).astype(np.int64) << 2 | ((hw >> 4) & 3)
        span = int(en.max())
        life = en - st
        nsimd = len(np.unique(simd))
        occ = life.sum() / (span * nsimd)
        # per SIMD: when its last wave ended (the SIMD then idles until the launch ends)
        last = {}
        for s_, e_ in zip(simd, en):
            last[s_] = max(last.get(s_, 0), e_)
        lastv = np.array(sorted(last.values()))
        q = [0, 0.1, 0.5, 0.9, 1]
        out.append({"launch": li, "waves": int(len(r)), "simds": int(nsimd), "span_ms": round(span * 1e-5, 3),
                    "mean_waves_per_simd": round(float(occ), 3),
                    "wave_life_ms_q": [round(float(x) * 1e-5, 3) for x in np.quantile(life, q)],
                    "start_ms_q": [round(float(x) * 1e-5, 3) for x in np.quantile(st, q)],
                    "simd_last_end_ms_q": [round(float(x) * 1e-5, 3) for x in np.quantile(lastv, q)]})
    print(json.dumps({"pairs": pairs, "launches": out[:6], "n_full_launches": len(out)}), flush=True)


if __name__ == "__main__":
    main()
