"""Driver for a timeline of the host-resident encrypt (bench.py's e2e_host_encrypt_pinned_per_s): one warm
call, then fthe_encrypt_u64 of N gradient plaintexts from page-locked host memory into page-locked host rows,
then the device-resident encrypt and (mode dec) three device-resident CRT decrypts of the same N ciphertexts.
    rocprofv3 --kernel-trace --memory-copy-trace --stats -d DIR -- python3 tools/e2e_trace.py [N] [dec]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedtree_amd import _lib  # noqa: E402
from fedtree_amd.paillier import Device, Paillier  # noqa: E402


def main():
    ne = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    lib = dev.lib
    mh = np.random.default_rng(1).integers(0, 2**62, ne, dtype=np.int64).view(np.uint64)
    mp = torch.from_numpy(mh.copy()).pin_memory()
    cp = torch.empty((ne, 2 * pl.n_words), dtype=torch.int32).pin_memory()
    res = {"ciphertexts": ne}
    for rep in range(3):
        t0 = time.perf_counter()
        _lib.check(lib.fthe_encrypt_u64(pl._key, dev.ctx, ctypes.c_void_p(mp.data_ptr()), ne, None, 0, 3,
                                        ctypes.c_void_p(cp.data_ptr()), 0), "encrypt")
        res[f"host_to_host_s_{rep}"] = round(time.perf_counter() - t0, 4)
        res[f"kernel_ms_{rep}"] = round(dev.last_kernel_ms(), 2)
    md = torch.from_numpy(mh.copy()).cuda()
    cd = torch.empty((ne, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    for rep in range(2):
        dev.sync()
        t0 = time.perf_counter()
        pl.encrypt_u64_dev(md, cd, seed=3)
        dev.sync()
        res[f"device_s_{rep}"] = round(time.perf_counter() - t0, 4)
    res["same"] = bool(torch.equal(cd.cpu(), cp))
    if len(sys.argv) > 2 and sys.argv[2] == "dec":
        low = torch.empty(ne, dtype=torch.int64, device="cuda")
        for rep in range(3):
            dev.sync()
            t0 = time.perf_counter()
            pl.decrypt_u64_dev(cd, low)
            dev.sync()
            res[f"decrypt_device_s_{rep}"] = round(time.perf_counter() - t0, 4)
        res["decrypt_ok"] = bool(torch.equal(low.cpu(), torch.from_numpy(mh.view(np.int64))))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
