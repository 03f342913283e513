"""Kernel-trace driver: exact fixed-base encrypt (known-order key, one generator) of
n Paillier-2048 ciphertexts, device-resident, after one warm-up call.
  rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 tools/prof_fb.py [n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1572864
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261016, known_order=True)
    pl.set_fixed_base_exact(seed=0)
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
    c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(m[:4096], c[:4096], seed=1, fixed_base_exact=True)
    dev.sync()
    pl.encrypt_u64_dev(m, c, seed=2, fixed_base_exact=True)
    dev.sync()
    print("exact known-order", n, "ms", dev.last_kernel_ms(), "rate", n / dev.last_kernel_ms() * 1e3)


if __name__ == "__main__":
    main()
