"""Small-batch probe for PMC passes on the s80 four-lane kernel: 8,192 Paillier-2048 ciphertexts
encrypted (device randomness) and decrypted three times each -- every exponentiation runs on s80."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from fedtree_amd.paillier import Device, Paillier
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=20261015)
    n = 8192
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda")
    c = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    low = torch.empty_like(m)
    for i in range(3):
        pl.encrypt_u64_dev(m, c, seed=1 + i)
        pl.decrypt_u64_dev(c, low)
    dev.sync()
    assert torch.equal(low, m)
    print("s80 probe ok")


if __name__ == "__main__":
    main()
