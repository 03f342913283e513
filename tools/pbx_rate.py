"""Party-side (public key) encrypt rates, device-resident: the default public formula
(per-ciphertext r^n mod n^2), the public exact fixed-base mode (published bases,
FTHE_ENC_FIXED_BASE_EXACT on a public key) and the subgroup fixed-base mode, at
Paillier-2048 (four-lane row kernel) and Paillier-1024 (one-lane n^2 kernel); one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rates(dev, bits, n, known_order=False):
    import torch
    from fedtree_amd.paillier import Paillier
    srv = Paillier(dev).keygen(bits, seed=20261015 + bits, known_order=known_order)
    t0 = time.perf_counter()
    hs = srv.public_bases()
    out = {"bases": len(hs), "bases_pick_s": round(time.perf_counter() - t0, 3)}
    t0 = time.perf_counter()
    party = srv.public(bases=hs)
    dev.sync()
    out["table_build_s"] = round(time.perf_counter() - t0, 3)
    m = torch.randint(0, 2**62, (n,), dtype=torch.int64, device="cuda:0")
    c = torch.empty((n, 2 * party.n_words), dtype=torch.int32, device="cuda:0")
    modes = [("public_exact", dict(fixed_base_exact=True))]
    if not known_order:
        modes += [("public_default", {}), ("public_fixed_base", dict(fixed_base=True))]
    for name, kw in modes:
        cnt = n if name != "public_default" else n // 4
        party.encrypt_u64_dev(m[:4096], c[:4096], seed=1, **kw)
        dev.sync()
        party.encrypt_u64_dev(m[:cnt], c[:cnt], seed=2, **kw)
        dev.sync()
        out[name + "_per_s"] = round(cnt / (dev.last_kernel_ms() * 1e-3))
        low = torch.empty_like(m[:cnt])
        srv.decrypt_u64_dev(c[:cnt], low)
        dev.sync()
        out[name + "_roundtrip_ok"] = bool(torch.equal(low, m[:cnt]))
    del party, srv
    torch.cuda.empty_cache()
    return out


def main():
    from fedtree_amd.paillier import Device
    dev = Device(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    res = {"ciphertexts": n}
    for bits, ko in ((2048, False), (2048, True), (1024, False)):
        res[f"p{bits}" + ("_known_order" if ko else "")] = rates(dev, bits, n, ko)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
