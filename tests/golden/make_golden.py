#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ (run in the build container).

Ciphertext vectors come from the REFERENCE's own Paillier_GMP
(src/FedTree/Encryption/paillier_gmp.cpp), compiled from /root/reference by
oracle/Makefile into oracle/_ref/libpaillier_gmp_ref.so and called through
oracle/ref_shim.cpp:
  keyGen(L)  paillier_gmp.cpp:108-239   (deterministic: unseeded MT)
  encrypt    paillier_gmp.cpp:37-73     (the shared unseeded-MT r)
  decrypt    paillier_gmp.cpp:75-85
  add / mul  paillier_gmp.cpp:16-28
The codec vectors come from the reference's C expressions (common.h:81,127,142)
compiled with gcc in oracle/paillier_oracle.c.

Usage: python tests/golden/make_golden.py   (writes ref_gmp_L*.json, codec.json)
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

# gradient values of the reference's plaintext histogram KATs
# (src/test/test_tree_builder.cpp:52-117) plus logistic-loss-shaped values.
KAT_FLOATS = [0.4, 0.6, 1.2, 1.4, 0.1, 0.2, 0.8, 1.0, 0.7, 0.8, 0.21, 0.42, 0.63, 0.84, 1.05, 1.26,
              -0.4, -0.6, -0.123456, 0.999999, -0.999999, 1e-7, -1e-7, 0.25, 1e-16, 0.5, -0.5,
              0.7310586, -0.2689414, 0.19661193]


def hexs(words):
    return hex(pyoracle.from_words(words))


def main():
    ref = pyoracle.RefGMP()
    ora = pyoracle.COracle()
    lib = ref.lib
    f32 = np.array(KAT_FLOATS, dtype=np.float32)
    enc_gmp = np.zeros(len(f32), dtype=np.uint64)
    enc_ntl = np.zeros(len(f32), dtype=np.uint64)
    ora.lib.po_encode_fixed_gmp.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p]
    ora.lib.po_encode_fixed_ntl.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p]
    ora.lib.po_decode_fixed.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p]
    ora.lib.po_encode_fixed_gmp(f32.ctypes.data, len(f32), enc_gmp.ctypes.data)
    ora.lib.po_encode_fixed_ntl(f32.ctypes.data, len(f32), enc_ntl.ctypes.data)
    # decode of encodings, of sums of encodings (mod 2^64) and of edge values
    sums = [(int(enc_gmp[i]) + int(enc_gmp[(i + 1) % len(f32)])) % 2**64 for i in range(len(f32))]
    dec_in = np.array(list(enc_gmp) + sums + [0, 1, 2**64 - 1, 2**63 - 1, 2**63, 123456789012345678],
                      dtype=np.uint64)
    dec_out = np.zeros(len(dec_in), dtype=np.float32)
    ora.lib.po_decode_fixed(dec_in.ctypes.data, len(dec_in), dec_out.ctypes.data)
    codec = {"source": "common.h:81,127,142 compiled by gcc (oracle/paillier_oracle.c)",
             "floats_f32_bits": [int(x) for x in f32.view(np.uint32)],
             "encode_gmp": [int(x) for x in enc_gmp], "encode_ntl": [int(x) for x in enc_ntl],
             "decode_in": [int(x) for x in dec_in],
             "decode_out_f32_bits": [int(x) for x in dec_out.view(np.uint32)]}
    with open(os.path.join(HERE, "codec.json"), "w") as f:
        json.dump(codec, f, indent=0)

    for L in (1024, 2048, 4096):
        h = lib.ref_keygen(L)
        nw = lib.ref_n_words(h)
        arrs = [np.zeros(nw, dtype=np.uint32) for _ in range(5)]
        lib.ref_export(h, nw, *[a.ctypes.data for a in arrs])
        n, pm1, qm1, lam, mu = arrs
        r = np.zeros(nw, dtype=np.uint32)
        lib.ref_shared_r(h, nw, r.ctypes.data)
        rng = np.random.default_rng(L)
        ms = [0, 1, 2, 2**64 - 1, 2**63 - 1, 2**63, 2**32, 2**32 - 1] + [int(x) for x in enc_gmp[:12]] + \
             [int(x) for x in rng.integers(0, 2**64, 8, dtype=np.uint64)]
        cw = 2 * nw
        cases = []
        cts = []
        for m in ms:
            c = np.zeros(cw, dtype=np.uint32)
            lib.ref_encrypt(h, nw, ctypes.c_uint64(m), c.ctypes.data)
            d = np.zeros(nw, dtype=np.uint32)
            lib.ref_decrypt(h, nw, c.ctypes.data, d.ctypes.data)
            cases.append({"m": m, "c": hexs(c), "dec": hexs(d)})
            cts.append(c)
        adds, muls = [], []
        for i in range(len(cts) - 1):
            o = np.zeros(cw, dtype=np.uint32)
            lib.ref_add(h, nw, cts[i].ctypes.data, cts[i + 1].ctypes.data, o.ctypes.data)
            d = np.zeros(nw, dtype=np.uint32)
            lib.ref_decrypt(h, nw, o.ctypes.data, d.ctypes.data)
            adds.append({"i": i, "j": i + 1, "c": hexs(o), "dec": hexs(d)})
        for i, k in ((3, 2**64 - 1), (8, 2**64 - 1), (9, 2**64 - 1), (10, 3), (11, 1), (12, 0)):
            o = np.zeros(cw, dtype=np.uint32)
            lib.ref_mul(h, nw, cts[i].ctypes.data, ctypes.c_uint64(k), o.ctypes.data)
            d = np.zeros(nw, dtype=np.uint32)
            lib.ref_decrypt(h, nw, o.ctypes.data, d.ctypes.data)
            muls.append({"i": i, "k": k, "c": hexs(o), "dec": hexs(d)})
        s = cts[0].copy()
        lib.ref_add_aliased(h, nw, s.ctypes.data, cts[1].ctypes.data)
        # 8-party merge of a 3x4-bin histogram (hist_tree_builder.cpp:1015-1058):
        # dest starts unencrypted -> first add encrypts 0 (common.h:157-170)
        parties, bins = 8, 12
        hm = rng.integers(0, 2**64, (parties, bins), dtype=np.uint64)
        pc = np.zeros((parties, bins, cw), dtype=np.uint32)
        for pi in range(parties):
            for b in range(bins):
                lib.ref_encrypt(h, nw, ctypes.c_uint64(int(hm[pi, b])), pc[pi, b].ctypes.data)
        e0 = np.zeros(cw, dtype=np.uint32)
        lib.ref_encrypt(h, nw, ctypes.c_uint64(0), e0.ctypes.data)
        merged, mdec = [], []
        for b in range(bins):
            acc = e0.copy()
            for pi in range(parties):
                o = np.zeros(cw, dtype=np.uint32)
                lib.ref_add(h, nw, acc.ctypes.data, pc[pi, b].ctypes.data, o.ctypes.data)
                acc = o
            d = np.zeros(nw, dtype=np.uint32)
            lib.ref_decrypt(h, nw, acc.ctypes.data, d.ctypes.data)
            merged.append(hexs(acc))
            mdec.append(hexs(d))
        out = {
            "source": "reference Paillier_GMP (paillier_gmp.cpp) compiled from /root/reference",
            "key_length_arg": L, "n_words": nw, "n_bits": int(pyoracle.from_words(n)).bit_length(),
            "n": hexs(n), "p_minus_1": hexs(pm1), "q_minus_1": hexs(qm1), "lambda": hexs(lam), "mu": hexs(mu),
            "shared_r": hexs(r), "cases": cases, "adds": adds, "muls": muls,
            "aliased_add_result": hexs(s),
            "hist": {"parties": parties, "bins": bins, "m": [[int(x) for x in row] for row in hm],
                     "ct": [[hexs(pc[pi, b]) for b in range(bins)] for pi in range(parties)],
                     "enc_zero": hexs(e0), "merged": merged, "merged_dec": mdec},
        }
        with open(os.path.join(HERE, f"ref_gmp_L{L}.json"), "w") as f:
            json.dump(out, f, indent=0)
        lib.ref_free(h)
        print(f"L={L}: n_bits={out['n_bits']} cases={len(cases)}")


if __name__ == "__main__":
    main()
