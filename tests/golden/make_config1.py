"""Make tests/golden/config1_p1024.json: BASELINE.json configs[1] at full size --
Paillier-1024 encryption of 100k synthetic gradient pairs (200k ciphertexts)
with injected r, computed by the C/GMP restatement of paillier.cpp:122-139
(oracle/paillier_oracle.c, itself pinned to the reference's Paillier_GMP by
tests/golden/ref_gmp_L*.json).  Stored: the key's primes, digests of the
plaintexts and r (so a test can tell an input mismatch from an output one),
the SHA-256 of all ciphertexts (little-endian u32 words, row-major) and of
each 10k-row block, and the first ciphertexts in hex.

Inputs (all integer-exact, identical on every host):
  key   primes from oracle next_prime over numpy PCG64(seed) words (512-bit each)
  m     encode_fixed of fedtree_amd.synth.exact_gradients(100000, SEED): g then h
  r     config1_inputs() below: PCG64 words, top word masked below n, r[0] = 1, r[1] = n - 1

  python tests/golden/make_config1.py        (about 1 min on 8 cores)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SEED = 20261015
PAIRS = 100_000
NBITS = 1024
BLOCK = 10_000


def config1_key(coracle):
    rng = np.random.default_rng(SEED + NBITS)
    hw = NBITS // 64
    return [coracle.next_prime(rng.integers(0, 2**32, hw, dtype=np.uint64).astype(np.uint32)) for _ in range(2)]


def config1_inputs(n):
    """m (2*PAIRS u64) and r (2*PAIRS x n_words u32) for modulus n."""
    from fedtree_amd.paillier import encode_fixed
    from fedtree_amd.synth import exact_gradients
    g, h = exact_gradients(PAIRS, SEED)
    m = np.ascontiguousarray(np.concatenate([encode_fixed(g), encode_fixed(h)]))
    nw = (n.bit_length() + 31) // 32
    rng = np.random.default_rng(SEED + 1)
    r = rng.integers(0, 2**32, (len(m), nw), dtype=np.uint64).astype(np.uint32)
    top = (n >> (32 * (nw - 1))) & 0xFFFFFFFF
    r[:, -1] &= np.uint32((1 << (top.bit_length() - 1)) - 1)      # r < 2^(bits(n)-1) < n
    r[:, 0] |= np.uint32(1)                                         # r != 0
    import pyoracle
    r[0] = pyoracle.to_words(1, nw)
    r[1] = pyoracle.to_words(n - 1, nw)
    return m, r


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    import pyoracle
    o = pyoracle.COracle()
    pw, qw = config1_key(o)
    p, q = pyoracle.from_words(pw), pyoracle.from_words(qw)
    n = p * q
    m, r = config1_inputs(n)
    key = o.key(pw, qw)
    t0 = time.time()
    c = key.encrypt_batch(m, r, threads=os.cpu_count() or 1)
    dt = time.time() - t0
    out = {
        "what": "BASELINE configs[1]: Paillier-1024 encrypt of 100k gradient pairs, injected r, C/GMP oracle",
        "seed": SEED, "pairs": PAIRS, "n_bits": n.bit_length(), "p": hex(p), "q": hex(q),
        "m_sha256": digest(m), "r_sha256": digest(r), "ct_words": c.shape[1],
        "ct_sha256": digest(c), "block": BLOCK,
        "block_sha256": [digest(c[i:i + BLOCK]) for i in range(0, len(c), BLOCK)],
        "first_ct": [hex(pyoracle.from_words(c[i])) for i in range(4)],
        "oracle_seconds": round(dt, 1),
    }
    with open(os.path.join(HERE, "config1_p1024.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(c)} ciphertexts in {dt:.1f} s -> config1_p1024.json")


if __name__ == "__main__":
    main()
