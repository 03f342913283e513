"""Small-batch latency paths: decrypts (paillier.cpp:141-157) and device-randomness
CRT encrypts (paillier.cpp:122-139) of at most one chunk (393,216 lanes) run the mod-q half on
the context's side stream, in a second slot region, beside the mod-p half; decrypts
of at most 16,384 ciphertexts of a Paillier-2048 key run both halves on the
four-lane s80 kernel (one quad of lanes per exponentiation).

The split must not change a single bit: the same seeded batch encrypted as a
large (one-stream) call and as small (two-stream) calls gives identical
ciphertexts, every one decrypts to its plaintext through both decrypt forms,
and the full plaintexts agree with the C oracle's decryption.
"""
import numpy as np
import pytest

import pyoracle
from conftest import golden_key, load_golden

pytestmark = pytest.mark.gpu

SPLIT_MAX = 393216    # dec_split_lanes() default = chunk_lanes() (one lane per ciphertext at P-1024, P-2048)
QUAD_MAX = 16384      # dec_quad_max() default


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


@pytest.mark.parametrize("name", ["ref_gmp_L2048.json", "ref_gmp_L1024.json"])
def test_split_matches_single_stream(dev, name):
    from fedtree_amd.paillier import Paillier
    g = load_golden(name)
    p, q = golden_key(g)
    pl = Paillier.from_primes(p, q, dev)
    rng = np.random.default_rng(11)
    big = SPLIT_MAX + 1000                       # above the threshold: one stream
    m = rng.integers(0, 2**64, big, dtype=np.uint64)
    m[:4] = [0, 1, 2**64 - 1, 2**63]
    c_big = pl.encrypt_u64(m, seed=77)
    for cnt in (1, 2, 3, 1000, QUAD_MAX, QUAD_MAX + 1, 20000, 200000):   # below: two streams (and s80 decrypts)
        c_small = pl.encrypt_u64(m[:cnt], seed=77)
        assert np.array_equal(c_small, c_big[:cnt]), cnt
        lo, full = pl.decrypt_u64(c_big[:cnt], full=True)
        assert np.array_equal(lo, m[:cnt]), cnt
        assert [pyoracle.from_words(w) for w in full] == [int(x) for x in m[:cnt]]
    assert np.array_equal(pl.decrypt_u64(c_big), m)
    # decrypt side: a small batch of sums (plaintexts need the full CRT) equals the large-call result
    s = pl.add_batch(c_big[:2048], c_big[2048:4096])
    want = (m[:2048] + m[2048:4096])               # mod 2^64
    _, f_small = pl.decrypt_u64(s, full=True)
    assert np.array_equal(pl.decrypt_u64(s), want)
    key = pyoracle.keygen_from_primes(p, q)
    ints = pyoracle.words_to_ints(s[:8])
    assert [pyoracle.from_words(w) for w in f_small[:8]] == [pyoracle.decrypt(key, x) for x in ints]


def test_split_injected_r_golden(dev):
    """Injected r keeps the two-stage single-stream encrypt; the split decrypt returns the
    reference's plaintexts on its golden ciphertexts (all P-2048 cases in one small call
    and one at a time)."""
    from fedtree_amd.paillier import Paillier
    g = load_golden("ref_gmp_L2048.json")
    p, q = golden_key(g)
    pl = Paillier.from_primes(p, q, dev)
    cts = pyoracle.ints_to_words([int(c["c"], 16) for c in g["cases"]], 2 * g["n_words"])
    want = np.array([c["m"] for c in g["cases"]], dtype=np.uint64)
    assert np.array_equal(pl.decrypt_u64(cts), want)
    for i in range(3):
        assert pl.decrypt_u64(cts[i:i + 1])[0] == want[i]


_SPLIT_ALL_PROBE = r'''
import hashlib, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from conftest import golden_key, load_golden
from fedtree_amd.paillier import Device, Paillier
p, q = golden_key(load_golden("ref_gmp_L2048.json"))
pl = Paillier.from_primes(p, q, Device(0))
n = int(sys.argv[2])
m = np.random.default_rng(5).integers(0, 2**64, n, dtype=np.uint64)
c = pl.encrypt_u64(m, seed=91)                       # host rows (the staged path)
ok = bool(np.array_equal(pl.decrypt_u64(c), m))
md = torch.from_numpy(m.view(np.int64)).cuda()       # device-resident (the bench's path: chunks pipelined)
cd = torch.empty((n, 2 * pl.n_words), dtype=torch.int32, device="cuda")
pl.encrypt_u64_dev(md, cd, seed=91)
pl.dev.sync()
cdh = cd.cpu().numpy().view(np.uint32)
low = torch.empty(n, dtype=torch.int64, device="cuda")
pl.decrypt_u64_dev(cd, low)
pl.dev.sync()
ok = ok and bool(np.array_equal(low.cpu().numpy().view(np.uint64), m))
print(hashlib.sha256(c.tobytes()).hexdigest(), hashlib.sha256(cdh.tobytes()).hexdigest(), ok)
'''


def test_split_all_large_calls_bit_identical(tmp_path):
    """Large CRT encrypts and decrypts run each chunk's p and q halves side by side on two streams (fthe.hip
    split_all, the default), and under FTHE_ENC_PIPE=1 device-resident encrypts pipeline the chunks over two
    slot-region pairs (enc_pipe, opt-in); FTHE_SPLIT_ALL=0 runs the halves in turn on one stream.
    Three chunks of 786,432 lanes and a partial fourth, host rows and device rows: the seeded ciphertexts are
    byte-identical all three ways (and host = device) and decrypt to their plaintexts."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    probe = tmp_path / "probe.py"
    probe.write_text(_SPLIT_ALL_PROBE)
    outs = []
    for split, piped in (("0", "0"), ("1", "0"), ("1", "1")):
        r = subprocess.run([sys.executable, str(probe), root, str(3 * 786432 + 5000)], capture_output=True, text=True,
                           timeout=600, env=dict(os.environ, FTHE_SPLIT_ALL=split, FTHE_ENC_PIPE=piped))
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(r.stdout.split())
    for o in outs:
        assert o[2] == "True"
        assert o[0] == o[1]                               # host rows = device rows
    assert outs[0][0] == outs[1][0] == outs[2][0]


def test_mem_limit_one_region_fallback():
    """the two-stream form of a large CRT encrypt / decrypt needs a second slot region; when the
    context's cap (fthe_ctx_set_mem_limit, standing in for a full device) cannot hold it, the call takes the
    one-region form instead of failing.  Caps falling by 0.8x from 16 GB down to the first that cannot hold even
    one region: every call above it returns the uncapped call's ciphertexts and plaintexts; the cap just above
    the failure is < 2x the one-region size, so that call ran the fallback; the failing cap reports NOMEM."""
    from fedtree_amd import _lib
    from fedtree_amd.paillier import Device, Paillier
    g = load_golden("ref_gmp_L2048.json")
    p, q = golden_key(g)
    n = SPLIT_MAX + 6789                          # above the small split: the large (split_all) form
    m = np.random.default_rng(21).integers(0, 2**64, n, dtype=np.uint64)
    want = Paillier.from_primes(p, q, Device(0)).encrypt_u64(m, seed=404)
    cap, ok_caps, failed = 16 << 30, [], None
    while cap > (64 << 20):
        d = Device(0)
        d.set_mem_limit(cap)
        pl = Paillier.from_primes(p, q, d)
        try:
            c = pl.encrypt_u64(m, seed=404)
        except _lib.FtheError as ex:
            assert ex.status == _lib.FTHE_ERR_NOMEM, ex
            failed = cap
            break
        assert np.array_equal(c, want), cap
        assert np.array_equal(pl.decrypt_u64(c), m), cap
        ok_caps.append(cap)
        cap = int(cap * 0.8)
    assert failed is not None and ok_caps and ok_caps[-1] < 2 * failed, (ok_caps, failed)
