"""Bit-exact pin of the headline encrypt path: the key holder's CRT encrypt with
device-drawn randomness (the "direct-y" path that bench.py times).

That path never forms r: it draws y_p in [1, p), y_q in [1, q) and computes
(1 + m n) y_P^P mod P^2.  The ciphertext is the reference's
encryption c = PowerMod(g, m, n^2) PowerMod(r, n, n^2) % n^2 (paillier.cpp:134-137)
under r = CRT(y_p^(q^-1 mod p-1) mod p, y_q^(p^-1 mod q-1) mod q), because
r^q = y_p (mod p) and x = y (mod P) implies x^P = y^P (mod P^2).  The test hook
fthe_debug_direct_y returns the drawn (y_p, y_q); r is rebuilt here and every
sampled ciphertext is compared with the C oracle's encrypt(m, r) -- the full
PowerMod formula, no CRT, no 1 + mn shortcut (oracle/paillier_oracle.c).

Covered: the four-lane small-batch path (<= 16,384 ciphertexts), the two-stream
split path (one chunk, <= 393,216), and the chunked large-batch path across its 786,432-lane
launch boundary (enc_chunk_lanes(), twice the engine's chunk).  Integer work: exact equality.
"""
import numpy as np
import pytest

import pyoracle

pytestmark = pytest.mark.gpu

SEED = 20261015
CHUNK = 393216                  # chunk_lanes() of the engine (fthe.hip)
ENC_CHUNK = 2 * CHUNK           # enc_chunk_lanes(): the large direct-y batches' launches


@pytest.fixture(scope="module")
def setup(coracle):
    from fedtree_amd.paillier import Device, Paillier, encode_fixed
    from fedtree_amd.synth import logistic_gradients
    dev = Device(0)
    pl = Paillier(dev).keygen(2048, seed=SEED)
    pw = (max(pl.p.bit_length(), pl.q.bit_length()) + 31) // 32
    ok = coracle.key(pyoracle.to_words(pl.p, pw), pyoracle.to_words(pl.q, pw))
    g, h = logistic_gradients(ENC_CHUNK // 2 + 4096, SEED)
    m = np.concatenate([encode_fixed(g), encode_fixed(h)])
    return dev, pl, ok, m


def _rebuild_r(pl, yp, yq):
    """r = CRT(y_p^(q^-1 mod p-1) mod p, y_q^(p^-1 mod q-1) mod q) mod n."""
    p, q, n = pl.p, pl.q, pl.modulus
    ep, eq = pow(q, -1, p - 1), pow(p, -1, q - 1)
    qinv = pow(q, -1, p)
    out = []
    for a, b in zip(pyoracle.words_to_ints(yp), pyoracle.words_to_ints(yq)):
        assert 0 < a < p and 0 < b < q
        rp, rq = pow(a, ep, p), pow(b, eq, q)
        out.append((rq + q * ((rp - rq) * qinv % p)) % n)
    return out


def _check(pl, ok, m, c, seed, idx):
    """Host rows c (the ciphertexts of indices idx, plaintexts m) against the oracle's
    encrypt(m, r) with r rebuilt from the draws of those indices."""
    idx = np.asarray(idx, dtype=np.int64)
    yps, yqs = [], []
    for lo, hi in _runs(idx):                          # the hook draws contiguous index ranges
        yp, yq = pl.direct_y(seed, lo, hi - lo)
        yps.append(yp)
        yqs.append(yq)
    yp, yq = np.concatenate(yps), np.concatenate(yqs)
    rs = _rebuild_r(pl, yp, yq)
    want = ok.encrypt_batch(m, pyoracle.ints_to_words(rs, pl.n_words))
    assert c.shape == want.shape
    bad = np.nonzero(~np.all(c == want, axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {len(idx)} ciphertexts differ, first at index {int(idx[bad[0]])}"


def _runs(idx):
    start = prev = int(idx[0])
    for x in idx[1:]:
        x = int(x)
        if x != prev + 1:
            yield start, prev + 1
            start = x
        prev = x
    yield start, prev + 1


def test_small_batch_quad_path(setup):
    dev, pl, ok, m = setup
    cnt = 1024                                         # four-lane s80 kernel, p and q on two streams
    c = pl.encrypt_u64(m[:cnt], seed=SEED + 1)
    _check(pl, ok, m[:cnt], c, SEED + 1, np.arange(cnt))


def test_split_path(setup):
    dev, pl, ok, m = setup
    cnt = 20000                                        # s74, q half on the side stream
    c = pl.encrypt_u64(m[:cnt], seed=SEED + 2)
    idx = np.concatenate([np.arange(0, 512), np.arange(cnt - 512, cnt)])
    _check(pl, ok, m[idx], c[idx], SEED + 2, idx)


def test_large_batch_across_chunk_boundary(setup):
    """The bench's call: device-resident m and c (fthe_encrypt_u64_dev), one full launch
    plus 4,096 more; 4,096 sampled ciphertexts on both sides of the boundary, 3,072 around the
    engine's chunk_lanes() (inside the first launch)."""
    import torch
    dev, pl, ok, m = setup
    cnt = ENC_CHUNK + 4096
    md = torch.from_numpy(m[:cnt].view(np.int64)).to("cuda:0")
    cd = torch.empty((cnt, 2 * pl.n_words), dtype=torch.int32, device="cuda:0")
    pl.encrypt_u64_dev(md, cd, seed=SEED + 3)
    dev.sync()
    idx = np.concatenate([np.arange(0, 512), np.arange(CHUNK - 1536, CHUNK + 1536),
                          np.arange(ENC_CHUNK - 1536, ENC_CHUNK + 1536), np.arange(cnt - 512, cnt)])
    c = cd[torch.from_numpy(idx).to("cuda:0")].cpu().numpy().view(np.uint32)
    _check(pl, ok, m[idx], c, SEED + 3, idx)
    # and the whole batch decrypts (CRT decrypt, the same key)
    low = torch.empty(cnt, dtype=torch.int64, device="cuda:0")
    pl.decrypt_u64_dev(cd, low)
    dev.sync()
    assert torch.equal(low, md)


def test_hook_matches_any_chunking(setup):
    """The draws are a function of the ciphertext index: one range or two give the same y."""
    dev, pl, ok, m = setup
    a = pl.direct_y(SEED + 9, 100, 300)
    b1 = pl.direct_y(SEED + 9, 100, 120)
    b2 = pl.direct_y(SEED + 9, 220, 180)
    assert np.array_equal(a[0], np.concatenate([b1[0], b2[0]]))
    assert np.array_equal(a[1], np.concatenate([b1[1], b2[1]]))
    assert not np.array_equal(pl.direct_y(SEED + 10, 100, 300)[0], a[0])
