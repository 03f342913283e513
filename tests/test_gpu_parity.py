"""Parity of the HIP engine (libfthe.so, through the C ABI) with the oracle.

* golden vectors of the reference's own Paillier_GMP (tests/golden/), bit-exact;
* seeded random keys / messages / r against the C oracle, bit-exact;
* full-size properties (encrypt -> decrypt round trips across chunk
  boundaries, homomorphic sums, scalar-multiplication linearity).
Integer work: every comparison is exact.
"""
import ctypes

import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN_KEYS, golden_key, load_golden
from fedtree_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from fedtree_amd.paillier import Device
    return Device(0)


@pytest.fixture(scope="module", params=GOLDEN_KEYS)
def gold(request):
    return load_golden(request.param)


def _pl(dev, p, q):
    from fedtree_amd.paillier import Paillier
    return Paillier.from_primes(p, q, dev)


def _cts(gold):
    return pyoracle.ints_to_words([int(c["c"], 16) for c in gold["cases"]], 2 * gold["n_words"])


def _public_supported(pl):
    return pl.lib.fthe_kernel_limbs(2 * pl.keyLength) != 0


# ---------------------------------------------------------------- golden vectors
def test_golden_key(dev, gold):
    p, q = golden_key(gold)
    pl = _pl(dev, p, q)
    assert pl.modulus == int(gold["n"], 16)
    assert pl.lambda_ == int(gold["lambda"], 16)
    assert pl.u == int(gold["mu"], 16)
    assert pl.n_words == gold["n_words"]


def test_golden_encrypt_crt(dev, gold):
    p, q = golden_key(gold)
    pl = _pl(dev, p, q)
    ms = np.array([c["m"] for c in gold["cases"]], dtype=np.uint64)
    r = np.tile(pyoracle.to_words(int(gold["shared_r"], 16), pl.n_words), (len(ms), 1))
    assert np.array_equal(pl.encrypt_u64(ms, r=r), _cts(gold))


def test_golden_encrypt_public(dev, gold):
    p, q = golden_key(gold)
    pl = _pl(dev, p, q)
    ms = np.array([c["m"] for c in gold["cases"]], dtype=np.uint64)
    r = np.tile(pyoracle.to_words(int(gold["shared_r"], 16), pl.n_words), (len(ms), 1))
    if not _public_supported(pl):
        with pytest.raises(_lib.FtheError) as e:
            pl.encrypt_u64(ms, r=r, public=True)
        assert e.value.status == _lib.FTHE_ERR_UNSUPPORTED
        return
    assert np.array_equal(pl.encrypt_u64(ms, r=r, public=True), _cts(gold))
    # a public-key-only copy (Paillier::operator=) encrypts identically
    pub = pl.public()
    assert not pub.has_private
    assert np.array_equal(pub.encrypt_u64(ms, r=r), _cts(gold))


def test_golden_decrypt(dev, gold):
    p, q = golden_key(gold)
    pl = _pl(dev, p, q)
    low, full = pl.decrypt_u64(_cts(gold), full=True)
    assert [int(x) for x in low] == [c["m"] % 2**64 for c in gold["cases"]]
    assert [pyoracle.from_words(f) for f in full] == [int(c["dec"], 16) for c in gold["cases"]]
    # decrypts of the reference's homomorphic results
    adds = pyoracle.ints_to_words([int(a["c"], 16) for a in gold["adds"]], 2 * pl.n_words)
    _, full = pl.decrypt_u64(adds, full=True)
    assert [pyoracle.from_words(f) for f in full] == [int(a["dec"], 16) for a in gold["adds"]]


def test_golden_add_mul(dev, gold):
    p, q = golden_key(gold)
    pl = _pl(dev, p, q)
    cts = _cts(gold)
    a_idx = [a["i"] for a in gold["adds"]]
    b_idx = [a["j"] for a in gold["adds"]]
    if not _public_supported(pl):
        with pytest.raises(_lib.FtheError):
            pl.add_batch(cts[a_idx], cts[b_idx])
        return
    out = pl.add_batch(cts[a_idx], cts[b_idx])
    assert [pyoracle.from_words(x) for x in out] == [int(a["c"], 16) for a in gold["adds"]]
    for m in gold["muls"]:
        got = pl.scalar_mul(cts[m["i"]][None], m["k"])
        assert pyoracle.from_words(got[0]) == int(m["c"], 16), m["k"]


def test_golden_hist_merge(dev, gold):
    """k-party merge with the reference's encrypt(0)-first semantics."""
    p, q = golden_key(gold)
    pl = _pl(dev, p, q)
    h = gold["hist"]
    cw = 2 * pl.n_words
    if not _public_supported(pl):
        pytest.skip("mod n^2 products at 4096 bits: round-2 kernel")
    stack = [np.tile(pyoracle.to_words(int(h["enc_zero"], 16), cw), (h["bins"], 1))]
    for pi in range(h["parties"]):
        stack.append(pyoracle.ints_to_words([int(x, 16) for x in h["ct"][pi]], cw))
    out = pl.reduce_kway(np.stack(stack))
    assert [pyoracle.from_words(x) for x in out] == [int(x, 16) for x in h["merged"]]
    low = pl.decrypt_u64(out)
    assert [int(x) for x in low] == [sum(h["m"][pi][b] for pi in range(h["parties"])) % 2**64
                                     for b in range(h["bins"])]


# ---------------------------------------------------------------- seeded random vs C oracle
def _det_primes(coracle, nbits, seed):
    rng = np.random.default_rng(seed)
    hw = nbits // 64
    return [coracle.next_prime(rng.integers(0, 2**32, hw, dtype=np.uint64).astype(np.uint32)) for _ in range(2)]


@pytest.mark.parametrize("nbits", [512, 1024, 2048])
def test_random_vs_c_oracle(dev, coracle, nbits):
    pw, qw = _det_primes(coracle, nbits, 20261015 + nbits)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    ok = coracle.key(pw, qw)
    n = pl.modulus
    rng = np.random.default_rng(nbits + 1)
    cnt = 777
    m = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    m[:5] = [0, 1, 2**64 - 1, 2**63 - 1, 2**63]
    rs = [int.from_bytes(rng.bytes(pl.n_words * 4), "little") % (n - 1) + 1 for _ in range(cnt)]
    rs[0], rs[1] = 1, n - 1
    r = pyoracle.ints_to_words(rs, pl.n_words)
    want = ok.encrypt_batch(m, r)
    assert np.array_equal(pl.encrypt_u64(m, r=r), want)
    if _public_supported(pl):
        assert np.array_equal(pl.encrypt_u64(m, r=r, public=True), want)
    low, full = pl.decrypt_u64(want, full=True)
    assert np.array_equal(low, m)
    assert np.array_equal(full, ok.decrypt_batch(want))


# ---------------------------------------------------------------- full-size properties
def test_p2048_roundtrip_across_chunks(dev, coracle):
    """Device CSPRNG r, count crossing the 262144-lane chunk boundary."""
    pw, qw = _det_primes(coracle, 2048, 7)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    cnt = 262144 + 777
    m = np.random.default_rng(3).integers(0, 2**64, cnt, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=11)
    assert np.array_equal(pl.decrypt_u64(c), m)
    # ciphertexts are fresh (no shared r): no two equal
    assert len({bytes(c[i]) for i in range(0, cnt, 997)}) == len(range(0, cnt, 997))
    # independent check of a sample by the C oracle
    ok = coracle.key(pw, qw)
    idx = np.arange(0, cnt, cnt // 40)
    dec = ok.decrypt_batch(c[idx])
    assert [pyoracle.from_words(d) for d in dec] == [int(x) for x in m[idx]]
    # same seed -> same ciphertexts; different seed -> different
    c2 = pl.encrypt_u64(m[:1000], seed=11)
    assert np.array_equal(c2, c[:1000])
    c3 = pl.encrypt_u64(m[:1000], seed=12)
    assert not np.array_equal(c3, c[:1000])


def test_homomorphic_sum_and_scalar(dev, coracle):
    pw, qw = _det_primes(coracle, 1024, 9)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    k, cnt = 8, 4099
    m = np.random.default_rng(5).integers(0, 2**64, (k, cnt), dtype=np.uint64)
    c = pl.encrypt_u64(m.reshape(-1), seed=1).reshape(k, cnt, -1)
    s = pl.reduce_kway(c)
    want = np.zeros(cnt, dtype=np.uint64)
    for j in range(k):
        want = want + m[j]            # wraps mod 2^64 == low 64 bits of the sum
    assert np.array_equal(pl.decrypt_u64(s), want)
    # subtraction through scalar mul by 2^64-1 (common.h:311-317)
    neg = pl.scalar_mul(c[1], 2**64 - 1)
    d = pl.add_batch(c[0], neg)
    assert np.array_equal(pl.decrypt_u64(d), m[0] - m[1])
    # linearity c^k -> k m
    t = pl.scalar_mul(c[2], 12345)
    assert np.array_equal(pl.decrypt_u64(t), m[2] * np.uint64(12345))
    # alias safety: out == a through the device API
    import torch
    ta = torch.from_numpy(c[0].copy()).cuda()
    tb = torch.from_numpy(c[1].copy()).cuda()
    pl.add_dev(ta, tb, ta)
    pl.dev.sync()
    assert np.array_equal(pl.decrypt_u64(ta.cpu().numpy()), m[0] + m[1])


@pytest.mark.parametrize("cnt", [0, 1, 255, 257])
def test_edge_counts(dev, coracle, cnt):
    pw, qw = _det_primes(coracle, 1024, 13)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    m = np.arange(cnt, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    c = pl.encrypt_u64(m, seed=3)
    assert c.shape == (cnt, 2 * pl.n_words)
    assert np.array_equal(pl.decrypt_u64(c), m)
    assert pl.add_batch(c, c).shape == c.shape


def test_device_codec_and_dev_api(dev, coracle):
    import torch
    from fedtree_amd.paillier import decode_fixed, encode_fixed
    g = load_golden("codec.json")
    f = np.array(g["floats_f32_bits"], dtype=np.uint32).view(np.float32)
    rng = np.random.default_rng(0)
    f = np.concatenate([f, rng.normal(size=5000).astype(np.float32), rng.uniform(-1, 1, 5000).astype(np.float32)])
    lib = dev.lib
    tf = torch.from_numpy(f).cuda()
    tm = torch.zeros(len(f), dtype=torch.int64, device="cuda")
    dev.order_in()                   # direct C-ABI calls: order after torch's fills and copies
    _lib.check(lib.fthe_encode_fixed_dev(dev.ctx, ctypes.c_void_p(tf.data_ptr()), len(f),
                                         ctypes.c_void_p(tm.data_ptr())))
    dev.sync()
    m = tm.cpu().numpy().view(np.uint64)
    assert np.array_equal(m, encode_fixed(f))
    din = np.array(g["decode_in"], dtype=np.uint64)
    allin = np.concatenate([din, m])
    tin = torch.from_numpy(allin.view(np.int64)).cuda()
    tout = torch.zeros(len(allin), dtype=torch.float32, device="cuda")
    dev.order_in()
    _lib.check(lib.fthe_decode_fixed_dev(dev.ctx, ctypes.c_void_p(tin.data_ptr()), len(allin),
                                         ctypes.c_void_p(tout.data_ptr())))
    dev.sync()
    assert np.array_equal(tout.cpu().numpy().view(np.uint32), decode_fixed(allin).view(np.uint32))
    # device-resident encrypt/decrypt through torch buffers
    pw, qw = _det_primes(coracle, 2048, 21)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    tc = torch.zeros((len(m), 2 * pl.n_words), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(tm, tc, seed=5)
    tl = torch.zeros(len(m), dtype=torch.int64, device="cuda")
    pl.decrypt_u64_dev(tc, tl)
    dev.sync()
    assert np.array_equal(tl.cpu().numpy().view(np.uint64), m)
    host = pl.encrypt_u64(m, seed=5)
    assert np.array_equal(tc.cpu().numpy().view(np.uint32), host)


def test_keygen(dev):
    from fedtree_amd.paillier import Paillier
    a = Paillier(dev).keygen(2048, seed=42)
    b = Paillier(dev).keygen(2048, seed=42)
    c = Paillier(dev).keygen(2048, seed=43)
    assert a.keyLength == 2048 and a.modulus == b.modulus != c.modulus
    assert a.p * a.q == a.modulus
    m = np.arange(1000, dtype=np.uint64) * np.uint64(2**40 + 7)
    assert np.array_equal(a.decrypt_u64(a.encrypt_u64(m)), m)
    # reference single-value signatures
    x = a.encrypt(123456789)
    assert a.decrypt(x) == 123456789
    assert 0 < x < a.modulus ** 2


def test_ghpair_server_party_flow(dev):
    """Server/Party HE flow on the reference's histogram KAT values
    (test_tree_builder.cpp:52-91): decrypt(sum of encrypted) == plaintext sum
    within the 1e-6 fixed-point quantum."""
    from fedtree_amd.paillier import GHPairs, HEParty, HEServer
    srv = HEServer(dev)
    srv.homo_init(1024, seed=1)
    party = HEParty()
    srv.send_key(party)
    assert not party.paillier.has_private
    g = np.array([0.4, 1.2, 0.1, 0.8, 0.7], np.float32)
    h = np.array([0.6, 1.4, 0.2, 1.0, 0.8], np.float32)
    a = srv.encrypt_gh_pairs(GHPairs(g, h))
    assert a.encrypted and not a.g.any()
    b = party.encrypt_histogram(GHPairs(g * 2, h * 2))
    s = a + b                                   # homomorphic
    z = GHPairs(np.zeros(5, np.float32)) + a    # unencrypted lhs: fresh encrypt(0) first (Q10)
    d = s - a                                   # subtraction via x^(2^64-1)
    srv.decrypt_gh_pairs(s)
    srv.decrypt_gh_pairs(z)
    srv.decrypt_gh_pairs(d)
    np.testing.assert_allclose(s.g, 3 * g, atol=3e-6)
    np.testing.assert_allclose(s.h, 3 * h, atol=3e-6)
    np.testing.assert_allclose(z.g, g, atol=2e-6)
    np.testing.assert_allclose(d.g, 2 * g, atol=3e-6)


def test_sharded_two_contexts(dev, coracle):
    """ShardedPaillier on two engine contexts (here both on cuda:0): threads x streams,
    contiguous shards, results identical to the single-context call."""
    from fedtree_amd.multi import ShardedPaillier
    from fedtree_amd.paillier import Device
    pw, qw = _det_primes(coracle, 1024, 31)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    sp = ShardedPaillier(pl, [Device(0), Device(0)])
    m = np.random.default_rng(8).integers(0, 2**64, 10_001, dtype=np.uint64)
    c = sp.encrypt_u64(m, seed=4)
    assert c.shape == (len(m), 2 * pl.n_words)
    # a seeded batch draws per position (fthe_encrypt_u64_at): the shards give the one-context ciphertexts
    assert np.array_equal(c, pl.encrypt_u64(m, seed=4))
    assert np.array_equal(sp.encrypt_u64(m[:999], seed=4, public=True), pl.encrypt_u64(m[:999], seed=4, public=True))
    assert np.array_equal(sp.decrypt_u64(c), m)
    assert np.array_equal(pl.decrypt_u64(c), m)
    s = sp.add_batch(c, c[::-1].copy())
    assert np.array_equal(s, pl.add_batch(c, c[::-1].copy()))
    assert np.array_equal(sp.sub_batch(c[:500], c[500:1000]), pl.sub_batch(c[:500], c[500:1000]))
    assert np.array_equal(sp.scalar_mul(c[:300], 12345), pl.scalar_mul(c[:300], 12345))
    assert np.array_equal(sp.decrypt_u64(c, short=True), m)
    # the N-to-1 root sum (tree.cpp:20-34): per-context partial products, combined on one context = one product
    root = sp.sum(c)
    assert np.array_equal(root, pl.reduce_segments(c, np.array([0, len(c)]))[0])
    assert int(pl.decrypt_u64(root[None, :])[0]) == int(m.sum(dtype=np.uint64))
    # parties: public-key copies with published bases on every context
    pub = ShardedPaillier(pl.public(), [Device(0), Device(0)], bases=pl.public_bases(seed=2))
    cp = pub.encrypt_u64(m, seed=6, fixed_base_exact=True)
    assert np.array_equal(pl.decrypt_u64(cp), m)
    assert np.array_equal(pub.encrypt_u64(m, seed=6, fixed_base_exact=True), cp)
    one = pl.public()
    one.set_public_bases(pl.public_bases(seed=2))
    assert np.array_equal(one.encrypt_u64(m, seed=6, fixed_base_exact=True), cp)


# ---------------------------------------------------------------- segmented product / histogram
@pytest.mark.parametrize("nbits", [1024, 2048])
def test_reduce_segments_vs_oracle(dev, coracle, nbits):
    """Ragged segments (empty, singletons, one multi-pass segment of 700), a
    gather index with repeats, bit-exact against the oracle's fold of add."""
    pw, qw = _det_primes(coracle, nbits, 31 + nbits)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    key = pyoracle.keygen_from_primes(pl.p, pl.q)
    rng = np.random.default_rng(nbits)
    cnt = 1200
    m = rng.integers(0, 2**50, cnt, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=5)
    lens = np.concatenate([[0, 1, 0, 700, 9, 8, 17, 64, 65, 1], rng.integers(0, 20, 50)])
    seg_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    idx = rng.integers(0, cnt, seg_ptr[-1]).astype(np.int64)
    got = pl.reduce_segments(c, seg_ptr, idx)
    cts = pyoracle.words_to_ints(c)
    want = pyoracle.segment_product(key, cts, list(seg_ptr), list(idx))
    assert [pyoracle.from_words(x) for x in got] == want
    sums = [int(m[idx[seg_ptr[s]:seg_ptr[s + 1]]].sum(dtype=np.uint64)) for s in range(len(lens))]
    assert [int(x) for x in pl.decrypt_u64(got)] == sums
    # contiguous form (idx = None) == the identity gather
    seg_c = np.array([0, 3, 3, 600, cnt], np.int64)
    got_c = pl.reduce_segments(c, seg_c)
    assert [pyoracle.from_words(x) for x in got_c] == pyoracle.segment_product(key, cts, list(seg_c))


def test_reduce_segments_root_sum_full_size(dev, coracle):
    """Root sum of 300,000 ciphertexts (tree.cpp:20-34): one segment, several
    passes and chunks; property check through decryption."""
    pw, qw = _det_primes(coracle, 2048, 41)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    cnt = 300000
    m = np.random.default_rng(7).integers(0, 2**62, cnt, dtype=np.uint64)
    import torch
    tm = torch.from_numpy(m.view(np.int64)).cuda()
    c = torch.empty((cnt, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    pl.encrypt_u64_dev(tm, c, seed=9)
    out = torch.empty((2, 2 * pl.n_words), dtype=torch.int32, device="cuda")
    seg = np.array([0, cnt, cnt + 3], np.int64)
    idx = np.concatenate([np.arange(cnt), [5, 5, 5]]).astype(np.int64)
    pl.reduce_segments_dev(c, seg, out, idx=idx)
    pl.dev.sync()
    low = pl.decrypt_u64(out.cpu().numpy().view(np.uint32))
    assert int(low[0]) == int(m.sum(dtype=np.uint64))
    assert int(low[1]) == int(m[5] * np.uint64(3))


def test_histogram_vs_reference_loop(dev, coracle):
    """HEParty.compute_histogram against the oracle's restatement of
    hist_tree_builder.cpp:574-595 (g and h), then decrypt."""
    from fedtree_amd.paillier import GHPairs, HEParty
    pw, qw = _det_primes(coracle, 1024, 51)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    key = pyoracle.keygen_from_primes(pl.p, pl.q)
    rng = np.random.default_rng(3)
    n_inst, n_col, max_bin = 500, 5, 32
    per = rng.integers(1, max_bin + 1, n_col)
    cut = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    bins = np.stack([np.where(rng.random(n_inst) < 0.05, max_bin, rng.integers(0, per[f], n_inst))
                     for f in range(n_col)], 1).astype(np.uint8)
    g0 = rng.standard_normal(n_inst).astype(np.float32)
    h0 = rng.random(n_inst).astype(np.float32)
    gh = GHPairs(g0, h0)
    gh.homo_encrypt(pl, seed=4)
    hist = HEParty(pl).compute_histogram(gh, bins.reshape(-1), cut, max_bin)
    for enc, name in ((gh.g_enc, "g"), (gh.h_enc, "h")):
        want = pyoracle.histogram(key, pyoracle.words_to_ints(enc), bins.reshape(-1), list(cut), max_bin)
        got = hist.g_enc if name == "g" else hist.h_enc
        assert [pyoracle.from_words(x) for x in got] == [1 if w is None else w for w in want]
    assert np.array_equal(hist.bin_encrypted, [w is not None for w in want])
    # decrypted bins == decode(sum mod 2^64 of the encoded members)
    from fedtree_amd.paillier import decode_fixed, encode_fixed, histogram_segments
    seg_ptr, idx = histogram_segments(bins.reshape(-1), cut, max_bin)
    hist.homo_decrypt(pl)
    for arr, x0 in ((hist.g, g0), (hist.h, h0)):
        e = encode_fixed(x0)
        want = [e[idx[seg_ptr[b]:seg_ptr[b + 1]]].sum(dtype=np.uint64) for b in range(cut[-1])]
        assert np.array_equal(arr, decode_fixed(np.array(want, np.uint64)))


@pytest.mark.parametrize("nbits", [1024, 2048])
def test_sub_vs_oracle(dev, coracle, nbits):
    """GHPair::operator- (common.h:311-317): a * b^(2^64-1), bit-exact; low 64
    bits of the plaintext are ma - mb mod 2^64."""
    pw, qw = _det_primes(coracle, nbits, 61 + nbits)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    key = pyoracle.keygen_from_primes(pl.p, pl.q)
    rng = np.random.default_rng(nbits + 5)
    cnt = 300
    ma = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    mb = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    ca, cb = pl.encrypt_u64(ma, seed=1), pl.encrypt_u64(mb, seed=2)
    got = pl.sub_batch(ca, cb)
    want = [pyoracle.sub(key, pyoracle.from_words(x), pyoracle.from_words(y)) for x, y in zip(ca[:40], cb[:40])]
    assert [pyoracle.from_words(x) for x in got[:40]] == want
    assert np.array_equal(pl.decrypt_u64(got), ma - mb)
    # scalar mul by 2^64-1 (all-ones chain) + add == fused sub
    assert np.array_equal(pl.add_batch(ca, pl.scalar_mul(cb, 2**64 - 1)), got)


@pytest.mark.parametrize("nbits", [1024, 2048])
def test_scan_segments_vs_oracle(dev, coracle, nbits):
    """Segmented inclusive scan (hist_tree_builder.cpp:695-708), ragged segments
    including empty, single and a 300-long one (three radix-8 passes)."""
    pw, qw = _det_primes(coracle, nbits, 71 + nbits)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    key = pyoracle.keygen_from_primes(pl.p, pl.q)
    rng = np.random.default_rng(nbits + 9)
    lens = [3, 0, 1, 300, 8, 9, 64, 65, 0, 17]
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    N = int(seg[-1])
    m = rng.integers(0, 2**40, N, dtype=np.uint64)
    c = pl.encrypt_u64(m, seed=3)
    got = pl.scan_segments(c, seg)
    want = pyoracle.scan_segments(key, pyoracle.words_to_ints(c), list(seg))
    assert [pyoracle.from_words(x) for x in got] == want
    want_m = np.concatenate([np.cumsum(m[seg[s]:seg[s + 1]], dtype=np.uint64) for s in range(len(lens))])
    assert np.array_equal(pl.decrypt_u64(got), want_m)


def test_level_histogram_flow(dev, coracle):
    """One tree level on the party side (hist_tree_builder.cpp:627-708): the
    smaller child's histogram by segmented product, the sibling as father -
    child (fused sub), then the per-feature prefix scan; every decrypted bin
    equals the fixed-point sum over the right instances."""
    from fedtree_amd.paillier import GHPairs, HEParty, decode_fixed, encode_fixed, histogram_segments
    pw, qw = _det_primes(coracle, 1024, 81)
    pl = _pl(dev, pyoracle.from_words(pw), pyoracle.from_words(qw))
    rng = np.random.default_rng(8)
    n_inst, n_col, max_bin = 400, 4, 16
    per = rng.integers(2, max_bin + 1, n_col)
    cut = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    bins = np.stack([rng.integers(0, per[f], n_inst) for f in range(n_col)], 1).astype(np.uint8)
    g0 = rng.standard_normal(n_inst).astype(np.float32)
    h0 = rng.random(n_inst).astype(np.float32)
    gh = GHPairs(g0, h0).homo_encrypt(pl, seed=6)
    party = HEParty(pl)
    left = rng.random(n_inst) < 0.3

    def sub_gh(mask):
        s = GHPairs(np.zeros(mask.sum(), np.float32), None, pl)
        s.g_enc, s.h_enc, s.encrypted = gh.g_enc[mask], gh.h_enc[mask], True
        return s

    father = party.compute_histogram(gh, bins.reshape(-1), cut, max_bin)
    child = party.compute_histogram(sub_gh(left), bins[left].reshape(-1), cut, max_bin)
    sib = party.sibling_histogram(father, child)
    scanned = party.prefix_histogram(sib, cut)
    scanned.homo_decrypt(pl)
    sib.homo_decrypt(pl)
    right = ~left
    for arr_s, arr_p, x0 in ((sib.g, scanned.g, g0), (sib.h, scanned.h, h0)):
        e = encode_fixed(x0[right])
        seg_ptr, idx = histogram_segments(bins[right].reshape(-1), cut, max_bin)
        per_bin = np.array([e[idx[seg_ptr[b]:seg_ptr[b + 1]]].sum(dtype=np.uint64) for b in range(cut[-1])], np.uint64)
        assert np.array_equal(arr_s, decode_fixed(per_bin))
        pref = np.concatenate([np.cumsum(per_bin[cut[f]:cut[f + 1]], dtype=np.uint64) for f in range(n_col)])
        assert np.array_equal(arr_p, decode_fixed(pref))


def _next_prime(x):
    """Smallest probable prime >= x (Miller-Rabin, 40 fixed bases; test keys only)."""
    x |= 1
    while True:
        if all(x % sp for sp in (3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)):
            d, s = x - 1, 0
            while d % 2 == 0:
                d, s = d // 2, s + 1
            for a in range(2, 42):
                y = pow(a, d, x)
                if y in (1, x - 1):
                    continue
                for _ in range(s - 1):
                    y = y * y % x
                    if y == x - 1:
                        break
                else:
                    break
            else:
                return x
        x += 2


@pytest.mark.parametrize("shape", ["q_over_p_1.9", "p_over_q_1.9", "q_24_bits_longer"])
def test_unbalanced_primes_vs_c_oracle(dev, coracle, shape):
    """CRT recombination for any prime ratio: u = c_p + K - c_q needs K > q^2 (was 2 p^2,
    wrong once q > sqrt(2) p) -- CRT/public encrypt and decrypt bit-exact vs the oracle."""
    rng = np.random.default_rng(len(shape))
    hw = 17
    base = int.from_bytes(rng.bytes(62), "little") | (1 << 495) | (1 << 511)
    base &= (1 << 512) - 1
    if shape == "q_24_bits_longer":
        p = _next_prime(base >> 12)                               # 500 bits
        q = _next_prime(base << 12)                               # 524 bits
    else:
        a = _next_prime(base >> 1)                                # 511 bits
        b = _next_prime(a * 19 // 10)                             # ~1.9 a, 512 bits
        p, q = (a, b) if shape == "q_over_p_1.9" else (b, a)
    pl = _pl(dev, p, q)
    ok = coracle.key(pyoracle.to_words(p, hw), pyoracle.to_words(q, hw))
    n = pl.modulus
    cnt = 300
    m = rng.integers(0, 2**64, cnt, dtype=np.uint64)
    m[:3] = [0, 1, 2**64 - 1]
    rs = [int.from_bytes(rng.bytes(pl.n_words * 4), "little") % (n - 1) + 1 for _ in range(cnt)]
    rs[0], rs[1] = 1, n - 1
    r = pyoracle.ints_to_words(rs, pl.n_words)
    r_or = np.zeros((cnt, 2 * hw), np.uint32)                     # oracle rows: 2 * hw words
    r_or[:, :pl.n_words] = r
    want_or = ok.encrypt_batch(m, r_or)
    assert not want_or[:, 2 * pl.n_words:].any()
    want = np.ascontiguousarray(want_or[:, :2 * pl.n_words])
    assert np.array_equal(pl.encrypt_u64(m, r=r), want)
    if _public_supported(pl):
        assert np.array_equal(pl.encrypt_u64(m, r=r, public=True), want)
    low, full = pl.decrypt_u64(want, full=True)
    assert np.array_equal(low, m)
    assert np.array_equal(full, ok.decrypt_batch(want_or)[:, :pl.n_words])
    c = pl.encrypt_u64(m, seed=4)                                 # device randomness (direct y)
    assert np.array_equal(pl.decrypt_u64(c), m)
    assert np.array_equal(pl.decrypt_u64(pl.encrypt_u64(m, seed=5, fixed_base_exact=True)), m)
