"""The CPU oracle pinned against the reference's own outputs (tests/golden/).

Golden ciphertexts were produced by FedTree's Paillier_GMP compiled from the
reference sources (tests/golden/make_golden.py).  Both restatements -- the
pure-Python one (oracle/pyoracle.py) and the C/GMP one
(oracle/paillier_oracle.c) -- must reproduce them bit for bit when fed the
reference's key and its shared r.
"""
import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN_KEYS, golden_key, load_golden


@pytest.fixture(scope="module", params=GOLDEN_KEYS)
def gold(request):
    return load_golden(request.param)


def test_key_derivation(gold):
    p, q = golden_key(gold)
    k = pyoracle.keygen_from_primes(p, q)
    assert k["n"] == int(gold["n"], 16)
    assert k["n"].bit_length() == gold["n_bits"]
    assert k["lam"] == int(gold["lambda"], 16)
    assert k["mu"] == int(gold["mu"], 16)


def test_python_oracle_encrypt_decrypt(gold):
    p, q = golden_key(gold)
    k = pyoracle.keygen_from_primes(p, q)
    r = int(gold["shared_r"], 16)
    cases = gold["cases"] if gold["n_bits"] <= 1100 else gold["cases"][:10]
    for c in cases:
        assert pyoracle.encrypt(k, c["m"], r) == int(c["c"], 16)
        assert pyoracle.decrypt(k, int(c["c"], 16)) == int(c["dec"], 16) == c["m"]


def test_python_oracle_add_mul(gold):
    p, q = golden_key(gold)
    k = pyoracle.keygen_from_primes(p, q)
    cts = [int(c["c"], 16) for c in gold["cases"]]
    for a in gold["adds"]:
        assert pyoracle.add(k, cts[a["i"]], cts[a["j"]]) == int(a["c"], 16)
        ms = gold["cases"]
        assert int(a["dec"], 16) == (ms[a["i"]]["m"] + ms[a["j"]]["m"]) % k["n"]
    for m in gold["muls"]:
        assert pyoracle.mul(k, cts[m["i"]], m["k"]) == int(m["c"], 16)
        assert int(m["dec"], 16) == gold["cases"][m["i"]]["m"] * m["k"] % k["n"]


def test_subtraction_decodes_low64(gold):
    """operator- = add(a, b^(2^64-1)); the low 64 bits decode to a - b."""
    p, q = golden_key(gold)
    k = pyoracle.keygen_from_primes(p, q)
    cs = gold["cases"]
    a, b = cs[12], cs[13]
    d = pyoracle.decrypt(k, pyoracle.add(k, int(a["c"], 16), pyoracle.mul(k, int(b["c"], 16), 2**64 - 1)))
    assert d % 2**64 == (a["m"] - b["m"]) % 2**64


def test_c_oracle_batch(gold, coracle):
    p, q = golden_key(gold)
    nw = gold["n_words"]
    hw = (nw + 1) // 2
    key = coracle.key(pyoracle.to_words(p, hw), pyoracle.to_words(q, hw))
    assert key.nw == 2 * hw
    kw = key.nw
    r = int(gold["shared_r"], 16)
    ms = np.array([c["m"] for c in gold["cases"]], dtype=np.uint64)
    rr = np.tile(pyoracle.to_words(r, kw), (len(ms), 1))
    ct = key.encrypt_batch(ms, rr)
    want = pyoracle.ints_to_words([int(c["c"], 16) for c in gold["cases"]], 2 * kw)
    assert np.array_equal(ct, want)
    dec = key.decrypt_batch(ct)
    assert [pyoracle.from_words(d) for d in dec] == [int(c["dec"], 16) for c in gold["cases"]]
    a = gold["adds"][0]
    s = key.add_batch(want[a["i"]:a["i"] + 1], want[a["j"]:a["j"] + 1])
    assert pyoracle.from_words(s[0]) == int(a["c"], 16)
    m0 = gold["muls"][0]
    assert pyoracle.from_words(key.mul_u64(want[m0["i"]], m0["k"])) == int(m0["c"], 16)


def test_aliased_add_zeroes(gold):
    """the reference's add(s, s, c) zeroes s; the engine is alias-safe instead."""
    assert int(gold["aliased_add_result"], 16) == 0


def test_hist_merge_semantics(gold):
    """8-party merge (hist_tree_builder.cpp:1015-1058) with the first add into an
    unencrypted zero being a fresh encrypt(0)."""
    p, q = golden_key(gold)
    k = pyoracle.keygen_from_primes(p, q)
    h = gold["hist"]
    e0 = int(h["enc_zero"], 16)
    for b in range(h["bins"]):
        acc = e0
        for pi in range(h["parties"]):
            acc = pyoracle.add(k, acc, int(h["ct"][pi][b], 16))
        assert acc == int(h["merged"][b], 16)
        assert int(h["merged_dec"][b], 16) == sum(h["m"][pi][b] for pi in range(h["parties"])) % k["n"]


def test_codec_matches_reference_expressions():
    g = load_golden("codec.json")
    f = np.array(g["floats_f32_bits"], dtype=np.uint32).view(np.float32)
    enc = pyoracle.encode_fixed(f)
    assert [int(x) for x in enc] == g["encode_gmp"] == g["encode_ntl"]
    dec = pyoracle.decode_fixed(np.array(g["decode_in"], dtype=np.uint64))
    assert [int(x) for x in dec.view(np.uint32)] == g["decode_out_f32_bits"]


def test_host_codec_matches_golden():
    """fedtree_amd's host-side codec (the marshalling of paillier_gpu.cu:240-251)."""
    from fedtree_amd.paillier import decode_fixed, encode_fixed
    g = load_golden("codec.json")
    f = np.array(g["floats_f32_bits"], dtype=np.uint32).view(np.float32)
    assert [int(x) for x in encode_fixed(f)] == g["encode_gmp"]
    dec = decode_fixed(np.array(g["decode_in"], dtype=np.uint64))
    assert [int(x) for x in dec.view(np.uint32)] == g["decode_out_f32_bits"]


def _ref_or_skip():
    try:
        return pyoracle.RefGMP()
    except OSError:
        pytest.skip("oracle/_ref not built (reference sources absent)")


def test_ref_key_from_primes_reproduces_reference(gold):
    """ref_key_from_primes (the CPU baseline's same-key handle) leaves the fields the
    reference's keyGen leaves, and the reference's own encrypt / decrypt / add / merge run on
    it reproduce the golden vectors (its unseeded MT draws the same shared r for this n)."""
    ref = _ref_or_skip()
    p, q = golden_key(gold)
    h = ref.key_from_primes(p, q)
    try:
        nw = gold["n_words"]
        assert ref.lib.ref_n_words(h) == nw
        bufs = [np.zeros(nw, np.uint32) for _ in range(5)]
        ref.lib.ref_export(h, nw, *[b.ctypes.data for b in bufs])
        n, pm1, qm1, lam, mu = (pyoracle.from_words(b) for b in bufs)
        assert (n, pm1, qm1, lam, mu) == (int(gold["n"], 16), int(gold["p_minus_1"], 16), int(gold["q_minus_1"], 16),
                                          int(gold["lambda"], 16), int(gold["mu"], 16))
        cases = gold["cases"][:6]
        ms = np.array([c["m"] for c in cases], dtype=np.uint64)
        ct = np.zeros((len(ms), 2 * nw), np.uint32)
        ref.lib.ref_encrypt_batch(h, nw, ms.ctypes.data, len(ms), ct.ctypes.data, 2)
        want = pyoracle.ints_to_words([int(c["c"], 16) for c in cases], 2 * nw)
        assert np.array_equal(ct, want)
        lo = np.zeros(len(ms), np.uint64)
        ref.lib.ref_decrypt_batch(h, nw, want.ctypes.data, len(ms), lo.ctypes.data, 2)
        assert np.array_equal(lo, ms)
        allc = pyoracle.ints_to_words([int(c["c"], 16) for c in gold["cases"]], 2 * nw)
        a = np.ascontiguousarray(allc[[x["i"] for x in gold["adds"]]])
        b = np.ascontiguousarray(allc[[x["j"] for x in gold["adds"]]])
        s = np.zeros_like(a)
        ref.lib.ref_add_batch(h, nw, a.ctypes.data, b.ctypes.data, len(a), s.ctypes.data, 2)
        assert [pyoracle.from_words(x) for x in s] == [int(x["c"], 16) for x in gold["adds"]]
        hist = gold["hist"]
        x = np.stack([pyoracle.ints_to_words([int(hist["enc_zero"], 16)] * hist["bins"], 2 * nw)] +
                     [pyoracle.ints_to_words([int(v, 16) for v in hist["ct"][pi]], 2 * nw)
                      for pi in range(hist["parties"])])
        x = np.ascontiguousarray(x)
        out = np.zeros((hist["bins"], 2 * nw), np.uint32)
        ref.lib.ref_merge_batch(h, nw, x.ctypes.data, x.shape[0], hist["bins"], out.ctypes.data, 2)
        assert [pyoracle.from_words(v) for v in out] == [int(v, 16) for v in hist["merged"]]
    finally:
        ref.lib.ref_free(h)
