"""Ciphertext wire formats (host only): the reference's decimal GHEncBatch
strings (fedtree.proto:82-99; `stream << g_enc`, NTL::to_ZZ) and the binary
FTHW frame.  Python's str(int) is the canonical base-10 form the reference
writes."""
import numpy as np
import pytest

import pyoracle
from fedtree_amd import _lib
from fedtree_amd.paillier import ct_from_decimal, ct_to_decimal, wire_decode, wire_encode


def _rows(n, words, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2**32, (n, words), dtype=np.uint64).astype(np.uint32)
    if n > 0:
        a[0] = 0                   # zero -> "0"
    if n > 1:
        a[1] = 0
        a[1, 0] = 7                # single digit
    if n > 2:
        a[2] = 0xFFFFFFFF          # all ones: the longest string
    if n > 3:
        a[3, words // 2:] = 0      # short value, leading zero words
    return a


@pytest.mark.parametrize("words,n", [(128, 300), (64, 5), (32, 1), (128, 0)])
def test_decimal_matches_python_and_roundtrips(words, n):
    a = _rows(n, words, words + n)
    s = ct_to_decimal(a, threads=4)
    assert s == [str(pyoracle.from_words(r)) for r in a]
    assert np.array_equal(ct_from_decimal(s, words, threads=3), a)


def test_decimal_rejects_garbage():
    with pytest.raises(_lib.FtheError):
        ct_from_decimal(["12x4"], 4)
    with pytest.raises(_lib.FtheError):
        ct_from_decimal([""], 4)
    with pytest.raises(_lib.FtheError):
        ct_from_decimal([str(2**128)], 4)      # does not fit in 4 words
    assert np.array_equal(ct_from_decimal([str(2**128 - 1)], 4), np.full((1, 4), 0xFFFFFFFF, np.uint32))


def test_binary_frame_roundtrip_and_checks():
    g, h = _rows(50, 128, 1), _rows(50, 128, 2)
    f = wire_encode(g, h)
    assert f[:4] == b"FTHW" and len(f) == 24 + 2 * 50 * 512
    g2, h2 = wire_decode(f, 128)
    assert np.array_equal(g2, g) and np.array_equal(h2, h)
    f1 = wire_encode(g)
    g3, h3 = wire_decode(f1, 128)
    assert np.array_equal(g3, g) and h3 is None
    with pytest.raises(_lib.FtheError):
        wire_decode(f[:-4], 128)             # truncated
    with pytest.raises(_lib.FtheError):
        wire_decode(b"XXXX" + f[4:], 128)     # bad magic
    with pytest.raises(_lib.FtheError):
        wire_decode(f, 64)                   # wrong width
