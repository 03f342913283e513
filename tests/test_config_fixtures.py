"""CPU checks of the full-size config fixtures (no GPU): the fixture inputs are
regenerated bit-identically on this host and the C oracle reproduces the
fixture's first ciphertext block (tests/golden/make_config1.py)."""
import hashlib
import os
import sys

import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN, load_golden

sys.path.insert(0, GOLDEN)
import make_config1 as cfg1   # noqa: E402


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def fix():
    return load_golden("config1_p1024.json")


def test_config1_inputs_regenerate(coracle, fix):
    pw, qw = cfg1.config1_key(coracle)
    p, q = pyoracle.from_words(pw), pyoracle.from_words(qw)
    assert (hex(p), hex(q)) == (fix["p"], fix["q"])
    m, r = cfg1.config1_inputs(p * q)
    assert len(m) == 2 * fix["pairs"]
    assert _sha(m) == fix["m_sha256"]
    assert _sha(r) == fix["r_sha256"]


def test_config1_oracle_reproduces_first_block(coracle, fix):
    pw, qw = cfg1.config1_key(coracle)
    n = pyoracle.from_words(pw) * pyoracle.from_words(qw)
    m, r = cfg1.config1_inputs(n)
    b = fix["block"]
    c = coracle.key(pw, qw).encrypt_batch(m[:b], r[:b], threads=os.cpu_count() or 1)
    assert [hex(pyoracle.from_words(c[i])) for i in range(4)] == fix["first_ct"]
    assert _sha(c) == fix["block_sha256"][0]
