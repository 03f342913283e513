import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; run with -m gpu")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


GOLDEN_KEYS = ["ref_gmp_L1024.json", "ref_gmp_L2048.json", "ref_gmp_L4096.json"]


@pytest.fixture(scope="session")
def coracle():
    import pyoracle
    return pyoracle.COracle()


def golden_key(g):
    """Primes of a golden key (the reference's p, q fields hold p-1, q-1: SURVEY Q5)."""
    p = int(g["p_minus_1"], 16) + 1
    q = int(g["q_minus_1"], 16) + 1
    return p, q
