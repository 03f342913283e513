"""CPU checks of the matrix-core Barrett of fthe_padic_m37 (gen_padic_mfma.py):
the bit-exact model (tools/padic_mfma_model.py: column sums of the i8 tiles, chunk accumulation, clamping,
digit bounds) on squarings / products / LOADP at the digit bounds, and the host's LDS tile image
(fedtree_amd/csrc/padic_tiles.hpp) byte for byte against the model's."""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import padic_model as pm  # noqa: E402
import padic_mfma_model as mm  # noqa: E402


@pytest.fixture(autouse=True)
def mfma_barrett():
    saved = pm.barrett
    mm.install()
    yield
    pm.barrett = saved


@pytest.mark.parametrize("bits", [1009, 1030])
def test_mfma_barrett_digit_bounds(bits):
    rng = random.Random(bits)
    P = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    key = mm.MfmaKey(P)
    key.check_skipped_tiles()
    P2 = P * P
    K = mm.K
    for x0v, x1v in ((5 * P - 1, 5 * P - 1), (1, 0), (0, 1), (rng.randrange(5 * P), rng.randrange(5 * P))):
        z0, z1 = pm.sqr(key, pm.limbs(x0v, K), pm.limbs(x1v, K))
        X = x0v + x1v * P
        assert (pm.value(z0) + pm.value(z1) * P) % P2 == X * X % P2
        pm.check_digit(key, z0)
        pm.check_digit(key, z1)
    a = [pm.limbs(rng.randrange(5 * P), K) for _ in range(4)]
    z0, z1 = pm.mul(key, *a)
    want = (pm.value(a[0]) + pm.value(a[1]) * P) * (pm.value(a[2]) + pm.value(a[3]) * P) % P2
    assert (pm.value(z0) + pm.value(z1) * P) % P2 == want
    clamped = 0
    for X in (0, 1, (1 << 1008) - 1, 1 << 1008, 50 * P2 - 1):
        q3, r, cl = mm.barrett(key, pm.limbs(X, 2 * K))
        clamped += cl
        assert pm.value(r) < 5 * P and pm.value(q3) * P + pm.value(r) == X
    assert clamped >= 2                        # X = 0, 1: q1 = 0


def test_host_tile_image_matches_model(tmp_path):
    exe = tmp_path / "padic_tiles_dump"
    r = subprocess.run(["g++", "-O1", "-idirafter", "/opt/conda/include", "-o", str(exe),
                        os.path.join(ROOT, "tools", "padic_tiles_dump.cpp"), "-l:libgmp.so.10"],
                       capture_output=True, text=True)
    if r.returncode:
        pytest.skip("no g++/GMP to build the host tile builder: " + r.stderr[-200:])
    rng = random.Random(5)
    for bits in (1009, 1024, 1030):
        P = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        out = tmp_path / f"img{bits}.bin"
        subprocess.run([str(exe), format(P, "x"), str(out)], check=True)
        assert out.read_bytes() == mm.MfmaKey(P).tile_image() + bytes(1024)


# moduli whose bytes make the balanced-digit conversion carry everywhere (0x80 / 0x7f / 0xff runs) or sit at
# the ends of the 1009..1030-bit range; Barrett needs no primality, so these need not be prime
STRUCTURED = [
    int("80" * 128, 16) | 1,                                  # 1024 bits, every byte 0x80
    int("7f" * 128, 16) | (1 << 1023) | 1,
    (1 << 1030) - 1,                                          # all ones, the largest P
    (1 << 1008) + 1,                                          # the smallest P (1009 bits)
    (1 << 1029) | int("ff" * 64, 16) << 300 | 1,
]


@pytest.mark.parametrize("P", STRUCTURED, ids=["x80", "x7f", "max", "min", "ffrun"])
def test_mfma_barrett_structured_moduli(P, tmp_path):
    key = mm.MfmaKey(P)
    key.check_skipped_tiles()
    K = mm.K
    P2 = P * P
    for x0v, x1v in ((5 * P - 1, 5 * P - 1), (1, 0), (P - 1, 1), (int("80" * 128, 16) % (5 * P), P // 3)):
        z0, z1 = pm.sqr(key, pm.limbs(x0v, K), pm.limbs(x1v, K))
        X = x0v + x1v * P
        assert (pm.value(z0) + pm.value(z1) * P) % P2 == X * X % P2
        pm.check_digit(key, z0)
        pm.check_digit(key, z1)
    for X in (0, 1, P2 - 1, 50 * P2 - 1, int("80" * 256, 16) % (50 * P2)):
        q3, r, _ = mm.barrett(key, pm.limbs(X, 2 * K))
        assert pm.value(r) < 5 * P and pm.value(q3) * P + pm.value(r) == X
    exe = tmp_path / "padic_tiles_dump"
    rc = subprocess.run(["g++", "-O1", "-idirafter", "/opt/conda/include", "-o", str(exe),
                         os.path.join(ROOT, "tools", "padic_tiles_dump.cpp"), "-l:libgmp.so.10"],
                        capture_output=True, text=True).returncode
    if rc:
        pytest.skip("no g++/GMP to build the host tile builder")
    out = tmp_path / "img.bin"
    subprocess.run([str(exe), format(P, "x"), str(out)], check=True)
    assert out.read_bytes() == key.tile_image() + bytes(1024)
