"""The FedTree drop-in class (integration/paillier_hip.h) compiles against
FedTree-shaped types and links libfthe.so; on a GPU it runs the Server/Party
HE call sequence (server.h:58-135, party.h:118-142)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTEG = os.path.join(ROOT, "integration")


def _build(out, src="shim_test.cpp", extra=()):
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", *extra, "-I" + INTEG, "-I" + os.path.join(INTEG, "mock"),
           "-I" + os.path.join(ROOT, "include"), "-idirafter", "/opt/conda/include",
           os.path.join(INTEG, src), "-o", out, "-L" + os.path.join(ROOT, "fedtree_amd"), "-lfthe",
           "-Wl,-rpath," + os.path.join(ROOT, "fedtree_amd"), "-l:libgmp.so.10"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def test_shim_compiles_and_links(tmp_path):
    exe = _build(str(tmp_path / "shim_test"))
    assert os.path.exists(exe)
    assert os.path.exists(_build(str(tmp_path / "concurrency_test"), "concurrency_test.cpp"))
    assert os.path.exists(_build(str(tmp_path / "shim_abort"), extra=("-DFTHE_SHIM_ABORT",)))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["default", "exact", "exact_known_order", "public_exact", "short", "helpers", "big"])
def test_shim_runs_server_party_flow(tmp_path, mode):
    exe = _build(str(tmp_path / "shim_test"))
    r = subprocess.run([exe, "1024", mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "shim OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["default", "exact", "public_exact"])
def test_shim_concurrent_threads_share_one_key(tmp_path, mode):
    """16 host threads, one shared key, a context per thread (the OpenMP call pattern)."""
    exe = _build(str(tmp_path / "concurrency_test"), "concurrency_test.cpp")
    r = subprocess.run([exe, "1024", "16", "24", mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "concurrency OK" in r.stdout, r.stdout + r.stderr
