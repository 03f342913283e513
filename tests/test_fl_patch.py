"""The Server / Party side of the drop-in: integration/server_party_h_use_hip.patch, the
USE_HIP change to the reference's server.h:47-51,58-135 and party.h:16-18,118-142,181-185, applies to the
reference's real headers, and with -DUSE_HIP the preprocessor selects Paillier_HIP and the batch branches
(`paillier.encrypt(raw)`, `paillier.decrypt(encrypted)`, ...) that Paillier_HIP implements, while the
USE_CUDA and CPU builds preprocess to exactly what they were.

The headers cannot be compiled here: party.h:19 includes diffie_hellman.h -> NTL/ZZ.h, absent from this
image.  The test therefore works on the preprocessor level: #include lines are dropped and
`cpp -P` evaluates the conditionals of the patched and the original files."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCH = os.path.join(ROOT, "integration", "server_party_h_use_hip.patch")
REF = "/root/reference"
FILES = ("include/FedTree/FL/server.h", "include/FedTree/FL/party.h")

pytestmark = pytest.mark.skipif(not all(os.path.exists(os.path.join(REF, f)) for f in FILES),
                                reason="reference sources absent (GPU box)")


def _tree(tmp_path, patched):
    d = tmp_path / ("patched" if patched else "orig")
    for f in FILES:
        os.makedirs(d / os.path.dirname(f), exist_ok=True)
        shutil.copy(os.path.join(REF, f), d / f)
    if patched:
        r = subprocess.run(["patch", "-s", "-p1", "-d", str(d), "-i", PATCH], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    return d


def _cpp(path, *defs):
    text = "".join(ln for ln in open(path) if not ln.lstrip().startswith("#include"))
    r = subprocess.run(["cpp", "-P", "-w", *[f"-D{d}" for d in defs], "-"], input=text, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    return [ln.strip() for ln in r.stdout.splitlines() if ln.strip()]


def test_patch_applies_to_the_reference_headers(tmp_path):
    # dry run against the reference tree itself (nothing is written), then a real application to copies
    r = subprocess.run(["patch", "--dry-run", "-s", "-p1", "-d", REF, "-i", PATCH], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    _tree(tmp_path, True)


def test_use_hip_selects_the_engine_class_and_batch_branches(tmp_path):
    d = _tree(tmp_path, True)
    srv = _cpp(d / FILES[0], "USE_HIP")
    par = _cpp(d / FILES[1], "USE_HIP")
    assert "Paillier_HIP paillier;" in srv and "Paillier_HIP paillier;" in par
    assert "Paillier paillier;" not in srv and "Paillier_GPU paillier;" not in srv
    # homo_init(keylength) keeps FLParam.key_length (server.h:64-65 of the CPU build, NTL semantics: n of
    # key_length bits, parser.cpp:50), not the USE_CUDA branch's argument-less keygen()
    assert "paillier.keygen(keylength);" in srv and "paillier.keygen();" not in srv
    assert re.search(r"void keygen\(int keyLength\)", open(os.path.join(ROOT, "integration", "paillier_hip.h")).read())
    for call in ("paillier.decrypt(gh);", "paillier.decrypt(encrypted);",
                 "paillier.encrypt(raw);", "raw_data[i].paillier = paillier.paillier_cpu;"):
        assert call in srv, call
    assert "paillier.encrypt(hist);" in par and "hist_data[i].paillier = paillier.paillier_cpu;" in par
    assert not any("homo_encrypt(paillier)" in ln for ln in srv + par)   # the NTL per-element loops are gone
    # the members those branches use exist on the drop-in class
    hip = open(os.path.join(ROOT, "integration", "paillier_hip.h")).read()
    for pat in (r"void keygen\(\)", r"void encrypt\(SyncArray<GHPair> &", r"void decrypt\(SyncArray<GHPair> &",
                r"void decrypt\(GHPair &", r"\bpaillier_cpu\b", r"Paillier_HIP &operator=\(const Paillier_HIP &"):
        assert re.search(pat, hip), pat
    # the include of the engine header replaces paillier_gpu.h under USE_HIP
    text = open(d / FILES[1]).read()
    assert '#if defined(USE_HIP)\n#include "FedTree/Encryption/paillier_hip.h"' in text


@pytest.mark.parametrize("defs", [(), ("USE_CUDA",)])
def test_other_builds_unchanged(tmp_path, defs):
    o, p = _tree(tmp_path, False), _tree(tmp_path, True)
    for f in FILES:
        assert _cpp(p / f, *defs) == _cpp(o / f, *defs), f
