"""The FedTree drop-in (integration/paillier_hip.h, integration/fthe_ghpair_key.h) compiles against
FedTree-shaped types and links libfthe.so; on a GPU it runs the Server/Party HE call sequence
(server.h:58-135, party.h:118-142) and GHPair's operators (common.h:150-337) on the engine,
bit-exact against the reference's golden vectors."""
import os
import re
import subprocess

import pytest

import pyoracle
from conftest import golden_key, load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTEG = os.path.join(ROOT, "integration")
REF_COMMON = "/root/reference/include/FedTree/common.h"


def _build(out, src="shim_test.cpp", extra=(), check=True):
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", *extra, "-I" + INTEG, "-I" + os.path.join(INTEG, "mock"),
           "-I" + os.path.join(ROOT, "include"), "-idirafter", "/opt/conda/include",
           os.path.join(INTEG, src), "-o", out, "-L" + os.path.join(ROOT, "fedtree_amd"), "-lfthe",
           "-Wl,-rpath," + os.path.join(ROOT, "fedtree_amd"), "-l:libgmp.so.10"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if check:
        assert r.returncode == 0, r.stderr
    return r


NONREF = ("-DFTHE_ENABLE_NONREFERENCE_MODES",)


def test_shim_compiles_and_links(tmp_path):
    _build(str(tmp_path / "shim_test"))
    _build(str(tmp_path / "shim_nonref"), extra=NONREF)
    _build(str(tmp_path / "concurrency_test"), "concurrency_test.cpp")
    _build(str(tmp_path / "shim_abort"), extra=("-DFTHE_SHIM_ABORT",))
    _build(str(tmp_path / "ghpair_test"), "ghpair_test.cpp", extra=("-DFTHE_REFERENCE_SHARED_R",))
    _build(str(tmp_path / "ghpair_rate"), "ghpair_rate.cpp", extra=("-fopenmp",))
    _build(str(tmp_path / "host_ops_test"), "host_ops_test.cpp", extra=("-fopenmp",))
    _build(str(tmp_path / "pool_test"), "pool_test.cpp", extra=("-fopenmp",))
    _build(str(tmp_path / "shim_refkeylen"), extra=("-DFTHE_REFERENCE_GPU_KEYLEN",))
    _build(str(tmp_path / "multidev_test"), "multidev_test.cpp")
    _build(str(tmp_path / "ghpair_e2e"), "ghpair_e2e.cpp", extra=("-fopenmp",))


def test_default_key_length_is_2048_unless_reference_keylen_requested(tmp_path):
    """keygen() with no argument makes a 2048-bit n; the reference GPU build's factorable 512-bit n
    (paillier_gpu.cu:119-121) only with -DFTHE_REFERENCE_GPU_KEYLEN."""
    src = tmp_path / "kl.cpp"
    src.write_text('#include "paillier_hip.h"\n#include <cstdio>\n'
                   'int main() { Paillier_HIP s; std::printf("%u\\n", s.key_length); return 0; }\n')
    for extra, want in (((), "2048"), (("-DFTHE_REFERENCE_GPU_KEYLEN",), "512")):
        exe = str(tmp_path / ("kl" + str(len(extra))))
        r = subprocess.run(["g++", "-std=c++17", "-pthread", *extra, "-I" + INTEG, "-I" + os.path.join(INTEG, "mock"),
                            "-I" + os.path.join(ROOT, "include"), "-idirafter", "/opt/conda/include", str(src), "-o",
                            exe, "-L" + os.path.join(ROOT, "fedtree_amd"), "-lfthe",
                            "-Wl,-rpath," + os.path.join(ROOT, "fedtree_amd"), "-l:libgmp.so.10"],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        out = subprocess.run([exe], capture_output=True, text=True)
        assert out.returncode == 0 and out.stdout.strip() == want, out.stdout + out.stderr


def _adds_fixture(path, name):
    g = load_golden(name)
    p, q = golden_key(g)
    cts = [int(c["c"], 16) for c in g["cases"]]
    lines = [f"{p * q:x}"] + [f"{cts[a['i']]:x} {cts[a['j']]:x} {_hx(a['c'])}" for a in g["adds"]]
    path.write_text("\n".join(lines) + "\n")


REF_INC = "/root/reference/include"
PATCH = os.path.join(INTEG, "common_h_use_hip.patch")


def _cmake_configure(template, out):
    """config.h from the reference's config.h.in the way CMake's configure_file writes it with none of the
    options set (every `#cmakedefine VAR ...` becomes `/* #undef VAR */`): the generated header of a
    plain build, produced by the same rule, not a stand-in written for the test."""
    lines = []
    for ln in open(template).read().splitlines():
        m = re.match(r"#cmakedefine\s+(\w+)", ln)
        lines.append(f"/* #undef {m.group(1)} */" if m else ln)
    out.write_text("\n".join(lines) + "\n")


@pytest.mark.skipif(not os.path.exists(REF_COMMON), reason="reference sources absent (GPU box)")
@pytest.mark.parametrize("name", ["ref_gmp_L1024.json", "ref_gmp_L4096.json"])
def test_reference_common_h_patched_compiles_and_adds(tmp_path, name):
    """The reference's own common.h, copied into a temporary tree and patched with
    integration/common_h_use_hip.patch, compiles with -DUSE_HIP against
    fthe_ghpair_key.h (hipcc: common.h includes thrust/tuple.h), and its unchanged operator bodies give
    the golden adds through operator+, += and dest = dest + src on a host-bound key."""
    fed = tmp_path / "inc" / "FedTree"
    fed.mkdir(parents=True)
    (fed / "common.h").write_text(open(REF_COMMON).read())
    r = subprocess.run(["patch", "-s", "-p3", "-d", str(fed), "-i", PATCH], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    _cmake_configure(os.path.join(REF_INC, "FedTree", "config.h.in"), fed / "config.h")
    exe = str(tmp_path / "real_common_test")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-DUSE_HIP", "--offload-arch=gfx950",
                        "-I" + str(tmp_path / "inc"), "-I" + REF_INC, "-I" + INTEG, "-I" + os.path.join(ROOT, "include"),
                        "-idirafter", "/opt/conda/include", os.path.join(INTEG, "real_common_test.cpp"), "-o", exe,
                        "-L" + os.path.join(ROOT, "fedtree_amd"), "-lfthe", "-Wl,-rpath," + os.path.join(ROOT, "fedtree_amd"),
                        "-l:libgmp.so.10", "-pthread"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    fx = tmp_path / "adds.txt"
    _adds_fixture(fx, name)
    r = subprocess.run([exe, str(fx)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "real common.h OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("name", ["ref_gmp_L1024.json", "ref_gmp_L2048.json", "ref_gmp_L4096.json"])
def test_ghpair_host_add_bit_exact_without_gpu(tmp_path, name):
    """The GHPair key's add runs on the host (one product x y mod n^2, as paillier_gpu.cu:57-61): bound to
    a public n only, operator+, the aliased += and add(s, s, c) give the reference's golden adds, also for
    unreduced operands; key copies share one cell and read n, n^2, g through views (no GPU needed)."""
    fx = tmp_path / "adds.txt"
    _adds_fixture(fx, name)
    exe = str(tmp_path / "host_ops_test")
    _build(exe, "host_ops_test.cpp", extra=("-fopenmp",))
    r = subprocess.run([exe, "check", str(fx)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "host ops OK" in r.stdout, r.stdout + r.stderr


def test_nonreference_modes_need_the_build_opt_in(tmp_path):
    """The subgroup randomizer (FTHE_ENC_FIXED_BASE) and known-order primes (FTHE_KEYGEN_KNOWN_ORDER)
    are not the reference's distributions: without FTHE_ENABLE_NONREFERENCE_MODES the drop-in class
    cannot even name them; the shared-r compat randomness needs FTHE_REFERENCE_SHARED_R."""
    src = tmp_path / "nonref.cpp"
    src.write_text('#include "paillier_hip.h"\nint main() { Paillier_HIP s;\n'
                   '  s.enc_mode = Paillier_HIP::EncMode::FixedBaseSubgroup;\n'
                   '  s.keygen_mode = Paillier_HIP::KeygenMode::KnownOrder; return 0; }\n')
    shr = tmp_path / "sharedr.cpp"
    shr.write_text('#include "paillier_hip.h"\nint main() { Paillier_HIP_Pub k; mpz_t r; mpz_init(r);\n'
                   '  k.set_shared_r(r); return 0; }\n')

    def build(path, extra):
        cmd = ["g++", "-std=c++17", "-fsyntax-only", *extra, "-I" + INTEG, "-I" + os.path.join(INTEG, "mock"),
               "-I" + os.path.join(ROOT, "include"), "-idirafter", "/opt/conda/include", str(path)]
        return subprocess.run(cmd, capture_output=True, text=True)

    r = build(src, ())
    assert r.returncode != 0 and "FixedBaseSubgroup" in r.stderr and "KnownOrder" in r.stderr
    assert build(src, NONREF).returncode == 0
    assert build(shr, ()).returncode != 0
    assert build(shr, ("-DFTHE_REFERENCE_SHARED_R",)).returncode == 0


def _key_calls(text):
    """`paillier.add(...)` / `paillier.mul(...)` calls with three arguments (the mpz_t forms of the
    USE_CUDA branches), whitespace removed, comments dropped."""
    text = re.sub(r"//[^\n]*", "", text)
    calls = re.findall(r"((?:rhs\.)?paillier\.(?:add|mul)\(([^;()]*)\));", text)
    return sorted({re.sub(r"\s+", "", c) for c, args in calls if args.count(",") == 2})


@pytest.mark.skipif(not os.path.exists(REF_COMMON), reason="reference sources absent (GPU box)")
def test_mock_operators_make_the_reference_key_calls():
    """Every key call in the reference's GHPair operator bodies (common.h:150-337, mpz_t branches)
    appears in the shim's GHPair with the same receiver and arguments, so ghpair_test exercises the
    reference's call sequence -- including the aliased add(g_enc, g_enc, ...) of operator+=."""
    ref = open(REF_COMMON).read().splitlines()
    ref_ops = "\n".join(ref[149:337])
    mock = open(os.path.join(INTEG, "mock", "FedTree", "common.h")).read()
    want = _key_calls(ref_ops)
    assert len(want) >= 12, want
    have = set(_key_calls(mock))
    missing = [c for c in want if c not in have]
    assert not missing, missing
    assert "paillier.add(g_enc,g_enc,rhs.g_enc)" in want


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["default", "exact", "exact_known_order", "public_exact", "short", "helpers", "big"])
def test_shim_runs_server_party_flow(tmp_path, mode):
    exe = str(tmp_path / "shim_test")
    _build(exe, extra=NONREF if mode == "exact_known_order" else ())
    r = subprocess.run([exe, "1024", mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "shim OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["default", "exact", "public_exact"])
def test_shim_concurrent_threads_share_one_key(tmp_path, mode):
    """16 host threads, one shared key, a context per thread (the OpenMP call pattern)."""
    exe = str(tmp_path / "concurrency_test")
    _build(exe, "concurrency_test.cpp")
    r = subprocess.run([exe, "1024", "16", "24", mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "concurrency OK" in r.stdout, r.stdout + r.stderr


def _hx(v):
    """Plain lower-case hex (the golden files write 0x-prefixed strings)."""
    return f"{int(v, 16) if isinstance(v, str) else int(v):x}"


def _ghpair_fixture(path, name):
    g = load_golden(name)
    p, q = golden_key(g)
    key = pyoracle.keygen_from_primes(p, q)
    r = int(g["shared_r"], 16)
    cts = [int(c["c"], 16) for c in g["cases"]]
    tok = [f"{p:x}", f"{q:x}", f"{r:x}", str(len(cts))] + [f"{c:x}" for c in cts]
    tok += [str(len(g["adds"]))]
    for a in g["adds"]:
        tok += [str(a["i"]), str(a["j"]), _hx(a["c"])]
    h = g["hist"]
    tok += [str(h["parties"]), str(h["bins"])]
    for pi in range(h["parties"]):
        tok += [_hx(v) for v in h["ct"][pi]]
    tok += [_hx(v) for v in h["merged"]]
    subs = [(12, 13), (0, 2), (3, 1), (5, 5)]
    tok += [str(len(subs))]
    for i, j in subs:
        tok += [str(i), str(j), f"{pyoracle.sub(key, cts[i], cts[j]):x}"]
    import numpy as np
    gf, hf, j = np.float32(0.5), np.float32(-0.25), 7
    mg, mh = (int(pyoracle.encode_fixed(np.array([v]))[0]) for v in (gf, hf))
    tok += [repr(float(gf)), repr(float(hf)), str(j),
            f"{pyoracle.add(key, pyoracle.encrypt(key, mg, r), pyoracle.mul(key, cts[j], 2**64 - 1)):x}",
            f"{pyoracle.add(key, pyoracle.encrypt(key, mh, r), pyoracle.mul(key, cts[j], 2**64 - 1)):x}"]
    path.write_text(" ".join(tok) + "\n")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref_gmp_L1024.json", "ref_gmp_L4096.json"])
def test_ghpair_operators_bit_exact_on_engine(tmp_path, name):
    """dest = dest + src, dest += src (aliased), dest - src, add(s, s, c) and the 8-party merge from an
    unencrypted zero (Q10) through the USE_HIP GHPair key: the reference's golden ciphertexts."""
    fx = tmp_path / "fixture.txt"
    _ghpair_fixture(fx, name)
    exe = str(tmp_path / "ghpair_test")
    _build(exe, "ghpair_test.cpp", extra=("-DFTHE_REFERENCE_SHARED_R",))
    r = subprocess.run([exe, str(fx)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ghpair OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def _rebuild_r(p, q, yp, yq):
    """r = CRT(y_p^(q^-1 mod p-1) mod p, y_q^(p^-1 mod q-1) mod q) (the direct-y draw, tests/test_gpu_direct_y.py)."""
    ep, eq, qinv = pow(q, -1, p - 1), pow(p, -1, q - 1), pow(q, -1, p)
    rp, rq = pow(yp, ep, p), pow(yq, eq, q)
    return (rq + q * ((rp - rq) * qinv % p)) % (p * q)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref_gmp_L1024.json", "ref_gmp_L4096.json"])
def test_pooled_promotions_equal_oracle_encrypt(tmp_path, name):
    """GHPair promotions (homo_encrypt, common.h:75-97) from the key's randomizer pool: (1 + m n) rho mod n^2
    with rho an engine Enc(0).  With deterministic pool batches, the r behind each pooled row is rebuilt
    from the engine's direct-y draws and the promoted ciphertext equals the oracle's full-PowerMod
    encrypt(m, r) (paillier.cpp:134-137), across three pool batches, for m = 0, 1, 2^64 - 1 and codec values."""
    from fedtree_amd.paillier import Device, Paillier
    g = load_golden(name)
    p, q = golden_key(g)
    key = pyoracle.keygen_from_primes(p, q)
    ms = [0, 1, 2**64 - 1, 2**63, 123456789, (2**64 - 300000), 5, 0, 77, 2**32 + 1, 999999, 42, 0, 3, 2**62 + 7]
    exe = str(tmp_path / "pool_test")
    _build(exe, "pool_test.cpp", extra=("-fopenmp",))
    seed0, batch = 7001, 6
    r = subprocess.run([exe, "trace", f"{p:x}", f"{q:x}", str(seed0), str(batch)] + [str(m) for m in ms],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [ln.split() for ln in r.stdout.strip().splitlines()]
    assert len(rows) == len(ms)
    pl = Paillier.from_primes(p, q, Device(0))
    pw = (max(p.bit_length(), q.bit_length()) + 31) // 32
    for k, (m_s, seed_s, idx_s, c_hex) in enumerate(rows):
        m, seed, idx = int(m_s), int(seed_s), int(idx_s)
        assert m == ms[k] and seed == seed0 + k // batch and idx == k % batch
        yp, yq = pl.direct_y(seed, idx, 1)
        r_ = _rebuild_r(p, q, pyoracle.words_to_ints(yp.reshape(1, pw))[0], pyoracle.words_to_ints(yq.reshape(1, pw))[0])
        assert int(c_hex, 16) == pyoracle.encrypt(key, m, r_), (k, m)


@pytest.mark.gpu
def test_pooled_promotions_from_threads(tmp_path):
    """16 OpenMP threads promote 2 x 16 x 300 plain GHPairs (codec values and zeros) at once: every pair
    decrypts to its codec values and no pooled randomizer is used twice (all 19,200 ciphertexts distinct)."""
    g = load_golden("ref_gmp_L4096.json")
    p, q = golden_key(g)
    exe = str(tmp_path / "pool_test")
    _build(exe, "pool_test.cpp", extra=("-fopenmp",))
    r = subprocess.run([exe, "threads", f"{p:x}", f"{q:x}", "16", "300"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "pool OK" in r.stdout, r.stdout + r.stderr


def test_marshalling_round_trip_and_shards(tmp_path):
    """The batch calls' host marshalling (Paillier_HIP::encode_pairs / rows_to_pairs / pairs_to_rows /
    decode_pairs; the limb-copy fast path of fthe_ghpair_key.h) is lossless for 1 and 2 concurrent shards
    (integration/marshal_rate.cpp, no kernels; the bench runs it at 1M pairs per shard)."""
    import json
    exe = str(tmp_path / "marshal_rate")
    _build(exe, "marshal_rate.cpp", extra=("-fopenmp",))
    r = subprocess.run([exe, "2048", "3000", "1", "1,2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["round_trip_ok"] and [s["shards"] for s in out["shards"]] == [1, 2]
    for bits in ("1024", "2016"):                                  # other row widths (edge rows self-checked)
        r = subprocess.run([exe, bits, "777", "1", "1"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1])["round_trip_ok"], r.stderr


def test_shard_plan_arithmetic(tmp_path):
    """The drop-in's shard arithmetic (fthe_shim::shard_plan / shard_plan_segments, no GPU): configs[4]'s 80M
    pairs (160M rows) over 8 devices are 8 contiguous shards of 20M rows; random sizes are covered contiguously,
    balanced to +-1 row with at least FTHE_SHARD_ROWS per shard; segment plans of random and skewed CSRs are
    contiguous, non-empty and balanced by member count."""
    import json
    exe = str(tmp_path / "multidev_test")
    _build(exe, "multidev_test.cpp")
    r = subprocess.run([exe, "plan"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["plan_ok"] and out["config4_shard_rows"] == 20_000_000


def test_device_list_parsing(tmp_path):
    """FTHE_DEVICES is parsed before any engine call (no GPU): a list, repeats allowed; garbage is an error."""
    src = tmp_path / "dl.cpp"
    src.write_text('#include "paillier_hip.h"\n#include <cstdio>\nint main(int c, char **v) {\n'
                   '  for (int d : fthe_shim::parse_devices(v[1])) std::printf("%d ", d);\n  return 0; }\n')
    exe = str(tmp_path / "dl")
    _build(exe, str(src))
    for arg, want in (("0,1,2,3", "0 1 2 3"), ("0,0", "0 0"), ("5", "5"), ("1, 3", "1 3")):
        r = subprocess.run([exe, arg], capture_output=True, text=True, timeout=30)
        assert r.returncode == 0 and r.stdout.strip() == want, (arg, r.stdout, r.stderr)
    r = subprocess.run([exe, "a,b"], capture_output=True, text=True, timeout=30)
    assert r.returncode != 0 and "not a device list" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["ref_gmp_L2048.json"])
def test_sharded_drop_in_identical_to_one_context(tmp_path, name):
    """Paillier_HIP's batch calls sharded over two and three contexts on device 0 (FTHE_DEVICES=0,0 / 0,0,0, small
    FTHE_SHARD_ROWS so 3,000 pairs split) give byte-identical ciphertexts to the one-context run for the seeded
    key holder's and party's encrypts (default and published-bases exact), the zero-first histogram, the zero-first
    3-party merge, subtract, prefix and the large merge / subtract; every decrypt is checked against the codec
    values (server.h:58-135, party.h:118-142, paillier_gpu.cu:211-313, 448-494)."""
    g = load_golden(name)
    p, q = golden_key(g)
    exe = str(tmp_path / "multidev_test")
    _build(exe, "multidev_test.cpp")
    outs = {}
    for devs, rep in (("0", "0"), ("0,0", "1"), ("0,0,0", "0")):
        # "0,0" also with FTHE_SHIM_REPLICATE=1: every shard on a key replica (from p, q for the key holder, from n
        # and the published bases for the party), the path of a second physical GPU
        env = dict(os.environ, FTHE_DEVICES=devs, FTHE_SHARD_ROWS="256", FTHE_SHIM_REPLICATE=rep)
        r = subprocess.run([exe, "run", f"{p:x}", f"{q:x}", "3000"], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0 and "multidev OK" in r.stdout, devs + ": " + r.stdout[-3000:] + r.stderr[-3000:]
        lines = r.stdout.strip().splitlines()
        assert f"devices {len(devs.split(','))}" in lines
        outs[devs] = [ln for ln in lines if not ln.startswith("devices")]
    assert outs["0,0"] == outs["0"] and outs["0,0,0"] == outs["0"], outs


@pytest.mark.gpu
@pytest.mark.parametrize("rows", ["2", "100000"])
def test_shim_concurrent_threads_sharded(tmp_path, rows):
    """16 host threads on one key with the batch calls sharded over three contexts (FTHE_DEVICES=0,0,0): batches of
    6 rows split into 3 shards that queue on the shard workers (FTHE_SHARD_ROWS=2), or run whole on each thread's
    home slot (100000); every result checked (the OpenMP call pattern of FLtrainer.cpp:275-306, 758-764)."""
    exe = str(tmp_path / "concurrency_test")
    _build(exe, "concurrency_test.cpp")
    env = dict(os.environ, FTHE_DEVICES="0,0,0", FTHE_SHARD_ROWS=rows, FTHE_SHIM_REPLICATE="1")
    r = subprocess.run([exe, "1024", "16", "12", "default"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "concurrency OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_ghpair_e2e_two_shards(tmp_path):
    """ghpair_e2e (Server::encrypt_gh_pairs / decrypt_gh_pairs at FedTree's types) with its batch split over two
    contexts on device 0: every plaintext round-trips."""
    import json
    exe = str(tmp_path / "ghpair_e2e")
    _build(exe, "ghpair_e2e.cpp", extra=("-fopenmp",))
    r = subprocess.run([exe, "2048", "20000", "1", "0,0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["shards"] == 2


def _gpu_count():
    import torch                                   # device_count() does not initialise HIP on this image
    return torch.cuda.device_count()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["physical", "emulated"])
def test_sharded_drop_in_every_device(tmp_path, mode):
    """configs[4]'s path through the class FedTree calls (Server::encrypt_gh_pairs / decrypt_gh_pairs,
    server.h:105-135 -> Paillier_HIP -> ShardPool, paillier_gpu.cu:211-313): "physical" shards every batch call of
    multidev_test over every visible GPU (FTHE_DEVICES=0,1,..,k-1: a worker thread, context and key replica per
    device, fthe_shim::ctx_on(d != 0), key_on's replicas incl. the key holder's exact tables) and must give the
    one-device run's digests byte for byte -- seeded encrypts (default, party published-bases exact, key-holder
    exact), histogram, merges, subtracts, prefix -- with every decrypt checked; then ghpair_e2e round-trips
    20,000 pairs per device over all of them.  Skipped with fewer than 2 GPUs.  "emulated" is the same over two
    contexts on device 0 with every shard on a key replica (FTHE_SHIM_REPLICATE=1), the path a one-GPU box runs, and
    ghpair_e2e over eight contexts of device 0 (configs[4]'s eight shards and worker threads)."""
    import json
    n = _gpu_count()
    if mode == "physical" and n < 2:
        pytest.skip(f"{n} GPU visible: the physical multi-device case needs 2 or more")
    devs = ",".join(str(i) for i in range(n)) if mode == "physical" else "0,0"
    g = load_golden("ref_gmp_L2048.json")
    p, q = golden_key(g)
    exe = str(tmp_path / "multidev_test")
    _build(exe, "multidev_test.cpp")
    outs = {}
    for dl, rep in (("0", "0"), (devs, "0" if mode == "physical" else "1")):
        env = dict(os.environ, FTHE_DEVICES=dl, FTHE_SHARD_ROWS="256", FTHE_SHIM_REPLICATE=rep)
        r = subprocess.run([exe, "run", f"{p:x}", f"{q:x}", "3000"], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0 and "multidev OK" in r.stdout, dl + ": " + r.stdout[-3000:] + r.stderr[-3000:]
        lines = r.stdout.strip().splitlines()
        assert f"devices {len(dl.split(','))}" in lines
        outs[dl] = [ln for ln in lines if not ln.startswith("devices")]
    assert any(ln.startswith("server_encrypt_exact ") for ln in outs["0"])
    assert outs[devs] == outs["0"], outs
    exe2 = str(tmp_path / "ghpair_e2e")
    _build(exe2, "ghpair_e2e.cpp", extra=("-fopenmp",))
    e2e_devs = devs if mode == "physical" else ",".join(["0"] * 8)    # emulated: configs[4]'s eight shards
    k = len(e2e_devs.split(","))
    r = subprocess.run([exe2, "2048", str(20000 * k), "1", e2e_devs], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, FTHE_SHIM_REPLICATE="0" if mode == "physical" else "1"))
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["shards"] == k
