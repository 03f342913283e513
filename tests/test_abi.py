"""The C-ABI library: it loads, exports every symbol include/fthe.h declares,
validates arguments and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import subprocess
import sys

import pytest

from fedtree_amd import _lib


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding declares a prototype for each of them
    assert set(syms) == set(_lib._PROTOS), set(syms) ^ set(_lib._PROTOS)


def test_nm_dynamic_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in _lib.header_symbols():
        assert s in exported, s


def test_strerror_and_version():
    lib = _lib.load()
    assert lib.fthe_version() >= 100
    for st in (0, -1, -2, -3, -4, -5, -6):
        assert lib.fthe_strerror(st)
    assert b"unknown" in lib.fthe_strerror(-99)


def test_kernel_limbs():
    lib = _lib.load()
    assert lib.fthe_kernel_limbs(1024) == 37
    assert lib.fthe_kernel_limbs(2048) == 74     # p^2 of Paillier-2048, n^2 of Paillier-1024
    assert lib.fthe_kernel_limbs(4096) == 152    # n^2 of Paillier-2048: four lanes per ciphertext, radix 2^27
    assert lib.fthe_kernel_limbs(4200) == 0


def test_null_arguments_rejected():
    lib = _lib.load()
    assert lib.fthe_ctx_create(0, None) == _lib.FTHE_ERR_ARG
    assert lib.fthe_key_generate(None, 1024, 0, None) == _lib.FTHE_ERR_ARG
    assert lib.fthe_encrypt_u64_dev(None, None, None, 0, None, 0, 0, None, 0) == _lib.FTHE_ERR_ARG
    assert lib.fthe_encrypt_u64_at_dev(None, None, None, 0, None, 0, 0, 5, None, 0) == _lib.FTHE_ERR_ARG
    assert lib.fthe_encrypt_u64_at(None, None, None, 0, None, 0, 0, 5, None, 0) == _lib.FTHE_ERR_ARG
    assert lib.fthe_decrypt_dev(None, None, None, 0, None, None) == _lib.FTHE_ERR_ARG
    assert lib.fthe_decrypt_shared(None, None, 0, None, None, 0) == _lib.FTHE_ERR_ARG
    assert lib.fthe_encrypt_shared(None, None, 0, None, 0) == _lib.FTHE_ERR_ARG
    assert lib.fthe_add_dev(None, None, None, None, 0, None) == _lib.FTHE_ERR_ARG
    assert lib.fthe_reduce_segments_dev(None, None, None, 0, None, None, 0, None) == _lib.FTHE_ERR_ARG
    assert lib.fthe_reduce_segments(None, None, None, 0, None, None, 0, None) == _lib.FTHE_ERR_ARG
    assert lib.fthe_key_n_words(None) == 0


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure mode")
def test_no_gpu_fails_loudly():
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.fthe_ctx_create(0, ctypes.byref(ctx)) == _lib.FTHE_ERR_HIP
    assert lib.fthe_device_count() == 0                      # the drop-in then has no shard to run on
    from fedtree_amd.paillier import Device
    with pytest.raises(_lib.FtheError):
        Device(0)


def test_missing_library_raises(tmp_path):
    code = ("import sys; sys.path.insert(0, %r); from fedtree_amd import _lib\n"
            "try:\n    _lib.load(%r)\nexcept OSError:\n    print('raised')\n") % (
        str(_lib._HERE).rsplit("/", 1)[0], str(tmp_path / "nope.so"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True).stdout
    assert "raised" in out
