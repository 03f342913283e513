"""ctypes binding of libfthe.so (include/fthe.h).

The engine is native only: if libfthe.so is missing or no gfx950 device is
visible, every compute entry point raises -- there is no CPU fallback.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FTHE_LIB") or os.path.join(_HERE, "libfthe.so")   # FTHE_LIB: A/B builds only
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "fthe.h")

FTHE_OK = 0
FTHE_ERR_ARG = -1
FTHE_ERR_HIP = -2
FTHE_ERR_NOPRIV = -3
FTHE_ERR_UNSUPPORTED = -4
FTHE_ERR_KEY = -5
FTHE_ERR_NOMEM = -6
FTHE_ENC_DEFAULT = 0
FTHE_ENC_PUBLIC = 1
FTHE_ENC_FIXED_BASE = 2
FTHE_ENC_FIXED_BASE_EXACT = 4
FTHE_KEYGEN_KNOWN_ORDER = 1


class FtheError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        msg = _lib.fthe_strerror(status).decode() if _lib is not None else str(status)
        super().__init__(f"{what}: {msg} ({status})" if what else f"{msg} ({status})")


_lib = None

_P = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t
_I = ctypes.c_int

_PROTOS = {
    "fthe_version": (_I, []),
    "fthe_strerror": (ctypes.c_char_p, [_I]),
    "fthe_device_count": (_I, []),
    "fthe_ctx_create": (_I, [_I, _PP]),
    "fthe_ctx_destroy": (None, [_P]),
    "fthe_ctx_sync": (_I, [_P]),
    "fthe_ctx_stream": (_P, [_P]),
    "fthe_ctx_device": (_I, [_P]),
    "fthe_ctx_set_mem_limit": (_I, [_P, _SZ]),
    "fthe_host_alloc": (_I, [_SZ, _PP]),
    "fthe_debug_addb_image": (_I, [_P, _I, _P, _SZ, _P]),
    "fthe_debug_nadicb_image": (_I, [_P, _I, _P, _SZ, _P]),
    "fthe_debug_nadicb_prog": (_I, [_P, _P, _P, _I, _P, _I, _SZ, _I, _P]),
    "fthe_host_free": (None, [_P]),
    "fthe_key_generate": (_I, [_P, _I, _U64, _PP]),
    "fthe_key_generate_ex": (_I, [_P, _I, _U64, _I, _PP]),
    "fthe_key_from_primes": (_I, [_P, _P, _P, _I, _PP]),
    "fthe_key_from_n": (_I, [_P, _P, _I, _PP]),
    "fthe_key_destroy": (None, [_P]),
    "fthe_key_n_words": (_I, [_P]),
    "fthe_key_n_bits": (_I, [_P]),
    "fthe_key_has_private": (_I, [_P]),
    "fthe_key_export": (_I, [_P, _P, _P, _P, _P, _P]),
    "fthe_key_fixed_base": (_I, [_P, _P, _P, _I]),
    "fthe_key_fixed_base_info": (_I, [_P, _P, _P, _P]),
    "fthe_key_fixed_base_exact": (_I, [_P, _P, _U64]),
    "fthe_key_fixed_base_exact_info": (_I, [_P, _I, _I, _P, _P]),
    "fthe_key_fixed_base_exact_set": (_I, [_P, _P, _I, _P]),
    "fthe_key_fixed_base_exact_bases": (_I, [_P]),
    "fthe_next_prime": (_I, [_P, _I, _P, _I]),
    "fthe_key_public_bases": (_I, [_P, _U64, _P, _P, _P]),
    "fthe_key_set_public_bases": (_I, [_P, _P, _P, _I, _P]),
    "fthe_key_public_bases_info": (_I, [_P, _P, _P]),
    "fthe_encrypt_u64_dev": (_I, [_P, _P, _P, _SZ, _P, _I, _U64, _P, _I]),
    "fthe_encrypt_u64": (_I, [_P, _P, _P, _SZ, _P, _I, _U64, _P, _I]),
    "fthe_encrypt_u64_at_dev": (_I, [_P, _P, _P, _SZ, _P, _I, _U64, _U64, _P, _I]),
    "fthe_encrypt_u64_at": (_I, [_P, _P, _P, _SZ, _P, _I, _U64, _U64, _P, _I]),
    "fthe_encrypt_words_dev": (_I, [_P, _P, _P, _I, _SZ, _P, _I, _U64, _P, _I]),
    "fthe_encrypt_words": (_I, [_P, _P, _P, _I, _SZ, _P, _I, _U64, _P, _I]),
    "fthe_decrypt_dev": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "fthe_decrypt": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "fthe_decrypt_short_dev": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "fthe_decrypt_short": (_I, [_P, _P, _P, _SZ, _P, _P]),
    "fthe_decrypt_shared": (_I, [_P, _P, _SZ, _P, _P, _I]),
    "fthe_encrypt_shared": (_I, [_P, _P, _SZ, _P, _I]),
    "fthe_add_dev": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_to_mont_dev": (_I, [_P, _P, _P, _SZ, _P]),
    "fthe_from_mont_dev": (_I, [_P, _P, _P, _SZ, _P]),
    "fthe_add_mont_dev": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_add": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_add_shared": (_I, [_P, _P, _P, _SZ, _P]),
    "fthe_scalar_mul_u64_shared": (_I, [_P, _P, _U64, _SZ, _P]),
    "fthe_scalar_mul_u64_dev": (_I, [_P, _P, _P, _U64, _SZ, _P]),
    "fthe_scalar_mul_u64": (_I, [_P, _P, _P, _U64, _SZ, _P]),
    "fthe_scalar_mul_words_dev": (_I, [_P, _P, _P, _P, _I, _SZ, _P]),
    "fthe_scalar_mul_words": (_I, [_P, _P, _P, _P, _I, _SZ, _P]),
    "fthe_reduce_kway_dev": (_I, [_P, _P, _P, _I, _SZ, _P]),
    "fthe_reduce_kway": (_I, [_P, _P, _P, _I, _SZ, _P]),
    "fthe_decimal_max_len": (_SZ, [_I]),
    "fthe_ct_to_decimal": (_I, [_P, _I, _SZ, _P, _SZ, _P, _I]),
    "fthe_ct_from_decimal": (_I, [_P, _P, _SZ, _I, _P, _I]),
    "fthe_ct_to_decimal_dev": (_I, [_P, _P, _I, _SZ, _P, _SZ, _P]),
    "fthe_ct_from_decimal_dev": (_I, [_P, _P, _P, _SZ, _I, _P]),
    "fthe_wire_size": (_SZ, [_SZ, _I, _I]),
    "fthe_wire_encode": (_I, [_P, _P, _SZ, _I, _P, _SZ, _P]),
    "fthe_wire_decode": (_I, [_P, _SZ, _I, _P, _P, _SZ, _P]),
    "fthe_sub_dev": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_sub": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_scan_segments_dev": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_scan_segments": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "fthe_reduce_segments_dev": (_I, [_P, _P, _P, _SZ, _P, _P, _SZ, _P]),
    "fthe_reduce_segments": (_I, [_P, _P, _P, _SZ, _P, _P, _SZ, _P]),
    "fthe_reduce_segments_csr_dev": (_I, [_P, _P, _P, _SZ, _P, _P, _SZ, _P]),
    "fthe_histogram_dev": (_I, [_P, _P, _P, _SZ, _I, _P, _I, _P, _I, _P, _SZ, _P]),
    "fthe_histogram_zero_first_dev": (_I, [_P, _P, _P, _SZ, _I, _P, _I, _P, _I, _P, _SZ, _P, _P]),
    "fthe_reduce_segments_zero_first_dev": (_I, [_P, _P, _P, _SZ, _P, _P, _SZ, _P, _P]),
    "fthe_encode_fixed_dev": (_I, [_P, _P, _SZ, _P]),
    "fthe_decode_fixed_dev": (_I, [_P, _P, _SZ, _P]),
    "fthe_last_kernel_ms": (ctypes.c_double, [_P]),
    "fthe_last_montmuls": (ctypes.c_double, [_P]),
    "fthe_kernel_limbs": (_I, [_I]),
    "fthe_debug_direct_y": (_I, [_P, _P, _U64, _U64, _SZ, _P, _P]),
    "fthe_prof_enable": (_I, [_P, _I]),
    "fthe_prof_variant": (_I, [_P, _I, _P, _P]),
    "fthe_prof_exec_macs": (_I, [_P, _P]),
    "fthe_prof_read": (_I, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "fthe_prof_busy": (_I, [_P, _P, _P]),
}


def header_symbols(path=HEADER_PATH):
    """Every function declared in include/fthe.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fthe_[a-z0-9_]+)\s*\(", src)))


def load(path=LIB_PATH):
    """Load libfthe.so and bind prototypes.  Raises OSError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"libfthe.so not built at {path} (run python fedtree_amd/build.py)")
    # One HIP runtime per process: when PyTorch is present (device buffers, streams),
    # load it first so libfthe.so binds to the libamdhip64.so.7 it already mapped;
    # loading ours first would bring up a second HIP/HSA runtime and torch then
    # reports "No HIP GPUs are available".
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status, what=""):
    if status != FTHE_OK:
        raise FtheError(status, what)
    return status
