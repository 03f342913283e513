"""Host-side mirror of FedTree's homomorphic-encryption interface over libfthe.so.

Reference interface (FedTree, file:line):
  Paillier            include/FedTree/Encryption/paillier.h:6-41, src/.../paillier.cpp
  Paillier_GPU        include/FedTree/Encryption/paillier_gpu.h:28-94, paillier_gpu.cu
  GHPair HE codec     include/FedTree/common.h:65-412
  Server HE methods   include/FedTree/FL/server.h:58-135
  Party HE methods    include/FedTree/FL/party.h:118-142

Every computation goes through the HIP engine (libfthe.so).  There is no CPU
fallback: without the library or a gfx950 device the constructors raise.
Ciphertexts are numpy uint32 arrays of shape (count, 2*n_words), the
little-endian word order of mpz_export(order=-1) (paillier_gpu.cu:7,18); batch
calls also accept torch tensors resident on the device (the *_dev paths).
"""
import ctypes
import functools
import threading

import numpy as np

from . import _lib

MINUS_ONE = 2**64 - 1   # (unsigned long)-1, common.h:264-267 / :311


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _words(x, nw):
    return np.array([(x >> (32 * i)) & 0xFFFFFFFF for i in range(nw)], dtype=np.uint32)


def _int(w):
    v = 0
    for x in np.asarray(w, dtype=np.uint64)[::-1]:
        v = (v << 32) | int(x)
    return v


# --------------------------------------------------------------------------
# codec (common.h:81-86, 127-128, 140-143): host marshalling, as the reference
# does it on the host (paillier_gpu.cu:240-251, 480-489).
def encode_fixed(x):
    """(uint64)(long)((double)x * 1e6), truncating toward zero."""
    v = np.trunc(np.asarray(x, dtype=np.float32).astype(np.float64) * 1e6)
    return v.astype(np.int64).view(np.uint64)


def decode_fixed(m):
    """(float)((float)(long)low64 / 1e6)."""
    v = np.asarray(m, dtype=np.uint64).view(np.int64)
    return (v.astype(np.float32).astype(np.float64) / 1e6).astype(np.float32)


# --------------------------------------------------------------------------
class Device:
    """One engine context (HIP stream + workspace) on one GPU.

    The C ABI context is single-threaded; Device.current() hands each host
    thread its own context, so callers may enter from OpenMP-style thread
    pools as FedTree does (FLtrainer.cpp:275-306)."""

    _tls = threading.local()

    def __init__(self, device=0):
        self.lib = _lib.load()
        self.ctx = ctypes.c_void_p()
        _lib.check(self.lib.fthe_ctx_create(int(device), ctypes.byref(self.ctx)), "fthe_ctx_create")
        self.device = int(device)

    @classmethod
    def current(cls, device=0):
        d = getattr(cls._tls, "devs", None)
        if d is None:
            d = cls._tls.devs = {}
        if device not in d:
            d[device] = cls(device)
        return d[device]

    def sync(self):
        _lib.check(self.lib.fthe_ctx_sync(self.ctx), "sync")

    def set_mem_limit(self, nbytes):
        """Cap the slot region a call may grow on this context (0: none); calls whose two-stream form does not
        fit take the one-region form, bit-identical (include/fthe.h fthe_ctx_set_mem_limit)."""
        _lib.check(self.lib.fthe_ctx_set_mem_limit(self.ctx, int(nbytes)), "set_mem_limit")

    # Stream order with torch: the engine runs on its own HIP stream, so a device-resident
    # call first waits for the work torch has queued on its current stream (the producers of
    # the inputs, e.g. a torch.zeros fill of the output), and torch's stream then waits for
    # the engine, so consumers of the outputs see them -- no host synchronisation.
    def _ext_stream(self):
        import torch
        st = getattr(self, "_ext", None)
        if st is None:
            st = self._ext = torch.cuda.ExternalStream(self.lib.fthe_ctx_stream(self.ctx),
                                                       device=torch.device("cuda", self.device))
        return st

    def order_in(self):
        import torch
        self._ext_stream().wait_stream(torch.cuda.current_stream(self.device))

    def order_out(self):
        import torch
        torch.cuda.current_stream(self.device).wait_stream(self._ext_stream())

    def last_kernel_ms(self):
        return self.lib.fthe_last_kernel_ms(self.ctx)

    def last_montmuls(self):
        return self.lib.fthe_last_montmuls(self.ctx)

    def close(self):
        if self.ctx:
            self.lib.fthe_ctx_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream_ordered(fn):
    """Device-resident method: ordered after torch's queued work, torch ordered after it."""
    @functools.wraps(fn)
    def wrap(self, *a, **k):
        self.dev.order_in()
        try:
            return fn(self, *a, **k)
        finally:
            self.dev.order_out()
    return wrap


class PublicBases(list):
    """Published fixed-base bases hs_i (ints) and the bits of each base's exponent."""

    def __init__(self, hs, exp_bits):
        super().__init__(hs)
        self.exp_bits = list(exp_bits)



def _check_out(out, shape, what):
    """A caller's output rows: the engine writes count x row words straight into them, so they must be a
    C-contiguous uint32 array of exactly the operand's shape (a converted copy would take the result)."""
    if not (isinstance(out, np.ndarray) and out.dtype == np.uint32 and out.flags.c_contiguous
            and out.flags.writeable and out.shape == tuple(shape)):
        raise ValueError(f"{what}: out must be a writable C-contiguous uint32 array of shape {tuple(shape)}")
    return out

class Paillier:
    """Paillier key + batch engine (mirror of Paillier / Paillier_GPU).

    Public fields follow paillier.h: modulus, generator, keyLength, p, q,
    lambda_ (lambda), u (mu).  `keyLength` is the bit length of n, as in the
    NTL build (paillier.cpp:53-54)."""

    def __init__(self, device=None):
        self.dev = device if isinstance(device, Device) else Device.current(device or 0)
        self.lib = self.dev.lib
        self._key = None
        self.modulus = self.generator = None
        self.keyLength = 0
        self.p = self.q = self.lambda_ = self.u = None

    # ---- key management -------------------------------------------------
    def _adopt(self, key):
        if self._key:
            self.lib.fthe_key_destroy(self._key)
        self._key = key
        self.n_words = self.lib.fthe_key_n_words(key)
        nw = self.n_words
        n = np.zeros(nw, np.uint32)
        if self.lib.fthe_key_has_private(key):
            lam, mu = np.zeros(nw, np.uint32), np.zeros(nw, np.uint32)
            p, q = np.zeros((nw + 1) // 2, np.uint32), np.zeros((nw + 1) // 2, np.uint32)
            _lib.check(self.lib.fthe_key_export(key, _ptr(n), _ptr(lam), _ptr(mu), _ptr(p), _ptr(q)), "export")
            self.lambda_, self.u, self.p, self.q = _int(lam), _int(mu), _int(p), _int(q)
        else:
            _lib.check(self.lib.fthe_key_export(key, _ptr(n), None, None, None, None), "export")
        self.modulus = _int(n)
        self.generator = self.modulus + 1
        self.keyLength = self.modulus.bit_length()
        self.n2 = self.modulus * self.modulus
        return self

    def keygen(self, keyLength, seed=0, known_order=False):
        """Paillier::keygen(int keyLength) (paillier.cpp:66-90).  known_order: primes with a
        factored P - 1 (FTHE_KEYGEN_KNOWN_ORDER: one generator per prime in the exact
        fixed-base mode; not the reference's prime distribution)."""
        key = ctypes.c_void_p()
        flags = _lib.FTHE_KEYGEN_KNOWN_ORDER if known_order else 0
        _lib.check(self.lib.fthe_key_generate_ex(self.dev.ctx, int(keyLength), int(seed), flags, ctypes.byref(key)),
                   "keygen")
        return self._adopt(key)

    @classmethod
    def from_primes(cls, p, q, device=None):
        self = cls(device)
        hw = max((p.bit_length() + 31) // 32, (q.bit_length() + 31) // 32)
        pw, qw = _words(p, hw), _words(q, hw)
        key = ctypes.c_void_p()
        _lib.check(self.lib.fthe_key_from_primes(self.dev.ctx, _ptr(pw), _ptr(qw), hw, ctypes.byref(key)),
                   "key_from_primes")
        return self._adopt(key)

    @classmethod
    def from_public(cls, n, device=None):
        self = cls(device)
        nw = (n.bit_length() + 31) // 32
        w = _words(n, nw)
        key = ctypes.c_void_p()
        _lib.check(self.lib.fthe_key_from_n(self.dev.ctx, _ptr(w), nw, ctypes.byref(key)), "key_from_n")
        return self._adopt(key)

    def public(self, bases=None):
        """Paillier::operator= (paillier.h:12-18): copies modulus, generator, keyLength only.
        bases: published public_bases() to build the party's exact fixed-base tables with."""
        pub = Paillier.from_public(self.modulus, self.dev)
        if bases is not None:
            pub.set_public_bases(bases)
        return pub

    @property
    def has_private(self):
        return bool(self._key) and bool(self.lib.fthe_key_has_private(self._key))

    def __del__(self):
        try:
            if self._key:
                self.lib.fthe_key_destroy(self._key)
        except Exception:
            pass

    # ---- batch API (host arrays) ---------------------------------------------
    def _cw(self):
        return 2 * self.n_words

    @staticmethod
    def _flags(public, fixed_base, fixed_base_exact=False):
        return (_lib.FTHE_ENC_PUBLIC if public else _lib.FTHE_ENC_DEFAULT) | \
            (_lib.FTHE_ENC_FIXED_BASE if fixed_base else 0) | \
            (_lib.FTHE_ENC_FIXED_BASE_EXACT if fixed_base_exact else 0)

    def set_fixed_base(self, h=None):
        """(Re)build the fixed-base randomizer tables for base h (None: random h)."""
        hw = None if h is None else _words(int(h), self.n_words)
        _lib.check(self.lib.fthe_key_fixed_base(self._key, self.dev.ctx, _ptr(hw), self.n_words if hw is not None else 0),
                   "key_fixed_base")

    def fixed_base_info(self):
        """(alpha_bits_public, alpha_bits_crt, hs) of the built fixed-base tables."""
        ap, ac = ctypes.c_int(), ctypes.c_int()
        hs = np.zeros(self._cw(), dtype=np.uint32)
        _lib.check(self.lib.fthe_key_fixed_base_info(self._key, ctypes.byref(ap), ctypes.byref(ac), _ptr(hs)),
                   "key_fixed_base_info")
        return ap.value, ac.value, int.from_bytes(hs.tobytes(), "little")

    def set_fixed_base_exact(self, seed=0):
        """(Re)build the exact fixed-base tables (key holder; seed 0: bases from /dev/urandom)."""
        _lib.check(self.lib.fthe_key_fixed_base_exact(self._key, self.dev.ctx, int(seed)), "key_fixed_base_exact")

    def fixed_base_exact_info(self):
        """([[gam_p1, ...], [gam_q1, ...]], words per exponent): 3 bases per prime, or 1 (a
        generator) for known-order keys."""
        gam, ew = [[], []], ctypes.c_int()
        buf = np.zeros(self.n_words, dtype=np.uint32)
        nb = self.lib.fthe_key_fixed_base_exact_bases(self._key)
        for side in (0, 1):
            for b in range(nb):
                _lib.check(self.lib.fthe_key_fixed_base_exact_info(self._key, side, b, _ptr(buf), ctypes.byref(ew)),
                           "key_fixed_base_exact_info")
                gam[side].append(int.from_bytes(buf.tobytes(), "little"))
        return gam, ew.value

    def public_bases(self, seed=0):
        """Key holder: bases hs_i = t_i^n mod n^2 with <t_i> = Z_n^* (checked), to publish with n
        (fthe_key_public_bases).  Returns a PublicBases list of 3 ints (2 for known-order keys)
        carrying the exponent bits of each base (.exp_bits)."""
        nb = ctypes.c_int()
        _lib.check(self.lib.fthe_key_public_bases(self._key, int(seed), None, ctypes.byref(nb), None),
                   "key_public_bases")
        hs = np.zeros((nb.value, self._cw()), dtype=np.uint32)
        eb = np.zeros(nb.value, dtype=np.int32)
        _lib.check(self.lib.fthe_key_public_bases(self._key, int(seed), _ptr(hs), ctypes.byref(nb), _ptr(eb)),
                   "key_public_bases")
        return PublicBases([int.from_bytes(row.tobytes(), "little") for row in hs], [int(x) for x in eb])

    def set_public_bases(self, hs, exp_bits=None):
        """Build the public exact fixed-base tables for published bases (any key); exp_bits
        from a PublicBases list, or given, or None (full-length exponents)."""
        if exp_bits is None:
            exp_bits = getattr(hs, "exp_bits", None)
        arr = np.stack([_words(int(h), self._cw()) for h in hs])
        eb = None if exp_bits is None else np.ascontiguousarray(exp_bits, dtype=np.int32)
        _lib.check(self.lib.fthe_key_set_public_bases(self._key, self.dev.ctx, _ptr(arr), len(hs), _ptr(eb)),
                   "key_set_public_bases")

    @property
    def has_public_bases(self):
        return bool(self._key) and self.lib.fthe_key_public_bases_info(self._key, None, None) == 0

    def public_bases_info(self):
        """(bases, [words per injected exponent of each base]) of the built public tables."""
        nb, ew = ctypes.c_int(), np.zeros(3, dtype=np.int32)
        _lib.check(self.lib.fthe_key_public_bases_info(self._key, ctypes.byref(nb), _ptr(ew)),
                   "key_public_bases_info")
        return nb.value, [int(x) for x in ew[:nb.value]]

    def encrypt_u64(self, m, r=None, seed=0, public=False, fixed_base=False, fixed_base_exact=False, index0=0):
        """c = g^m r^n mod n^2 for every m (paillier.cpp:134-137).
        index0: m is the shard starting at element index0 of a larger batch (fthe_encrypt_u64_at): with a
           nonzero seed its device-drawn randomness is that of the whole batch's call at those positions.
        r: None -> fresh uniform r per ciphertext from the device CSPRNG;
           else (count, n_words) uint32 words or a list of ints.
        fixed_base: r = h^alpha from the key's fixed-base tables (include/fthe.h);
           r then injects alpha (ints or (count, words) uint32) instead of r.
        fixed_base_exact: r^n mod p^2, q^2 from the exact generator tables (key holder);
           r then injects the 2 * bases exponents per ciphertext ((count, 2 * bases * n_words/2)
           uint32 or tuples of ints; bases from fixed_base_exact_info).  On a public key (or
           with public=True): r^n = prod hs_i^y_i from the published bases (set_public_bases);
           r injects the `bases` exponents y_i (tuples of ints, see public_bases_info)."""
        m = np.ascontiguousarray(m, dtype=np.uint64).reshape(-1)
        cnt = len(m)
        out = np.zeros((cnt, self._cw()), dtype=np.uint32)
        rw = None
        if r is not None:
            if not isinstance(r, np.ndarray) and fixed_base_exact:
                if public or not self.has_private:  # tuples of `bases` exponents (public_bases_info)
                    hws = self.public_bases_info()[1]
                else:                               # tuples of 2 * bases exponents (fixed_base_exact_info)
                    hws = [self.n_words // 2] * 6
                r = np.stack([np.concatenate([_words(int(x), hw) for x, hw in zip(t, hws)]) for t in r]) if cnt \
                    else np.zeros((0, sum(hws)), np.uint32)
            if not isinstance(r, np.ndarray):
                nw = self.n_words + (2 if fixed_base else 0)
                if fixed_base and cnt:
                    nw = max(1, max((int(x).bit_length() + 31) // 32 for x in r))
                r = np.stack([_words(int(x), nw) for x in r]) if cnt else np.zeros((0, nw), np.uint32)
            rw = np.ascontiguousarray(r, dtype=np.uint32).reshape(cnt, -1)
        flags = self._flags(public, fixed_base, fixed_base_exact)
        _lib.check(self.lib.fthe_encrypt_u64_at(self._key, self.dev.ctx, _ptr(m), cnt, _ptr(rw),
                                                rw.shape[1] if rw is not None else 0, int(seed), int(index0),
                                                _ptr(out), flags), "encrypt")
        return out

    def direct_y(self, seed, index0, count):
        """(y_p, y_q) words ((count, pq_words) uint32 each) that encrypt_u64[_dev](r=None, seed=seed)
        draws for ciphertexts [index0, index0 + count) on the key holder's direct-y path
        (fthe_debug_direct_y, test hook): r = CRT(y_p^(q^-1 mod p-1), y_q^(p^-1 mod q-1))."""
        if not seed:
            raise ValueError("direct_y needs the nonzero seed of the encrypt call")
        pw = (max(self.p.bit_length(), self.q.bit_length()) + 31) // 32
        yp = np.zeros((count, pw), dtype=np.uint32)
        yq = np.zeros((count, pw), dtype=np.uint32)
        _lib.check(self.lib.fthe_debug_direct_y(self._key, self.dev.ctx, int(seed), int(index0), int(count),
                                                _ptr(yp), _ptr(yq)), "debug_direct_y")
        return yp, yq

    def decrypt_u64(self, c, full=False, short=False):
        """Low 64 bits of m = L(c^lambda mod n^2) mu mod n (paillier.cpp:153-156).
        short: plaintexts known to be < p (FedTree's codec values and their sums):
        the p half of the CRT only (fthe_decrypt_short), half the work."""
        c = np.ascontiguousarray(c, dtype=np.uint32).reshape(-1, self._cw())
        cnt = len(c)
        low = np.zeros(cnt, dtype=np.uint64)
        fullw = np.zeros((cnt, self.n_words), dtype=np.uint32) if full else None
        fn = self.lib.fthe_decrypt_short if short else self.lib.fthe_decrypt
        _lib.check(fn(self._key, self.dev.ctx, _ptr(c), cnt, _ptr(low), _ptr(fullw)), "decrypt")
        return (low, fullw) if full else low

    def encrypt_u64_shared(self, m, public=False):
        """encrypt_u64 with fresh device randomness through the key's coalescing queue
        (fthe_encrypt_shared): thread-safe on one Paillier object, concurrent calls share a launch."""
        m = np.ascontiguousarray(m, dtype=np.uint64).reshape(-1)
        out = np.zeros((len(m), self._cw()), dtype=np.uint32)
        flags = _lib.FTHE_ENC_PUBLIC if public else 0
        _lib.check(self.lib.fthe_encrypt_shared(self._key, _ptr(m), len(m), _ptr(out), flags), "encrypt_shared")
        return out

    def decrypt_u64_shared(self, c, full=False, short=False):
        """decrypt_u64 through the key's coalescing queue (fthe_decrypt_shared): safe to call from
        many threads on one Paillier object; concurrent calls are merged into one batch
        (decrypt_gh per node from OpenMP threads, FLtrainer.cpp:758-764)."""
        c = np.ascontiguousarray(c, dtype=np.uint32).reshape(-1, self._cw())
        cnt = len(c)
        low = np.zeros(cnt, dtype=np.uint64)
        fullw = np.zeros((cnt, self.n_words), dtype=np.uint32) if full else None
        _lib.check(self.lib.fthe_decrypt_shared(self._key, _ptr(c), cnt, _ptr(low), _ptr(fullw), int(short)),
                   "decrypt_shared")
        return (low, fullw) if full else low

    def add_batch(self, a, b):
        """x*y mod n^2 (paillier.cpp:103), alias-safe."""
        a = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, self._cw())
        b = np.ascontiguousarray(b, dtype=np.uint32).reshape(-1, self._cw())
        out = np.zeros_like(a)
        _lib.check(self.lib.fthe_add(self._key, self.dev.ctx, _ptr(a), _ptr(b), len(a), _ptr(out)), "add")
        return out

    def add_shared(self, a, b, out=None):
        """add_batch through the key's coalescing queue (fthe_add_shared): thread-safe on one
        Paillier object, concurrent calls share a launch; out may be a or b (alias-safe)."""
        a = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, self._cw())
        b = np.ascontiguousarray(b, dtype=np.uint32).reshape(-1, self._cw())
        if b.shape != a.shape:
            raise ValueError(f"add_shared: operand shapes differ ({a.shape} vs {b.shape})")
        out = np.zeros_like(a) if out is None else _check_out(out, a.shape, "add_shared")
        _lib.check(self.lib.fthe_add_shared(self._key, _ptr(a), _ptr(b), len(a), _ptr(out)), "add_shared")
        return out

    def scalar_mul_shared(self, x, k, out=None):
        """scalar_mul through the key's coalescing queue (fthe_scalar_mul_u64_shared)."""
        x = np.ascontiguousarray(x, dtype=np.uint32).reshape(-1, self._cw())
        out = np.zeros_like(x) if out is None else _check_out(out, x.shape, "scalar_mul_shared")
        _lib.check(self.lib.fthe_scalar_mul_u64_shared(self._key, _ptr(x), int(k), len(x), _ptr(out)),
                   "scalar_mul_shared")
        return out

    def sub_batch(self, a, b):
        """a * b^(2^64-1) mod n^2: GHPair::operator- with both sides encrypted
        (common.h:311-317), one fused device program."""
        a = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, self._cw())
        b = np.ascontiguousarray(b, dtype=np.uint32).reshape(-1, self._cw())
        out = np.zeros_like(a)
        _lib.check(self.lib.fthe_sub(self._key, self.dev.ctx, _ptr(a), _ptr(b), len(a), _ptr(out)), "sub")
        return out

    def scan_segments(self, x, seg_ptr):
        """Inclusive prefix products inside each segment (hist_tree_builder.cpp:695-708)."""
        x = np.ascontiguousarray(x, dtype=np.uint32).reshape(-1, self._cw())
        seg = np.ascontiguousarray(seg_ptr, dtype=np.int64)
        out = np.zeros((int(seg[-1]), self._cw()), dtype=np.uint32)
        _lib.check(self.lib.fthe_scan_segments(self._key, self.dev.ctx, _ptr(x), _ptr(seg), len(seg) - 1, _ptr(out)),
                   "scan_segments")
        return out

    def reduce_kway(self, x):
        """x: (k, count, 2nw) -> prod over k (hist_tree_builder.cpp:1015-1058 merge)."""
        x = np.ascontiguousarray(x, dtype=np.uint32)
        k, cnt = x.shape[0], x.shape[1]
        out = np.zeros((cnt, self._cw()), dtype=np.uint32)
        _lib.check(self.lib.fthe_reduce_kway(self._key, self.dev.ctx, _ptr(x), k, cnt, _ptr(out)), "reduce_kway")
        return out

    def reduce_segments(self, x, seg_ptr, idx=None):
        """out[s] = prod x[idx[t]] over t in [seg_ptr[s], seg_ptr[s+1]) mod n^2
        (histogram scatter hist_tree_builder.cpp:565-595, root sum tree.cpp:20-34).
        Empty segments give 1."""
        x = np.ascontiguousarray(x, dtype=np.uint32).reshape(-1, self._cw())
        seg = np.ascontiguousarray(seg_ptr, dtype=np.int64)
        ix = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        out = np.zeros((len(seg) - 1, self._cw()), dtype=np.uint32)
        _lib.check(self.lib.fthe_reduce_segments(self._key, self.dev.ctx, _ptr(x), len(x), _ptr(seg), _ptr(ix),
                                                 len(seg) - 1, _ptr(out)), "reduce_segments")
        return out

    def scalar_mul(self, x, k):
        """x^k mod n^2 (paillier.cpp:118), k < 2^64."""
        x = np.ascontiguousarray(x, dtype=np.uint32).reshape(-1, self._cw())
        out = np.zeros_like(x)
        _lib.check(self.lib.fthe_scalar_mul_u64(self._key, self.dev.ctx, _ptr(x), int(k), len(x), _ptr(out)),
                   "scalar_mul")
        return out

    # ---- device-resident batch API (torch tensors on this device) -------------
    @_stream_ordered
    def encrypt_u64_dev(self, m, out, r=None, seed=0, public=False, fixed_base=False, fixed_base_exact=False,
                        index0=0):
        flags = self._flags(public, fixed_base, fixed_base_exact)
        rp = ctypes.c_void_p(r.data_ptr()) if r is not None else None
        rw = r.shape[-1] if r is not None else 0
        _lib.check(self.lib.fthe_encrypt_u64_at_dev(self._key, self.dev.ctx, ctypes.c_void_p(m.data_ptr()),
                                                    m.numel(), rp, rw, int(seed), int(index0),
                                                    ctypes.c_void_p(out.data_ptr()), flags), "encrypt_dev")
        return out

    @_stream_ordered
    def decrypt_u64_dev(self, c, out_low, short=False):
        cnt = c.numel() // self._cw()
        fn = self.lib.fthe_decrypt_short_dev if short else self.lib.fthe_decrypt_dev
        _lib.check(fn(self._key, self.dev.ctx, ctypes.c_void_p(c.data_ptr()), cnt,
                      ctypes.c_void_p(out_low.data_ptr()), None), "decrypt_dev")
        return out_low

    @_stream_ordered
    def to_mont_dev(self, x, out):
        """Montgomery-resident rows: out = x R mod n^2 (fthe_to_mont_dev)."""
        _lib.check(self.lib.fthe_to_mont_dev(self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()),
                                             x.numel() // self._cw(), ctypes.c_void_p(out.data_ptr())), "to_mont_dev")
        return out

    @_stream_ordered
    def from_mont_dev(self, x, out):
        """Montgomery-resident rows back to ciphertexts: out = x R^-1 mod n^2."""
        _lib.check(self.lib.fthe_from_mont_dev(self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()),
                                               x.numel() // self._cw(), ctypes.c_void_p(out.data_ptr())),
                   "from_mont_dev")
        return out

    @_stream_ordered
    def add_mont_dev(self, a, b, out):
        """Homomorphic add of Montgomery-resident rows, one product: (aR)(bR)R^-1 = (ab)R."""
        _lib.check(self.lib.fthe_add_mont_dev(self._key, self.dev.ctx, ctypes.c_void_p(a.data_ptr()),
                                              ctypes.c_void_p(b.data_ptr()), a.numel() // self._cw(),
                                              ctypes.c_void_p(out.data_ptr())), "add_mont_dev")
        return out

    @_stream_ordered
    def add_dev(self, a, b, out):
        cnt = a.numel() // self._cw()
        _lib.check(self.lib.fthe_add_dev(self._key, self.dev.ctx, ctypes.c_void_p(a.data_ptr()),
                                         ctypes.c_void_p(b.data_ptr()), cnt, ctypes.c_void_p(out.data_ptr())),
                   "add_dev")
        return out

    @_stream_ordered
    def sub_dev(self, a, b, out):
        cnt = a.numel() // self._cw()
        _lib.check(self.lib.fthe_sub_dev(self._key, self.dev.ctx, ctypes.c_void_p(a.data_ptr()),
                                         ctypes.c_void_p(b.data_ptr()), cnt, ctypes.c_void_p(out.data_ptr())),
                   "sub_dev")
        return out

    @_stream_ordered
    def scan_segments_dev(self, x, seg_ptr, out):
        seg = np.ascontiguousarray(seg_ptr, dtype=np.int64)
        _lib.check(self.lib.fthe_scan_segments_dev(self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()), _ptr(seg),
                                                   len(seg) - 1, ctypes.c_void_p(out.data_ptr())), "scan_segments_dev")
        return out

    @_stream_ordered
    def reduce_kway_dev(self, x, k, out):
        cnt = out.numel() // self._cw()
        _lib.check(self.lib.fthe_reduce_kway_dev(self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()), int(k),
                                                 cnt, ctypes.c_void_p(out.data_ptr())), "reduce_kway_dev")
        return out

    @_stream_ordered
    def reduce_segments_dev(self, x, seg_ptr, out, idx=None):
        """Device tensors x (count, 2nw) and out (nseg, 2nw); host seg_ptr / idx."""
        seg = np.ascontiguousarray(seg_ptr, dtype=np.int64)
        ix = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        cnt = x.numel() // self._cw()
        _lib.check(self.lib.fthe_reduce_segments_dev(self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()), cnt,
                                                     _ptr(seg), _ptr(ix), len(seg) - 1,
                                                     ctypes.c_void_p(out.data_ptr())), "reduce_segments_dev")
        return out

    @_stream_ordered
    def reduce_segments_csr_dev(self, x, seg_ptr, out, idx=None):
        """Segmented product with the CSR (int64 seg_ptr, optional int64 idx) on the device."""
        cnt = x.numel() // self._cw()
        _lib.check(self.lib.fthe_reduce_segments_csr_dev(
            self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()), cnt, ctypes.c_void_p(seg_ptr.data_ptr()),
            ctypes.c_void_p(idx.data_ptr()) if idx is not None else None, seg_ptr.numel() - 1,
            ctypes.c_void_p(out.data_ptr())), "reduce_segments_csr_dev")
        return out

    @_stream_ordered
    def histogram_dev(self, x, count, planes, bin_ids, cut_col_ptr, max_num_bin, out, inst=None, enc_zero=None):
        """Node histogram on the device (hist_tree_builder.cpp:565-595, :640-664).
        x: device (planes*count, 2nw) ciphertexts (g plane, h plane); bin_ids: device
        uint8 (count, n_col); inst: device int32 instance ids of the node or None;
        out: device (planes*n_bins, 2nw).  enc_zero: device (planes*n_bins, 2nw) Enc(0) rows folded
        into every populated bin -- the reference's first add into an unencrypted zero
        (common.h:156-160; fthe_histogram_zero_first_dev)."""
        cut = np.ascontiguousarray(cut_col_ptr, dtype=np.int32)
        n_col = len(cut) - 1
        n_sel = inst.numel() if inst is not None else count
        args = [self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()), int(count), int(planes),
                ctypes.c_void_p(bin_ids.data_ptr()), n_col, _ptr(cut), int(max_num_bin),
                ctypes.c_void_p(inst.data_ptr()) if inst is not None else None, int(n_sel)]
        if enc_zero is None:
            _lib.check(self.lib.fthe_histogram_dev(*args, ctypes.c_void_p(out.data_ptr())), "histogram_dev")
        else:
            _lib.check(self.lib.fthe_histogram_zero_first_dev(*args, ctypes.c_void_p(enc_zero.data_ptr()),
                                                              ctypes.c_void_p(out.data_ptr())), "histogram_zero_first")
        return out

    @_stream_ordered
    def reduce_segments_zero_first_dev(self, x, seg_ptr, enc_zero, out, idx=None):
        """reduce_segments_dev with an Enc(0) row per segment folded into every populated one
        (the reference's Q10 sequence, fthe_reduce_segments_zero_first_dev)."""
        seg = np.ascontiguousarray(seg_ptr, dtype=np.int64)
        ix = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        cnt = x.numel() // self._cw()
        _lib.check(self.lib.fthe_reduce_segments_zero_first_dev(
            self._key, self.dev.ctx, ctypes.c_void_p(x.data_ptr()), cnt, _ptr(seg), _ptr(ix), len(seg) - 1,
            ctypes.c_void_p(enc_zero.data_ptr()), ctypes.c_void_p(out.data_ptr())), "reduce_segments_zero_first")
        return out

    def encrypt_words(self, m, r=None, seed=0, public=False, fixed_base_exact=False):
        """General plaintexts (Paillier::encrypt(const ZZ&), paillier.cpp:122-139): m is a list of
        ints (any size up to n_words words) or a (count, words) uint32 array; r as encrypt_u64
        (fixed_base_exact: r = None, the device draws the exponents)."""
        if fixed_base_exact and r is not None:
            raise ValueError("encrypt_words: injected exponents go through encrypt_u64")
        if not isinstance(m, np.ndarray):
            m = np.stack([_words(int(x), self.n_words) for x in m]) if len(m) else np.zeros((0, self.n_words), np.uint32)
        m = np.ascontiguousarray(m, dtype=np.uint32)
        cnt, mw = m.shape
        out = np.zeros((cnt, self._cw()), dtype=np.uint32)
        rw = None
        if r is not None:
            rw = r if isinstance(r, np.ndarray) else np.stack([_words(int(x), self.n_words) for x in r])
            rw = np.ascontiguousarray(rw, dtype=np.uint32).reshape(cnt, -1)
        _lib.check(self.lib.fthe_encrypt_words(self._key, self.dev.ctx, _ptr(m), mw, cnt, _ptr(rw),
                                               rw.shape[1] if rw is not None else 0, int(seed), _ptr(out),
                                               self._flags(public, False, fixed_base_exact)), "encrypt_words")
        return out

    # ---- reference single-value signatures (batch of one) ------------------
    def encrypt(self, message, r=None):
        """Paillier::encrypt(const ZZ&) (paillier.cpp:122): any plaintext that fits in n_words."""
        message = int(message)
        if 0 <= message < 2**64:
            c = self.encrypt_u64(np.array([message], np.uint64), None if r is None else [int(r)])
        else:
            if message < 0 or message.bit_length() > 32 * self.n_words:
                raise ValueError("plaintext must be a non-negative integer of at most n_words words")
            c = self.encrypt_words([message], None if r is None else [int(r)])
        return _int(c[0])

    def decrypt(self, ciphertext):
        """Paillier::decrypt(const ZZ&) (paillier.cpp:141): the full plaintext."""
        c = _words(int(ciphertext), self._cw())[None]
        _, full = self.decrypt_u64(c, full=True)
        return _int(full[0])

    def add(self, x, y):
        """Paillier::add (paillier.cpp:92)."""
        return _int(self.add_batch(_words(int(x), self._cw())[None], _words(int(y), self._cw())[None])[0])

    def mul(self, x, y):
        """Paillier::mul (paillier.cpp:107): x^y mod n^2 for any y >= 0."""
        y = int(y)
        if y < 0:
            raise ValueError("exponent must be non-negative")
        xw = _words(int(x), self._cw())[None]
        if y < 2**64:
            return _int(self.scalar_mul(xw, y)[0])
        ew = _words(y, (y.bit_length() + 31) // 32)
        out = np.zeros_like(xw)
        _lib.check(self.lib.fthe_scalar_mul_words(self._key, self.dev.ctx, _ptr(xw), _ptr(ew), len(ew), 1, _ptr(out)),
                   "scalar_mul_words")
        return _int(out[0])


# --------------------------------------------------------------------------
class GHPairs:
    """A batch of GHPair (common.h:65-412): float g, h plus ciphertexts g_enc,
    h_enc and the `encrypted` flag.  Arrays are numpy; ciphertexts are
    (count, 2*n_words) uint32."""

    def __init__(self, g, h=None, paillier=None):
        self.g = np.ascontiguousarray(g, dtype=np.float32).copy()
        self.h = np.ascontiguousarray(h if h is not None else g, dtype=np.float32).copy()
        self.encrypted = False
        self.g_enc = self.h_enc = None
        self.paillier = paillier

    def __len__(self):
        return len(self.g)

    def homo_encrypt(self, pl, r_g=None, r_h=None, seed=0, fixed_base_exact=False):
        """GHPair::homo_encrypt (common.h:125-134): encrypt g,h, zero them, set encrypted.
        fixed_base_exact: the table-driven randomizer (key holder: same distribution; public
        key with published bases: within 2^-62 of it; otherwise the default path)."""
        if self.encrypted:
            return self
        m = np.concatenate([encode_fixed(self.g), encode_fixed(self.h)])
        r = None
        if r_g is not None:
            r = np.concatenate([np.asarray(r_g, np.uint32).reshape(len(self), -1),
                                np.asarray(r_h, np.uint32).reshape(len(self), -1)])
        fbx = fixed_base_exact and r is None and (pl.has_private or pl.has_public_bases)
        c = pl.encrypt_u64(m, r=r, seed=seed, fixed_base_exact=fbx)
        self.g_enc, self.h_enc = c[:len(self)], c[len(self):]
        self.paillier = pl
        self.g[:] = 0
        self.h[:] = 0
        self.encrypted = True
        return self

    def homo_decrypt(self, pl, short=False, shared=False):
        """GHPair::homo_decrypt (common.h:136-146): g = (float)(long)dec / 1e6.
        short: plaintexts known < p (codec values and their sums): p half of the CRT only.
        shared: through the key's coalescing queue (thread-safe on one key, fthe_decrypt_shared)."""
        if not self.encrypted:
            return self
        dec = pl.decrypt_u64_shared if shared else pl.decrypt_u64
        low = dec(np.concatenate([self.g_enc, self.h_enc]), short=short)
        self.g = decode_fixed(low[:len(self)])
        self.h = decode_fixed(low[len(self):])
        self.encrypted = False
        return self

    def _enc_side(self, pl):
        t = GHPairs(self.g, self.h)
        return t.homo_encrypt(pl)

    def __add__(self, rhs):
        """GHPair::operator+ (common.h:150-195).  An unencrypted side is first
        encrypted with a fresh r."""
        if not self.encrypted and not rhs.encrypted:
            return GHPairs(self.g + rhs.g, self.h + rhs.h)
        pl = rhs.paillier if not self.encrypted else self.paillier
        lhs = self if self.encrypted else self._enc_side(pl)
        r = rhs if rhs.encrypted else rhs._enc_side(pl)
        res = GHPairs(np.zeros(len(self), np.float32), np.zeros(len(self), np.float32), pl)
        both = pl.add_batch(np.concatenate([lhs.g_enc, lhs.h_enc]), np.concatenate([r.g_enc, r.h_enc]))
        res.g_enc, res.h_enc = both[:len(self)], both[len(self):]
        res.encrypted = True
        return res

    def __sub__(self, rhs):
        """GHPair::operator- (common.h:253-337): rhs^(2^64-1) then add; an
        unencrypted rhs is negated and encrypted."""
        if not self.encrypted and not rhs.encrypted:
            return GHPairs(self.g - rhs.g, self.h - rhs.h)
        if not rhs.encrypted:
            neg = GHPairs(-rhs.g, -rhs.h)
            return self + neg._enc_side(self.paillier)
        pl = rhs.paillier if not self.encrypted else self.paillier
        lhs = self if self.encrypted else self._enc_side(pl)
        both = pl.sub_batch(np.concatenate([lhs.g_enc, lhs.h_enc]), np.concatenate([rhs.g_enc, rhs.h_enc]))
        res = GHPairs(np.zeros(len(rhs), np.float32), np.zeros(len(rhs), np.float32), pl)
        res.g_enc, res.h_enc = both[:len(rhs)], both[len(rhs):]
        res.encrypted = True
        return res


def histogram_segments(bin_ids, cut_col_ptr, max_num_bin):
    """CSR form of the histogram scatter of hist_tree_builder.cpp:574-595:
    segment b (= cut_col_ptr[fid] + bid) lists, in the reference's accumulation
    order (instance order), the instances whose feature fid falls in bin bid;
    bid == max_num_bin (missing value) is skipped.
    bin_ids: uint8 (n_instances * n_columns), row-major by instance."""
    cut = np.asarray(cut_col_ptr, dtype=np.int64)
    n_col = len(cut) - 1
    b = np.asarray(bin_ids, dtype=np.int64).reshape(-1, n_col)
    n_inst = b.shape[0]
    valid = b != int(max_num_bin)
    key = b + cut[None, :-1]
    iid = np.broadcast_to(np.arange(n_inst, dtype=np.int64)[:, None], b.shape)
    key, iid = key[valid], iid[valid]
    order = np.argsort(key, kind="stable")      # stable: instance order inside a bin
    n_bins = int(cut[-1])
    counts = np.bincount(key, minlength=n_bins)[:n_bins]
    seg_ptr = np.zeros(n_bins + 1, dtype=np.int64)
    np.cumsum(counts, out=seg_ptr[1:])
    return seg_ptr, iid[order]


class HEServer:
    """Server HE members (server.h:47-135)."""

    def __init__(self, device=None):
        self.paillier = Paillier(device)

    def homo_init(self, keylength, seed=0):
        """server.h:58-67 (NTL build: keygen(keylength))."""
        self.paillier.keygen(keylength, seed)
        self._bases = None                      # published bases belong to the previous key

    def send_key(self, party, bases=False):
        """server.h:53-55: party.paillier = paillier (public part only).
        bases: also publish checked fixed-base bases (Paillier.public_bases) for the
        parties' FTHE_ENC_FIXED_BASE_EXACT histogram encryption."""
        if bases and getattr(self, "_bases", None) is None:
            self._bases = self.paillier.public_bases()
        party.paillier = self.paillier.public(self._bases if bases else None)

    def encrypt_gh_pairs(self, raw, seed=0, fixed_base_exact=False):
        """server.h:113-135."""
        return raw.homo_encrypt(self.paillier, seed=seed, fixed_base_exact=fixed_base_exact)

    def decrypt_gh_pairs(self, encrypted, short=False):
        """server.h:80-111.  short: see GHPairs.homo_decrypt (opt-in, ~2x)."""
        return encrypted.homo_decrypt(self.paillier, short=short)

    def decrypt_gh(self, gh):
        """server.h:69-78 (single pair).  FedTree calls it per tree node from OpenMP threads
        (FLtrainer.cpp:758-764): it goes through the key's coalescing queue, so concurrent
        calls share one launch and threads need no context of their own."""
        return gh.homo_decrypt(self.paillier, shared=True)


class HEParty:
    """Party HE members (party.h:118-142, 181-185)."""

    def __init__(self, paillier=None):
        self.paillier = paillier

    def encrypt_histogram(self, hist, seed=0, fixed_base_exact=False):
        """party.h:118-142.  fixed_base_exact: the published-bases randomizer (send_key(bases=True))."""
        return hist.homo_encrypt(self.paillier, seed=seed, fixed_base_exact=fixed_base_exact)

    def compute_histogram(self, gh, bin_ids, cut_col_ptr, max_num_bin):
        """Histogram of one node (hist_tree_builder.cpp:565-595, n_nodes_in_level == 1):
        hist[cut_col_ptr[fid] + bid] = sum of gh[iid] over the instances in that bin.

        Encrypted gh: one segmented product on the device for g and h together.
        Bins without instances stay unencrypted zero, as in the reference; a
        populated bin is the product of its members (the reference's first add
        also folds in a fresh Enc(0) from promoting the zero accumulator,
        common.h:156-160 -- same plaintext, different randomness).
        Plain gh: float32 accumulation in instance order (dest.g += src.g)."""
        seg_ptr, idx = histogram_segments(bin_ids, cut_col_ptr, max_num_bin)
        n_bins = len(seg_ptr) - 1
        if not gh.encrypted:
            key = np.repeat(np.arange(n_bins), np.diff(seg_ptr))
            hist = GHPairs(np.zeros(n_bins, np.float32), np.zeros(n_bins, np.float32))
            np.add.at(hist.g, key, gh.g[idx])
            np.add.at(hist.h, key, gh.h[idx])
            return hist
        pl = gh.paillier
        n = len(gh)
        both = np.concatenate([gh.g_enc, gh.h_enc])
        seg2 = np.concatenate([seg_ptr, seg_ptr[1:] + seg_ptr[-1]])
        idx2 = np.concatenate([idx, idx + n])
        prod = pl.reduce_segments(both, seg2, idx2)
        hist = GHPairs(np.zeros(n_bins, np.float32), np.zeros(n_bins, np.float32), pl)
        hist.g_enc, hist.h_enc = prod[:n_bins], prod[n_bins:]
        hist.encrypted = True
        hist.bin_encrypted = np.diff(seg_ptr) > 0
        return hist

    def prefix_histogram(self, hist, cut_col_ptr):
        """inclusive_scan_by_key over features (hist_tree_builder.cpp:695-708):
        bin b of feature f becomes the sum of bins cut_col_ptr[f] .. b.  One
        segmented scan on the device for g and h together.  (An untouched bin
        enters as the ciphertext 1; the reference would promote its zero with a
        fresh Enc(0) -- same plaintexts.)"""
        cut = np.asarray(cut_col_ptr, dtype=np.int64)
        n_bins = int(cut[-1])
        if not hist.encrypted:
            out = GHPairs(hist.g.copy(), hist.h.copy())
            for f in range(len(cut) - 1):
                out.g[cut[f]:cut[f + 1]] = np.cumsum(hist.g[cut[f]:cut[f + 1]], dtype=np.float32)
                out.h[cut[f]:cut[f + 1]] = np.cumsum(hist.h[cut[f]:cut[f + 1]], dtype=np.float32)
            return out
        pl = hist.paillier
        seg2 = np.concatenate([cut, cut[1:] + n_bins])
        sc = pl.scan_segments(np.concatenate([hist.g_enc, hist.h_enc]), seg2)
        out = GHPairs(np.zeros(n_bins, np.float32), np.zeros(n_bins, np.float32), pl)
        out.g_enc, out.h_enc = sc[:n_bins], sc[n_bins:]
        out.encrypted = True
        return out

    @staticmethod
    def sibling_histogram(father, computed):
        """hist_tree_builder.cpp:670-680: the larger child's histogram as
        father - computed (GHPair::operator-, one fused device op per bin)."""
        return father - computed


# --------------------------------------------------------------------------
# wire formats (fthe_wire.cpp): no device needed
def ct_to_decimal(ct, threads=0):
    """Ciphertext rows -> the reference's GHEncBatch decimal strings
    (`stream << g_enc`, distributed_server.cpp:37-54)."""
    lib = _lib.load()
    ct = np.ascontiguousarray(ct, dtype=np.uint32)
    cnt, words = ct.shape
    buf = np.zeros(max(1, cnt * lib.fthe_decimal_max_len(words)), dtype=np.uint8)
    offs = np.zeros(cnt + 1, dtype=np.uint64)
    _lib.check(lib.fthe_ct_to_decimal(_ptr(ct), words, cnt, _ptr(buf), buf.nbytes, _ptr(offs), threads), "to_decimal")
    raw = buf[: int(offs[-1])].tobytes()
    return [raw[int(offs[i]):int(offs[i + 1])].decode() for i in range(cnt)]


def ct_from_decimal(strings, words, threads=0):
    """NTL::to_ZZ(str) of the receiving side (distributed_party.cpp:1267-1273)."""
    lib = _lib.load()
    enc = [s.encode() for s in strings]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in enc]) if enc else []
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    out = np.zeros((len(enc), words), dtype=np.uint32)
    _lib.check(lib.fthe_ct_from_decimal(_ptr(buf), _ptr(offs), len(enc), words, _ptr(out), threads), "from_decimal")
    return out


def ct_to_decimal_dev(dev, ct):
    dev.order_in()
    try:
        return _ct_to_decimal_dev(dev, ct)
    finally:
        dev.order_out()


def _ct_to_decimal_dev(dev, ct):
    """Device ciphertext rows (torch int32/uint32, (count, words)) -> (buf, offsets): the
    strings of ct_to_decimal concatenated in a device uint8 tensor and count+1 int64
    device offsets, computed on the GPU (fthe_ct_to_decimal_dev)."""
    import torch
    cnt, words = ct.shape
    buf = torch.empty(max(1, cnt * dev.lib.fthe_decimal_max_len(words)), dtype=torch.uint8, device=ct.device)
    offs = torch.empty(cnt + 1, dtype=torch.int64, device=ct.device)
    _lib.check(dev.lib.fthe_ct_to_decimal_dev(dev.ctx, ctypes.c_void_p(ct.data_ptr()), words, cnt,
                                              ctypes.c_void_p(buf.data_ptr()), buf.numel(),
                                              ctypes.c_void_p(offs.data_ptr())), "to_decimal_dev")
    return buf, offs


def ct_from_decimal_dev(dev, buf, offs, words):
    dev.order_in()
    try:
        return _ct_from_decimal_dev(dev, buf, offs, words)
    finally:
        dev.order_out()


def _ct_from_decimal_dev(dev, buf, offs, words):
    """(buf, offsets) device tensors of decimal strings -> (count, words) int32 device rows."""
    import torch
    cnt = offs.numel() - 1
    out = torch.empty((cnt, words), dtype=torch.int32, device=buf.device)
    _lib.check(dev.lib.fthe_ct_from_decimal_dev(dev.ctx, ctypes.c_void_p(buf.data_ptr()),
                                                ctypes.c_void_p(offs.data_ptr()), cnt, words,
                                                ctypes.c_void_p(out.data_ptr())), "from_decimal_dev")
    return out


def wire_encode(g, h=None):
    """Binary "FTHW" frame of raw little-endian words."""
    lib = _lib.load()
    g = np.ascontiguousarray(g, dtype=np.uint32)
    cnt, words = g.shape
    hh = None if h is None else np.ascontiguousarray(h, dtype=np.uint32)
    out = np.zeros(lib.fthe_wire_size(cnt, words, hh is not None), dtype=np.uint8)
    ln = ctypes.c_size_t()
    _lib.check(lib.fthe_wire_encode(_ptr(g), _ptr(hh), cnt, words, _ptr(out), out.nbytes, ctypes.byref(ln)), "wire_encode")
    return out.tobytes()


def wire_decode(frame, words):
    lib = _lib.load()
    buf = np.frombuffer(frame, dtype=np.uint8).copy()
    cnt = ctypes.c_size_t()
    lib.fthe_wire_decode(_ptr(buf), buf.nbytes, words, None, None, 0, ctypes.byref(cnt))
    n = cnt.value
    g = np.zeros((n, words), np.uint32)
    h = np.zeros((n, words), np.uint32)
    with_h = len(frame) >= 8 and (frame[6] & 1)
    _lib.check(lib.fthe_wire_decode(_ptr(buf), buf.nbytes, words, _ptr(g), _ptr(h) if with_h else None, n,
                                    ctypes.byref(cnt)), "wire_decode")
    return (g, h) if with_h else (g, None)
