"""pyoracle.py -- TEST INFRASTRUCTURE ONLY.

Python view of the CPU oracle:
  * a pure-Python restatement of FedTree's NTL Paillier (paillier.cpp) for
    small cases (Python big-int pow), each function citing the reference;
  * a ctypes binding of oracle/liboracle.so (the C/GMP restatement,
    paillier_oracle.c) for batch checks and the bench's cpu_baseline leg;
  * a ctypes binding of oracle/_ref/libpaillier_gmp_ref.so, the reference's
    own Paillier_GMP compiled from /root/reference (present only in the build
    container; the golden vectors under tests/golden/ were made with it).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use it.
"""
import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpaillier_gmp_ref.so")


# --------------------------------------------------------------------------
# pure-Python restatement (paillier.cpp)
def L(x, n):
    """paillier.h:40  L_function(x) = (x - 1) / n."""
    return (x - 1) // n


def keygen_from_primes(p, q):
    """paillier.cpp:80-87 with injected primes."""
    n = p * q
    g = n + 1
    lam = (p - 1) * (q - 1) // math.gcd(p - 1, q - 1)
    mu = pow(L(pow(g, lam, n * n), n), -1, n)
    return dict(n=n, g=g, lam=lam, mu=mu, p=p, q=q, n2=n * n)


def encrypt(key, m, r):
    """paillier.cpp:134-137: PowerMod(g, m, n^2) * PowerMod(r, n, n^2) % n^2."""
    n2 = key["n2"]
    return pow(key["g"], m, n2) * pow(r, key["n"], n2) % n2


def decrypt(key, c):
    """paillier.cpp:153-156."""
    return L(pow(c, key["lam"], key["n2"]), key["n"]) * key["mu"] % key["n"]


def add(key, x, y):
    """paillier.cpp:103."""
    return x * y % key["n2"]


def mul(key, x, y):
    """paillier.cpp:118."""
    return pow(x, y, key["n2"])


def sub(key, a, b):
    """GHPair::operator- on two ciphertexts (common.h:311-317, NTL branch):
    add(a, mul(b, (unsigned long)-1))."""
    return add(key, a, mul(key, b, 2**64 - 1))


def scan_segments(key, cts, seg_ptr):
    """inclusive_scan_by_key (hist_tree_builder.cpp:695-708) with the add of
    paillier.cpp:103 as the operator: running products inside each segment."""
    out = list(cts[:seg_ptr[-1]])
    for s in range(len(seg_ptr) - 1):
        for t in range(seg_ptr[s] + 1, seg_ptr[s + 1]):
            out[t] = add(key, out[t - 1], cts[t])
    return out


def segment_product(key, cts, seg_ptr, idx=None):
    """Products of ciphertext segments (the add of paillier.cpp:103 folded over
    each segment, in member order).  An empty segment gives 1."""
    out = []
    for s in range(len(seg_ptr) - 1):
        acc = 1
        for t in range(seg_ptr[s], seg_ptr[s + 1]):
            acc = add(key, acc, cts[idx[t] if idx is not None else t])
        out.append(acc)
    return out


def histogram(key, gh_cts, bin_ids, cut_col_ptr, max_num_bin, enc_zero=None):
    """hist_tree_builder.cpp:574-595 (single node in level): for each feature
    fid and instance iid with bid = dense_bin_id[iid*n_col + fid] != max_num_bin,
    hist[cut_col_ptr[fid] + bid] = hist[...] + gh[iid].  Ciphertexts only (one
    of g or h); the first add promotes the unencrypted zero with
    Enc(0) (common.h:156-160) -- `enc_zero` stands for that fresh encryption
    (None: the multiplicative identity).  Untouched bins are None
    (unencrypted zero)."""
    n_col = len(cut_col_ptr) - 1
    n_inst = len(bin_ids) // n_col
    hist = [None] * cut_col_ptr[-1]
    for fid in range(n_col):
        for iid in range(n_inst):
            bid = int(bin_ids[iid * n_col + fid])
            if bid == max_num_bin:
                continue
            b = cut_col_ptr[fid] + bid
            if hist[b] is None:
                hist[b] = 1 if enc_zero is None else enc_zero
            hist[b] = add(key, hist[b], gh_cts[iid])
    return hist


def encode_fixed(x):
    """common.h:81-86 / :127: (uint64)(int64)((double)x * 1e6), truncating."""
    v = np.trunc(np.asarray(x, dtype=np.float32).astype(np.float64) * 1e6).astype(np.int64)
    return v.view(np.uint64)


def decode_fixed(m):
    """common.h:140-143 / paillier_gpu.cu:487: (float)((float)(long)v / 1e6)."""
    v = np.asarray(m, dtype=np.uint64).view(np.int64)
    return (v.astype(np.float32).astype(np.float64) / 1e6).astype(np.float32)


# --------------------------------------------------------------------------
# word helpers (little-endian u32, mpz_export order -1 / paillier_gpu.cu:7,18)
def to_words(x, nw):
    return np.array([(x >> (32 * i)) & 0xFFFFFFFF for i in range(nw)], dtype=np.uint32)


def from_words(w):
    w = np.asarray(w, dtype=np.uint64)
    v = 0
    for i in range(len(w) - 1, -1, -1):
        v = (v << 32) | int(w[i])
    return v


def ints_to_words(xs, nw):
    out = np.zeros((len(xs), nw), dtype=np.uint32)
    for i, x in enumerate(xs):
        out[i] = to_words(int(x), nw)
    return out


def words_to_ints(a):
    a = np.asarray(a)
    return [from_words(row) for row in a]


# --------------------------------------------------------------------------
# C oracle (paillier_oracle.c)
class COracle:
    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise OSError(f"{path} not built (make -C oracle)")
        lib = ctypes.CDLL(path)
        P, U32P = ctypes.c_void_p, ctypes.c_void_p
        lib.po_key_from_primes.restype = P
        lib.po_key_from_primes.argtypes = [U32P, U32P, ctypes.c_int]
        lib.po_key_from_n.restype = P
        lib.po_key_from_n.argtypes = [U32P, ctypes.c_int]
        lib.po_key_free.argtypes = [P]
        lib.po_key_export.argtypes = [P, U32P, U32P, U32P]
        lib.po_encrypt.argtypes = [P, ctypes.c_uint64, U32P, U32P]
        lib.po_decrypt.argtypes = [P, U32P, U32P]
        lib.po_decrypt.restype = ctypes.c_int
        lib.po_add.argtypes = [P, U32P, U32P, U32P]
        lib.po_mul_u64.argtypes = [P, U32P, ctypes.c_uint64, U32P]
        lib.po_encrypt_batch.argtypes = [P, U32P, U32P, ctypes.c_long, U32P, ctypes.c_int]
        lib.po_decrypt_batch.argtypes = [P, U32P, ctypes.c_long, U32P, ctypes.c_int]
        lib.po_decrypt_batch.restype = ctypes.c_int
        lib.po_add_batch.argtypes = [P, U32P, U32P, ctypes.c_long, U32P, ctypes.c_int]
        lib.po_next_prime.argtypes = [U32P, ctypes.c_int, U32P]
        lib.po_num_threads.restype = ctypes.c_int
        self.lib = lib

    def num_threads(self):
        return self.lib.po_num_threads()

    def next_prime(self, seed_words):
        seed_words = np.ascontiguousarray(seed_words, dtype=np.uint32)
        out = np.zeros_like(seed_words)
        self.lib.po_next_prime(seed_words.ctypes.data, len(seed_words), out.ctypes.data)
        return out

    def key(self, p_words, q_words):
        p_words = np.ascontiguousarray(p_words, dtype=np.uint32)
        q_words = np.ascontiguousarray(q_words, dtype=np.uint32)
        k = self.lib.po_key_from_primes(p_words.ctypes.data, q_words.ctypes.data, len(p_words))
        if not k:
            raise ValueError("oracle: invalid primes")
        return OracleKey(self, k, 2 * len(p_words))


class OracleKey:
    def __init__(self, o, handle, nw):
        self.o, self.h, self.nw = o, handle, nw

    def __del__(self):
        try:
            self.o.lib.po_key_free(self.h)
        except Exception:
            pass

    def encrypt_batch(self, m, r, threads=0):
        m = np.ascontiguousarray(m, dtype=np.uint64)
        r = np.ascontiguousarray(r, dtype=np.uint32)
        out = np.zeros((len(m), 2 * self.nw), dtype=np.uint32)
        self.o.lib.po_encrypt_batch(self.h, m.ctypes.data, r.ctypes.data, len(m), out.ctypes.data, threads)
        return out

    def decrypt_batch(self, c, threads=0):
        c = np.ascontiguousarray(c, dtype=np.uint32)
        out = np.zeros((len(c), self.nw), dtype=np.uint32)
        rc = self.o.lib.po_decrypt_batch(self.h, c.ctypes.data, len(c), out.ctypes.data, threads)
        assert rc == 0
        return out

    def add_batch(self, a, b, threads=0):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros_like(a)
        self.o.lib.po_add_batch(self.h, a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data, threads)
        return out

    def mul_u64(self, x, k):
        x = np.ascontiguousarray(x, dtype=np.uint32)
        out = np.zeros_like(x)
        self.o.lib.po_mul_u64(self.h, x.ctypes.data, ctypes.c_uint64(k), out.ctypes.data)
        return out


# --------------------------------------------------------------------------
# reference Paillier_GMP (compiled from /root/reference; build container only)
class RefGMP:
    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise OSError(f"{path} not built (make -C oracle ref)")
        lib = ctypes.CDLL(path)
        P = ctypes.c_void_p
        lib.ref_keygen.restype = P
        lib.ref_keygen.argtypes = [ctypes.c_uint32]
        lib.ref_free.argtypes = [P]
        lib.ref_n_words.restype = ctypes.c_int
        lib.ref_n_words.argtypes = [P]
        lib.ref_export.argtypes = [P, ctypes.c_int, P, P, P, P, P]
        lib.ref_encrypt.argtypes = [P, ctypes.c_int, ctypes.c_uint64, P]
        lib.ref_decrypt.argtypes = [P, ctypes.c_int, P, P]
        lib.ref_add.argtypes = [P, ctypes.c_int, P, P, P]
        lib.ref_add_aliased.argtypes = [P, ctypes.c_int, P, P]
        lib.ref_mul.argtypes = [P, ctypes.c_int, P, ctypes.c_uint64, P]
        lib.ref_shared_r.argtypes = [P, ctypes.c_int, P]
        lib.ref_encrypt_batch.argtypes = [P, ctypes.c_int, P, ctypes.c_long, P, ctypes.c_int]
        lib.ref_num_threads.restype = ctypes.c_int
        lib.ref_key_from_primes.restype = P
        lib.ref_key_from_primes.argtypes = [P, P, ctypes.c_int]
        lib.ref_decrypt_batch.argtypes = [P, ctypes.c_int, P, ctypes.c_long, P, ctypes.c_int]
        lib.ref_add_batch.argtypes = [P, ctypes.c_int, P, P, ctypes.c_long, P, ctypes.c_int]
        lib.ref_merge_batch.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_long, P, ctypes.c_int]
        self.lib = lib

    def key_from_primes(self, p, q):
        """Handle of a Paillier_GMP holding the key of primes p, q (ints); free with lib.ref_free."""
        w = (max(p.bit_length(), q.bit_length()) + 31) // 32
        pw, qw = to_words(p, w), to_words(q, w)
        h = self.lib.ref_key_from_primes(pw.ctypes.data, qw.ctypes.data, w)
        if not h:
            raise ValueError("reference key: mu not invertible")
        return h
