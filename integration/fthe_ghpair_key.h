// fthe_ghpair_key.h -- the key a GHPair carries in a FedTree build with USE_HIP.
//
// In the reference's GPU build every GHPair holds a `Paillier_GMP paillier` (common.h:72) and its
// operators run on it on the host: operator+ / += call paillier.add(res, x, y) (common.h:150-237),
// operator- calls paillier.mul(res, x, (unsigned long)-1) then add (common.h:253-309), and an
// unencrypted operand is promoted by homo_encrypt(pl) -> pl.encrypt(enc, m) (common.h:75-97).
// Paillier_GMP::add zeroes an aliased accumulator (mpz_init(result) before the multiply,
// paillier_gmp.cpp:16-20), so `+=` (common.h:207, 221, 229) loses the sum.
//
// Paillier_HIP_Pub has the members the operator text uses -- encrypt / add / mul with
// Paillier_GMP's signatures, the public fields n, n_square, generator, key_length, public-part
// assignment -- and computes them on the engine:
//   add     -> fthe_add_shared             (alias-safe: res may be x or y)
//   mul     -> fthe_scalar_mul_u64_shared  (fthe_scalar_mul_words for exponents above 64 bits)
//   encrypt -> fthe_encrypt_shared         (a fresh uniform r per ciphertext)
// The *_shared calls are thread-safe without a context and merge concurrent callers of one key
// (FedTree's OpenMP loops over bins / features) into one launch.  The maintainer's change to
// common.h is the member type and the branch condition:
//     #if defined(USE_HIP)
//         #include "fthe_ghpair_key.h"
//         typedef Paillier_HIP_Pub GHPairKey;
//     #elif defined(USE_CUDA) ... typedef Paillier_GMP GHPairKey;
//     struct GHPair { ... GHPairKey paillier; ... }   and `#ifdef USE_CUDA` -> `#if defined(USE_CUDA) || defined(USE_HIP)`
// so the operator bodies compile unchanged.
#pragma once
#include <gmp.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fthe.h"

namespace fthe_shim {
// Engine status codes become exceptions.  The reference aborts on engine errors (CUDA_CHECK ->
// CHECK_EQ, exit(1); common.h:47-52, paillier_gpu.cu:13-16): uncaught, an exception does the same
// (std::terminate), and a caller that wants to recover can catch it.  Define FTHE_SHIM_ABORT to
// print and abort() instead, as LOG(FATAL) would.
inline void check(int st, const char *what) {
    if (st == FTHE_OK) return;
#ifdef FTHE_SHIM_ABORT
    std::fprintf(stderr, "fthe: %s: %s\n", what, fthe_strerror(st));
    std::abort();
#else
    throw std::runtime_error(std::string(what) + ": " + fthe_strerror(st));
#endif
}
// One engine context per host thread (the boundary is entered from OpenMP
// regions, FLtrainer.cpp:275-306); device from FTHE_DEVICE (default 0).
inline fthe_ctx *thread_ctx() {
    static thread_local fthe_ctx *c = nullptr;
    if (!c) {
        const char *d = std::getenv("FTHE_DEVICE");
        check(fthe_ctx_create(d ? std::atoi(d) : 0, &c), "fthe_ctx_create");
    }
    return c;
}
// mpz <-> little-endian u32 words (paillier_gpu.cu:7,18 order)
inline void to_words(const mpz_t x, uint32_t *w, int nw) {
    size_t cnt = 0;
    for (int i = 0; i < nw; i++) w[i] = 0;
    if (mpz_sgn(x) < 0) throw std::runtime_error("negative operand");
    if (mpz_sizeinbase(x, 2) > (size_t)nw * 32) throw std::runtime_error("operand does not fit");
    mpz_export(w, &cnt, -1, 4, 0, 0, x);
}
inline void from_words(mpz_t x, const uint32_t *w, int nw) { mpz_import(x, (size_t)nw, -1, 4, 0, 0, w); }
inline size_t words_of(const mpz_t x) { return (mpz_sizeinbase(x, 2) + 31) / 32; }
}  // namespace fthe_shim

// The engine key shared by every copy of a handle (copies are cheap: GHPair copies its key on every
// operator, common.h:170, 190, 384).  Keys are immutable in the engine and usable from any thread.
using fthe_key_ref = std::shared_ptr<fthe_key>;
inline fthe_key_ref fthe_key_adopt(fthe_key *k) { return fthe_key_ref(k, [](fthe_key *p) { fthe_key_destroy(p); }); }

class Paillier_HIP_Pub {
public:
    Paillier_HIP_Pub() { mpz_init(n); mpz_init(n_square); mpz_init(generator); }
    Paillier_HIP_Pub(const Paillier_HIP_Pub &o) : Paillier_HIP_Pub() { *this = o; }
    ~Paillier_HIP_Pub() { mpz_clear(n); mpz_clear(n_square); mpz_clear(generator); }
    // Paillier_GMP::operator= (paillier_gmp.h:12-21): the public part only
    Paillier_HIP_Pub &operator=(const Paillier_HIP_Pub &o) {
        if (this == &o) return *this;
        mpz_set(n, o.n);
        mpz_set(n_square, o.n_square);
        mpz_set(generator, o.generator);
        key_length = o.key_length;
        key_ = o.key_;
#ifdef FTHE_REFERENCE_SHARED_R
        shared_r_ = o.shared_r_;
#endif
        return *this;
    }

    // Bind to an engine key (Paillier_HIP::keygen / key_from_primes / parameters_cpu_to_gpu).
    void bind(const fthe_key_ref &k, uint32_t keyLength) {
        key_ = k;
        const int nw = fthe_key_n_words(k.get());
        std::vector<uint32_t> w(nw);
        fthe_shim::check(fthe_key_export(k.get(), w.data(), nullptr, nullptr, nullptr, nullptr), "export");
        fthe_shim::from_words(n, w.data(), nw);
        mpz_mul(n_square, n, n);
        mpz_add_ui(generator, n, 1);
        key_length = keyLength;
    }
    fthe_key *key() const { return key_.get(); }
    int n_words() const { return fthe_key_n_words(need()); }

    // Paillier_GMP::encrypt (paillier_gmp.cpp:37-73): r <- g^m r'^n mod n^2 with a fresh uniform r'.
    // GHPair::homo_encrypt passes the codec value (common.h:81-88): m < 2^64.
    void encrypt(mpz_t &r, const mpz_t &message) const {
        fthe_key *k = need();
        const int cw = 2 * fthe_key_n_words(k);
        std::vector<uint32_t> c(cw);
        if (mpz_sgn(message) < 0) throw std::runtime_error("encrypt: negative plaintext");
#ifdef FTHE_REFERENCE_SHARED_R
        if (!shared_r_.empty()) {                 // reference GMP / GPU semantics: one fixed r
            const int nw = fthe_key_n_words(k), mw = std::max<int>(1, (int)fthe_shim::words_of(message));
            std::vector<uint32_t> m(mw);
            fthe_shim::to_words(message, m.data(), mw);
            fthe_shim::check(fthe_encrypt_words(k, fthe_shim::thread_ctx(), m.data(), mw, 1, shared_r_.data(), nw, 0,
                                                c.data(), FTHE_ENC_PUBLIC), "encrypt");
            fthe_shim::from_words(r, c.data(), cw);
            return;
        }
#endif
        if (mpz_sizeinbase(message, 2) <= 64) {
            uint64_t m = 0;
            mpz_export(&m, nullptr, -1, 8, 0, 0, message);
            fthe_shim::check(fthe_encrypt_shared(k, &m, 1, c.data(), FTHE_ENC_DEFAULT), "encrypt");
        } else {                                  // Paillier::encrypt(ZZ) of any size (paillier.cpp:122)
            const int mw = (int)fthe_shim::words_of(message);
            std::vector<uint32_t> m(mw);
            fthe_shim::to_words(message, m.data(), mw);
            fthe_shim::check(fthe_encrypt_words(k, fthe_shim::thread_ctx(), m.data(), mw, 1, nullptr, 0, 0, c.data(),
                                                FTHE_ENC_DEFAULT), "encrypt");
        }
        fthe_shim::from_words(r, c.data(), cw);
    }

    // Paillier_GMP::add (paillier_gmp.cpp:16-21): r <- x y mod n^2.  Alias-safe: both operands are
    // read before r is written, so add(s, s, c) (common.h:207, 221, 229) gives s c, not 0.  r must be
    // initialised, as every GHPair operand is (common.h:347-386).
    void add(mpz_t &r, const mpz_t &x, const mpz_t &y) const {
        fthe_key *k = need();
        const int cw = 2 * fthe_key_n_words(k);
        uint32_t buf[3 * 256];
        std::vector<uint32_t> heap;
        uint32_t *a = buf;
        if (cw > 256) { heap.resize(3 * (size_t)cw); a = heap.data(); }
        uint32_t *b = a + cw, *o = b + cw;
        fthe_shim::to_words(x, a, cw);
        fthe_shim::to_words(y, b, cw);
        fthe_shim::check(fthe_add_shared(k, a, b, 1, o), "add");
        fthe_shim::from_words(r, o, cw);
    }

    // Paillier_GMP::mul (paillier_gmp.cpp:24-28): r <- x^y mod n^2.  Like the reference it
    // initialises r: operator- passes an uninitialised mpz_t (common.h:270-272).  Alias-safe.
    void mul(mpz_t &r, const mpz_t &x, const mpz_t &y) const {
        fthe_key *k = need();
        const int cw = 2 * fthe_key_n_words(k);
        std::vector<uint32_t> a(cw), o(cw);
        fthe_shim::to_words(x, a.data(), cw);
        if (mpz_sgn(y) < 0) throw std::runtime_error("mul: negative exponent");
        if (mpz_sizeinbase(y, 2) <= 64) {
            uint64_t e = 0;
            mpz_export(&e, nullptr, -1, 8, 0, 0, y);
            fthe_shim::check(fthe_scalar_mul_u64_shared(k, a.data(), e, 1, o.data()), "mul");
        } else {
            std::vector<uint32_t> e(fthe_shim::words_of(y));
            fthe_shim::to_words(y, e.data(), (int)e.size());
            fthe_shim::check(fthe_scalar_mul_words(k, fthe_shim::thread_ctx(), a.data(), e.data(), (int)e.size(), 1,
                                                   o.data()), "mul");
        }
        mpz_init(r);
        fthe_shim::from_words(r, o.data(), cw);
    }

#ifdef FTHE_REFERENCE_SHARED_R
    // Reference-compat randomness (opt-in at compile time): every encrypt() uses this one r, as
    // Paillier_GMP::encrypt does (its unseeded MT draws the same r on every call, paillier_gmp.cpp:40-52)
    // and as Paillier_GPU shares one r per batch (paillier_gpu.cu:262-272).  Reproduces the reference's
    // ciphertexts bit for bit (tests); not semantically secure -- never for production keys.
    void set_shared_r(const mpz_t rr) {
        shared_r_.assign((size_t)n_words(), 0u);
        fthe_shim::to_words(rr, shared_r_.data(), (int)shared_r_.size());
    }
#endif

    mpz_t n;
    mpz_t n_square;
    mpz_t generator;
    uint32_t key_length = 0;

private:
    fthe_key_ref key_;
#ifdef FTHE_REFERENCE_SHARED_R
    std::vector<uint32_t> shared_r_;
#endif
    fthe_key *need() const {
        if (!key_) throw std::runtime_error("Paillier_HIP_Pub: no key (keygen / assignment from a keyed object first)");
        return key_.get();
    }
};
