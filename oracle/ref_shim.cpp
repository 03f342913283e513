// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" wrapper around the reference's own Paillier_GMP class, compiled
// from /root/reference/src/FedTree/Encryption/paillier_gmp.cpp (never copied)
// by oracle/Makefile into oracle/_ref/libpaillier_gmp_ref.so.  Used by
// tests/golden/make_golden.py to generate golden vectors and by tests to
// cross-check the C oracle (oracle/paillier_oracle.c).
#include "FedTree/Encryption/paillier_gmp.h"   // /root/reference/include
#include <cstring>
#include <cstdint>
#ifdef _OPENMP
#include <omp.h>
#endif

static void exp_words(uint32_t *w, int nw, const mpz_t x) {
    size_t cnt = 0;
    std::memset(w, 0, (size_t)nw * 4);
    mpz_export(w, &cnt, -1, 4, 0, 0, x);
}
static void imp_words(mpz_t x, const uint32_t *w, int nw) { mpz_import(x, (size_t)nw, -1, 4, 0, 0, w); }

extern "C" {

// Paillier_GMP::keyGen (paillier_gmp.cpp:108-239).  Returns a handle.
void *ref_keygen(uint32_t key_length) {
    Paillier_GMP *k = new Paillier_GMP();
    k->keyGen(key_length);
    return k;
}
void ref_free(void *h) { delete (Paillier_GMP *)h; }

// Words of n.
int ref_n_words(void *h) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    return (int)((mpz_sizeinbase(k->n, 2) + 31) / 32);
}
// Export the fields.  NOTE: after keyGen p,q hold p-1, q-1.
void ref_export(void *h, int nw, uint32_t *n, uint32_t *pm1, uint32_t *qm1, uint32_t *lambda, uint32_t *mu) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    exp_words(n, nw, k->n);
    exp_words(pm1, nw, k->p);
    exp_words(qm1, nw, k->q);
    exp_words(lambda, nw, k->lambda);
    exp_words(mu, nw, k->mu);
}
// Paillier_GMP::encrypt (paillier_gmp.cpp:37-73) of a 64-bit message.
void ref_encrypt(void *h, int nw, uint64_t m, uint32_t *out) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    mpz_t mz, c; mpz_init(mz);
    mpz_import(mz, 1, -1, 8, 0, 0, &m);
    k->encrypt(c, mz);
    exp_words(out, 2 * nw, c);
    mpz_clear(mz); mpz_clear(c);
}
// Batch form for the CPU baseline: OpenMP over elements exactly as
// Server::encrypt_gh_pairs does (server.h:129-133), each element one call of
// the reference's Paillier_GMP::encrypt (full PowerMod formula).
void ref_encrypt_batch(void *h, int nw, const uint64_t *m, long count, uint32_t *out, int threads) {
    Paillier_GMP *k = (Paillier_GMP *)h;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    #pragma omp parallel for schedule(dynamic, 4)
    for (long i = 0; i < count; i++) {
        mpz_t mz, c; mpz_init(mz);
        uint64_t v = m[i];
        mpz_import(mz, 1, -1, 8, 0, 0, &v);
        k->encrypt(c, mz);
        exp_words(out + (size_t)i * 2 * nw, 2 * nw, c);
        mpz_clear(mz); mpz_clear(c);
    }
}
int ref_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

// Paillier_GMP::decrypt (paillier_gmp.cpp:75-85); out: nw words.
void ref_decrypt(void *h, int nw, const uint32_t *c, uint32_t *out) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    mpz_t cz, m; mpz_init(cz);
    imp_words(cz, c, 2 * nw);
    k->decrypt(m, cz);
    exp_words(out, nw, m);
    mpz_clear(cz); mpz_clear(m);
}
// Paillier_GMP::add (paillier_gmp.cpp:16-21), non-aliased result.
void ref_add(void *h, int nw, const uint32_t *x, const uint32_t *y, uint32_t *out) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    mpz_t a, b, r; mpz_init(a); mpz_init(b);
    imp_words(a, x, 2 * nw); imp_words(b, y, 2 * nw);
    k->add(r, a, b);
    exp_words(out, 2 * nw, r);
    mpz_clear(a); mpz_clear(b); mpz_clear(r);
}
// The aliasing call add(s, s, c) as GHPair::operator+= makes it in the GPU
// build (common.h:207,221,229) -- SURVEY Q11: result is 0.
void ref_add_aliased(void *h, int nw, uint32_t *s, const uint32_t *y) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    mpz_t a, b; mpz_init(a); mpz_init(b);
    imp_words(a, s, 2 * nw); imp_words(b, y, 2 * nw);
    k->add(a, a, b);
    exp_words(s, 2 * nw, a);
    mpz_clear(a); mpz_clear(b);
}
// Paillier_GMP::mul (paillier_gmp.cpp:24-28) with a 64-bit exponent.
void ref_mul(void *h, int nw, const uint32_t *x, uint64_t y, uint32_t *out) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    mpz_t a, e, r; mpz_init(a); mpz_init(e);
    imp_words(a, x, 2 * nw);
    mpz_import(e, 1, -1, 8, 0, 0, &y);
    k->mul(r, a, e);
    exp_words(out, 2 * nw, r);
    mpz_clear(a); mpz_clear(e); mpz_clear(r);
}
// The r every Paillier_GMP::encrypt call draws (paillier_gmp.cpp:40-52 and
// paillier_gpu.cu:262-272): first nonzero mpz_urandomm(n) of a freshly
// initialised, unseeded MT state.  Restated with the same GMP calls so the
// engine can be fed the reference's r.
void ref_shared_r(void *h, int nw, uint32_t *out) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    gmp_randstate_t st; gmp_randinit_mt(st);
    mpz_t r; mpz_init(r);
    while (true) { mpz_urandomm(r, st, k->n); if (mpz_cmp_ui(r, 0)) break; }
    exp_words(out, nw, r);
    mpz_clear(r); gmp_randclear(st);
}
}
