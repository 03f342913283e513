// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" wrapper around the reference's own Paillier_GMP class, compiled
// from /root/reference/src/FedTree/Encryption/paillier_gmp.cpp (never copied)
// by oracle/Makefile into oracle/_ref/libpaillier_gmp_ref.so.  Used by
// tests/golden/make_golden.py to generate golden vectors and by tests to
// cross-check the C oracle (oracle/paillier_oracle.c).
#include "FedTree/Encryption/paillier_gmp.h"   // /root/reference/include
#include <cstring>
#include <cstdint>
#include <vector>
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
// A Paillier_GMP whose fields hold the key of primes p, q (w words each): the state
// Paillier_GMP::keyGen leaves behind (paillier_gmp.cpp:185-210) -- n, n^2, g = n + 1,
// the p, q fields holding p - 1, q - 1, lambda = lcm(p-1, q-1),
// mu = L(g^lambda mod n^2)^-1 mod n -- for injected primes, so the CPU baseline runs
// the reference's own encrypt / decrypt / add on the bench's key.  NULL if mu is not
// invertible.
void *ref_key_from_primes(const uint32_t *pw, const uint32_t *qw, int w) {
    Paillier_GMP *k = new Paillier_GMP();
    mpz_t P, Q, t;
    mpz_init(P); mpz_init(Q); mpz_init(t);
    imp_words(P, pw, w); imp_words(Q, qw, w);
    mpz_mul(k->n, P, Q);
    mpz_add_ui(k->generator, k->n, 1);
    mpz_sub_ui(k->p, P, 1);
    mpz_sub_ui(k->q, Q, 1);
    mpz_lcm(k->lambda, k->p, k->q);
    mpz_mul(k->n_square, k->n, k->n);
    k->key_length = (uint32_t)(2 * mpz_sizeinbase(k->n, 2));      // GMP semantics: n has key_length / 2 bits
    mpz_powm(t, k->generator, k->lambda, k->n_square);
    k->L_function(k->mu, t, k->n);
    int ok = mpz_invert(k->mu, k->mu, k->n);
    mpz_clear(P); mpz_clear(Q); mpz_clear(t);
    if (!ok) { delete k; return nullptr; }
    return k;
}

static void set_threads(int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
}

// Server::decrypt_gh_pairs' CPU loop (server.h:105-109): OpenMP over elements, each one
// Paillier_GMP::decrypt (paillier_gmp.cpp:75-85, PowerMod(c, lambda, n^2), no CRT).
// out: low 64 bits of each plaintext.
void ref_decrypt_batch(void *h, int nw, const uint32_t *c, long count, uint64_t *out, int threads) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    set_threads(threads);
    #pragma omp parallel for schedule(dynamic, 4)
    for (long i = 0; i < count; i++) {
        mpz_t cz, m; mpz_init(cz);
        imp_words(cz, c + (size_t)i * 2 * nw, 2 * nw);
        k->decrypt(m, cz);
        uint64_t lo = 0; size_t cnt = 0;
        uint32_t w[2] = {0, 0};
        if (mpz_sizeinbase(m, 2) <= 64) mpz_export(w, &cnt, -1, 4, 0, 0, m);
        else { mpz_t t; mpz_init(t); mpz_fdiv_r_2exp(t, m, 64); mpz_export(w, &cnt, -1, 4, 0, 0, t); mpz_clear(t); }
        lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        out[i] = lo;
        mpz_clear(cz); mpz_clear(m);
    }
}

// Pairwise homomorphic adds, Paillier_GMP::add (paillier_gmp.cpp:16-21), OpenMP over elements.
void ref_add_batch(void *h, int nw, const uint32_t *a, const uint32_t *b, long count, uint32_t *out, int threads) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    set_threads(threads);
    #pragma omp parallel for schedule(static)
    for (long i = 0; i < count; i++) {
        mpz_t x, y, r; mpz_init(x); mpz_init(y);
        imp_words(x, a + (size_t)i * 2 * nw, 2 * nw);
        imp_words(y, b + (size_t)i * 2 * nw, 2 * nw);
        k->add(r, x, y);
        exp_words(out + (size_t)i * 2 * nw, 2 * nw, r);
        mpz_clear(x); mpz_clear(y); mpz_clear(r);
    }
}

// The k-party merge of merge_histograms_server_propose (hist_tree_builder.cpp:1026-1037):
// for each party after the first, `omp parallel for` over bins of dest = dest + src, each a
// Paillier_GMP::add into a fresh result (non-aliased).  x: k * count rows (party-major);
// out: count rows, starting as party 0's histogram.  (k - 1) * count adds.
void ref_merge_batch(void *h, int nw, const uint32_t *x, int kparties, long count, uint32_t *out, int threads) {
    Paillier_GMP *k = (Paillier_GMP *)h;
    set_threads(threads);
    const size_t cw = 2 * (size_t)nw;
    std::vector<__mpz_struct> acc(count);
    #pragma omp parallel for schedule(static)
    for (long j = 0; j < count; j++) { mpz_init(&acc[j]); imp_words(&acc[j], x + (size_t)j * cw, (int)cw); }
    for (int i = 1; i < kparties; i++) {
        const uint32_t *src = x + (size_t)i * count * cw;
        #pragma omp parallel for schedule(static)
        for (long j = 0; j < count; j++) {
            mpz_t y, r; mpz_init(y);
            imp_words(y, src + (size_t)j * cw, (int)cw);
            mpz_t a; a[0] = acc[j];
            k->add(r, a, y);
            mpz_swap(&acc[j], r);
            mpz_clear(y); mpz_clear(r);
        }
    }
    #pragma omp parallel for schedule(static)
    for (long j = 0; j < count; j++) { exp_words(out + (size_t)j * cw, (int)cw, &acc[j]); mpz_clear(&acc[j]); }
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
