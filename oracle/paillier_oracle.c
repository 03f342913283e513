/*
 * paillier_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C/GMP restatement of FedTree's CPU Paillier path, used ONLY by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
 * product (fedtree_amd/, libfthe.so) never links or calls this file.
 *
 * Every function follows the reference formula literally (no CRT, no
 * (1+mn) shortcut, full PowerMod), so the oracle is an independent check of
 * the GPU engine's algebraic shortcuts:
 *   keygen from primes   paillier.cpp:80-87   (n=pq, g=n+1, lambda=lcm(p-1,q-1),
 *                                              mu = L(g^lambda mod n^2)^-1 mod n)
 *   encrypt              paillier.cpp:134-137 (c = g^m * r^n mod n^2, r injected
 *                                              instead of Gen_Coprime, paillier.cpp:9-25)
 *   decrypt              paillier.cpp:153-156 (m = L(c^lambda mod n^2) * mu mod n)
 *   add                  paillier.cpp:103     (x*y mod n^2)
 *   mul                  paillier.cpp:118     (x^y mod n^2)
 *   L_function           paillier.h:40        ((x-1)/n)
 * The GMP build (paillier_gmp.cpp:16-85) computes the same residues.
 *
 * Parity is pinned by tests/golden/ref_gmp_*.json, which were produced by the
 * reference's own Paillier_GMP compiled from /root/reference (oracle/Makefile,
 * oracle/ref_shim.cpp, tests/golden/make_golden.py).
 *
 * Big integers cross this ABI as little-endian arrays of uint32 words (the
 * order of paillier_gpu.cu:7,18: mpz_import/export order -1, 4-byte words).
 */
#include <gmp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int nw;          /* words of n */
    mpz_t n, n2, g, lambda, mu, p, q;
    int has_priv;
} po_key;

static void imp(mpz_t x, const uint32_t *w, int nw) { mpz_import(x, (size_t)nw, -1, 4, 0, 0, w); }
static void exp_(uint32_t *w, int nw, const mpz_t x) {
    size_t cnt = 0;
    memset(w, 0, (size_t)nw * 4);
    if (mpz_sizeinbase(x, 2) > (size_t)nw * 32) { /* does not fit: mark with all-ones */
        memset(w, 0xff, (size_t)nw * 4); return;
    }
    mpz_export(w, &cnt, -1, 4, 0, 0, x);
}

static po_key *key_alloc(void) {
    po_key *k = (po_key *)calloc(1, sizeof(po_key));
    mpz_inits(k->n, k->n2, k->g, k->lambda, k->mu, k->p, k->q, NULL);
    return k;
}

/* paillier.cpp:80-87 with injected primes (GenPrimePair replaced by caller's p,q). */
void *po_key_from_primes(const uint32_t *p, const uint32_t *q, int hw) {
    po_key *k = key_alloc();
    mpz_t pm1, qm1, gl;
    mpz_inits(pm1, qm1, gl, NULL);
    imp(k->p, p, hw); imp(k->q, q, hw);
    mpz_mul(k->n, k->p, k->q);                 /* modulus = p*q            :82 */
    mpz_add_ui(k->g, k->n, 1);                  /* generator = modulus + 1  :83 */
    mpz_sub_ui(pm1, k->p, 1); mpz_sub_ui(qm1, k->q, 1);
    mpz_lcm(k->lambda, pm1, qm1);               /* lcm(p-1,q-1)             :84 */
    mpz_mul(k->n2, k->n, k->n);
    mpz_powm(gl, k->g, k->lambda, k->n2);       /* lambda_power             :85 */
    mpz_sub_ui(gl, gl, 1); mpz_tdiv_q(gl, gl, k->n);   /* L_function paillier.h:40 */
    if (!mpz_invert(k->mu, gl, k->n)) { mpz_clears(pm1, qm1, gl, NULL); return NULL; } /* :86 */
    k->nw = 2 * hw;
    k->has_priv = 1;
    mpz_clears(pm1, qm1, gl, NULL);
    return k;
}

/* Public-key-only copy (Paillier::operator=, paillier.h:12-18). */
void *po_key_from_n(const uint32_t *n, int nw) {
    po_key *k = key_alloc();
    imp(k->n, n, nw);
    mpz_add_ui(k->g, k->n, 1);
    mpz_mul(k->n2, k->n, k->n);
    k->nw = nw;
    return k;
}

void po_key_free(void *kp) {
    po_key *k = (po_key *)kp;
    if (!k) return;
    mpz_clears(k->n, k->n2, k->g, k->lambda, k->mu, k->p, k->q, NULL);
    free(k);
}

/* Export n, lambda, mu (nw words each). */
void po_key_export(void *kp, uint32_t *n, uint32_t *lambda, uint32_t *mu) {
    po_key *k = (po_key *)kp;
    if (n) exp_(n, k->nw, k->n);
    if (lambda) exp_(lambda, k->nw, k->lambda);
    if (mu) exp_(mu, k->nw, k->mu);
}

/* Paillier::encrypt, paillier.cpp:134-137, r injected. m is the 64-bit codec
 * output (common.h:127: NTL::to_ZZ((unsigned long)(g*1e6))).  out: 2*nw words. */
static void encrypt_one(po_key *k, uint64_t m, const uint32_t *r, uint32_t *out, mpz_t t1, mpz_t t2, mpz_t mz, mpz_t rz) {
    mpz_import(mz, 1, -1, 8, 0, 0, &m);
    imp(rz, r, k->nw);
    mpz_powm(t1, k->g, mz, k->n2);
    mpz_powm(t2, rz, k->n, k->n2);
    mpz_mul(t1, t1, t2);
    mpz_mod(t1, t1, k->n2);
    exp_(out, 2 * k->nw, t1);
}

void po_encrypt(void *kp, uint64_t m, const uint32_t *r, uint32_t *out) {
    po_key *k = (po_key *)kp;
    mpz_t t1, t2, mz, rz; mpz_inits(t1, t2, mz, rz, NULL);
    encrypt_one(k, m, r, out, t1, t2, mz, rz);
    mpz_clears(t1, t2, mz, rz, NULL);
}

/* Paillier::decrypt, paillier.cpp:153-156.  out: nw words (full plaintext). */
static void decrypt_one(po_key *k, const uint32_t *c, uint32_t *out, mpz_t cz, mpz_t t) {
    imp(cz, c, 2 * k->nw);
    mpz_powm(t, cz, k->lambda, k->n2);
    mpz_sub_ui(t, t, 1); mpz_tdiv_q(t, t, k->n);
    mpz_mul(t, t, k->mu);
    mpz_mod(t, t, k->n);
    exp_(out, k->nw, t);
}

int po_decrypt(void *kp, const uint32_t *c, uint32_t *out) {
    po_key *k = (po_key *)kp;
    if (!k->has_priv) return -1;
    mpz_t cz, t; mpz_inits(cz, t, NULL);
    decrypt_one(k, c, out, cz, t);
    mpz_clears(cz, t, NULL);
    return 0;
}

/* Paillier::add, paillier.cpp:103. */
void po_add(void *kp, const uint32_t *x, const uint32_t *y, uint32_t *out) {
    po_key *k = (po_key *)kp;
    mpz_t a, b; mpz_inits(a, b, NULL);
    imp(a, x, 2 * k->nw); imp(b, y, 2 * k->nw);
    mpz_mul(a, a, b); mpz_mod(a, a, k->n2);
    exp_(out, 2 * k->nw, a);
    mpz_clears(a, b, NULL);
}

/* Paillier::mul, paillier.cpp:118: x^y mod n^2, y given as 64-bit scalar
 * (common.h:311 uses (unsigned long)-1 for subtraction). */
void po_mul_u64(void *kp, const uint32_t *x, uint64_t y, uint32_t *out) {
    po_key *k = (po_key *)kp;
    mpz_t a, e; mpz_inits(a, e, NULL);
    imp(a, x, 2 * k->nw);
    mpz_import(e, 1, -1, 8, 0, 0, &y);
    mpz_powm(a, a, e, k->n2);
    exp_(out, 2 * k->nw, a);
    mpz_clears(a, e, NULL);
}

/* Batch forms: OpenMP over elements, as Server::encrypt_gh_pairs /
 * decrypt_gh_pairs do (server.h:106-109, 129-133).  threads<=0: OMP default. */
void po_encrypt_batch(void *kp, const uint64_t *m, const uint32_t *r, long count, uint32_t *out, int threads) {
    po_key *k = (po_key *)kp;
    int nw = k->nw;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    #pragma omp parallel
    {
        mpz_t t1, t2, mz, rz; mpz_inits(t1, t2, mz, rz, NULL);
        #pragma omp for schedule(dynamic, 4)
        for (long i = 0; i < count; i++)
            encrypt_one(k, m[i], r + (size_t)i * nw, out + (size_t)i * 2 * nw, t1, t2, mz, rz);
        mpz_clears(t1, t2, mz, rz, NULL);
    }
}

int po_decrypt_batch(void *kp, const uint32_t *c, long count, uint32_t *out, int threads) {
    po_key *k = (po_key *)kp;
    int nw = k->nw;
    if (!k->has_priv) return -1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    #pragma omp parallel
    {
        mpz_t cz, t; mpz_inits(cz, t, NULL);
        #pragma omp for schedule(dynamic, 4)
        for (long i = 0; i < count; i++)
            decrypt_one(k, c + (size_t)i * 2 * nw, out + (size_t)i * nw, cz, t);
        mpz_clears(cz, t, NULL);
    }
    return 0;
}

void po_add_batch(void *kp, const uint32_t *x, const uint32_t *y, long count, uint32_t *out, int threads) {
    po_key *k = (po_key *)kp;
    int w = 2 * k->nw;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    #pragma omp parallel
    {
        mpz_t a, b; mpz_inits(a, b, NULL);
        #pragma omp for schedule(static)
        for (long i = 0; i < count; i++) {
            imp(a, x + (size_t)i * w, w); imp(b, y + (size_t)i * w, w);
            mpz_mul(a, a, b); mpz_mod(a, a, k->n2);
            exp_(out + (size_t)i * w, w, a);
        }
        mpz_clears(a, b, NULL);
    }
}

/* Deterministic test-key prime: nextprime of a seeded value with the top two
 * bits set, so that p*q has exactly 2*bits bits (SURVEY.md 8(d) "Keys").
 * words: little-endian uint32 seed material of bits/32 words. */
void po_next_prime(const uint32_t *seed_words, int hw, uint32_t *out) {
    mpz_t x; mpz_init(x);
    imp(x, seed_words, hw);
    mpz_setbit(x, (mp_bitcnt_t)hw * 32 - 1);
    mpz_setbit(x, (mp_bitcnt_t)hw * 32 - 2);
    mpz_nextprime(x, x);
    exp_(out, hw, x);
    mpz_clear(x);
}

int po_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* Fixed-point codec exactly as the reference writes it (float_type = float):
 *   GMP/GPU build  common.h:81      long g_ul = (long)(g * 1e6);
 *   NTL build      common.h:127     NTL::to_ZZ((unsigned long)(g * 1e6))
 *   decode         common.h:142     g = (float_type)g_dec / 1e6;
 *                  paillier_gpu.cu:487 (float_type)g_ul / 1e6          */
void po_encode_fixed_gmp(const float *g, long n, uint64_t *out) {
    for (long i = 0; i < n; i++) { long v = (long)(g[i] * 1e6); out[i] = (uint64_t)v; }
}
void po_encode_fixed_ntl(const float *g, long n, uint64_t *out) {
    for (long i = 0; i < n; i++) out[i] = (unsigned long)(g[i] * 1e6);
}
void po_decode_fixed(const uint64_t *m, long n, float *out) {
    for (long i = 0; i < n; i++) { long v = (long)m[i]; out[i] = (float)v / 1e6; }
}
