/*
 * fthe.h -- C ABI of the MI355X batch Paillier engine ("FedTree HE").
 *
 * Drop-in boundary for FedTree's homomorphic-encryption interface.  Every
 * entry point below replaces a reference call (file:line relative to the
 * FedTree source tree); INTEGRATION.md shows the C++ shim a FedTree build
 * would compile (USE_HIP) and the ctypes binding used by the Python mirror.
 *
 * Conventions
 *   - Big integers are little-endian arrays of uint32 words, the order of
 *     mpz_import/mpz_export(order=-1, size=4) used by the reference GPU path
 *     (paillier_gpu.cu:7,18).  A key of n_words words has ciphertexts of
 *     2*n_words words.
 *   - Plaintexts are the 64-bit fixed-point codec values of common.h:81-86 /
 *     :127 ((uint64)(int64)((double)x*1e6)); decryption returns the low 64
 *     bits, which is what the reference decodes (paillier_gpu.cu:485-488).
 *   - "_dev" calls take device pointers and are asynchronous on the context's
 *     stream; the plain calls take host pointers and are synchronous.
 *   - All calls return FTHE_OK (0) or a negative status; nothing aborts.
 *   - Thread safety: a context may be used by one host thread at a time;
 *     create one context per host thread / device (callers enter the boundary
 *     from OpenMP regions, FLtrainer.cpp:275-306).  Keys are immutable after
 *     creation and may be shared between contexts on the same device.
 *   - There is no CPU fallback: without a gfx950 device every compute call
 *     fails with FTHE_ERR_HIP.
 */
#ifndef FTHE_H
#define FTHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FTHE_OK               0
#define FTHE_ERR_ARG         -1   /* bad argument / size */
#define FTHE_ERR_HIP         -2   /* HIP runtime failure, no device, kernel load */
#define FTHE_ERR_NOPRIV      -3   /* private key required (decrypt, CRT) */
#define FTHE_ERR_UNSUPPORTED -4   /* modulus size not built */
#define FTHE_ERR_KEY         -5   /* invalid key material (mu not invertible, p==q, ...) */
#define FTHE_ERR_NOMEM       -6

/* fthe_encrypt flags */
#define FTHE_ENC_DEFAULT      0   /* CRT when the private key is present */
#define FTHE_ENC_PUBLIC       1   /* force the public-key (no CRT) formula */
#define FTHE_ENC_FIXED_BASE   2   /* fixed-base randomizer r = h^alpha (see fthe_key_fixed_base) */
#define FTHE_ENC_FIXED_BASE_EXACT 4  /* key holder: tables with the reference's r^n distribution (see fthe_key_fixed_base_exact) */

typedef struct fthe_ctx fthe_ctx;
typedef struct fthe_key fthe_key;

int         fthe_version(void);
const char *fthe_strerror(int status);

/* ---- device context (one HIP stream + workspace) ------------------------ */
/* Every call is ordered on the context stream.  Small decrypts and device-
 * randomness encrypts (<= one chunk, 393,216 lanes; <= 16,384 ciphertexts of a
 * Paillier-2048 key also switch to the four-lane s80 kernel) fork their mod-q
 * half onto a private side stream and join it back before any output is
 * written, so callers see one stream: fthe_ctx_sync / an event on
 * fthe_ctx_stream cover all of it.  Results are bit-identical whichever path
 * a batch size takes. */
/* Visible gfx950 devices (0 without a GPU or HIP runtime).  The drop-in class shards its batch calls over
 * them (integration/paillier_hip.h, FTHE_DEVICES), as the 8 GPUs of a node would take Server::encrypt_gh_pairs'
 * batch (server.h:105-121) in independent contiguous shards. */
int   fthe_device_count(void);
int   fthe_ctx_create(int device, fthe_ctx **out);
void  fthe_ctx_destroy(fthe_ctx *ctx);
int   fthe_ctx_sync(fthe_ctx *ctx);
void *fthe_ctx_stream(fthe_ctx *ctx);       /* hipStream_t */
int   fthe_ctx_device(fthe_ctx *ctx);
/* Cap (bytes, 0 = none) on the slot region a call may grow on this context.  Large CRT encrypts and decrypts
 * prefer two slot regions (both halves of a chunk on two streams, 7.4 GB at Paillier-2048); when the cap or
 * the device cannot hold them they take the one-region form, bit-identical.  For many contexts on one GPU
 * (the drop-in's per-thread and per-device contexts). */
int   fthe_ctx_set_mem_limit(fthe_ctx *ctx, size_t bytes);
/* Page-locked host memory for caller row buffers: host-resident calls then DMA straight from / into
 * it instead of staging through the context's pinned chunks (the drop-in class keeps one per thread for
 * encrypt / decrypt(SyncArray<GHPair>&), reused across calls: pinning is paid once). */
int   fthe_host_alloc(size_t bytes, void **out);
void  fthe_host_free(void *p);

/* ---- keys ----------------------------------------------------------------
 * fthe_key_generate      Paillier::keygen(int keyLength), paillier.cpp:66-90:
 *                        n has exactly n_bits bits (NTL semantics),
 *                        g = n+1, lambda = lcm(p-1,q-1), mu = L(g^lambda)^-1.
 *                        seed 0 draws primes from /dev/urandom; a nonzero seed
 *                        is deterministic (tests, benchmarks).
 * fthe_key_from_primes   same derivation from caller primes (injected keys).
 * fthe_key_from_n        public key only: Paillier::operator=, paillier.h:12-18
 *                        (copies modulus/generator/keyLength only).
 */
int  fthe_key_generate(fthe_ctx *ctx, int n_bits, uint64_t seed, fthe_key **out);
/* fthe_key_generate_ex   flags 0: fthe_key_generate.  FTHE_KEYGEN_KNOWN_ORDER: p and q
 *                        (top two bits set, n of n_bits bits) of the form 2 s P' + 1 with
 *                        P' a random prime and s a product of random primes < 2^16, the
 *                        factorisation of p - 1, q - 1 kept with the key, so that the exact
 *                        fixed-base mode uses one generator per prime (64 instead of 192
 *                        gathered products at P-2048) and is exact without a probability
 *                        bound.  Not the reference's prime distribution (paillier.cpp:43-62
 *                        draws unconstrained random primes); opt-in. */
#define FTHE_KEYGEN_KNOWN_ORDER 1
int  fthe_key_generate_ex(fthe_ctx *ctx, int n_bits, uint64_t seed, int flags, fthe_key **out);
/* fthe_next_prime        host only (no device): the smallest prime > start (words
 *                        little-endian u32) into out, as mpz_nextprime; the keygen's prime
 *                        search, sieved and tested on up to 16 host threads. */
int  fthe_next_prime(const uint32_t *start, int words, uint32_t *out, int out_words);
int  fthe_key_from_primes(fthe_ctx *ctx, const uint32_t *p, const uint32_t *q,
                          int pq_words, fthe_key **out);
int  fthe_key_from_n(fthe_ctx *ctx, const uint32_t *n, int n_words, fthe_key **out);
void fthe_key_destroy(fthe_key *key);
int  fthe_key_n_words(const fthe_key *key);
int  fthe_key_n_bits(const fthe_key *key);
int  fthe_key_has_private(const fthe_key *key);
/* Each output (nullable) is n_words words; p and q are n_words/2 words. */
int  fthe_key_export(const fthe_key *key, uint32_t *n, uint32_t *lambda,
                     uint32_t *mu, uint32_t *p, uint32_t *q);

/* ---- encrypt: c = g^m * r^n mod n^2 (paillier.cpp:134-137) ----------------
 * Replaces Paillier::encrypt (paillier.cpp:122), Paillier_GMP::encrypt
 * (paillier_gmp.cpp:37) and Paillier_GPU::encrypt (paillier_gpu.cu:211).
 * r:       NULL -> a fresh uniform r in [1,n) per ciphertext from a device
 *          ChaCha20 stream keyed by rng_seed (0 -> /dev/urandom);
 *          else count*r_words words, r < n (injected randomness: parity,
 *          reference-compat shared r of paillier_gpu.cu:262-272).
 * c:       count * 2*n_words words. */
int fthe_encrypt_u64_dev(fthe_key *key, fthe_ctx *ctx, const uint64_t *m, size_t count,
                         const uint32_t *r, int r_words, uint64_t rng_seed,
                         uint32_t *c, int flags);
int fthe_encrypt_u64(fthe_key *key, fthe_ctx *ctx, const uint64_t *m, size_t count,
                     const uint32_t *r, int r_words, uint64_t rng_seed,
                     uint32_t *c, int flags);
/* A shard of a larger batch: plaintext i of this call is element index0 + i of the caller's whole batch.
 * With device randomness (r == NULL) and a nonzero rng_seed, ciphertext i draws the randomness element
 * index0 + i of that seed's stream, so contiguous shards encrypted on several contexts or devices give
 * exactly the ciphertexts of one fthe_encrypt_u64 call over the whole batch (the multi-GPU drop-in,
 * integration/paillier_hip.h).  index0 = 0 is fthe_encrypt_u64[_dev]. */
int fthe_encrypt_u64_at_dev(fthe_key *key, fthe_ctx *ctx, const uint64_t *m, size_t count,
                            const uint32_t *r, int r_words, uint64_t rng_seed, uint64_t index0,
                            uint32_t *c, int flags);
int fthe_encrypt_u64_at(fthe_key *key, fthe_ctx *ctx, const uint64_t *m, size_t count,
                        const uint32_t *r, int r_words, uint64_t rng_seed, uint64_t index0,
                        uint32_t *c, int flags);
/* General plaintexts (Paillier::encrypt(const ZZ&), paillier.cpp:122-139): m_words little-
 * endian words per plaintext (m_words <= n_words); otherwise as fthe_encrypt_u64.  Any m that
 * fits is encrypted exactly as PowerMod(g, m, n^2) r^n (g^m = 1 + m n mod n^2 for every m). */
int fthe_encrypt_words_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *m, int m_words, size_t count,
                           const uint32_t *r, int r_words, uint64_t rng_seed, uint32_t *c, int flags);
int fthe_encrypt_words(fthe_key *key, fthe_ctx *ctx, const uint32_t *m, int m_words, size_t count,
                       const uint32_t *r, int r_words, uint64_t rng_seed, uint32_t *c, int flags);

/* ---- fixed-base randomizer (flag FTHE_ENC_FIXED_BASE) -----------------------
 * Not in the reference: an opt-in encryption mode for throughput.  One random
 * h per key; c = (1 + m n) * hs^alpha mod n^2 with hs = h^n mod n^2, i.e. a
 * Paillier encryption of m under r = h^alpha (Damgard-Jurik-Nielsen fixed-base
 * randomizer).  Decryption, add, mul are unchanged.  alpha is drawn per
 * ciphertext from the device ChaCha20 stream (r == NULL: alpha_bits random
 * bits, 64 more than the bits of the modulus, independently mod p^2 and q^2
 * under CRT), or injected through the r / r_words arguments of
 * fthe_encrypt_u64[_dev] (little-endian words, alpha < 2^alpha_bits; the same
 * alpha for both CRT halves).  16-bit windows (FTHE_FB_WINDOW=8: 8-bit): one
 * gathered product per window from precomputed tables (hs^(d 65536^j), 65536
 * entries per window, ~4.4 GB public + 2 x 1.4 GB CRT at P-2048, widened on the
 * device from host-built 8-bit tables) instead of ~1.2 log2(n) products.
 * fthe_key_fixed_base        (re)build the tables for base h (h_words words,
 *                            1 <= h < n); h == NULL draws h from /dev/urandom.
 *                            Built on first use otherwise.  Not concurrent with
 *                            calls that use the key.
 * fthe_key_fixed_base_info   exponent bits per form (0 if unavailable) and hs
 *                            (2*n_words words, nullable), after a build. */
int fthe_key_fixed_base(fthe_key *key, fthe_ctx *ctx, const uint32_t *h, int h_words);
int fthe_key_fixed_base_info(fthe_key *key, int *alpha_bits_public, int *alpha_bits_crt, uint32_t *hs);

/* ---- exact fixed-base randomizer (flag FTHE_ENC_FIXED_BASE_EXACT) -----------
 * Key holder (CRT; public keys: see fthe_key_set_public_bases).  The reference's r is
 * uniform in Z_n^* (paillier.cpp:127-133); then r^n mod P^2 (P = p, q) is
 * uniform over G_P = {x^P mod P^2}, cyclic of order P - 1, independently for p
 * and q.  Here, per prime, three bases gam_i = t_i^P mod P^2 with
 * <t_1, t_2, t_3> = Z_P^* (checked at every prime l < 2^24 dividing P - 1; a
 * larger l escapes with probability < 2^-66 per key) and exponents y_i uniform
 * in [1, P) from the device ChaCha20 stream give r^n mod P^2 = prod gam_i^y_i,
 * exactly uniform over G_P: the reference's ciphertext distribution, computed as
 * 3 * ceil(bits(P)/16) gathered products from 16-bit-window tables (~3.8 GB
 * per prime at P-2048) instead of ~1.2 bits(P) squarings and products.
 * Injected exponents (parity): r = y, r_words = 6 * (n_words / 2): per
 * ciphertext y_{p,1}, y_{p,2}, y_{q,1}, ... (see fthe_key_fixed_base_exact_bases;
 * 3 bases, or 1 for FTHE_KEYGEN_KNOWN_ORDER keys), n_words/2 little-endian words
 * each, each y < 2^(16 * ceil(bits(P)/16)).
 * fthe_key_fixed_base_exact       (re)build bases and tables; seed 0 draws the
 *                                 bases from /dev/urandom, else deterministic.
 *                                 Built on first use otherwise.  Not concurrent
 *                                 with calls that use the key.
 * fthe_key_fixed_base_exact_info  gam_{side,base} (side 0 = p, 1 = q; n_words
 *                                 words, nullable) and the words per exponent. */
int fthe_key_fixed_base_exact(fthe_key *key, fthe_ctx *ctx, uint64_t seed);
int fthe_key_fixed_base_exact_info(fthe_key *key, int side, int base, uint32_t *gamma, int *exp_words);
/* (Re)build the exact tables from given generators instead of fresh ones: gammas = the nb gam of side 0, then
 * the nb of side 1 (n_words words each, as fthe_key_fixed_base_exact_info returns them) of a key with the same
 * primes -- a key replica on another device then draws r^n exactly as the original for the same exponents, so a
 * seeded batch encrypt does not depend on how it was sharded (integration/paillier_hip.h key_on).  nb must be
 * this key's bases per prime (3, or 1 for FTHE_KEYGEN_KNOWN_ORDER).  Not concurrent with calls using the key. */
int fthe_key_fixed_base_exact_set(fthe_key *key, fthe_ctx *ctx, int nb, const uint32_t *gammas);
/* bases per prime of the built exact tables: 3, or 1 for FTHE_KEYGEN_KNOWN_ORDER keys
 * (one generator); 0 before a build.  Injected exponents then take 2 * bases * (n_words/2)
 * words per ciphertext (y_{p,1..bases}, y_{q,1..bases}). */
int fthe_key_fixed_base_exact_bases(fthe_key *key);

/* ---- public exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT, public form) ----
 * Parties hold only n (party.h:181-185) and encrypt with the public formula
 * (Party::encrypt_histogram, party.h:118-142; paillier.cpp:122-139), r uniform in
 * Z_n^*.  r^n mod n^2 depends on r mod n only and is multiplicative, so with bases
 * hs_i = t_i^n mod n^2 for t_1 .. t_nb generating Z_n^*, r^n = prod hs_i^y_i for
 * exponents y_i uniform modulo the group order.  Holding n alone, the encrypting
 * side draws y_i uniform below 2^(16 nwin), nwin = ceil((bits(n) + 64) / 16): the
 * ciphertext distribution is within nb * 2^-64 (statistical distance) of the
 * reference's, from nb * nwin gathered products of 16-bit-window tables (~13 GB
 * at P-2048 with 3 bases) instead of ~1.2 bits(n) products mod n^2.
 * fthe_key_public_bases      key holder (FTHE_ERR_NOPRIV otherwise): draws t_i and
 *                            checks <t_i> = Z_n^* at every prime l < 2^24 dividing
 *                            p-1 or q-1 (rank 2 over GF(l) where l divides both;
 *                            a larger l escapes with probability < 2^-65), at every
 *                            l for FTHE_KEYGEN_KNOWN_ORDER keys; writes hs_i (nb *
 *                            2*n_words words; hs NULL: *nb only) and the bits of
 *                            each base's exponent (exp_bits[nb], nullable; published
 *                            with the bases).  nb = 3 with 16 nwin bits each, or for
 *                            known-order keys with gcd(p-1, q-1) < 2^64: 2, the first
 *                            of order lcm(p-1, q-1) (16 nwin bits), the second
 *                            generating the quotient Z_gcd (128 bits: 140 instead of
 *                            264 products at P-2048).  seed 0: /dev/urandom.  Host only.
 * fthe_key_set_public_bases  any key with the public form: builds the tables for the
 *                            published hs (nb * 2*n_words words, 1 <= nb <= 3) and
 *                            exp_bits (multiples of 16, <= 16 nwin; NULL: 16 nwin
 *                            each); then FTHE_ENC_FIXED_BASE_EXACT on a public key (or
 *                            with FTHE_ENC_PUBLIC) uses them.  Not concurrent with
 *                            calls that use the key.
 * fthe_key_public_bases_info nb and the words per injected exponent of each base
 *                            (exp_words[nb]); injected exponents (parity): r = y,
 *                            r_words = sum exp_words, y_i < 2^exp_bits_i. */
int fthe_key_public_bases(fthe_key *key, uint64_t seed, uint32_t *hs, int *nb, int *exp_bits);
int fthe_key_set_public_bases(fthe_key *key, fthe_ctx *ctx, const uint32_t *hs, int nb, const int *exp_bits);
int fthe_key_public_bases_info(fthe_key *key, int *nb, int *exp_words);

/* ---- decrypt: m = L(c^lambda mod n^2) * mu mod n (paillier.cpp:153-156) ---
 * Computed with CRT over p^2, q^2 (identical canonical result).
 * Replaces Paillier::decrypt (paillier.cpp:141), Paillier_GMP::decrypt
 * (paillier_gmp.cpp:75), Paillier_GPU::decrypt (paillier_gpu.cu:448,497).
 * m_low:   count uint64 (low 64 bits of the plaintext), nullable.
 * m_full:  count * n_words words (full plaintext), nullable. */
int fthe_decrypt_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *c, size_t count,
                     uint64_t *m_low, uint32_t *m_full);
int fthe_decrypt(fthe_key *key, fthe_ctx *ctx, const uint32_t *c, size_t count,
                 uint64_t *m_low, uint32_t *m_full);

/* Short-plaintext decryption (opt-in): only the p half of the CRT,
 * m = L_p(c^(p-1) mod p^2) h_p mod p -- equal to the plaintext when it is
 * below p.  FedTree's plaintexts always are: 64-bit fixed-point codes and
 * sums / differences of them (common.h:81-86, 253-337) stay below 2^130 for
 * any batch that fits in memory, and p has n_bits/2 >= 256 bits.  Half the
 * work of fthe_decrypt; a plaintext >= p decrypts to m mod p. */
int fthe_decrypt_short_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *c, size_t count,
                           uint64_t *m_low, uint32_t *m_full);
int fthe_decrypt_short(fthe_key *key, fthe_ctx *ctx, const uint32_t *c, size_t count,
                       uint64_t *m_low, uint32_t *m_full);

/* Coalescing host-resident decrypt for many concurrent callers of one key:
 * Server::decrypt_gh per tree node from OpenMP threads (server.h:69-78,
 * FLtrainer.cpp:758-764).  Thread-safe, no context argument: requests that
 * arrive while a batch runs are merged into the next one, run by one of the
 * waiting callers on a context the key owns, so N concurrent single-pair
 * calls cost about one batch latency instead of N (small launches from
 * separate contexts share the process's few hardware queues and serialise).
 * A new leader lingers until the previous round's callers are back, at most
 * FTHE_LINGER_US (200 us) or a quarter of the previous batch (0: off).
 * short_pt != 0: fthe_decrypt_short semantics.  Same results as fthe_decrypt. */
int fthe_decrypt_shared(fthe_key *key, const uint32_t *c, size_t count,
                        uint64_t *m_low, uint32_t *m_full, int short_pt);

/* The same queue for encryption (a second leader and context): concurrent
 * fthe_encrypt_u64 calls with fresh device randomness (r = NULL, seed from
 * /dev/urandom per batch) on one key -- single GHPair encrypts from threads
 * (GHPair::homo_encrypt, common.h:125-133; party.h:118-142 per party) --
 * merged into one launch per flags value.  c: count * 2*n_words words. */
int fthe_encrypt_shared(fthe_key *key, const uint64_t *m, size_t count, uint32_t *c, int flags);

/* ---- homomorphic add: x*y mod n^2 (paillier.cpp:103) ------------------------
 * Replaces Paillier::add / Paillier_GMP::add (paillier_gmp.cpp:16) and
 * Paillier_GPU::add (paillier_gpu.cu:58).  Alias-safe: out may equal a or b
 * (fixes SURVEY Q11, where add(s,s,c) zeroes s). */
int fthe_add_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *a, const uint32_t *b,
                 size_t count, uint32_t *out);
int fthe_add(fthe_key *key, fthe_ctx *ctx, const uint32_t *a, const uint32_t *b,
             size_t count, uint32_t *out);

/* Coalescing host-resident add / scalar mul for many concurrent single-pair callers of one key:
 * GHPair::operator+, += and - of the USE_HIP build (common.h:150-337; integration/fthe_ghpair_key.h)
 * from FedTree's OpenMP loops (hist_tree_builder.cpp:574-591, 1031-1047; tree.cpp:24).  Thread-safe,
 * no context argument: calls arriving while a batch runs are merged into the next launch (adds
 * together, scalar muls per exponent) on a context the key owns.  Alias-safe: out may equal a,
 * b or x (the reference's add(s, s, c) zeroes s).  Same results as fthe_add /
 * fthe_scalar_mul_u64. */
int fthe_add_shared(fthe_key *key, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out);
int fthe_scalar_mul_u64_shared(fthe_key *key, const uint32_t *x, uint64_t k, size_t count, uint32_t *out);

/* ---- Montgomery-resident rows (device; not in the reference) ---------------
 * A fresh add costs two Montgomery products (x y R^-1, then a product by R^2
 * mod n^2).  Rows kept resident in Montgomery form, x R mod n^2 (same 2 n_words
 * layout, canonical < n^2), multiply with one: (aR)(bR)R^-1 = (ab)R.  For
 * device-resident chains of adds (tree sums, repeated merges): convert once,
 * add many times, convert back; the converted-back rows are bit-identical to
 * fthe_add_dev's.  Alias-safe.
 * fthe_to_mont_dev    out = x R mod n^2   (one product)
 * fthe_from_mont_dev  out = x R^-1 mod n^2 (one product): canonical ciphertexts
 * fthe_add_mont_dev   out = a b R^-1 mod n^2 (one product): Mont(a) Mont(b) -> Mont(ab) */
int fthe_to_mont_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count, uint32_t *out);
int fthe_from_mont_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count, uint32_t *out);
int fthe_add_mont_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *a, const uint32_t *b,
                      size_t count, uint32_t *out);

/* out[i] = a[i] * b[i]^(2^64-1) mod n^2: GHPair::operator- with both sides
 * encrypted (common.h:253-337 -- Paillier::add(a, Paillier::mul(b, (unsigned
 * long)-1))), fused into one program (all-ones addition chain).  The sibling
 * histogram father - child (hist_tree_builder.cpp:678) and missing_gh (:724). */
int fthe_sub_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *a, const uint32_t *b,
                 size_t count, uint32_t *out);
int fthe_sub(fthe_key *key, fthe_ctx *ctx, const uint32_t *a, const uint32_t *b,
             size_t count, uint32_t *out);


/* ---- scalar mul: x^k mod n^2 (paillier.cpp:118), one k for the batch ------
 * The reference only multiplies by (unsigned long)-1 (subtraction,
 * common.h:264-267,311-317). */
int fthe_scalar_mul_u64_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, uint64_t k,
                            size_t count, uint32_t *out);
int fthe_scalar_mul_u64(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, uint64_t k,
                        size_t count, uint32_t *out);
/* x^e mod n^2 with an exponent of e_words little-endian words (Paillier::mul(x, ZZ y),
 * paillier.cpp:107-120, any y), one exponent for the batch. */
int fthe_scalar_mul_words_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, const uint32_t *e, int e_words,
                              size_t count, uint32_t *out);
int fthe_scalar_mul_words(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, const uint32_t *e, int e_words,
                          size_t count, uint32_t *out);

/* ---- k-way product (k-party histogram merge) ---------------------------
 * out[i] = prod_{j<k} x[j*count + i] mod n^2.
 * merge_histograms_server_propose, hist_tree_builder.cpp:1015-1058 (the
 * reference's first add into an unencrypted zero is a fresh encrypt(0),
 * pass that ciphertext as one of the k inputs to reproduce it). */
int fthe_reduce_kway_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, int k,
                         size_t count, uint32_t *out);
int fthe_reduce_kway(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, int k,
                     size_t count, uint32_t *out);

/* ---- segmented product ----------------------------------------------------
 * out[s] = prod_{t in [seg_ptr[s], seg_ptr[s+1])} x[idx ? idx[t] : t] mod n^2.
 * The histogram scatter of hist_tree_builder.cpp:565-595 (hist[bin] += gh[iid],
 * segments = the instances of each (feature, bin)), root / node sums
 * (tree.cpp:20-34, tree_builder.cpp:268-274).  An empty segment yields 1 (the
 * reference keeps an unencrypted zero GHPair there).  seg_ptr (nseg+1 entries)
 * and idx are HOST arrays; x / out are device (_dev) or host pointers. */
int fthe_reduce_segments_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count,
                             const int64_t *seg_ptr, const int64_t *idx, size_t nseg, uint32_t *out);
int fthe_reduce_segments(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count,
                         const int64_t *seg_ptr, const int64_t *idx, size_t nseg, uint32_t *out);

/* The same with the CSR in device memory (seg_ptr: nseg+1 int64, idx: int64 or
 * NULL for the identity), planned on the device: no host-side index work. */
int fthe_reduce_segments_csr_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count,
                                 const int64_t *seg_ptr, const int64_t *idx, size_t nseg, uint32_t *out);

/* ---- homomorphic histogram of one tree node, all on the device ------------
 * Replaces the scatter loop of HistTreeBuilder::compute_histogram_in_a_level
 * (hist_tree_builder.cpp:565-595 root, :640-664 smaller child of a sibling
 * pair: hist[cut_col_ptr[fid] + bid] = hist[...] + gh[iid], bid =
 * dense_bin_id[iid*n_col + fid] != max_num_bin).
 *   x        planes * count ciphertexts (plane p = x[p*count ..]: g_enc, h_enc)
 *   bin_ids  device, count * n_col bytes (dense_bin_id, row-major by instance)
 *   cut_col_ptr  HOST, n_col + 1 int32 (cut.cut_col_ptr)
 *   inst     device int32 instance ids of the node (node_idx range), or NULL
 *            for instances 0 .. n_sel-1
 *   out      device, planes * n_bins ciphertexts; a bin without members is
 *            the integer 1 (the reference keeps an unencrypted zero there). */
int fthe_histogram_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count, int planes,
                       const uint8_t *bin_ids, int n_col, const int32_t *cut_col_ptr, int max_num_bin,
                       const int32_t *inst, size_t n_sel, uint32_t *out);

/* The reference's exact sequence for a bin: its accumulator starts as an unencrypted
 * zero GHPair, and the first `hist[bin] = hist[bin] + gh[iid]` encrypts that zero with a fresh r
 * (GHPair::operator+, common.h:156-160), so a populated bin is Enc(0) * prod(members) mod n^2.
 * enc_zero: device, one Enc(0) row per segment (planes * n_bins rows for the histogram; a fresh
 * encryption each, e.g. fthe_encrypt_u64_dev of zeros, or the reference's shared r to reproduce
 * its ciphertexts); folded into every populated segment, while an empty one stays the integer 1.
 * Same arguments otherwise as fthe_histogram_dev / fthe_reduce_segments_dev. */
int fthe_histogram_zero_first_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count, int planes,
                                  const uint8_t *bin_ids, int n_col, const int32_t *cut_col_ptr, int max_num_bin,
                                  const int32_t *inst, size_t n_sel, const uint32_t *enc_zero, uint32_t *out);
int fthe_reduce_segments_zero_first_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, size_t count,
                                        const int64_t *seg_ptr, const int64_t *idx, size_t nseg,
                                        const uint32_t *enc_zero, uint32_t *out);

/* Segmented inclusive scan: out[t] = prod of x[seg_start(t) .. t] mod n^2 --
 * the inclusive_scan_by_key of the histogram over (node, feature)
 * (hist_tree_builder.cpp:695-708).  seg_ptr (nseg+1 entries) is a HOST array;
 * the elements are x[0 .. seg_ptr[nseg]). */
int fthe_scan_segments_dev(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, const int64_t *seg_ptr,
                           size_t nseg, uint32_t *out);
int fthe_scan_segments(fthe_key *key, fthe_ctx *ctx, const uint32_t *x, const int64_t *seg_ptr,
                       size_t nseg, uint32_t *out);

/* ---- ciphertext wire formats (host only; fthe_wire.cpp) --------------------
 * Decimal: the reference's GHEncBatch strings (fedtree.proto:82-99), written
 * by `stream << g_enc` (distributed_server.cpp:37-54, distributed_party.cpp:
 * 1285-1300) and read by NTL::to_ZZ (distributed_party.cpp:1267-1273,
 * distributed_server.cpp:1427-1433); byte-identical both ways.  Strings are
 * concatenated in buf; offsets has count+1 entries (offsets[count] = total
 * bytes; when buf_len is too small the call fails with FTHE_ERR_ARG and
 * offsets[count] tells the size needed).  threads <= 0: all cores.
 * Binary: the "FTHW" frame of raw little-endian words. */
size_t fthe_decimal_max_len(int words);
int fthe_ct_to_decimal(const uint32_t *ct, int words, size_t count, char *buf, size_t buf_len,
                       size_t *offsets, int threads);
int fthe_ct_from_decimal(const char *buf, const size_t *offsets, size_t count, int words,
                         uint32_t *ct, int threads);
/* The same decimal strings computed on the GPU (fthe_dec.hip): ct, buf and offsets
 * (count+1 entries, size_t) in device memory, words <= 128.  to: offsets[count] =
 * bytes; buf_len too small -> FTHE_ERR_ARG with the offsets filled (size needed in
 * offsets[count]).  from: FTHE_ERR_ARG on an empty, non-decimal or oversized string.
 * Both synchronise the context stream once (the size / error flag). */
int fthe_ct_to_decimal_dev(fthe_ctx *ctx, const uint32_t *ct, int words, size_t count, char *buf,
                           size_t buf_len, size_t *offsets);
int fthe_ct_from_decimal_dev(fthe_ctx *ctx, const char *buf, const size_t *offsets, size_t count,
                             int words, uint32_t *ct);
size_t fthe_wire_size(size_t count, int words, int with_h);
int fthe_wire_encode(const uint32_t *g, const uint32_t *h, size_t count, int words,
                     uint8_t *out, size_t cap, size_t *len);
int fthe_wire_decode(const uint8_t *in, size_t len, int words, uint32_t *g, uint32_t *h,
                     size_t cap, size_t *count);

/* ---- fixed-point codec (common.h:81-86,127-128,140-143) ------------------- */
int fthe_encode_fixed_dev(fthe_ctx *ctx, const float *x, size_t count, uint64_t *m);
int fthe_decode_fixed_dev(fthe_ctx *ctx, const uint64_t *m, size_t count, float *x);

/* ---- test hook: the randomness of the direct-y CRT encrypt ----------------
 * A key holder's fthe_encrypt_u64[_dev] with r == NULL draws, per ciphertext,
 * y_p uniform in [1, p) and y_q uniform in [1, q) and computes
 * (1 + m n) y_P^P mod P^2 for P = p, q: the encryption under
 * r = CRT(y_p^(q^-1 mod p-1) mod p, y_q^(p^-1 mod q-1) mod q).  This returns the
 * (y_p, y_q) a call with this nonzero rng_seed draws for ciphertexts
 * [index0, index0 + count) (the draws depend on the index only, not on the
 * chunking), pq_words = words of max(p, q) each, little-endian, into host yp /
 * yq (count * pq_words words), so tests can pin device-drawn ciphertexts
 * against PowerMod(g, m, n^2) PowerMod(r, n, n^2) (paillier.cpp:134-137). */
int fthe_debug_direct_y(fthe_key *key, fthe_ctx *ctx, uint64_t rng_seed, uint64_t index0, size_t count,
                        uint32_t *yp, uint32_t *yq);

/* ---- test hook: the per-key context of the matrix-core Barrett add ---------
 * The bytes fthe_addb_q152 reads (mu and N copies, column corrections, N), built
 * on the host from n (n_words little-endian words) exactly as at key set-up;
 * out == NULL: only *len.  FTHE_ERR_UNSUPPORTED unless n^2 has 4095-4096 bits.
 * Host only (tests compare it with tools/addb_model.py addb_image). */
int fthe_debug_addb_image(const uint32_t *n, int n_words, uint8_t *out, size_t cap, size_t *len);
/* The per-key context of fthe_nadic_b76, the parties' public-key encrypt on base-n digits with matrix-core
 * Barrett reductions (party.h:118-142 -> paillier.cpp:122-139): mu and n copies, column corrections, n's 27-bit
 * limbs, built on the host from n exactly as at key set-up; out == NULL: only *len.  FTHE_ERR_UNSUPPORTED
 * unless n is odd with 2041..2048 bits.  Host only (tests compare it with tools/nadicb_model.py). */
int fthe_debug_nadicb_image(const uint32_t *n, int n_words, uint8_t *out, size_t cap, size_t *len);
/* Test hook of fthe_nadic_b76: run the op program `prog` (prog_words uint32) over `count` ciphertexts whose slots
 * 0 .. nslots-1 are given as host limbs (nslots x count x 152 limbs of 27 bits: x0 in 0..75, x1 in 76..151) and
 * return slot out_slot the same way.  FTHE_ERR_UNSUPPORTED unless the key runs fthe_nadic_b76 (n of 2041..2048
 * bits).  For tests and bring-up only. */
int fthe_debug_nadicb_prog(fthe_key *key, fthe_ctx *ctx, const uint32_t *prog, int prog_words, const uint32_t *in,
                           int nslots, size_t count, int out_slot, uint32_t *out);

/* ---- profiling hooks: time of the last call's kernels on the stream ------ */
double fthe_last_kernel_ms(fthe_ctx *ctx);
/* Montgomery products executed by the last call (for roofline accounting). */
double fthe_last_montmuls(fthe_ctx *ctx);
/* Per-launch timing of the Montgomery program kernel (HIP events on the
 * context stream, bracketing each launch).  fthe_prof_read drains the stream,
 * returns totals since the last read/enable and resets them:
 *   kernel_ms      summed launch durations
 *   launches       number of launches
 *   lane_montmuls  sum over launches of (live lanes x Montgomery products)
 *   lanes          sum over launches of live lanes
 *   expo_ms/_launches  the same restricted to exponentiation launches
 *                  (programs of >= 64 products per lane)
 *   alg_macs       algorithmic work of those launches in 32-bit MACs: live lanes x
 *                  products x W(s), W(s) = 2 s^2 + s with s = 32-bit words of the
 *                  modulus, and for the P-adic kernel its own count
 *                  (digit products + Barrett reductions) -- independent of the radix */
int    fthe_prof_enable(fthe_ctx *ctx, int on);
int    fthe_prof_read(fthe_ctx *ctx, double *kernel_ms, double *launches,
                      double *lane_montmuls, double *lanes,
                      double *expo_ms, double *expo_launches, double *alg_macs);
/* The union of the launch intervals of the last fthe_prof_read window (time with at least one launch running,
 * all launches / exponentiation launches): launches on the context's two compute streams overlap when a large
 * CRT encrypt or decrypt runs its p and q halves side by side, so summed durations then count that time twice. */
int    fthe_prof_busy(fthe_ctx *ctx, double *busy_ms, double *expo_busy_ms);
/* Per kernel variant (limb count S: 37, 74, 152, 80; 1037 = the P-adic kernel mod
 * p^2 / q^2) exponentiation-launch time and count of the last fthe_prof_read window. */
int    fthe_prof_variant(fthe_ctx *ctx, int S, double *expo_ms, double *expo_launches);
/* Multiply-add instructions (v_mad, per lane, summed over live lanes) the P-adic
 * kernel's launches executed since the last fthe_prof_enable / fthe_prof_read;
 * read it before fthe_prof_read, which resets it. */
int    fthe_prof_exec_macs(fthe_ctx *ctx, double *exec_macs);
/* limb count S of the radix-2^28 kernel used for a modulus of `bits` bits
 * (0 if unsupported). */
int    fthe_kernel_limbs(int bits);

#ifdef __cplusplus
}
#endif
#endif /* FTHE_H */
