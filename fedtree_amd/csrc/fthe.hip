// fthe.hip -- host side of the MI355X batch Paillier engine: C ABI (include/fthe.h),
// key set-up, program construction, chunked launch of the montprog kernel and
// the glue kernels.
//
// Data flow of one batch call (device-resident variant):
//   inputs (AoS u32 words / u64 plaintexts)  --pack-->  slots (radix-2^28, limb-major)
//   montprog kernel (one ciphertext per lane, uniform op program per modulus)
//   glue (canonicalise, CRT recombine)  --unpack-->  outputs (AoS u32 words)
// Batches are processed in chunks of L lanes (default 262144) so the
// per-lane window tables fit comfortably in HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <mutex>
#include <new>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>
#include <fcntl.h>
#include <unistd.h>

#include "../../include/fthe.h"
#include "bn_host.hpp"
#include "padic_tiles.hpp"
#include "addb_image.hpp"
#include "nadicb_image.hpp"
#include "fthe_glue.h"
#include "gen/montprog_blobs.h"

using namespace fthe;

#define HIPOK(x) do { if ((x) != hipSuccess) return FTHE_ERR_HIP; } while (0)

namespace {

constexpr int MAX_VARIANTS = 10;
// s80: four lanes per element mod p^2 / q^2 of Paillier-2048 (small-batch decrypt latency);
// 1000 + K: the P-adic exponentiation kernels mod P^2 (gen_padic.py, digits of K limbs, slots of 2K
// limbs; the "S" here only names the variant): K = 37 runs on the s74 slots of Paillier-2048,
// K = 19 on slots of its own (38 limbs) for Paillier-1024;
// 1137: the K = 37 P-adic kernel with matrix-core (MFMA) Barrett reductions (gen_padic_mfma.py), same
// slots and programs, no fixed-base table ops;
// 2000 + 76: the n-adic four-lane kernel (gen_nadic.py, base-n digits of 76 limbs) on the s152 slots;
// 2100 + 76: its Montgomery form (gen_nadic.py mont: LSB-first reductions, no quotient estimates)
// 2200 + 76: its matrix-core Barrett form (gen_nadicb.py: the products on the VALU, both Barrett reductions by n
// on i8 MFMA; workgroups of kNbWaves waves, n of 2041..2048 bits)
constexpr int kPadicS = 1037, kPadicK = 37, kPadicSmallK = 19, kNadicS = 2076, kPadicMfmaS = 1137,
              kNadicMontS = 2176, kNadicBarS = 2276;
const Shape kVariants[MAX_VARIANTS] = {{37, 28, 1}, {74, 28, 1}, {152, 27, 4}, {80, 27, 4},
                                       {1000 + kPadicK, 28, 1}, {1000 + kPadicSmallK, 28, 1}, {kNadicS, 27, 4},
                                       {kPadicMfmaS, 28, 1}, {kNadicMontS, 27, 4}, {kNadicBarS, 27, 4}};
constexpr Shape kLatShape{80, 27, 4};
constexpr int kAddbBlob = 3152;           // fthe_addb_q152's code object in gen/montprog_blobs.h

int variant_index(int S) {
    for (int i = 0; i < MAX_VARIANTS; i++) if (kVariants[i].S == S) return i;
    return -1;
}

// n bytes from the kernel CSPRNG (/dev/urandom; std::random_device if it cannot be read)
void urandom_bytes(void *dst, size_t n) {
    uint8_t *p = (uint8_t *)dst;
    size_t got = 0;
    int fd = open("/dev/urandom", O_RDONLY);
    if (fd >= 0) {
        while (got < n) {
            ssize_t r = read(fd, p + got, n - got);
            if (r <= 0) break;
            got += (size_t)r;
        }
        close(fd);
    }
    if (got < n) {
        std::random_device rd;
        for (; got < n; got++) p[got] = (uint8_t)rd();
    }
}

// splitmix64 (seeded key generation / rng keys)
uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ChaCha20 key + nonce of a device randomness stream.  seed 0: 320 bits straight from
// /dev/urandom; a nonzero seed (tests, benchmarks) expands deterministically with
// splitmix64.  `tweak` separates the streams of the different randomizer modes.
RngKey make_rng_key(uint64_t seed, uint64_t tweak) {
    RngKey rk{};
    if (!seed) {
        urandom_bytes(rk.k, sizeof rk.k);
        urandom_bytes(&rk.nonce, sizeof rk.nonce);
        return rk;
    }
    uint64_t s = seed;
    for (int i = 0; i < 8; i += 2) { uint64_t v = splitmix64(s); rk.k[i] = (uint32_t)v; rk.k[i + 1] = (uint32_t)(v >> 32); }
    rk.nonce = splitmix64(s) ^ tweak;
    return rk;
}

// GMP random state for key material: seed 0 -> 256 bits from /dev/urandom, else a
// deterministic 128-bit expansion of the seed (tests, benchmarks).
void seed_gmp_state(gmp_randstate_t st, uint64_t seed, uint64_t tweak) {
    Mpz sd;
    if (!seed) {
        uint32_t w[8];
        urandom_bytes(w, sizeof w);
        mpz_import(sd, 8, -1, 4, 0, 0, w);
    } else {
        uint64_t s = seed;
        mpz_set_ui(sd, (unsigned long)splitmix64(s));
        mpz_mul_2exp(sd, sd, 64);
        mpz_add_ui(sd, sd, (unsigned long)(splitmix64(s) ^ tweak));
    }
    gmp_randseed(st, sd);
}

size_t chunk_lanes() {
    static size_t v = [] {
        const char *e = getenv("FTHE_CHUNK");
        // 393216 lanes = 6144 waves: whole rounds at 2 waves/SIMD (s74) and 3 (s37, s152) on 1024 SIMDs
        size_t c = e ? (size_t)strtoull(e, nullptr, 10) : 393216;
        c = (c + 255) / 256 * 256;
        return c < 256 ? (size_t)256 : c;
    }();
    return v;
}

// CRT decrypts and device-randomness encrypts of at most this many lanes run their p and q halves on
// two streams, so the two launches share the chip: the waves of a batch that is not a whole number of
// rounds per half (200,000 Paillier-1024 ciphertexts: 3,125 waves per half, 3,072 resident) fill one
// tail instead of two -- 16.4 ms instead of 19.4 ms, and 91.7 ms instead of 106.7 ms at Paillier-2048
// (profiles/r02zzn_split_*.jsonl).  Default: one chunk; FTHE_DEC_SPLIT overrides, 0 turns this small-batch split
// off.  Larger calls split as well while split_all() is on (the default), so a one-stream A/B needs
// FTHE_DEC_SPLIT=0 and FTHE_SPLIT_ALL=0 together.
size_t dec_split_lanes() {
    static size_t v = [] {
        const char *e = getenv("FTHE_DEC_SPLIT");
        return e ? (size_t)strtoull(e, nullptr, 10) : chunk_lanes();
    }();
    return v;
}

// Large CRT encrypts / decrypts with both halves on two streams as well (each chunk's p and q launches share the
// chip, so one launch's tail of finishing waves overlaps the other's instead of idling SIMDs: +1.0% encrypts/s and
// decrypts/s at 10M pairs, profiles/r05c_split_ab.jsonl; a second slot region, 7.4 GB at P-2048).
// FTHE_SPLIT_ALL=0 keeps the halves in turn on one stream (A/B).
bool split_all() {
    static const bool v = [] {
        const char *e = getenv("FTHE_SPLIT_ALL");
        return e ? atoi(e) != 0 : true;
    }();
    return v;
}

// Decrypts of at most this many ciphertexts take the four-lane s80 kernel (Paillier-2048 keys);
// FTHE_DEC_QUAD overrides, 0 turns it off (A/B).
size_t dec_quad_max() {
    static size_t v = [] {
        const char *e = getenv("FTHE_DEC_QUAD");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)16384;
    }();
    return v;
}

// Launch size of the row-I/O ops (four-lane kernel, no slots but the R^k constant):
// 4 chunks; FTHE_ROWIO_CHUNK overrides (A/B)
size_t rowio_chunk_lanes() {
    static size_t v = [] {
        const char *e = getenv("FTHE_ROWIO_CHUNK");
        size_t c = e ? (size_t)strtoull(e, nullptr, 10) : 4 * chunk_lanes();
        c = (c + 1023) / 1024 * 1024;
        return c < 1024 ? (size_t)1024 : c;
    }();
    return v;
}

// Large CRT encrypts with device randomness pipelined across chunks: the p half of chunk i + 1 starts as soon as
// the p half of chunk i has finished (the q half and the recombination of chunk i still running on the side
// stream), so the chip never drains between chunks; two slot-region pairs alternate (15 GB more at P-2048).
// Measured neutral (2.721 / 2.707M vs 2.729 / 2.706M encrypts/s, profiles/r05j_enc_pipe_ab.jsonl): the split
// chunks already keep the chip full -- a chunk's p and q launches share it until the last round of waves -- so
// it is opt-in, FTHE_ENC_PIPE=1 (bit-identical, tests/test_gpu_split_streams.py).
bool enc_pipe() {
    static const bool v = [] {
        const char *e = getenv("FTHE_ENC_PIPE");
        return e ? atoi(e) != 0 : false;
    }();
    return v;
}

// the key holder's large encrypt batches with device randomness (the direct-y path bench.py times) launch
// twice chunk_lanes() per exponentiation: 786,432 lanes = six rounds of the P-adic kernel instead of three,
// +1.5% encrypts/s (1.8% at 1,572,864; profiles/r04q_chunk_ab.jsonl); FTHE_ENC_CHUNK overrides
size_t enc_chunk_lanes() {
    static const size_t v = [] {
        const char *e = getenv("FTHE_ENC_CHUNK");
        size_t c = e ? (size_t)strtoull(e, nullptr, 10) : 2 * chunk_lanes();
        return c < 1024 ? (size_t)1024 : c;
    }();
    return v;
}

// the parties' public-key encrypt on fthe_nadic_b76 (persistent waves: more batches per wave balance the SIMDs
// better): lanes per launch, four per ciphertext; FTHE_PUB_CHUNK overrides
size_t pub_chunk_lanes() {
    static const size_t v = [] {
        const char *e = getenv("FTHE_PUB_CHUNK");
        size_t c = e ? (size_t)strtoull(e, nullptr, 10) : chunk_lanes();
        return c < 3072 ? (size_t)3072 : c;
    }();
    return v;
}

// window width minimising table + multiplications for an e-bit exponent
int best_window(size_t ebits) {
    int best = 1; double bc = 1e30;
    for (int w = 1; w <= 6; w++) {
        double c = (double)(1 << (w - 1)) + (double)ebits / (w + 1);
        if (c < bc) { bc = c; best = w; }
    }
    return best;
}

}  // namespace

// --------------------------------------------------------------------------
struct DevBuf {
    void *p = nullptr; size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return FTHE_OK;
        if (p) (void)hipFree(p);
        p = nullptr; n = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) return FTHE_ERR_NOMEM;
        n = bytes;
        return FTHE_OK;
    }
    ~DevBuf() { if (p) (void)hipFree(p); }
};

// Pinned host staging buffer (page-locked: truly asynchronous DMA).
struct PinBuf {
    void *p = nullptr; size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return FTHE_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr; n = 0;
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return FTHE_ERR_NOMEM;
        n = bytes;
        return FTHE_OK;
    }
    ~PinBuf() { if (p) (void)hipHostFree(p); }
};

struct fthe_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t copy = nullptr;               // host<->device staging copies, overlapped with compute
    hipStream_t side = nullptr;               // second compute stream: the q half of small decrypts
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t ev_cb[2] = {};                 // pipelined CRT encrypts: chunk i's recombination done (region i & 1)
    int n_cu = 256;                           // compute units (small-batch spreading)
    int static_lds[MAX_VARIANTS] = {};        // per-variant static LDS bytes per workgroup
    PinBuf stage_out[2], stage_in[2];
    hipEvent_t ev_done[2] = {}, ev_copied[2] = {}, ev_in[2] = {};
    hipModule_t mod[MAX_VARIANTS] = {};
    hipFunction_t fn[MAX_VARIANTS] = {};
    hipModule_t mod_addb = nullptr;           // fthe_addb_q152 (gen_addb.py): P-2048 adds, matrix-core Barrett
    hipFunction_t fn_addb = nullptr;
    uint32_t *d_jobctr = nullptr;             // job counters of persistent launches (one per launch, in turn)
    unsigned jobctr_i = 0;
    DevBuf slots, slots1, scratch, io[5];   // slots1: the small-modulus (mod p, q) programs
    size_t mem_limit = 0;                   // fthe_ctx_set_mem_limit: cap on the slot region grown for a call
    DevBuf hb[6];                           // histogram CSR / segmented-product plan (device)
    DevBuf ezm;                             // zero-first folds: Enc(0) rows masked to the populated segments
    DevBuf dec[3];                          // decimal codec: 9-digit chunks, lengths, leading chunk / error flag
    void *cub_tmp = nullptr; size_t cub_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_mm = 0;
    bool timed = false;
    // optional per-launch timing of the montprog kernel (bench roofline)
    bool prof = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev;
    std::vector<double> prof_mm;  // products per lane of each recorded launch
    std::vector<int> prof_vi;     // kernel variant of each recorded launch
    double var_ms[MAX_VARIANTS] = {}, var_n[MAX_VARIANTS] = {};   // last read, exponentiation launches
    size_t prof_used = 0;
    double prof_busy_ms = 0, prof_expo_busy_ms = 0;   // union of the launch intervals at the last fthe_prof_read
    double prof_lane_mm = 0;      // sum over launches of live lanes x products
    double prof_alg_macs = 0;     // sum over launches of live lanes x products x W(s), SURVEY 8(d)
    double prof_exec_macs = 0;    // P-adic launches: v_mad instructions x live lanes
    double prof_launch_lanes = 0; // sum over launches of live lanes
};

// Device copy of one Montgomery modulus.
struct DevMod {
    MontMod m;
    uint32_t *d_ctx = nullptr;     // N limbs (S) + nprime; P-adic: -P limbs, mu limbs
    int kernel_S = 0;              // kPadicS: the P-adic kernel on m's slot shape (m.N = P^2)
    int kernel_S_mfma = 0;         // kPadicMfmaS: the same programs on the MFMA-Barrett kernel (no table ops)
    // SURVEY 8(d) work unit: W(s) = 2 s^2 + s 32x32 MACs per Montgomery
    // product on s = ceil(bits/32) u32 limbs (algorithmic, kernel-independent)
    double w_alg() const {
        double s = (double)((mpz_sizeinbase(m.N, 2) + 31) / 32);
        return 2 * s * s + s;
    }
};

// Group-commit queue of fthe_decrypt_shared (one per key, created on first use).
struct DecReq {
    const uint32_t *ct; size_t count; uint64_t *m_low; uint32_t *m_full; bool short_pt;
    int rc = FTHE_OK; bool done = false;
};
struct EncReq {
    const uint64_t *m; size_t count; uint32_t *out; int flags;
    int rc = FTHE_OK; bool done = false;
};
struct OpReq {                               // fthe_add_shared / fthe_scalar_mul_u64_shared
    bool mul; const uint32_t *a, *b; uint64_t k; size_t count; uint32_t *out;
    int rc = FTHE_OK; bool done = false;
};
struct Coalescer {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<DecReq *> pending;
    std::vector<EncReq *> epending;          // fthe_encrypt_shared: its own leader and context
    std::vector<OpReq *> opending;           // fthe_add_shared / _scalar_mul_u64_shared: a third one
    bool leader = false, eleader = false, oleader = false;
    fthe_ctx *ctx = nullptr, *ectx = nullptr, *octx = nullptr;   // the key's own contexts, one leader each
    // group-commit linger (linger() below): requests in each queue's previous batch, a leader waiting
    std::condition_variable lcv;
    size_t last = 0, elast = 0, olast = 0;
    int64_t last_us = 0, elast_us = 0, olast_us = 0;   // the previous batch's duration
    bool lingering = false, elingering = false, olingering = false;
    std::vector<uint32_t> ct, full, eout, oa, ob, oout;
    std::vector<uint64_t> lo, em;
    ~Coalescer() {
        if (ctx) fthe_ctx_destroy(ctx);
        if (ectx) fthe_ctx_destroy(ectx);
        if (octx) fthe_ctx_destroy(octx);
    }
};

// A named constant (S limbs) on the device.
struct fthe_key {
    std::mutex co_mu;
    std::unique_ptr<Coalescer> co;           // released first in ~fthe_key (its context drains there)
    int device = 0;
    Shape spq{0, 0, 0}, sn2{0, 0, 0};   // kernel shapes: mod p^2/q^2/p/q and mod n^2
    int n_bits = 0, n_words = 0;
    bool priv = false, pub_ok = false;
    Mpz n, n2, g, p, q, lambda, mu;
    DevMod mn2, mp2, mq2, mp, mq, mp1, mq1;   // mp1/mq1: mod p, q on the small-limb kernel
    Shape sp1{0, 0, 0};
    // small-batch decrypt on the four-lane s80 kernel (each product spread over a quad of lanes)
    Shape slat{0, 0, 0};
    DevMod mp2l, mq2l;
    // P-adic exponentiation kernel mod p^2, q^2 (gen_padic.py): the CRT encrypt's y^P and the
    // decrypt's c^(P-1); s74 programs before / after it convert to and from Montgomery form
    bool padic = false;
    bool padic_own_slots = false;   // the P-adic kernel's slots are not the CRT region's (K = 19)
    DevMod mpA, mqA;
    // n-adic four-lane kernel (gen_nadic.py): the public-key encrypt's r^n mod n^2 on base-n digits
    bool nadic = false;
    DevMod mnA;                     // m: n^2 on the s152 slot shape; ctx: n on 76 limbs of 27 bits
    int c_n76 = -1;                 // n in 76 limbs (the output c = x0 + x1 n)
    // the Montgomery form of the n-adic kernel (default; FTHE_NADIC_CLASSICAL=1 keeps the classical one):
    // ctx as mnA's (n limbs, n' at word 76); K = R^(n+1) mod n^2 as digits (K mod n, K div n), R = 2^2052
    bool nadic_mont = false;
    DevMod mnM;
    int c_Kn = -1;
    // the matrix-core Barrett form (fthe_nadic_b76, the default for n of 2041..2048 bits; FTHE_NADIC_MONT=1
    // keeps the Montgomery form): ctx = nadicb_image.hpp (LDS image, n limbs); the classical program
    bool nadic_b = false;
    DevMod mnB;
    // Paillier-1024 public-key encrypt (n of 1009..1030 bits) on the P-adic kernel with P = n
    bool padic_pub = false;
    DevMod mnP;
    int cl_R2p = -1, cl_R3p = -1, cl_R2q = -1, cl_R3q = -1, cl_one = -1, cl_p2 = -1, cl_q2 = -1, cl_nRp = -1, cl_nRq = -1;
    int c1_R2p = -1, c1_R3p = -1, c1_R2q = -1, c1_R3q = -1, c1_one = -1;
    int kp = 0, kq = 0;             // limbs of p, q
    // device constants: one allocation, each its modulus' limb count
    std::vector<std::vector<uint32_t>> host_consts;
    std::vector<size_t> const_off;
    uint32_t *d_consts = nullptr;
    // programs: one allocation
    std::vector<uint32_t> host_progs;
    uint32_t *d_progs = nullptr;
    size_t n_words_dev_off = 0;     // offset (in u32) of n words in d_consts
    uint32_t *d_nwords = nullptr;
    uint32_t *d_pqwords = nullptr;  // p then q as pq_w u32 words each (device-drawn y_p, y_q)
    int pq_w = 0;
    ~fthe_key() {
        co.reset();
        for (DevMod *d : {&mn2, &mp2, &mq2, &mp, &mq, &mp1, &mq1, &mp2l, &mq2l, &mpA, &mqA, &mnA, &mnP, &mnM, &mnB})
            if (d->d_ctx) (void)hipFree(d->d_ctx);
        if (d_consts) (void)hipFree(d_consts);
        if (d_progs) (void)hipFree(d_progs);
        if (d_nwords) (void)hipFree(d_nwords);
        if (d_pqwords) (void)hipFree(d_pqwords);
        if (d_addb) (void)hipFree(d_addb);
        for (uint32_t *p : {fb.d_tab_pub, fb.d_tab_p, fb.d_tab_q, fb.d_prog}) if (p) (void)hipFree(p);
        for (uint32_t *p : {xb.d_tab[0], xb.d_tab[1], xb.d_prog}) if (p) (void)hipFree(p);
        if (pb.d_prog) (void)hipFree(pb.d_prog);           // pb.tab: shared, freed by its last key
    }
    // constant handles
    int add_const(const std::vector<uint32_t> &limbs) {
        size_t off = const_off.empty() ? 0 : const_off.back() + host_consts.back().size();
        host_consts.push_back(limbs);
        const_off.push_back(off);
        return (int)host_consts.size() - 1;
    }
    uint32_t *cst(int h) const { return d_consts + const_off[h]; }
    // programs
    // alg: algorithmic MACs per lane if not mm x W(s); exec: v_mad per lane (P-adic programs)
    struct PH { size_t off = 0; double mm = 0, alg = -1, exec = -1; };
    PH add_prog(const Prog &p) {
        PH h; h.off = host_progs.size(); h.mm = p.montmuls;
        host_progs.insert(host_progs.end(), p.w.begin(), p.w.end());
        return h;
    }
    const uint32_t *prog(const PH &h) const { return d_progs + h.off; }

    // ---- slot maps and programs --------------------------------------------
    int w_pub = 5, w_crt = 5, w_dec = 5, tabn_max = 16;
    // consts
    int c_one = -1, c_one_n2 = -1, c_R2n2 = -1, c_nRn2 = -1, c_n2 = -1;
    int c_R2p = -1, c_R3p = -1, c_nRp = -1, c_R2q = -1, c_R3q = -1, c_nRq = -1;
    int c_p2 = -1, c_q2 = -1, c_2p2 = -1, c_qinvRp2 = -1;
    int c_zero = -1;
    int c_p = -1, c_q = -1, c_2p = -1, c_pinv = -1, c_qinv2 = -1, c_hRp = -1, c_hRq = -1, c_qinvRp = -1;
    PH pr_add_w, pr_sub_w;     // row-I/O forms (four-lane kernel, 128-word rows)
    bool rowio = false;
    bool add_classical = false;               // pr_add_w is one classical product (no R^2 constant)
    void *d_addb = nullptr;                   // fthe_addb_q152's per-key context (addb_image.hpp): n of 2048 bits
    PH pr_enc_pub, pr_add, pr_sub, pr_enc_p, pr_enc_q, pr_enc_p_nt, pr_enc_tail, pr_dec_pl, pr_dec_ql, pr_enc_pl, pr_enc_ql, pr_dec_p, pr_dec_q, pr_dec_hp, pr_dec_hq, pr_dec_t;
    PH pr_encA_p, pr_encA_q;      // stage A of the CRT encrypt (mod p, q; small kernel)
    // P-adic form of stage B: the exponentiation (P-adic kernel), then the rest on s74
    PH prP_enc_p, prP_enc_q, prP_encB_p, prP_encB_q, prP_encB_p_nt;
    PH prP_dec_pre_p, prP_dec_pre_q, prP_dec_p, prP_dec_q, prP_dec_post_p, prP_dec_post_q;
    PH prN_enc_pub;                  // n-adic form of the public-key encrypt
    PH prM_enc_pub;                  // its Montgomery form (fthe_nadic_m76)
    PH prB_enc_pub;                  // its matrix-core Barrett form (fthe_nadic_b76)
    PH prP_enc_pub;                  // P-adic form (P = n) of the Paillier-1024 public-key encrypt

    // ---- fixed-base randomizer (FTHE_ENC_FIXED_BASE), built on first use -----
    // r^n = hs^alpha with hs = h^n mod n^2 for one random h per key: 8-bit-window
    // tables entry[j][d] = hs^(d 256^j) (Montgomery form) turn the exponentiation
    // into one gathered product per window (no squarings).
    struct FixedBase {
        bool ready = false;
        Mpz h, hs;
        int window = 16;                  // bits per window (digit width)
        int nwin_pub = 0, nwin_crt = 0;   // windows of alpha: public / per prime
        int ew_pub = 0, ew_crt = 0;       // words per table entry
        bool pub = false, pub_rows = false;
        uint32_t *d_tab_pub = nullptr, *d_tab_p = nullptr, *d_tab_q = nullptr, *d_prog = nullptr;
        size_t off_pub = 0, off_p = 0, off_q = 0;
        double mm_pub = 0, mm_crt = 0;
    } fb;
    std::mutex fb_mu;

    // ---- exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT, key holder) ----
    // Per prime P: three bases gam[i] = t_i^P mod P^2 whose t_i generate Z_P^*
    // (checked for every prime l < 2^24 dividing P - 1), tables of 16-bit windows
    // for exponents y_i < P; r^n mod P^2 is drawn as prod_i gam[i]^y_i.
    struct ExactBase {
        bool ready = false;
        int nb = 3;                       // bases per prime: 1 when P - 1 is factored (a generator), else 3
        int nwin = 0, ew = 0;             // 16-bit windows per exponent, words per entry
        Mpz gam[2][3];
        uint32_t *d_tab[2] = {nullptr, nullptr}, *d_prog = nullptr;
        size_t off[2] = {0, 0};
        double mm = 0;
        bool padic = false;               // tables in digit form, products on the P-adic kernel
    } xb;
    // ---- public exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT, public form) ----
    // Bases hs_i = t_i^n mod n^2 published by the key holder, <t_1 .. t_nb> = Z_n^*;
    // r^n = prod hs_i^y_i with y_i uniform below 2^(16 nwin) >= n 2^64.
    // The tables depend on (device, n, bases) only and are shared between the keys that hold
    // them: in FedTree's simulation every party has its own copy of the public key.
    struct SharedTab {
        uint32_t *d = nullptr;
        ~SharedTab() { if (d) (void)hipFree(d); }
    };
    struct PublicBase {
        bool ready = false, rows = false;
        bool nadic = false;               // digit-form entries, products on the n-adic kernel (P-2048)
        int nb = 0, ew = 0;               // bases, words per table entry
        int nwin[3] = {0, 0, 0};          // 16-bit windows of each base's exponent
        int wtot = 0;                     // windows of all bases
        Mpz hs[3];
        std::shared_ptr<SharedTab> tab;
        uint32_t *d_tab = nullptr, *d_prog = nullptr;
        double mm = 0;
    } pb;
    // prime factors of p - 1 and q - 1 when the key generator recorded them (FTHE_KEYGEN_KNOWN_ORDER)
    bool order_known = false;
    std::vector<Mpz> pm1_factors, qm1_factors;
};

// slot numbering shared by all programs
enum Slot : int {
    SL_IN0 = 0, SL_IN1 = 1, SL_C0 = 2, SL_C1 = 3, SL_C2 = 4, SL_C3 = 5,
    SL_OUTP = 6, SL_OUTQ = 7, SL_SAVED = 8, SL_SQ = 9, SL_T0 = 10, SL_T1 = 11,
    SL_T2 = 12, SL_T3 = 13, SL_T4 = 14, SL_T5 = 15, SL_TAB = 16
};

static int nslots_for(const fthe_key *k) { return SL_TAB + k->tabn_max; }

// The p half of every CRT encrypt program ends here: X = cp (< 2p^2) -> (cp + v) (q^2)^-1 mod p^2
// into T2, with v = K - cq in T0 (k_crt_prep_q, run after the q half) and Mont((q^2)^-1) in T1.
static void crt_tail(Prog &e) { e.addslot(SL_T0); e.mul(SL_T1); e.storex(SL_T2); }

// One-lane kernels prefetch multipliers into LDS (PREFA/MULA); FTHE_NO_LDSDMA=1 turns it off (A/B).
static bool lds_prefetch(const Shape &sh) {
    static const bool off = getenv("FTHE_NO_LDSDMA") != nullptr;
    return sh.lanes == 1 && !off;
}

// ---------------------------------------------------------------------------
extern "C" int fthe_version(void) { return 100; }

extern "C" const char *fthe_strerror(int s) {
    switch (s) {
        case FTHE_OK: return "ok";
        case FTHE_ERR_ARG: return "invalid argument";
        case FTHE_ERR_HIP: return "HIP runtime error (no gfx950 device or launch failure)";
        case FTHE_ERR_NOPRIV: return "private key required";
        case FTHE_ERR_UNSUPPORTED: return "modulus size not supported by the built kernels";
        case FTHE_ERR_KEY: return "invalid key material";
        case FTHE_ERR_NOMEM: return "device allocation failed";
        default: return "unknown status";
    }
}

extern "C" int fthe_kernel_limbs(int bits) { return kernel_limbs_for_bits(bits); }

extern "C" int fthe_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0 ? n : 0;
}

extern "C" int fthe_ctx_create(int device, fthe_ctx **out) {
    if (!out) return FTHE_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return FTHE_ERR_HIP;
    HIPOK(hipSetDevice(device));
    std::unique_ptr<fthe_ctx> c(new fthe_ctx);
    c->device = device;
    HIPOK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPOK(hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
    HIPOK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    HIPOK(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    HIPOK(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    for (auto &ev : c->ev_cb) HIPOK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int i = 0; i < 2; i++) {
        HIPOK(hipEventCreateWithFlags(&c->ev_done[i], hipEventDisableTiming));
        HIPOK(hipEventCreateWithFlags(&c->ev_copied[i], hipEventDisableTiming));
        HIPOK(hipEventCreateWithFlags(&c->ev_in[i], hipEventDisableTiming));
    }
    for (int i = 0; i < MAX_VARIANTS; i++) {
        const unsigned char *blob = fthe_montprog_blob(kVariants[i].S);
        if (!blob) return FTHE_ERR_HIP;
        HIPOK(hipModuleLoadData(&c->mod[i], blob));
        char name[64];
        if (kVariants[i].S > 2200) snprintf(name, sizeof name, "fthe_nadic_b%d", kVariants[i].S - 2200);
        else if (kVariants[i].S > 2100) snprintf(name, sizeof name, "fthe_nadic_m%d", kVariants[i].S - 2100);
        else if (kVariants[i].S > 2000) snprintf(name, sizeof name, "fthe_nadic_q%d", kVariants[i].S - 2000);
        else if (kVariants[i].S > 1100) snprintf(name, sizeof name, "fthe_padic_m%d", kVariants[i].S - 1100);
        else if (kVariants[i].S > 1000) snprintf(name, sizeof name, "fthe_padic_k%d", kVariants[i].S - 1000);
        else snprintf(name, sizeof name, "fthe_montprog_s%d", kVariants[i].S);
        HIPOK(hipModuleGetFunction(&c->fn[i], c->mod[i], name));
        HIPOK(hipFuncGetAttribute(&c->static_lds[i], HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, c->fn[i]));
    }
    if (const unsigned char *blob = fthe_montprog_blob(kAddbBlob)) {
        HIPOK(hipModuleLoadData(&c->mod_addb, blob));
        HIPOK(hipModuleGetFunction(&c->fn_addb, c->mod_addb, "fthe_addb_q152"));
    }
    HIPOK(hipEventCreate(&c->ev0));
    HIPOK(hipEventCreate(&c->ev1));
    HIPOK(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
    *out = c.release();
    return FTHE_OK;
}

extern "C" int fthe_host_alloc(size_t bytes, void **out) {
    if (!out) return FTHE_ERR_ARG;
    *out = nullptr;
    if (bytes == 0) return FTHE_OK;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) { *out = nullptr; return FTHE_ERR_HIP; }
    return FTHE_OK;
}

extern "C" void fthe_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

extern "C" void fthe_ctx_destroy(fthe_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    if (c->side) (void)hipStreamSynchronize(c->side);
    for (int i = 0; i < MAX_VARIANTS; i++) if (c->mod[i]) (void)hipModuleUnload(c->mod[i]);
    if (c->mod_addb) (void)hipModuleUnload(c->mod_addb);
    if (c->d_jobctr) (void)hipFree(c->d_jobctr);
    if (c->cub_tmp) (void)hipFree(c->cub_tmp);
    for (auto &e : c->prof_ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    for (auto &ev : c->ev_cb) if (ev) (void)hipEventDestroy(ev);
    for (int i = 0; i < 2; i++) {
        if (c->ev_done[i]) (void)hipEventDestroy(c->ev_done[i]);
        if (c->ev_copied[i]) (void)hipEventDestroy(c->ev_copied[i]);
        if (c->ev_in[i]) (void)hipEventDestroy(c->ev_in[i]);
    }
    delete c;
}

extern "C" int fthe_ctx_sync(fthe_ctx *c) {
    if (!c) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipStreamSynchronize(c->stream));
    return FTHE_OK;
}
extern "C" void *fthe_ctx_stream(fthe_ctx *c) { return c ? (void *)c->stream : nullptr; }
extern "C" int fthe_ctx_device(fthe_ctx *c) { return c ? c->device : -1; }

extern "C" int fthe_ctx_set_mem_limit(fthe_ctx *c, size_t bytes) {
    if (!c) return FTHE_ERR_ARG;
    c->mem_limit = bytes;
    return FTHE_OK;
}

extern "C" double fthe_last_kernel_ms(fthe_ctx *c) {
    if (!c || !c->timed) return 0.0;
    float ms = 0;
    if (hipEventSynchronize(c->ev1) != hipSuccess) return 0.0;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return 0.0;
    return ms;
}
extern "C" double fthe_last_montmuls(fthe_ctx *c) { return c ? c->last_mm : 0.0; }

extern "C" int fthe_prof_variant(fthe_ctx *c, int S, double *expo_ms, double *expo_launches) {
    if (!c) return FTHE_ERR_ARG;
    int vi = variant_index(S);
    if (vi < 0) return FTHE_ERR_ARG;
    if (expo_ms) *expo_ms = c->var_ms[vi];
    if (expo_launches) *expo_launches = c->var_n[vi];
    return FTHE_OK;
}

extern "C" int fthe_prof_enable(fthe_ctx *c, int on) {
    if (!c) return FTHE_ERR_ARG;
    c->prof = on != 0;
    c->prof_used = 0; c->prof_lane_mm = 0; c->prof_launch_lanes = 0; c->prof_alg_macs = 0;
    c->prof_exec_macs = 0;
    return FTHE_OK;
}

extern "C" int fthe_prof_busy(fthe_ctx *c, double *busy_ms, double *expo_busy_ms) {
    if (!c) return FTHE_ERR_ARG;
    if (busy_ms) *busy_ms = c->prof_busy_ms;
    if (expo_busy_ms) *expo_busy_ms = c->prof_expo_busy_ms;
    return FTHE_OK;
}

extern "C" int fthe_prof_exec_macs(fthe_ctx *c, double *exec_macs) {
    if (!c || !exec_macs) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipStreamSynchronize(c->stream));
    *exec_macs = c->prof_exec_macs;
    return FTHE_OK;
}

extern "C" int fthe_prof_read(fthe_ctx *c, double *kernel_ms, double *launches, double *lane_montmuls, double *lanes,
                              double *expo_ms, double *expo_launches, double *alg_macs) {
    if (!c) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipStreamSynchronize(c->stream));
    HIPOK(hipStreamSynchronize(c->side));
    double tot = 0, etot = 0, en = 0;
    for (int v = 0; v < MAX_VARIANTS; v++) c->var_ms[v] = c->var_n[v] = 0;
    // launches on the context's two compute streams may overlap (the CRT halves of FTHE_SPLIT_ALL): besides the
    // summed durations, the union of the launch intervals (time with at least one such launch running)
    std::vector<std::pair<double, double>> iv, eiv;
    for (size_t i = 0; i < c->prof_used; i++) {
        float ms = 0, t0 = 0;
        HIPOK(hipEventElapsedTime(&ms, c->prof_ev[i].first, c->prof_ev[i].second));
        HIPOK(hipEventElapsedTime(&t0, c->prof_ev[0].first, c->prof_ev[i].first));
        tot += ms;
        iv.emplace_back(t0, (double)t0 + ms);
        if (c->prof_mm[i] >= 64) {                            // exponentiation launches
            etot += ms; en += 1;
            c->var_ms[c->prof_vi[i]] += ms; c->var_n[c->prof_vi[i]] += 1;
            eiv.emplace_back(t0, (double)t0 + ms);
        }
    }
    auto union_ms = [](std::vector<std::pair<double, double>> &v) {
        std::sort(v.begin(), v.end());
        double u = 0, a = 0, b = -1e300;
        for (auto &x : v) {
            if (x.first > b) { if (b > a) u += b - a; a = x.first; b = x.second; }
            else b = std::max(b, x.second);
        }
        if (!v.empty() && b > a) u += b - a;
        return u;
    };
    c->prof_busy_ms = union_ms(iv);
    c->prof_expo_busy_ms = union_ms(eiv);
    if (kernel_ms) *kernel_ms = tot;
    if (expo_ms) *expo_ms = etot;
    if (expo_launches) *expo_launches = en;
    if (launches) *launches = (double)c->prof_used;
    if (lane_montmuls) *lane_montmuls = c->prof_lane_mm;
    if (lanes) *lanes = c->prof_launch_lanes;
    if (alg_macs) *alg_macs = c->prof_alg_macs;
    c->prof_used = 0; c->prof_lane_mm = 0; c->prof_launch_lanes = 0; c->prof_alg_macs = 0; c->prof_exec_macs = 0;
    return FTHE_OK;
}

// ---------------------------------------------------------------------------
// Key set-up
static int upload_mod(DevMod &d, const mpz_t N, Shape sh) {
    d.m.init(N, sh);
    if (hipMalloc(&d.d_ctx, d.m.ctx.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(d.d_ctx, d.m.ctx.data(), d.m.ctx.size() * 4, hipMemcpyHostToDevice));
    return FTHE_OK;
}

// P-adic kernel constants for P (gen_padic.py): -P in K radix-2^28 limbs (int32), zero words up to
// a multiple of 4 SGPRs, mu = floor(2^(56 K) / P) in K + 1 limbs; m is P^2 on the kernel's slot
// shape (2K limbs: slot strides, roofline units).  The digit size K for the CRT half shape sh:
//   K = 37 on the s74 slots (Paillier-2048): b^36 <= P and 50 P < b^37 -> P of 1009..1030 bits;
//   K = 19 on 38-limb slots of its own (Paillier-1024, sh = s37): P of 505..516 bits, which also
//     keeps its < 6 P^2 results within the 37 limbs of the s37 slots they are copied back to; the
//     s37 shape itself takes P^2 of <= 1028 bits (kernel_shape_for_bits), so in effect 505..514.
// 0: no P-adic kernel for this P.
static int padic_digits(const mpz_t P, Shape sh) {
    if (getenv("FTHE_NO_PADIC") || sh.B != 28 || sh.lanes != 1) return 0;
    const size_t b = mpz_sizeinbase(P, 2);
    if (sh.S == 2 * kPadicK && b >= 1009 && b <= 1030) return kPadicK;
    if (sh.S == 37 && b >= 505 && b <= 516) return kPadicSmallK;
    return 0;
}
// K = 37 also carries the LDS tile image of fthe_padic_m37 (padic_tiles.hpp) at byte 512 of the context,
// and the MFMA-Barrett kernel then runs the key's exponentiation programs; FTHE_NO_PADIC_MFMA=1 keeps
// them on fthe_padic_k37 (bit-identical results).
static int upload_padic(DevMod &d, const mpz_t P, int K) {
    Mpz P2; mpz_mul(P2, P, P);
    d.m.init(P2, Shape{2 * K, 28, 1});
    const int pad = ((20 + K + 3) & ~3) - 20 - K;          // gen_padic.py: mu from an aligned SGPR
    std::vector<uint8_t> tiles;
    if (K == kPadicK && !getenv("FTHE_NO_PADIC_MFMA")) tiles = padic_tiles::build(P);
    std::vector<uint32_t> w(tiles.empty() ? (size_t)2 * K + 1 + pad : 128 + tiles.size() / 4, 0u), l = to_limbs(P, K, 28);
    if (!tiles.empty()) std::memcpy(w.data() + 128, tiles.data(), tiles.size());
    for (int j = 0; j < K; j++) w[j] = (uint32_t)(-(int32_t)l[j]);
    Mpz mu; mpz_set_ui(mu, 1); mpz_mul_2exp(mu, mu, 56 * K); mpz_fdiv_q(mu, mu, P);
    std::vector<uint32_t> ml = to_limbs(mu, K + 1, 28);
    std::copy(ml.begin(), ml.end(), w.begin() + K + pad);
    if (hipMalloc(&d.d_ctx, w.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(d.d_ctx, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    d.kernel_S = 1000 + K;
    d.kernel_S_mfma = tiles.empty() ? 0 : kPadicMfmaS;
    return FTHE_OK;
}
// Algorithmic 32-bit MACs of a P-adic program (SURVEY 8(d) units, the executed algorithm): s = words
// of P; squaring s^2 (2 x0 x1) + s(s+1)/2 (x0^2) + 2 Barretts, product 3 s^2 + 2 Barretts, a Barrett
// (s+1)(s+2)/2 (upper half of q1 mu) + s(s+1)/2 (lower half of q3 P); LOADP one Barrett, STOREP s^2.
static double padic_alg(const Prog &p, const mpz_t P) {
    const double s = (double)((mpz_sizeinbase(P, 2) + 31) / 32);
    const double bar = (s + 1) * (s + 2) / 2 + s * (s + 1) / 2;
    const double sq = s * s + s * (s + 1) / 2 + 2 * bar, mul = 3 * s * s + 2 * bar;
    return p.squarings * sq + (p.montmuls - p.squarings) * mul + bar + s * s;
}
// v_mad instructions per lane of the same program in the kernel (K = 37 radix-2^28 limbs per digit),
// as emitted by gen_padic.py: a Barrett is K(K+1)/2 + 2K + 1 (q2 columns K-1..2K) + K(K+1)/2 + K
// (r columns 0..K-1, one init MAD each); squaring K^2 + K(K+1)/2 + 2 Barretts, product 3 K^2 +
// 2 Barretts, LOADP one Barrett, STOREP K^2 + K (5,108 / 7,143 / 1,518 / 1,406 at K = 37).
static double padic_exec(const Prog &p, int Kd) {
    const double K = Kd;
    const double bar = K * (K + 1) + 3 * K + 1;
    const double sq = K * K + K * (K + 1) / 2 + 2 * bar, mul = 3 * K * K + 2 * bar;
    return p.squarings * sq + (p.montmuls - p.squarings) * mul + bar + K * K + K;
}

// n-adic kernel (gen_nadic.py) for the public-key encrypt: n of 2042..2050 bits on the s152 slots (which
// hold n^2 of <= 4096 bits: in effect 2042..2048).
// ctx = MontMod(n, 76 limbs of 27 bits, four lanes).ctx (n limbs, nprime, quotient-estimate doubles).
constexpr Shape kNadicDigit{76, 27, 4};
static bool nadic_ok(const fthe_key *k) {
    const size_t b = mpz_sizeinbase(k->n, 2);
    return !getenv("FTHE_NO_NADIC") && k->sn2.S == 152 && k->sn2.B == 27 && k->sn2.lanes == 4 &&
           b >= 2042 && b <= 2050;
}
// its Montgomery form (fthe_nadic_m76, the default below 2041 bits) needs only an odd n with 8 n < R = 2^2052 and n^2 on the
// s152 slots: every n of 1033..2048 bits (no quotient estimate, so no lower bound of its own)
static bool nadic_mont_ok(const fthe_key *k) {
    return !getenv("FTHE_NO_NADIC") && !getenv("FTHE_NADIC_CLASSICAL") && k->sn2.S == 152 && k->sn2.B == 27 &&
           k->sn2.lanes == 4 && mpz_sizeinbase(k->n, 2) <= 2048;
}
// its matrix-core Barrett form (fthe_nadic_b76, the default for n of 2041..2048 bits, n^2 on the s152 slots;
// FTHE_NADIC_MONT=1 at key set-up keeps the Montgomery form): persistent waves and the fixed-pair hand-off made
// it 2.6% faster than fthe_nadic_m76 (555k vs 541k public-key encrypts/s in one process, tools/nadicb_ab.py,
// profiles/r04u_nadicb_3op_ab.json)
static bool nadicb_ok(const fthe_key *k) {
    return !getenv("FTHE_NO_NADIC") && !getenv("FTHE_NADIC_MONT") && !getenv("FTHE_NADIC_CLASSICAL") &&
           k->sn2.S == 152 && k->sn2.B == 27 && k->sn2.lanes == 4 && nadicb::n_ok(k->n);
}
static int upload_nadic(DevMod &d, const mpz_t n, const mpz_t n2, Shape slots, bool classical = true) {
    d.m.init(n2, slots);
    MontMod dm;
    dm.init(n, kNadicDigit);
    if (classical && !dm.classical_ok()) return FTHE_ERR_UNSUPPORTED;
    if (hipMalloc(&d.d_ctx, dm.ctx.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(d.d_ctx, dm.ctx.data(), dm.ctx.size() * 4, hipMemcpyHostToDevice));
    d.kernel_S = kNadicS;
    return FTHE_OK;
}
// Algorithmic 32-bit MACs of an n-adic program (s = words of n): a squaring is two classical products
// mod n, 2 (s^2 + s^2) (product + quotient-digit reduction), a general product 2 s^2 + 3 s^2.
static double nadic_alg(const Prog &p, const mpz_t n) {
    const double s = (double)((mpz_sizeinbase(n, 2) + 31) / 32);
    return p.squarings * 4 * s * s + (p.montmuls - p.squarings) * 5 * s * s;
}
// v_mad per lane of the same program in the kernel (76 steps of 4 x 19 / 5 x 19 MADs, quads of lanes)
static double nadic_exec(const Prog &p) {
    return p.squarings * 76.0 * 76 + (p.montmuls - p.squarings) * 76.0 * 95;
}

static int key_finish(fthe_key *k) {
    // choose kernel variants: CRT moduli (p^2, q^2, p, q) and n^2
    if (k->priv) {
        Mpz p2; mpz_mul(p2, k->p, k->p);
        Mpz q2; mpz_mul(q2, k->q, k->q);
        size_t b = std::max(p2.bits(), q2.bits());
        k->spq = kernel_shape_for_bits((int)b);
        if (!k->spq.S) return FTHE_ERR_UNSUPPORTED;
    }
    k->sn2 = kernel_shape_for_bits((int)k->n2.bits());
    k->pub_ok = k->sn2.S != 0;
    if (!k->pub_ok && !k->priv) return FTHE_ERR_UNSUPPORTED;
    Mpz one(1);

    if (k->pub_ok) {
        int rc = upload_mod(k->mn2, k->n2, k->sn2); if (rc) return rc;
        const MontMod &M = k->mn2.m;
        k->c_one_n2 = k->add_const(M.limbs(one));
        k->c_R2n2 = k->add_const(M.limbs(M.R2));
        k->c_nRn2 = k->add_const(M.mont(k->n));
        k->c_n2 = k->add_const(M.limbs(k->n2));
        // encrypt: X = r R; X^n; (1 + m n) X  (paillier.cpp:135-137 with g^m = 1 + m n)
        Prog e;
        e.lds_a = lds_prefetch(k->sn2);
        k->w_pub = best_window(k->n.bits());
        e.loadx(SL_IN0); e.mul(SL_C0);
        e.pow(k->n, SL_TAB, SL_SQ, k->w_pub);
        e.storex(SL_SAVED);
        e.loadx(SL_IN1); e.mul(SL_C1); e.addsmall(1); e.mul(SL_SAVED);
        e.storex(SL_OUTP); e.end();
        k->pr_enc_pub = k->add_prog(e);
        k->tabn_max = std::max(k->tabn_max, 1 << (k->w_pub - 1));
        // n-adic form (n of 2048 bits): X = r as base-n digits (r, 0); X^n; X (1 + m n) with the digits
        // (1, m) of slot C1; canonical digits -> c = x0 + x1 n by the output kernel (mul_add_out)
        k->nadic = nadic_ok(k);
        k->nadic_mont = nadic_mont_ok(k);
        if (k->nadic || k->nadic_mont) k->c_n76 = k->add_const(to_limbs(k->n, kNadicDigit.S, kNadicDigit.B));
        if (k->nadic) {
            if ((rc = upload_nadic(k->mnA, k->n, k->n2, k->sn2))) return rc;
            Prog x;
            x.loadx(SL_IN0); x.canon();
            x.pow(k->n, SL_TAB, SL_SQ, k->w_pub);
            x.mul(SL_C1); x.canon(); x.storex(SL_OUTP); x.end();
            fthe_key::PH h = k->add_prog(x);
            h.alg = nadic_alg(x, k->n);
            h.exec = nadic_exec(x);
            k->prN_enc_pub = h;
        }
        // matrix-core Barrett form (tools/nadicb_model.py): the classical program (digits in [0, 3n) between
        // products, CANON at the end); ctx: the LDS image and n's limbs (nadicb_image.hpp)
        k->nadic_b = nadicb_ok(k);
        if (k->nadic_b) {
            std::vector<uint8_t> img;
            if (!nadicb::build(k->n, img)) return FTHE_ERR_UNSUPPORTED;
            k->mnB.m.init(k->n2, k->sn2);
            if (hipMalloc(&k->mnB.d_ctx, img.size()) != hipSuccess) return FTHE_ERR_NOMEM;
            HIPOK(hipMemcpy(k->mnB.d_ctx, img.data(), img.size(), hipMemcpyHostToDevice));
            k->mnB.kernel_S = kNadicBarS;
            if (k->c_n76 < 0) k->c_n76 = k->add_const(to_limbs(k->n, kNadicDigit.S, kNadicDigit.B));
            Prog x;
            x.loadx(SL_IN0); x.canon();
            x.pow(k->n, SL_TAB, SL_SQ, k->w_pub);
            x.mul(SL_C1); x.canon(); x.storex(SL_OUTP); x.end();
            fthe_key::PH h = k->add_prog(x);
            h.alg = nadic_alg(x, k->n);
            h.exec = nadic_exec(x) / 2;             // the VALU half: the products (the reductions run on MFMA)
            k->prB_enc_pub = h;
        }
        {
            // Montgomery form (tools/nadic_mont_model.py): the raw r is a Montgomery residue (value r R^-1),
            // pow(n) gives r^n R^(1-n), MUL (1, m) and MUL K (slot C2) give (1 + m n) r^n; digits < 2n
            // between products, CANON at the end
            if (k->nadic_mont) {
                if ((rc = upload_nadic(k->mnM, k->n, k->n2, k->sn2, false))) return rc;
                k->mnM.kernel_S = kNadicMontS;
                Mpz Kc, R, e1, q0, q1;
                mpz_set_ui(R, 1); mpz_mul_2exp(R, R, (mp_bitcnt_t)kNadicDigit.B * kNadicDigit.S);
                mpz_add_ui(e1, k->n, 1);
                mpz_powm(Kc, R, e1, k->n2);
                mpz_fdiv_qr(q1, q0, Kc, k->n);
                std::vector<uint32_t> kl = to_limbs(q0, kNadicDigit.S, kNadicDigit.B);
                std::vector<uint32_t> kh = to_limbs(q1, kNadicDigit.S, kNadicDigit.B);
                kl.insert(kl.end(), kh.begin(), kh.end());
                k->c_Kn = k->add_const(kl);
                Prog y;
                y.loadx(SL_IN0); y.canon();
                y.pow(k->n, SL_TAB, SL_SQ, k->w_pub);
                y.mul(SL_C1); y.mul(SL_C2); y.canon(); y.storex(SL_OUTP); y.end();
                fthe_key::PH hm = k->add_prog(y);
                hm.alg = nadic_alg(y, k->n);
                hm.exec = nadic_exec(y);
                k->prM_enc_pub = hm;
            }
        }
        // Paillier-1024 (n of 1009..1030 bits, n^2 on the s74 slots): the P-adic kernel with P = n -- the
        // base-n digit arithmetic needs no factorisation.  X = r -> digits (LOADP), X^n, X (1 + m n) with the
        // raw digits (1, m) of slot C1, STOREP (< 6 n^2; the output kernel reduces it)
        k->padic_pub = padic_digits(k->n, k->sn2) == kPadicK;
        if (k->padic_pub) {
            if ((rc = upload_padic(k->mnP, k->n, kPadicK))) return rc;
            Prog x;
            x.loadp(SL_IN0);
            x.pow(k->n, SL_TAB, SL_SQ, k->w_pub);
            x.mul(SL_C1); x.storep(SL_OUTP); x.end();
            fthe_key::PH h = k->add_prog(x);
            h.alg = padic_alg(x, k->n);
            h.exec = padic_exec(x, kPadicK);
            k->prP_enc_pub = h;
        }
        // add: a b R^-1 -> * R2 -> a b mod n^2 (paillier.cpp:103)
        Prog a;
        a.loadx(SL_IN0); a.mul(SL_IN1); a.mul(SL_C0); a.storex(SL_OUTP); a.end();
        k->pr_add = k->add_prog(a);
        // sub: a * b^(2^64-1) mod n^2 (GHPair::operator-, common.h:311-317): b R; (b R)^(2^64-1)
        // in the Montgomery domain by the all-ones chain; times a (plain) leaves the plain product
        Prog sb;
        sb.lds_a = lds_prefetch(k->sn2);
        sb.loadx(SL_IN1); sb.mul(SL_C0); sb.pow_ones(64, SL_T0, SL_T1); sb.mul(SL_IN0);
        sb.storex(SL_OUTP); sb.end();
        k->pr_sub = k->add_prog(sb);
        // row-I/O forms: canonical rows read / written by the kernel itself (no layout kernels)
        k->rowio = k->sn2.lanes == 4 && 2 * k->n_words == 128 && !getenv("FTHE_NO_ROWIO");
        if (k->rowio) {
            // fresh add: one classical product a b mod n^2 when the modulus allows it (n of 2048 bits),
            // else a b R^-1 then the R^2 correction (two Montgomery products); FTHE_ADD_MONT=1: the latter
            Prog aw;
            k->add_classical = k->mn2.m.classical_ok() && !getenv("FTHE_ADD_MONT");
            if (k->add_classical) { aw.loadw(0); aw.canon(); aw.mulwc(1); aw.storew(2); }
            else { aw.loadw(0); aw.mulw(1); aw.mul(SL_C0); aw.storew(2); }
            aw.end();
            k->pr_add_w = k->add_prog(aw);
            Prog sw;
            sw.loadw(1); sw.mul(SL_C0); sw.pow_ones(64, SL_T0, SL_T1); sw.mulw(0); sw.storew(2); sw.end();
            k->pr_sub_w = k->add_prog(sw);
            // pairwise adds with the Barrett reduction on the matrix cores (fthe_addb_q152) when n has 2048
            // bits; FTHE_ADD_NO_ADDB=1 keeps the classical product on the four-lane kernel (bit-identical)
            std::vector<uint8_t> img;
            if (k->add_classical && !getenv("FTHE_ADD_NO_ADDB") && addb::build(k->n, img)) {
                HIPOK(hipMalloc(&k->d_addb, img.size()));
                HIPOK(hipMemcpy(k->d_addb, img.data(), img.size(), hipMemcpyHostToDevice));
            }
        }
    }
    if (k->priv) {
        int rc;
        Mpz p2, q2; mpz_mul(p2, k->p, k->p); mpz_mul(q2, k->q, k->q);
        const Shape sh = k->spq;
        const int S = sh.S, RB = sh.B;
        if ((rc = upload_mod(k->mp2, p2, sh))) return rc;
        if ((rc = upload_mod(k->mq2, q2, sh))) return rc;
        if ((rc = upload_mod(k->mp, k->p, sh))) return rc;
        if ((rc = upload_mod(k->mq, k->q, sh))) return rc;
        auto L_ = [&](const mpz_t x) { return to_limbs(x, S, RB); };
        k->c_one = k->add_const(L_(one));
        k->c_zero = k->add_const(std::vector<uint32_t>(1, 0u));
        k->kp = (int)((k->p.bits() + RB - 1) / RB);
        k->kq = (int)((k->q.bits() + RB - 1) / RB);
        // --- CRT encrypt constants
        Mpz np, nq, ep, eq, t;
        mpz_mod(np, k->n, p2); mpz_mod(nq, k->n, q2);
        Mpz pm1, qm1; mpz_sub_ui(pm1, k->p, 1); mpz_sub_ui(qm1, k->q, 1);
        mpz_mul(t, k->p, pm1); mpz_mod(ep, k->n, t);     // n mod p(p-1): order of (Z/p^2)^*
        mpz_mul(t, k->q, qm1); mpz_mod(eq, k->n, t);
        k->c_R2p = k->add_const(L_(k->mp2.m.R2));
        k->c_nRp = k->add_const(k->mp2.m.mont(np));
        k->c_R2q = k->add_const(L_(k->mq2.m.R2));
        k->c_nRq = k->add_const(k->mq2.m.mont(nq));
        k->c_R3p = k->add_const(L_(k->mp2.m.R3));
        k->c_R3q = k->add_const(L_(k->mq2.m.R3));
        k->c_p2 = k->add_const(L_(p2));
        k->c_q2 = k->add_const(L_(q2));
        // u = cp + (K - cq) (k_crt_prep_q + the p program's CRT tail) with K = p^2 (floor(q^2/p^2) + 1)
        // > q^2 > cq: u >= 0 and u = cp - cq (mod p^2) whatever the ratio q / p (K = 2 p^2 failed
        // for q > sqrt(2) p).  u < K + 2 p^2 must stay a valid Montgomery operand: < R / 2.
        mpz_fdiv_q(t, q2, p2); mpz_add_ui(t, t, 1); mpz_mul(t, t, p2);
        {
            Mpz lim; mpz_add(lim, t, p2); mpz_add(lim, lim, p2); mpz_mul_2exp(lim, lim, 1);   // cp + v < K + 2p^2
            if (mpz_cmp(lim, k->mp2.m.R) >= 0) return FTHE_ERR_UNSUPPORTED;
        }
        k->c_2p2 = k->add_const(L_(t));
        Mpz qi; if (!mpz_invert(qi, q2, p2)) return FTHE_ERR_KEY;
        k->c_qinvRp2 = k->add_const(k->mp2.m.mont(qi));
        (void)ep; (void)eq;
        // Two-stage CRT encrypt.  r^n mod P^2 = (r^Q mod P)^P mod P^2 for n = P Q:
        // x = y (mod P) implies x^P = y^P (mod P^2), and r^Q mod P = r^(Q mod (P-1)) mod P.
        // Stage A (mod P, small-limb kernel): y = r^(Q mod (P-1)) mod P, 1024-bit exponent
        // over a 1024-bit modulus; stage B (mod P^2): y^P (1024-bit exponent) then
        // (1 + m n) y^P.  Same canonical residue as PowerMod(r, n, n^2) (paillier.cpp:136),
        // 0.62x the products of the direct r^(n mod P(P-1)) mod P^2.
        {
            size_t pb = std::max(k->p.bits(), k->q.bits());
            k->sp1 = kernel_shape_for_bits((int)pb);
            if (!k->sp1.S) return FTHE_ERR_UNSUPPORTED;
            if ((rc = upload_mod(k->mp1, k->p, k->sp1))) return rc;
            if ((rc = upload_mod(k->mq1, k->q, k->sp1))) return rc;
            const MontMod &A = k->mp1.m, &Bq = k->mq1.m;
            k->c1_R2p = k->add_const(A.limbs(A.R2));
            k->c1_R3p = k->add_const(A.limbs(A.R3));
            k->c1_R2q = k->add_const(Bq.limbs(Bq.R2));
            k->c1_R3q = k->add_const(Bq.limbs(Bq.R3));
            k->c1_one = k->add_const(A.limbs(one));
            Mpz ea, eb;
            mpz_mod(ea, k->q, pm1);             // Q mod (P-1) for P = p
            mpz_mod(eb, k->p, qm1);             // and for P = q
            int wA = best_window(std::max(ea.bits(), eb.bits()));
            int wB = best_window(std::max(k->p.bits(), k->q.bits()));
            k->tabn_max = std::max(k->tabn_max, std::max(1 << (wA - 1), 1 << (wB - 1)));
            for (int side = 0; side < 2; side++) {
                Prog a;                                          // slots in the small region
                a.lds_a = lds_prefetch(k->sp1);
                a.loadx(SL_IN1); a.mul(side ? SL_C3 : SL_C1);    // r_hi R^2
                a.storex(SL_T0);
                a.loadx(SL_IN0); a.mul(side ? SL_C2 : SL_C0);    // r_lo R
                a.addslot(SL_T0);                                // r R mod P
                a.pow(side ? eb : ea, SL_TAB, SL_SQ, wA);         // r^Q R
                a.mul(SL_T5);                                    // out of Montgomery (< 2P)
                a.storex(side ? SL_OUTQ : SL_OUTP); a.end();
                (side ? k->pr_encA_q : k->pr_encA_p) = k->add_prog(a);
                Prog e;                                          // slots in the P^2 region
                e.lds_a = lds_prefetch(sh);
                e.loadx(side ? SL_T4 : SL_T3); e.mul(side ? SL_C2 : SL_C0);   // y R mod P^2
                e.pow(side ? k->q : k->p, SL_TAB, SL_SQ, wB);     // y^P R = r^n R
                e.storex(SL_SAVED);
                e.loadx(SL_IN1); e.mul(side ? SL_C3 : SL_C1);    // m (n mod P^2)
                e.addsmall(1); e.mul(SL_SAVED);                  // (1 + m n) r^n mod P^2
                if (side) {
                    e.storex(SL_OUTQ);
                } else {
                    // the split form (q half on the side stream) stops at c_p and runs the tail after the join
                    Prog nt = e; nt.storex(SL_OUTP); nt.end();
                    k->pr_enc_p_nt = k->add_prog(nt);
                    Prog t; t.loadx(SL_OUTP); crt_tail(t); t.end();
                    k->pr_enc_tail = k->add_prog(t);
                    crt_tail(e);
                }
                e.end();
                (side ? k->pr_enc_q : k->pr_enc_p) = k->add_prog(e);
            }
            // P-adic stage B (P of 1009..1030 bits: Paillier-2048): y^P mod P^2 on the P-adic kernel
            // (1.4x the products/s of the Montgomery s74 program), then (1 + m n) y^P and the CRT tail
            // on s74 after one product into Montgomery form.  FTHE_NO_PADIC=1: the s74 programs above.
            const int Kd = padic_digits(k->p, sh);
            k->padic = Kd && padic_digits(k->q, sh) == Kd;
            k->padic_own_slots = k->padic && 2 * Kd != sh.S;      // Paillier-1024: 38-limb slots of its own
            if (k->padic) {
                if ((rc = upload_padic(k->mpA, k->p, Kd))) return rc;
                if ((rc = upload_padic(k->mqA, k->q, Kd))) return rc;
                for (int side = 0; side < 2; side++) {
                    const Mpz &P = side ? k->q : k->p;
                    Prog a;                                          // P-adic kernel
                    a.loadp(side ? SL_T4 : SL_T3);
                    a.pow(P, SL_TAB, SL_SQ, wB);                     // y^P mod P^2 (< 6 P^2)
                    a.storep(SL_SAVED); a.end();
                    fthe_key::PH ha = k->add_prog(a);
                    ha.alg = padic_alg(a, P);
                    ha.exec = padic_exec(a, Kd);
                    (side ? k->prP_enc_q : k->prP_enc_p) = ha;
                    Prog e;                                          // s74
                    e.loadx(SL_SAVED); e.mul(side ? SL_C2 : SL_C0);  // y^P R
                    e.storex(SL_SAVED);
                    e.loadx(SL_IN1); e.mul(side ? SL_C3 : SL_C1);
                    e.addsmall(1); e.mul(SL_SAVED);                  // (1 + m n) r^n mod P^2
                    if (side) {
                        e.storex(SL_OUTQ);
                    } else {
                        Prog nt = e; nt.storex(SL_OUTP); nt.end();
                        k->prP_encB_p_nt = k->add_prog(nt);
                        crt_tail(e);
                    }
                    e.end();
                    (side ? k->prP_encB_q : k->prP_encB_p) = k->add_prog(e);
                }
            }
        }
        // --- CRT decrypt constants
        k->c_p = k->add_const(L_(k->p));
        k->c_q = k->add_const(L_(k->q));
        // d = m_p + K - m_q (k_crt_dec_prep), K = p (floor(q / p) + 1) > q > m_q: see c_2p2
        mpz_fdiv_q(t, k->q, k->p); mpz_add_ui(t, t, 1); mpz_mul(t, t, k->p);
        {
            Mpz lim; mpz_add(lim, t, k->p); mpz_mul_2exp(lim, lim, 1);
            if (mpz_cmp(lim, k->mp.m.R) >= 0) return FTHE_ERR_UNSUPPORTED;
        }
        k->c_2p = k->add_const(L_(t));
        Mpz m2k, pinv, qinv;
        mpz_set_ui(m2k, 1); mpz_mul_2exp(m2k, m2k, (mp_bitcnt_t)RB * k->kp);
        mpz_invert(pinv, k->p, m2k);
        k->c_pinv = k->add_const(L_(pinv));
        mpz_set_ui(m2k, 1); mpz_mul_2exp(m2k, m2k, (mp_bitcnt_t)RB * k->kq);
        mpz_invert(qinv, k->q, m2k);
        k->c_qinv2 = k->add_const(L_(qinv));
        // h_P = L_P(g^(P-1) mod P^2)^-1 mod P
        for (int side = 0; side < 2; side++) {
            const Mpz &P = side ? k->q : k->p;
            const Mpz &P2 = side ? q2 : p2;
            Mpz Pm1, x, hp; mpz_sub_ui(Pm1, P, 1);
            mpz_powm(x, k->g, Pm1, P2);
            mpz_sub_ui(x, x, 1); mpz_tdiv_q(x, x, P);
            if (!mpz_invert(hp, x, P)) return FTHE_ERR_KEY;
            int h = k->add_const((side ? k->mq : k->mp).m.mont(hp));
            (side ? k->c_hRq : k->c_hRp) = h;
        }
        Mpz qip; if (!mpz_invert(qip, k->q, k->p)) return FTHE_ERR_KEY;
        k->c_qinvRp = k->add_const(k->mp.m.mont(qip));
        k->w_dec = best_window(std::max(pm1.bits(), qm1.bits()));
        k->tabn_max = std::max(k->tabn_max, 1 << (k->w_dec - 1));
        for (int side = 0; side < 2; side++) {
            Prog d;
            d.lds_a = lds_prefetch(sh);
            d.loadx(SL_IN1); d.mul(side ? SL_C3 : SL_C1);        // c_hi R^2  (= Montgomery of c_hi R)
            d.storex(SL_T0);
            d.loadx(SL_IN0); d.mul(side ? SL_C2 : SL_C0);        // c_lo R
            d.addslot(SL_T0);                                    // c R mod P^2 (< 4P^2)
            d.pow(side ? qm1 : pm1, SL_TAB, SL_SQ, k->w_dec);     // c^(P-1) R
            d.mul(SL_T5);                                        // * 1 -> out of Montgomery
            d.storex(side ? SL_OUTQ : SL_OUTP); d.end();
            (side ? k->pr_dec_q : k->pr_dec_p) = k->add_prog(d);
        }
        // the same with c^(P-1) on the P-adic kernel: c mod P^2 on s74 (< 2 P^2, plain), the
        // exponentiation, then back to a residue < 2 P^2 on s74 for the L-function tail
        for (int side = 0; side < 2 && k->padic; side++) {
            Prog d;
            d.loadx(SL_IN1); d.mul(side ? SL_C3 : SL_C1);
            d.storex(SL_T0);
            d.loadx(SL_IN0); d.mul(side ? SL_C2 : SL_C0);
            d.addslot(SL_T0);                                    // c R mod P^2 (< 4 P^2)
            d.mul(SL_T5);                                        // c mod P^2 (< 2 P^2)
            d.storex(SL_SAVED); d.end();
            (side ? k->prP_dec_pre_q : k->prP_dec_pre_p) = k->add_prog(d);
            const Mpz &Pm1 = side ? qm1 : pm1;
            Prog a;
            a.loadp(SL_SAVED); a.pow(Pm1, SL_TAB, SL_SQ, k->w_dec); a.storep(SL_SAVED); a.end();
            fthe_key::PH ha = k->add_prog(a);
            ha.alg = padic_alg(a, side ? k->q : k->p);
            ha.exec = padic_exec(a, k->mpA.kernel_S - 1000);
            (side ? k->prP_dec_q : k->prP_dec_p) = ha;
            Prog t;
            t.loadx(SL_SAVED); t.mul(side ? SL_C2 : SL_C0); t.mul(SL_T5);   // (X R) * 1 R^-1: X mod P^2 < 2 P^2
            t.storex(side ? SL_OUTQ : SL_OUTP); t.end();
            (side ? k->prP_dec_post_q : k->prP_dec_post_p) = k->add_prog(t);
        }
        // the same exponentiations on the four-lane s80 kernel, for batches that leave the chip idle
        if (S == 74 && !getenv("FTHE_NO_QUAD_DEC") && p2.bits() + 8 <= (size_t)kLatShape.S * kLatShape.B &&
            q2.bits() + 8 <= (size_t)kLatShape.S * kLatShape.B) {
            const Shape ls = kLatShape;
            if ((rc = upload_mod(k->mp2l, p2, ls))) return rc;
            if ((rc = upload_mod(k->mq2l, q2, ls))) return rc;
            auto Q_ = [&](const mpz_t x) { return to_limbs(x, ls.S, ls.B); };
            k->cl_R2p = k->add_const(Q_(k->mp2l.m.R2)); k->cl_R3p = k->add_const(Q_(k->mp2l.m.R3));
            k->cl_R2q = k->add_const(Q_(k->mq2l.m.R2)); k->cl_R3q = k->add_const(Q_(k->mq2l.m.R3));
            k->cl_one = k->add_const(Q_(one));
            k->cl_p2 = k->add_const(Q_(p2)); k->cl_q2 = k->add_const(Q_(q2));
            for (int side = 0; side < 2; side++) {
                Prog d;
                d.loadx(SL_IN1); d.mul(side ? SL_C3 : SL_C1);
                d.storex(SL_T0);
                d.loadx(SL_IN0); d.mul(side ? SL_C2 : SL_C0);
                d.addslot(SL_T0);
                d.pow(side ? qm1 : pm1, SL_TAB, SL_SQ, k->w_dec);
                d.mul(SL_T5);
                d.storex(side ? SL_OUTQ : SL_OUTP); d.end();
                (side ? k->pr_dec_ql : k->pr_dec_pl) = k->add_prog(d);
            }
            // direct-y encrypt stage B, (1 + m n) y^P mod P^2, stopping at c_P (the CRT tail runs on s74)
            k->cl_nRp = k->add_const(k->mp2l.m.mont(np)); k->cl_nRq = k->add_const(k->mq2l.m.mont(nq));
            const int wB = best_window(std::max(k->p.bits(), k->q.bits()));
            for (int side = 0; side < 2; side++) {
                Prog e;
                e.loadx(side ? SL_T4 : SL_T3); e.mul(side ? SL_C2 : SL_C0);
                e.pow(side ? k->q : k->p, SL_TAB, SL_SQ, wB);
                e.storex(SL_SAVED);
                e.loadx(SL_IN1); e.mul(side ? SL_C3 : SL_C1);
                e.addsmall(1); e.mul(SL_SAVED);
                e.storex(side ? SL_OUTQ : SL_OUTP); e.end();
                (side ? k->pr_enc_ql : k->pr_enc_pl) = k->add_prog(e);
            }
            k->slat = ls;
        }
        for (int side = 0; side < 2; side++) {
            Prog d; d.loadx(side ? SL_T2 : SL_T1); d.mul(side ? SL_C1 : SL_C0);
            d.storex(side ? SL_OUTQ : SL_OUTP); d.end();
            (side ? k->pr_dec_hq : k->pr_dec_hp) = k->add_prog(d);
        }
        {
            Prog d; d.loadx(SL_T3); d.mul(SL_C2); d.storex(SL_T4); d.end();
            k->pr_dec_t = k->add_prog(d);
        }
    }
    // upload constants and programs
    std::vector<uint32_t> flat;
    for (auto &v : k->host_consts) flat.insert(flat.end(), v.begin(), v.end());
    if (hipMalloc(&k->d_consts, flat.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(k->d_consts, flat.data(), flat.size() * 4, hipMemcpyHostToDevice));
    if (hipMalloc(&k->d_progs, k->host_progs.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(k->d_progs, k->host_progs.data(), k->host_progs.size() * 4, hipMemcpyHostToDevice));
    if (k->priv) {
        k->pq_w = (int)((std::max(k->p.bits(), k->q.bits()) + 31) / 32);
        std::vector<uint32_t> pq(2 * (size_t)k->pq_w);
        mpz_to_words(k->p, pq.data(), k->pq_w);
        mpz_to_words(k->q, pq.data() + k->pq_w, k->pq_w);
        if (hipMalloc(&k->d_pqwords, pq.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
        HIPOK(hipMemcpy(k->d_pqwords, pq.data(), pq.size() * 4, hipMemcpyHostToDevice));
    }
    std::vector<uint32_t> nw(k->n_words);
    mpz_to_words(k->n, nw.data(), k->n_words);
    if (hipMalloc(&k->d_nwords, nw.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(k->d_nwords, nw.data(), nw.size() * 4, hipMemcpyHostToDevice));
    return FTHE_OK;
}

static int key_from_pq(fthe_ctx *ctx, const mpz_t p, const mpz_t q, fthe_key **out) {
    if (mpz_cmp(p, q) == 0 || mpz_even_p(p) || mpz_even_p(q) || mpz_cmp_ui(p, 2) <= 0 || mpz_cmp_ui(q, 2) <= 0)
        return FTHE_ERR_KEY;
    std::unique_ptr<fthe_key> k(new fthe_key);
    k->device = ctx->device;
    k->priv = true;
    mpz_set(k->p, p); mpz_set(k->q, q);
    mpz_mul(k->n, p, q);                                   // paillier.cpp:82
    mpz_add_ui(k->g, k->n, 1);                             // :83
    Mpz pm1, qm1, phi, gcd;
    mpz_sub_ui(pm1, p, 1); mpz_sub_ui(qm1, q, 1);
    mpz_mul(phi, pm1, qm1); mpz_gcd(gcd, phi, k->n);
    if (mpz_cmp_ui(gcd, 1) != 0) return FTHE_ERR_KEY;      // paillier.cpp:60
    mpz_lcm(k->lambda, pm1, qm1);                          // :84
    mpz_mul(k->n2, k->n, k->n);
    Mpz lp; mpz_powm(lp, k->g, k->lambda, k->n2);          // :85
    mpz_sub_ui(lp, lp, 1); mpz_tdiv_q(lp, lp, k->n);
    if (!mpz_invert(k->mu, lp, k->n)) return FTHE_ERR_KEY; // :86
    k->n_bits = (int)k->n.bits();
    k->n_words = (k->n_bits + 31) / 32;
    if (hipSetDevice(ctx->device) != hipSuccess) return FTHE_ERR_HIP;
    int rc = key_finish(k.get());
    if (rc) return rc;
    *out = k.release();
    return FTHE_OK;
}

extern "C" int fthe_key_from_primes(fthe_ctx *ctx, const uint32_t *p, const uint32_t *q, int w, fthe_key **out) {
    if (!ctx || !p || !q || w <= 0 || !out) return FTHE_ERR_ARG;
    Mpz P, Q; mpz_from_words(P, p, w); mpz_from_words(Q, q, w);
    return key_from_pq(ctx, P, Q, out);
}

// A prime P of hb bits (top two bits set) with P - 1 = 2 s P' fully factored: P' a random
// prime of hb - 42 bits, s a product of random primes below 2^16; P found by trying s.
// Returns the distinct prime factors of P - 1 in `factors`.
static void known_order_prime(gmp_randstate_t st, int hb, Mpz &P, std::vector<Mpz> &factors) {
    static const std::vector<uint32_t> sp = [] {
        std::vector<uint32_t> v;
        for (uint32_t i = 3; i < 65536; i += 2) {
            bool pr = true;
            for (uint32_t d = 3; d * d <= i; d += 2) if (i % d == 0) { pr = false; break; }
            if (pr) v.push_back(i);
        }
        return v;
    }();
    Mpz Pp, lo, hi, s, t, r;
    for (;;) {
        mpz_urandomb(Pp, st, hb - 42); mpz_setbit(Pp, hb - 43); mpz_nextprime(Pp, Pp);
        // 2 s P' + 1 in [3 * 2^(hb-2), 2^hb): s in [lo, hi)
        mpz_set_ui(t, 3); mpz_mul_2exp(t, t, hb - 2); mpz_fdiv_q(lo, t, Pp); mpz_fdiv_q_2exp(lo, lo, 1);
        mpz_set_ui(t, 1); mpz_mul_2exp(t, t, hb); mpz_fdiv_q(hi, t, Pp); mpz_fdiv_q_2exp(hi, hi, 1);
        for (int tries = 0; tries < 20000; tries++) {
            std::vector<uint32_t> used;
            mpz_set_ui(s, 1);
            for (;;) {                                    // random small primes while s * 2^16 < lo
                mpz_mul_2exp(t, s, 16);
                if (mpz_cmp(t, lo) >= 0) break;
                mpz_urandomm(r, st, Mpz((unsigned long)sp.size()));
                used.push_back(sp[mpz_get_ui(r)]);
                mpz_mul_ui(s, s, used.back());
            }
            // the last factor: a random small prime in [ceil(lo / s), ceil(hi / s))
            mpz_cdiv_q(t, lo, s);
            const unsigned long a = mpz_get_ui(t);
            mpz_cdiv_q(t, hi, s);
            const unsigned long b = std::min(mpz_get_ui(t), 65536ul);
            auto ia = std::lower_bound(sp.begin(), sp.end(), (uint32_t)a), ib = std::lower_bound(sp.begin(), sp.end(), (uint32_t)b);
            if (ia >= ib) continue;
            mpz_urandomm(r, st, Mpz((unsigned long)(ib - ia)));
            used.push_back(*(ia + mpz_get_ui(r)));
            mpz_mul_ui(s, s, used.back());
            mpz_mul(P, s, Pp); mpz_mul_2exp(P, P, 1); mpz_add_ui(P, P, 1);
            if (mpz_probab_prime_p(P, 30) == 0) continue;
            factors.clear();
            factors.emplace_back(2ul);
            std::sort(used.begin(), used.end());
            used.erase(std::unique(used.begin(), used.end()), used.end());
            for (uint32_t l : used) factors.emplace_back((unsigned long)l);
            factors.push_back(Pp);
            return;
        }
    }
}

extern "C" int fthe_key_generate_ex(fthe_ctx *ctx, int n_bits, uint64_t seed, int flags, fthe_key **out) {
    if (!(flags & FTHE_KEYGEN_KNOWN_ORDER)) return fthe_key_generate(ctx, n_bits, seed, out);
    if (!ctx || !out || n_bits < 128 || (n_bits & 1)) return FTHE_ERR_ARG;
    gmp_randstate_t st; gmp_randinit_mt(st);
    seed_gmp_state(st, seed, 0x6b6e6f776e6f7264ull);
    const int hb = n_bits / 2;
    int rc = FTHE_ERR_KEY;
    for (int tries = 0; tries < 64 && rc == FTHE_ERR_KEY; tries++) {
        Mpz p, q;
        std::vector<Mpz> fp, fq;
        known_order_prime(st, hb, p, fp);
        known_order_prime(st, hb, q, fq);
        Mpz nn; mpz_mul(nn, p, q);
        if (mpz_cmp(p, q) == 0 || nn.bits() != (size_t)n_bits) continue;
        rc = key_from_pq(ctx, p, q, out);
        if (rc == FTHE_OK) {
            (*out)->order_known = true;
            (*out)->pm1_factors = fp;
            (*out)->qm1_factors = fq;
        }
    }
    gmp_randclear(st);
    return rc;
}

// Smallest prime > start, the result of mpz_nextprime(start), searched on up to 16 host
// threads: windows of 2^14 odd candidates sieved by the odd primes below 2^16, survivors
// tested (mpz_probab_prime_p: BPSW + 1 Miller-Rabin round) in index order from a shared
// counter; a thread stops once its index passes the smallest prime found, so every
// smaller survivor has been tested when the threads join.  Prime generation is a
// per-round cost in FedTree's vertical simulation (FLtrainer.cpp:556).
static void next_prime_par(mpz_t out, const mpz_t start) {
    static const std::vector<uint32_t> sieve_primes = [] {      // odd primes below 2^16
        std::vector<uint8_t> c(65536, 0);
        std::vector<uint32_t> v;
        for (uint32_t i = 3; i < 65536; i += 2) {
            if (c[i]) continue;
            v.push_back(i);
            for (uint32_t j = i * i; j < 65536; j += 2 * i) c[j] = 1;
        }
        return v;
    }();
    if (mpz_cmp_ui(start, 1u << 20) < 0) { mpz_nextprime(out, start); return; }
    const int W = 1 << 14;
    const unsigned nt = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    Mpz base;
    mpz_add_ui(base, start, 1);
    if (mpz_even_p(base)) mpz_add_ui(base, base, 1);           // odd candidates base + 2i
    std::vector<uint8_t> comp(W);
    std::vector<uint32_t> surv;
    for (;;) {
        std::fill(comp.begin(), comp.end(), 0);
        for (uint32_t l : sieve_primes) {
            const uint64_t r = mpz_fdiv_ui(base, l);           // base + 2i = 0 mod l  <=>  i = -r / 2 mod l
            uint64_t i0 = (uint64_t)((l - r) % l) * ((l + 1) / 2) % l;
            for (uint64_t i = i0; i < (uint64_t)W; i += l) comp[i] = 1;
        }
        surv.clear();
        for (int i = 0; i < W; i++)
            if (!comp[i]) surv.push_back((uint32_t)i);
        std::atomic<size_t> next{0}, best{SIZE_MAX};
        auto work = [&] {
            Mpz cand;
            for (;;) {
                const size_t idx = next.fetch_add(1);
                if (idx >= surv.size() || idx > best.load()) return;
                mpz_add_ui(cand, base, 2u * surv[idx]);
                if (mpz_probab_prime_p(cand, 25)) {
                    size_t b = best.load();
                    while (idx < b && !best.compare_exchange_weak(b, idx)) {}
                    return;
                }
            }
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
        work();
        for (auto &x : th) x.join();
        if (best.load() != SIZE_MAX) {
            mpz_add_ui(out, base, 2u * surv[best.load()]);
            return;
        }
        mpz_add_ui(base, base, 2u * W);
    }
}

extern "C" int fthe_next_prime(const uint32_t *start, int words, uint32_t *out, int out_words) {
    if (!start || !out || words <= 0 || out_words <= 0) return FTHE_ERR_ARG;
    Mpz s, r;
    mpz_from_words(s, start, words);
    next_prime_par(r, s);
    if (r.bits() > (size_t)out_words * 32) return FTHE_ERR_ARG;
    mpz_to_words(r, out, out_words);
    return FTHE_OK;
}

extern "C" int fthe_key_generate(fthe_ctx *ctx, int n_bits, uint64_t seed, fthe_key **out) {
    if (!ctx || !out || n_bits < 64 || (n_bits & 1)) return FTHE_ERR_ARG;
    gmp_randstate_t st; gmp_randinit_mt(st);
    seed_gmp_state(st, seed, 0);
    int hb = n_bits / 2;
    int rc = FTHE_ERR_KEY;
    for (int tries = 0; tries < 64 && rc == FTHE_ERR_KEY; tries++) {
        Mpz p, q;
        // top two bits set -> p*q has exactly n_bits bits (GenPrimePair, paillier.cpp:51-61)
        mpz_urandomb(p, st, hb); mpz_setbit(p, hb - 1); mpz_setbit(p, hb - 2); next_prime_par(p, p);
        mpz_urandomb(q, st, hb); mpz_setbit(q, hb - 1); mpz_setbit(q, hb - 2); next_prime_par(q, q);
        if (p.bits() != (size_t)hb || q.bits() != (size_t)hb) continue;
        rc = key_from_pq(ctx, p, q, out);
    }
    gmp_randclear(st);
    return rc;
}

extern "C" int fthe_key_from_n(fthe_ctx *ctx, const uint32_t *n, int n_words, fthe_key **out) {
    if (!ctx || !n || n_words <= 0 || !out) return FTHE_ERR_ARG;
    std::unique_ptr<fthe_key> k(new fthe_key);
    k->device = ctx->device;
    mpz_from_words(k->n, n, n_words);
    if (mpz_even_p(k->n) || mpz_cmp_ui(k->n, 3) < 0) return FTHE_ERR_KEY;
    mpz_add_ui(k->g, k->n, 1);
    mpz_mul(k->n2, k->n, k->n);
    k->n_bits = (int)k->n.bits();
    k->n_words = (k->n_bits + 31) / 32;
    if (hipSetDevice(ctx->device) != hipSuccess) return FTHE_ERR_HIP;
    int rc = key_finish(k.get());
    if (rc) return rc;
    *out = k.release();
    return FTHE_OK;
}

extern "C" void fthe_key_destroy(fthe_key *k) { delete k; }
extern "C" int fthe_key_n_words(const fthe_key *k) { return k ? k->n_words : 0; }
extern "C" int fthe_key_n_bits(const fthe_key *k) { return k ? k->n_bits : 0; }
extern "C" int fthe_key_has_private(const fthe_key *k) { return k ? (int)k->priv : 0; }

extern "C" int fthe_key_export(const fthe_key *k, uint32_t *n, uint32_t *lambda, uint32_t *mu, uint32_t *p, uint32_t *q) {
    if (!k) return FTHE_ERR_ARG;
    int w = k->n_words;
    if (n) mpz_to_words(k->n, n, w);
    if ((lambda || mu || p || q) && !k->priv) return FTHE_ERR_NOPRIV;
    if (lambda) mpz_to_words(k->lambda, lambda, w);
    if (mu) mpz_to_words(k->mu, mu, w);
    if (p) mpz_to_words(k->p, p, (w + 1) / 2);
    if (q) mpz_to_words(k->q, q, (w + 1) / 2);
    return FTHE_OK;
}

// ---------------------------------------------------------------------------
// Launch helpers
namespace {

// Launch the montprog kernel, bracketed by profiling events when enabled.
constexpr int kSpreadLds = 84 * 1024;   // > 80 KB: one workgroup per CU (gfx950: 160 KB LDS per CU)

int launch_montprog(fthe_ctx *c, void *slots, int S, int L, const void *prog, const DevMod &mod, double lane_mm,
                    size_t live, const void *const *rows = nullptr, int nrows = 0, hipStream_t st = nullptr,
                    bool spread = false, double lane_alg = -1, double lane_exec = -1, bool table_free = false) {
    if (!st) st = c->stream;
    struct {
        void *s; const void *p; const void *cx; uint32_t ls, ss; uint32_t live, pad; const void *rows[16];
    } args = {slots, prog, mod.d_ctx, (uint32_t)L * 4, (uint32_t)((size_t)S * L * 4), (uint32_t)live, 0, {}};
    static_assert(sizeof(args) == 168, "kernarg layout of gen_montprog.py");
    if (nrows > 16) return FTHE_ERR_ARG;
    for (int i = 0; i < nrows; i++) args.rows[i] = rows[i];
#ifdef FTHE_STAMP_HOOK
    // timing builds only (FTHE_GEN_M37_AB=stamp, tools/m37_stamps.py; compiled in for FTHE_BUILD_OUT libraries,
    // never the in-tree one): FTHE_STAMP_PTR = a device buffer of FTHE_STAMP_LAUNCHES x 128 KiB, one 128 KiB
    // record area per launch in turn
    static const char *stamp_ptr = getenv("FTHE_STAMP_PTR");
    static std::atomic<unsigned> stamp_launch{0};
    if (stamp_ptr && nrows < 16) {
        static const unsigned nl = getenv("FTHE_STAMP_LAUNCHES") ? (unsigned)atoi(getenv("FTHE_STAMP_LAUNCHES")) : 1;
        const unsigned i = stamp_launch.fetch_add(1);
        if (i < nl) args.rows[15] = (const char *)(uintptr_t)strtoull(stamp_ptr, nullptr, 0) + (size_t)i * 131072;
    }
#endif
    size_t sz = sizeof(args);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    // programs without fixed-base table ops (the key's own) may take the MFMA-Barrett P-adic kernel
    const bool mfma = table_free && mod.kernel_S_mfma;
    int vi = variant_index(mfma ? mod.kernel_S_mfma : mod.kernel_S ? mod.kernel_S : S);
    if (vi < 0) return FTHE_ERR_UNSUPPORTED;
    if (mfma) lane_exec = -1;             // the v_mad counts of padic_exec are fthe_padic_k37's
    // only the workgroups that hold live elements (slot strides stay those of L)
    if (live > (size_t)L) return FTHE_ERR_ARG;
    if (live == 0) return FTHE_OK;
    // fthe_padic_m37 built with dynamic jobs (FTHE_GEN_M37_AB=dyn, A/B under FTHE_M37_DYN=1): the resident
    // workgroups only, a zeroed job counter per launch (gen_padic_mfma.py DYN)
    static const bool m37_dyn = getenv("FTHE_M37_DYN") && *getenv("FTHE_M37_DYN") == '1';
    const bool dyn = mfma && m37_dyn && nrows < 15;
    const bool nb = kVariants[vi].S == kNadicBarS;       // kNbPerWg ciphertexts per workgroup of kNbWaves waves
    if (nb && L % kNbPerWg) return FTHE_ERR_ARG;          // the kernel covers whole workgroups of the slots
    unsigned blocks = nb ? (unsigned)((live + kNbPerWg - 1) / kNbPerWg)
                         : (unsigned)((live * kVariants[vi].lanes + 255) / 256);
    if (nb) {                     // persistent: at most one workgroup per CU, batches from its LDS counter
        blocks = std::min(blocks, (unsigned)c->n_cu);
        args.pad = blocks;
    }
    if (dyn) {
        if (!c->d_jobctr) HIPOK(hipMalloc(&c->d_jobctr, 256 * sizeof(uint32_t)));
        blocks = std::min(blocks, 2u * (unsigned)c->n_cu);          // 249 VGPRs: two waves per SIMD
        uint32_t *ctr = c->d_jobctr + (c->jobctr_i++ % 256);
        args.pad = 4 * blocks;
        args.rows[14] = ctr;
        if (hipMemsetAsync(ctr, 0, sizeof(uint32_t), st) != hipSuccess) return FTHE_ERR_HIP;
    }
    std::pair<hipEvent_t, hipEvent_t> *ev = nullptr;
    if (c->prof) {
        if (c->prof_used == c->prof_ev.size()) {
            std::pair<hipEvent_t, hipEvent_t> e;
            HIPOK(hipEventCreate(&e.first));
            HIPOK(hipEventCreate(&e.second));
            c->prof_ev.push_back(e);
        }
        if (c->prof_mm.size() < c->prof_ev.size()) c->prof_mm.resize(c->prof_ev.size());
        if (c->prof_vi.size() < c->prof_ev.size()) c->prof_vi.resize(c->prof_ev.size());
        c->prof_mm[c->prof_used] = lane_mm;
        c->prof_vi[c->prof_used] = vi;
        ev = &c->prof_ev[c->prof_used++];
        HIPOK(hipEventRecord(ev->first, st));
    }
    // Two concurrent small launches (the p and q halves on two streams) would otherwise pack two
    // workgroups onto one CU -- two waves per SIMD, each at half speed.  Dynamic LDS beyond half
    // the CU's 160 KB keeps one workgroup per CU while both launches fit on the chip together.
    unsigned shm = 0;
    if (!nb && spread && 2 * blocks <= (unsigned)c->n_cu && c->static_lds[vi] < kSpreadLds)
        shm = (unsigned)(kSpreadLds - c->static_lds[vi]);
    if (hipModuleLaunchKernel(c->fn[vi], blocks, 1, 1, nb ? 64 * kNbWaves : 256, 1, 1, shm, st, nullptr, cfg) !=
        hipSuccess)
        return FTHE_ERR_HIP;
    if (ev) {
        HIPOK(hipEventRecord(ev->second, st));
        c->prof_lane_mm += lane_mm * (double)live;
        c->prof_alg_macs += (lane_alg >= 0 ? lane_alg : lane_mm * mod.w_alg()) * (double)live;
        if (lane_exec >= 0) c->prof_exec_macs += lane_exec * (double)live;
        c->prof_launch_lanes += (double)live;
    }
    return FTHE_OK;
}

// AoS rows <-> slot limbs through the LDS-tiled kernels (fthe_glue.hip).
void pack_rows(hipStream_t st, const uint32_t *in, int win, size_t count, int bit0, uint32_t *slot, int S, int L,
               int B, const int64_t *idx = nullptr) {
    hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)((L + PACK_TILE - 1) / PACK_TILE)), dim3(256),
                       (size_t)PACK_TILE * (win + 1) * 4, st, in, win, idx, count, bit0, slot, S, L, B);
}
void unpack_rows(hipStream_t st, uint32_t *x, const uint32_t *N, int S, int L, size_t count, uint32_t *out,
                 int wout, int B) {
    hipLaunchKernelGGL(k_unpack_rows, dim3((unsigned)((L + PACK_TILE - 1) / PACK_TILE)), dim3(256),
                       (size_t)(PACK_TILE + 1) * S * 4, st, x, N, S, L, count, out, wout, B);
}

struct Launch {
    fthe_ctx *c; const fthe_key *k; int L; int S; int B; double mm = 0; size_t live = 0;
    void *base = nullptr;          // slot region (c->slots, or c->slots1 for small-modulus programs)
    hipStream_t st = nullptr;      // compute stream (null: the context's main stream)
    bool spread = false;           // one workgroup per CU (small concurrent launches)
    uint32_t *slot(int s) const { return (uint32_t *)base + (size_t)s * S * L; }
    dim3 grid() const { return dim3((unsigned)(L / 256)); }
    int prog(const fthe_key::PH &ph, const DevMod &mod, const void *const *rows = nullptr, int nrows = 0) {
        if (mod.m.S != S) return FTHE_ERR_ARG;
        int rc = launch_montprog(c, base, S, L, k->prog(ph), mod, ph.mm, live, rows, nrows, st, spread, ph.alg,
                                 ph.exec, true);
        if (rc) return rc;
        mm += ph.mm * (double)live;
        return FTHE_OK;
    }
    int prog_raw(const uint32_t *p, double pmm, const DevMod &mod, const void *const *rows, int nrows) {
        if (mod.m.S != S) return FTHE_ERR_ARG;
        int rc = launch_montprog(c, base, S, L, p, mod, pmm, live, rows, nrows, st, spread);
        if (rc) return rc;
        mm += pmm * (double)live;
        return FTHE_OK;
    }
    void fill(int s, int h) {
        hipLaunchKernelGGL(k_fill_const, grid(), dim3(256), 0, st ? st : c->stream, k->cst(h), slot(s), S, L);
    }
};

// CRT stage B of the encrypt (side 0: p, 1: q; nt: the p program without the CRT tail) and the
// decrypt's c^(P-1) mod P^2: P-adic exponentiation + s74 programs when the key has them.
// The P-adic launch itself: on L's slots, or (padic_own_slots, Paillier-1024) on the region of pa
// with the input slot copied in and SAVED copied back (k_copy_limbs between the slot shapes).
static int padic_launch(Launch &L, Launch *pa, const fthe_key *k, const fthe_key::PH &ph, const DevMod &mA, int in) {
    if (!k->padic_own_slots) return L.prog(ph, mA);
    Launch &A = *pa;
    A.live = L.live;
    hipStream_t st = L.st ? L.st : L.c->stream;
    hipLaunchKernelGGL(k_copy_limbs, L.grid(), dim3(256), 0, st, L.slot(in), L.S, A.slot(in), A.S, L.L);
    if (int rc = A.prog(ph, mA)) return rc;
    L.mm += A.mm; A.mm = 0;
    hipLaunchKernelGGL(k_copy_limbs, L.grid(), dim3(256), 0, st, A.slot(SL_SAVED), A.S, L.slot(SL_SAVED), L.S, L.L);
    return FTHE_OK;
}
static bool padic_here(const fthe_key *k, const Launch *pa) { return k->padic && (!k->padic_own_slots || pa); }
int enc_stage_b(Launch &L, const fthe_key *k, int side, bool nt = false, Launch *pa = nullptr) {
    const DevMod &m2 = side ? k->mq2 : k->mp2;
    if (!padic_here(k, pa)) return L.prog(side ? k->pr_enc_q : (nt ? k->pr_enc_p_nt : k->pr_enc_p), m2);
    if (int rc = padic_launch(L, pa, k, side ? k->prP_enc_q : k->prP_enc_p, side ? k->mqA : k->mpA,
                              side ? SL_T4 : SL_T3)) return rc;
    return L.prog(side ? k->prP_encB_q : (nt ? k->prP_encB_p_nt : k->prP_encB_p), m2);
}
int dec_pow(Launch &L, const fthe_key *k, int side, Launch *pa = nullptr) {
    const DevMod &m2 = side ? k->mq2 : k->mp2;
    if (!padic_here(k, pa)) return L.prog(side ? k->pr_dec_q : k->pr_dec_p, m2);
    if (int rc = L.prog(side ? k->prP_dec_pre_q : k->prP_dec_pre_p, m2)) return rc;
    if (int rc = padic_launch(L, pa, k, side ? k->prP_dec_q : k->prP_dec_p, side ? k->mqA : k->mpA, SL_SAVED))
        return rc;
    return L.prog(side ? k->prP_dec_post_q : k->prP_dec_post_p, m2);
}
// The P-adic region of a call on a key with padic_own_slots: c->slots1 after the stage-A region of
// the small-limb kernel (sp1 slots of the same key, whose constants must survive across chunks).
static size_t padic_region_offset(const fthe_key *k, int L) { return (size_t)nslots_for(k) * k->sp1.S * L * 4; }
// paq (split calls): a second region after it for the q half on the side stream.
static int padic_region(fthe_ctx *c, const fthe_key *k, const Launch &Lc, Launch &pa, Launch *paq = nullptr) {
    pa = Lc;
    if (paq) { *paq = Lc; paq->st = c->side; }
    if (!k->padic_own_slots) return FTHE_OK;
    pa.S = 2 * (k->mpA.kernel_S - 1000);
    const size_t off = padic_region_offset(k, Lc.L), reg = (size_t)nslots_for(k) * pa.S * Lc.L * 4;
    if (int rc = c->slots1.ensure(off + (paq ? 2 : 1) * reg)) return rc;
    pa.base = (uint8_t *)c->slots1.p + off;
    if (paq) { paq->S = pa.S; paq->base = (uint8_t *)pa.base + reg; }
    return FTHE_OK;
}

int begin_call(fthe_ctx *c, const fthe_key *k, size_t count, Launch &Lc, int nslots, Shape sh,
               size_t chunk = 0) {
    if (!c || !k) return FTHE_ERR_ARG;
    if (k->device != c->device) return FTHE_ERR_ARG;
    if (!sh.S) return FTHE_ERR_UNSUPPORTED;
    HIPOK(hipSetDevice(c->device));
    // L: a multiple of 256 ciphertexts (the 256-thread glue grids cover the slots exactly), and of 768 on a
    // shape that may run fthe_nadic_b76, whose workgroups hold 192 ciphertexts (the public-key encrypt mod n^2)
    const size_t q = (k->nadic_b && sh.S == k->sn2.S && sh.lanes == k->sn2.lanes) ? 768 : 256;
    size_t ch = (chunk ? chunk : chunk_lanes()) / (size_t)sh.lanes;    // same slot footprint per chunk
    ch = (ch + q - 1) / q * q;
    size_t L = std::min(ch, (count + q - 1) / q * q);
    if (L == 0) L = q;
    Lc.c = c; Lc.k = k; Lc.L = (int)L; Lc.S = sh.S; Lc.B = sh.B;
    const size_t need = (size_t)nslots * sh.S * L * 4;
    if (c->mem_limit && need > c->mem_limit && need > c->slots.n) return FTHE_ERR_NOMEM;
    int rc = c->slots.ensure(need);
    Lc.base = c->slots.p;
    if (rc) return rc;
    HIPOK(hipEventRecord(c->ev0, c->stream));
    return FTHE_OK;
}

int end_call(fthe_ctx *c, Launch &Lc) {
    HIPOK(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    c->last_mm = Lc.mm;
    if (hipGetLastError() != hipSuccess) return FTHE_ERR_HIP;
    return FTHE_OK;
}

// Host-resident calls: chunked, double-buffered transfers through pinned
// staging on the context's copy stream.  Chunk i+1's input is staged (ahead of
// chunk i's output on the copy stream) and chunk i's output drained while the
// kernels of the neighbouring chunk run,
// so a host-to-host call costs ~max(compute, PCIe + host memcpy) rather than
// their sum.  Caller buffers that are already page-locked are DMA'd directly.
// Large host copies (pageable caller buffer <-> pinned staging) on several cores.
void par_memcpy(void *dst, const void *src, size_t n) {
    const size_t grain = (size_t)16 << 20;
    int nt = (int)std::min<size_t>(8, n / grain);
    if (nt <= 1) { memcpy(dst, src, n); return; }
    std::vector<std::thread> th;
    size_t per = (n + nt - 1) / nt;
    for (int t = 1; t < nt; t++) {
        size_t b = t * per, e = std::min(n, b + per);
        if (b < e) th.emplace_back([=] { memcpy((char *)dst + b, (const char *)src + b, e - b); });
    }
    memcpy(dst, src, std::min(n, per));
    for (auto &x : th) x.join();
}

struct HostPipe {
    struct In { const uint8_t *h; uint8_t *d; size_t row; bool pinned; };
    struct Out { uint8_t *h; const uint8_t *d; size_t row; bool pinned; };
    fthe_ctx *c;
    In in[2]; int nin = 0;
    Out out[2]; int nout = 0;
    size_t L = 0, count = 0;
    bool pend = false; int pend_slot = 0; size_t pend_off = 0, pend_cnt = 0;
    // compute-bound calls (encrypt, decrypt): the next chunk's input goes on the copy stream ahead of this
    // chunk's output drain, so the next kernels never wait behind a D2H.  Copy-bound calls (add / sub:
    // 1.5 KB of PCIe per product) keep the drain first, so the DMA engine works while the host copies the
    // next chunk into pinned staging.
    bool input_first = true;
    static bool is_pinned(const void *p) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return false; }
        return a.type == hipMemoryTypeHost;
    }
    void add_in(const void *h, void *d, size_t row) {
        in[nin++] = In{(const uint8_t *)h, (uint8_t *)d, row, is_pinned(h)};
    }
    void add_out(void *h, const void *d, size_t row) {
        out[nout++] = Out{(uint8_t *)h, (const uint8_t *)d, row, is_pinned(h)};
    }
    size_t in_row() const { size_t r = 0; for (int i = 0; i < nin; i++) r += in[i].row; return r; }
    size_t out_row() const { size_t r = 0; for (int i = 0; i < nout; i++) r += out[i].row; return r; }
    int stage(size_t off) {                     // input rows [off, off + L) -> device, slot (off / L) & 1
        if (off >= count) return FTHE_OK;
        const size_t cnt = std::min(L, count - off);
        const int sl = (int)((off / L) & 1);
        HIPOK(hipEventSynchronize(c->ev_in[sl]));   // the slot's previous H2D has drained
        uint8_t *st = (uint8_t *)c->stage_in[sl].p;
        for (int i = 0; i < nin; i++) {
            const size_t b = cnt * in[i].row, o = off * in[i].row;
            if (in[i].pinned) {
                HIPOK(hipMemcpyAsync(in[i].d + o, in[i].h + o, b, hipMemcpyHostToDevice, c->copy));
            } else {
                par_memcpy(st, in[i].h + o, b);
                HIPOK(hipMemcpyAsync(in[i].d + o, st, b, hipMemcpyHostToDevice, c->copy));
                st += b;
            }
        }
        HIPOK(hipEventRecord(c->ev_in[sl], c->copy));
        return FTHE_OK;
    }
    int finish_pending() {
        if (!pend) return FTHE_OK;
        HIPOK(hipEventSynchronize(c->ev_copied[pend_slot]));
        const uint8_t *st = (const uint8_t *)c->stage_out[pend_slot].p;
        for (int i = 0; i < nout; i++) {
            if (out[i].pinned) continue;
            const size_t b = pend_cnt * out[i].row;
            par_memcpy(out[i].h + pend_off * out[i].row, st, b);
            st += b;
        }
        pend = false;
        return FTHE_OK;
    }
    // before the kernels of chunk [off, off+cnt)
    int before(size_t off, size_t Lc, size_t cnt_total) {
        int rc;
        if (off == 0) {
            L = Lc; count = cnt_total;
            for (int i = 0; i < 2; i++) {
                if ((rc = c->stage_in[i].ensure(std::max<size_t>(1, L * in_row())))) return rc;
                if ((rc = c->stage_out[i].ensure(std::max<size_t>(1, L * out_row())))) return rc;
                HIPOK(hipEventRecord(c->ev_in[i], c->copy));
                HIPOK(hipEventRecord(c->ev_copied[i], c->copy));
            }
            if ((rc = stage(0))) return rc;
        }
        if (nin) HIPOK(hipStreamWaitEvent(c->stream, c->ev_in[(off / L) & 1], 0));
        return FTHE_OK;
    }
    // after the kernels of chunk [off, off+cnt) are enqueued
    int after(size_t off, size_t cnt) {
        int rc;
        const int sl = (int)((off / L) & 1);
        // the next chunk's input first: on the copy stream it must not queue behind this chunk's output
        // drain, which waits for this chunk's kernels -- the next chunk's kernels wait for their input, so
        // the other order serialised every D2H with the compute (3.5 ms of idle GPU per 393,216-row chunk,
        // profiles/r03zl_e2e_timeline.txt)
        if (input_first && (rc = stage(off + L))) return rc;
        if (nout) {
            HIPOK(hipEventRecord(c->ev_done[sl], c->stream));
            HIPOK(hipStreamWaitEvent(c->copy, c->ev_done[sl], 0));
            uint8_t *st = (uint8_t *)c->stage_out[sl].p;
            for (int i = 0; i < nout; i++) {
                const size_t b = cnt * out[i].row, o = off * out[i].row;
                if (out[i].pinned) {
                    HIPOK(hipMemcpyAsync(out[i].h + o, out[i].d + o, b, hipMemcpyDeviceToHost, c->copy));
                } else {
                    HIPOK(hipMemcpyAsync(st, out[i].d + o, b, hipMemcpyDeviceToHost, c->copy));
                    st += b;
                }
            }
            HIPOK(hipEventRecord(c->ev_copied[sl], c->copy));
        }
        if (!input_first && (rc = stage(off + L))) return rc;
        if ((rc = finish_pending())) return rc;      // previous chunk's output -> caller
        if (nout) { pend = true; pend_slot = sl; pend_off = off; pend_cnt = cnt; }
        return FTHE_OK;
    }
    int finish() {
        int rc = finish_pending();
        if (rc) return rc;
        HIPOK(hipStreamSynchronize(c->copy));
        HIPOK(hipStreamSynchronize(c->stream));
        return FTHE_OK;
    }
};

}  // namespace

// Programs built per call (k-way product, scalar exponent, table widening) go
// through a per-context device buffer; the stream is drained before it is rewritten.
static int upload_dyn_prog(fthe_ctx *c, const Prog &p, fthe_key::PH &ph, DevBuf &buf) {
    HIPOK(hipStreamSynchronize(c->stream));
    int rc = buf.ensure(p.w.size() * 4);
    if (rc) return rc;
    HIPOK(hipMemcpy(buf.p, p.w.data(), p.w.size() * 4, hipMemcpyHostToDevice));
    ph.off = 0; ph.mm = p.montmuls;
    return FTHE_OK;
}
namespace {
// Launch with an explicit (dynamic) program pointer.
int launch_dyn(Launch &Lc, const void *prog, double mm, const DevMod &mod, const void *const *rows = nullptr,
               int nrows = 0) {
    if (mod.m.S != Lc.S) return FTHE_ERR_ARG;
    int rc = launch_montprog(Lc.c, Lc.base, Lc.S, Lc.L, prog, mod, mm, Lc.live, rows, nrows);
    if (rc) return rc;
    Lc.mm += mm * (double)Lc.live;
    return FTHE_OK;
}
}  // namespace

// ---------------------------------------------------------------------------
// Encrypt
// Plaintexts of an encrypt call: the u64 codec values of FedTree (m64), or general plaintexts
// m < n as little-endian words (mw, mww words each: Paillier::encrypt(const ZZ&), paillier.cpp:122).
struct MsgSrc {
    const uint64_t *m64 = nullptr;
    const uint32_t *mw = nullptr;
    int mww = 0;
    // index of m[0] in the caller's whole batch: device-drawn randomness (r == NULL) of plaintext i is the
    // stream element idx0 + i, so the shards of a seeded batch (fthe_encrypt_u64_at) draw what one call would
    uint64_t idx0 = 0;
    bool null() const { return !m64 && !mw; }
    // plaintexts [off, off + cnt) -> the IN1 slot (radix-2^B limbs); g^m = 1 + m n follows in the programs
    void pack(hipStream_t st, dim3 grid, size_t off, size_t cnt, uint32_t *slot, int S, int L, int B) const {
        if (m64) hipLaunchKernelGGL(k_pack_u64, grid, dim3(256), 0, st, m64 + off, cnt, slot, S, L, B);
        else pack_rows(st, mw + off * (size_t)mww, mww, cnt, 0, slot, S, L, B);
    }
};

static int encrypt_fb_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *alpha,
                           int a_words, uint64_t rng_seed, uint32_t *out, bool crt, HostPipe *pipe);
// nonce tweak of the y_q stream of the direct-y CRT encrypt (y_p uses the key's own nonce)
constexpr uint64_t kYqStream = 0x7172737475767778ull;
static int encrypt_xb_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *y,
                           int y_words, uint64_t rng_seed, uint32_t *out, HostPipe *pipe);
static int encrypt_pb_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *y, int y_words,
                           uint64_t rng_seed, uint32_t *out, HostPipe *pipe);
static int encrypt_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *r, int r_words,
                        uint64_t rng_seed, uint32_t *out, int flags, HostPipe *pipe) {
    if (!k || !c || (m.null() && count) || (!out && count)) return FTHE_ERR_ARG;
    if (m.mw && (m.mww <= 0 || m.mww > k->n_words)) return FTHE_ERR_ARG;
    if (r && !(flags & (FTHE_ENC_FIXED_BASE | FTHE_ENC_FIXED_BASE_EXACT)) && (r_words <= 0 || r_words > k->n_words))
        return FTHE_ERR_ARG;
    bool crt = k->priv && !(flags & FTHE_ENC_PUBLIC);
    if (flags & FTHE_ENC_FIXED_BASE_EXACT) {
        if (crt) return encrypt_xb_impl(k, c, m, count, r, r_words, rng_seed, out, pipe);
        bool pb_ready;
        { std::lock_guard<std::mutex> g(k->fb_mu); pb_ready = k->pb.ready; }
        if (!pb_ready) return k->priv ? FTHE_ERR_UNSUPPORTED : FTHE_ERR_NOPRIV;
        return encrypt_pb_impl(k, c, m, count, r, r_words, rng_seed, out, pipe);
    }
    if (!crt && !k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (flags & FTHE_ENC_FIXED_BASE) return encrypt_fb_impl(k, c, m, count, r, r_words, rng_seed, out, crt, pipe);
    static const bool no_direct = getenv("FTHE_NO_DIRECT_Y") != nullptr;
    const bool direct_y = crt && !r && !no_direct;
    // small batches: the q half on the side stream in a second slot region, as decrypt_impl
    const int vi = variant_index(k->spq.S);
    // and smaller ones both halves on the four-lane s80 kernel (as decrypt_impl)
    // (one chunk by construction: FTHE_CHUNK below the quad limit sends the batch down the other paths)
    const bool quad = direct_y && k->slat.S && count > 0 && count <= dec_quad_max() && count <= chunk_lanes();
    const bool small_split = !quad && direct_y && vi >= 0 && count * (size_t)kVariants[vi].lanes <= dec_split_lanes();
    bool big_split = !quad && !small_split && direct_y && vi >= 0 && split_all();
    // big split calls of more than one chunk: chunks pipelined over two slot-region pairs (enc_pipe)
    bool piped = big_split && !pipe && !k->padic_own_slots && enc_pipe() && count > enc_chunk_lanes();
    const int nsl = nslots_for(k);
    Launch Lc;
    auto begin = [&] {
        return begin_call(c, k, count, Lc, piped ? 4 * nsl : (small_split || big_split) ? 2 * nsl : nsl,
                          crt ? k->spq : k->sn2,
                          direct_y && !small_split && !quad ? enc_chunk_lanes() : !crt && k->nadic_b ? pub_chunk_lanes() : 0);
    };
    int rc = begin();
    // the extra regions of the pipelined / two-stream forms are a speed option (+1%): when the device (or the
    // context's limit, fthe_ctx_set_mem_limit) cannot hold them, the call takes the one-region form, bit-identical
    while (rc == FTHE_ERR_NOMEM && (piped || big_split)) {
        if (piped) piped = false; else big_split = false;
        rc = begin();
    }
    const bool split = small_split || big_split;
    if (rc) return rc;
    const int S = Lc.S, L = Lc.L, nw = k->n_words, cw = 2 * nw;
    // Device-drawn randomness under CRT draws y_p, y_q uniform in [1,p), [1,q) and
    // skips stage A: r^n mod P^2 = (r^Q mod P)^P and r -> r^Q mod P is a bijection of
    // Z_P^* (gcd(n, phi(n)) = 1, checked at key set-up as paillier.cpp:60), so
    // y^P mod P^2 for uniform y has exactly the distribution of r^n mod P^2 for the
    // reference's uniform r, independently for P = p, q (CRT).  FTHE_NO_DIRECT_Y=1
    // keeps the explicit r (A/B).  Injected r always takes both stages (bit-exact).
    // scratch: AoS r words for the device RNG
    const int wl = (kLatShape.S * kLatShape.B + 31) / 32;   // u32 words of an s80 row
    if (!r && (rc = c->scratch.ensure(std::max((size_t)L * nw * 4 * (direct_y ? 2 : 1) * (piped ? 2 : 1),
                                               quad ? (size_t)L * (2 * k->pq_w + 2 * wl) * 4 : (size_t)0))))
        return rc;
    RngKey rk{};
    if (!r) rk = make_rng_key(rng_seed, 0);
    Launch L1 = Lc;                    // stage A: mod p, q on the small-limb kernel, own slot region
    Launch Lq = Lc;                    // split: q half, region 2 of the slots, side stream
    if (split) {
        Lq.base = (uint8_t *)Lc.base + (size_t)nsl * S * L * 4;
        Lq.st = c->side;
        Lc.spread = Lq.spread = true;
        HIPOK(hipEventRecord(c->ev_fork, c->stream));
        HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
        Lq.fill(SL_C2, k->c_R2q); Lq.fill(SL_C3, k->c_nRq);
    }
    Launch Lp4 = Lc, Lq4 = Lc;         // quad: s80 regions for the p and q halves (slots1)
    if (quad) {
        if (count > (size_t)L) return FTHE_ERR_ARG;        // one chunk by construction
        const size_t reg = (size_t)nsl * kLatShape.S * L * 4;
        if ((rc = c->slots1.ensure(2 * reg))) return rc;
        Lp4.S = kLatShape.S; Lp4.B = kLatShape.B; Lp4.base = c->slots1.p; Lp4.spread = true;
        Lq4 = Lp4; Lq4.base = (uint8_t *)c->slots1.p + reg; Lq4.st = c->side;
        Lp4.fill(SL_C0, k->cl_R2p); Lp4.fill(SL_C1, k->cl_nRp);
        Lq4.fill(SL_C2, k->cl_R2q); Lq4.fill(SL_C3, k->cl_nRq);
    }
    Launch Lpa, Lpaq;                  // the P-adic kernel's own slots (Paillier-1024; else Lc's)
    if (crt && (rc = padic_region(c, k, Lc, Lpa, split ? &Lpaq : nullptr))) return rc;
    if (direct_y) {
        Lc.fill(SL_C0, k->c_R2p); Lc.fill(SL_C1, k->c_nRp);
        Lc.fill(SL_C2, k->c_R2q); Lc.fill(SL_C3, k->c_nRq);
        Lc.fill(SL_T1, k->c_qinvRp2);
    } else if (crt) {
        L1.S = k->sp1.S; L1.B = k->sp1.B;
        if ((rc = c->slots1.ensure(std::max((size_t)nslots_for(k) * L1.S * L * 4,
                                            k->padic_own_slots ? padic_region_offset(k, L) +
                                                (size_t)nslots_for(k) * Lpa.S * L * 4 : (size_t)0))))
            return rc;
        L1.base = c->slots1.p;                 // stage A; the P-adic region (if any) follows it
        if (k->padic_own_slots) Lpa.base = (uint8_t *)c->slots1.p + padic_region_offset(k, L);
        L1.fill(SL_C0, k->c1_R2p); L1.fill(SL_C1, k->c1_R3p);
        L1.fill(SL_C2, k->c1_R2q); L1.fill(SL_C3, k->c1_R3q);
        L1.fill(SL_T5, k->c1_one);
        Lc.fill(SL_C0, k->c_R2p); Lc.fill(SL_C1, k->c_nRp);
        Lc.fill(SL_C2, k->c_R2q); Lc.fill(SL_C3, k->c_nRq);
        Lc.fill(SL_T1, k->c_qinvRp2);
    } else {
        Lc.fill(SL_C0, k->c_R2n2); Lc.fill(SL_C1, k->c_nRn2);
    }
    if (piped) {
        // region pair b = chunk & 1: the p half (main stream) on Rp[b], the q half and the recombination (side
        // stream) on Rq[b].  Chunk i's p half waits only for the recombination of chunk i - 2 (the last user of
        // its region pair and of its y buffers), so it runs beside the q half of chunk i - 1.
        Launch Rp[2] = {Lc, Lc}, Rq[2] = {Lq, Lq};
        Rp[1].base = (uint8_t *)Lc.base + (size_t)2 * nsl * S * L * 4;
        Rq[1].base = (uint8_t *)Lc.base + (size_t)3 * nsl * S * L * 4;
        Rp[1].fill(SL_C0, k->c_R2p); Rp[1].fill(SL_C1, k->c_nRp);
        Rp[1].fill(SL_C2, k->c_R2q); Rp[1].fill(SL_C3, k->c_nRq);
        Rp[1].fill(SL_T1, k->c_qinvRp2);
        Rq[1].fill(SL_C2, k->c_R2q); Rq[1].fill(SL_C3, k->c_nRq);
        double mm_tail = 0;
        size_t i = 0;
        for (size_t off = 0; off < count; off += L, i++) {
            const int b = (int)(i & 1);
            const size_t cnt = std::min((size_t)L, count - off);
            Launch &P = Rp[b], &Q = Rq[b];
            P.live = Q.live = cnt;
            uint32_t *yp = (uint32_t *)c->scratch.p + (size_t)b * 2 * L * k->pq_w, *yq = yp + (size_t)L * k->pq_w;
            RngKey rq = rk; rq.nonce ^= kYqStream;
            if (i >= 2) HIPOK(hipStreamWaitEvent(c->stream, c->ev_cb[b], 0));
            hipLaunchKernelGGL(k_rng_r, Lc.grid(), dim3(256), 0, c->stream, k->d_pqwords, k->pq_w, (int)k->p.bits(),
                               rk, m.idx0 + off, cnt, yp);
            m.pack(c->stream, Lc.grid(), off, cnt, P.slot(SL_IN1), S, L, Lc.B);
            pack_rows(c->stream, yp, k->pq_w, cnt, 0, P.slot(SL_T3), S, L, Lc.B);
            if ((rc = enc_stage_b(P, k, 0, true, &Lpa))) return rc;
            HIPOK(hipEventRecord(c->ev_fork, c->stream));
            hipLaunchKernelGGL(k_rng_r, Lc.grid(), dim3(256), 0, c->side, k->d_pqwords + k->pq_w, k->pq_w,
                               (int)k->q.bits(), rq, m.idx0 + off, cnt, yq);
            m.pack(c->side, Lc.grid(), off, cnt, Q.slot(SL_IN1), S, L, Lc.B);
            pack_rows(c->side, yq, k->pq_w, cnt, 0, Q.slot(SL_T4), S, L, Lc.B);
            if ((rc = enc_stage_b(Q, k, 1, false, &Lpaq))) return rc;
            HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
            Launch T = P;                  // the recombination: P's slots, on the side stream
            T.st = c->side; T.mm = 0;
            hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->side, Q.slot(SL_OUTQ), k->cst(k->c_q2),
                               k->cst(k->c_2p2), P.slot(SL_T0), S, L, Lc.B);
            if ((rc = T.prog(k->pr_enc_tail, k->mp2))) return rc;
            mm_tail += T.mm;
            hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->side, P.slot(SL_T2), k->cst(k->c_p2), S, L, Lc.B);
            mul_add_out(c->side, Lc.grid(), Q.slot(SL_OUTQ), S, k->cst(k->c_q2), S, P.slot(SL_T2), S, L, cnt,
                        out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
            HIPOK(hipEventRecord(c->ev_cb[b], c->side));
        }
        HIPOK(hipEventRecord(c->ev_join, c->side));
        HIPOK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
        Lc.mm = Rp[0].mm + Rp[1].mm + Rq[0].mm + Rq[1].mm + mm_tail;
        return end_call(c, Lc);
    }
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt; L1.live = cnt; Lq.live = cnt;
        if (pipe && (rc = pipe->before(off, L, count))) return rc;
        const uint32_t *rw = r + (r ? off * r_words : 0);
        int rwn = r_words;
        if (direct_y) {
            uint32_t *yp = (uint32_t *)c->scratch.p, *yq = yp + (size_t)L * k->pq_w;
            RngKey rq = rk; rq.nonce ^= kYqStream;                    // an independent stream for y_q
            hipLaunchKernelGGL(k_rng_r, Lc.grid(), dim3(256), 0, c->stream, k->d_pqwords, k->pq_w, (int)k->p.bits(),
                               rk, m.idx0 + off, cnt, yp);
            hipLaunchKernelGGL(k_rng_r, Lc.grid(), dim3(256), 0, c->stream, k->d_pqwords + k->pq_w, k->pq_w,
                               (int)k->q.bits(), rq, m.idx0 + off, cnt, yq);
            m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_IN1), S, L, Lc.B);
            pack_rows(c->stream, yp, k->pq_w, cnt, 0, Lc.slot(SL_T3), S, L, Lc.B);
            pack_rows(c->stream, yq, k->pq_w, cnt, 0, Lc.slot(SL_T4), S, L, Lc.B);
            if (quad) {
                const int S4 = kLatShape.S, B4 = kLatShape.B;
                uint32_t *rowp = yq + (size_t)L * k->pq_w, *rowq = rowp + (size_t)L * wl;
                Lp4.live = cnt; Lq4.live = cnt;
                m.pack(c->stream, Lc.grid(), off, cnt, Lp4.slot(SL_IN1), S4, L, B4);
                m.pack(c->stream, Lc.grid(), off, cnt, Lq4.slot(SL_IN1), S4, L, B4);
                pack_rows(c->stream, yp, k->pq_w, cnt, 0, Lp4.slot(SL_T3), S4, L, B4);
                pack_rows(c->stream, yq, k->pq_w, cnt, 0, Lq4.slot(SL_T4), S4, L, B4);
                HIPOK(hipEventRecord(c->ev_fork, c->stream));
                HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
                if ((rc = Lq4.prog(k->pr_enc_ql, k->mq2l))) return rc;
                HIPOK(hipEventRecord(c->ev_join, c->side));
                if ((rc = Lp4.prog(k->pr_enc_pl, k->mp2l))) return rc;
                // canonical c_p, c_q rows -> the s74 slots of the CRT tail
                unpack_rows(c->stream, Lp4.slot(SL_OUTP), k->cst(k->cl_p2), S4, L, cnt, rowp, wl, B4);
                pack_rows(c->stream, rowp, wl, cnt, 0, Lc.slot(SL_OUTP), S, L, Lc.B);
                HIPOK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
                unpack_rows(c->stream, Lq4.slot(SL_OUTQ), k->cst(k->cl_q2), S4, L, cnt, rowq, wl, B4);
                pack_rows(c->stream, rowq, wl, cnt, 0, Lc.slot(SL_OUTQ), S, L, Lc.B);
                Lc.mm += Lp4.mm + Lq4.mm; Lp4.mm = Lq4.mm = 0;
                hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTQ),
                                   k->cst(k->c_q2), k->cst(k->c_2p2), Lc.slot(SL_T0), S, L, Lc.B);
                if ((rc = Lc.prog(k->pr_enc_tail, k->mp2))) return rc;
                hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T2), k->cst(k->c_p2), S,
                                   L, Lc.B);
                mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTQ), S, k->cst(k->c_q2), S, Lc.slot(SL_T2), S, L, cnt,
                            out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
                if (pipe && (rc = pipe->after(off, cnt))) return rc;
                continue;
            }
            if (split) {
                m.pack(c->stream, Lc.grid(), off, cnt, Lq.slot(SL_IN1), S, L, Lc.B);
                pack_rows(c->stream, yq, k->pq_w, cnt, 0, Lq.slot(SL_T4), S, L, Lc.B);
                HIPOK(hipEventRecord(c->ev_fork, c->stream));
                HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
                if ((rc = enc_stage_b(Lq, k, 1, false, &Lpaq))) return rc;
                HIPOK(hipEventRecord(c->ev_join, c->side));
                if ((rc = enc_stage_b(Lc, k, 0, true, &Lpa))) return rc;
                HIPOK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
                hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->stream, Lq.slot(SL_OUTQ),
                                   k->cst(k->c_q2), k->cst(k->c_2p2), Lc.slot(SL_T0), S, L, Lc.B);
                if ((rc = Lc.prog(k->pr_enc_tail, k->mp2))) return rc;
                hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T2), k->cst(k->c_p2), S,
                                   L, Lc.B);
                mul_add_out(c->stream, Lc.grid(), Lq.slot(SL_OUTQ), S, k->cst(k->c_q2), S, Lc.slot(SL_T2), S, L, cnt,
                            out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
                if (pipe && (rc = pipe->after(off, cnt))) return rc;
                continue;
            }
            if ((rc = enc_stage_b(Lc, k, 1, false, &Lpa))) return rc;
            hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTQ), k->cst(k->c_q2),
                               k->cst(k->c_2p2), Lc.slot(SL_T0), S, L, Lc.B);
            if ((rc = enc_stage_b(Lc, k, 0, false, &Lpa))) return rc;                 // ends with h = (cp - cq) q^-2 in T2
            hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T2), k->cst(k->c_p2), S, L, Lc.B);
            mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTQ), S,
                        k->cst(k->c_q2), S, Lc.slot(SL_T2), S, L, cnt, out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
            if (pipe && (rc = pipe->after(off, cnt))) return rc;
            continue;
        }
        if (!r) {
            hipLaunchKernelGGL(k_rng_r, Lc.grid(), dim3(256), 0, c->stream, k->d_nwords, nw, k->n_bits, rk,
                               m.idx0 + off, cnt, (uint32_t *)c->scratch.p);
            rw = (const uint32_t *)c->scratch.p; rwn = nw;
        }
        m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_IN1), S, L, Lc.B);
        if (crt) {
            // r (< n) -> low / high halves in the small layout
            pack_rows(c->stream, rw, rwn, cnt, 0,
                               L1.slot(SL_IN0), L1.S, L, L1.B);
            pack_rows(c->stream, rw, rwn, cnt, L1.B * L1.S,
                               L1.slot(SL_IN1), L1.S, L, L1.B);
            if ((rc = L1.prog(k->pr_encA_p, k->mp1))) return rc;
            if ((rc = L1.prog(k->pr_encA_q, k->mq1))) return rc;
            if (L1.B != Lc.B) return FTHE_ERR_UNSUPPORTED;
            hipLaunchKernelGGL(k_copy_limbs, Lc.grid(), dim3(256), 0, c->stream, L1.slot(SL_OUTP), L1.S,
                               Lc.slot(SL_T3), S, L);
            hipLaunchKernelGGL(k_copy_limbs, Lc.grid(), dim3(256), 0, c->stream, L1.slot(SL_OUTQ), L1.S,
                               Lc.slot(SL_T4), S, L);
            if ((rc = enc_stage_b(Lc, k, 1, false, &Lpa))) return rc;
            hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTQ), k->cst(k->c_q2),
                               k->cst(k->c_2p2), Lc.slot(SL_T0), S, L, Lc.B);
            if ((rc = enc_stage_b(Lc, k, 0, false, &Lpa))) return rc;                 // ends with h = (cp - cq) q^-2 in T2
            hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T2), k->cst(k->c_p2), S, L, Lc.B);
            // c = cq + q^2 h   (< p^2 q^2 = n^2)
            mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTQ), S,
                        k->cst(k->c_q2), S, Lc.slot(SL_T2), S, L, cnt, out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
        } else if (k->nadic || k->nadic_mont || k->nadic_b) {
            // n-adic kernel: digits (r, 0) in IN0, (1, m) in C1; out = x0 + x1 n (x0, x1 < n: c < n^2)
            const int D = kNadicDigit.S;
            pack_rows(c->stream, rw, rwn, cnt, 0, Lc.slot(SL_IN0), S, L, Lc.B);
            Lc.fill(SL_C1, k->c_one_n2);
            m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_C1) + (size_t)D * L, D, L, Lc.B);
            if (k->nadic_b) {
                if ((rc = Lc.prog(k->prB_enc_pub, k->mnB))) return rc;
            } else if (k->nadic_mont) {
                Lc.fill(SL_C2, k->c_Kn);
                if ((rc = Lc.prog(k->prM_enc_pub, k->mnM))) return rc;
            } else if ((rc = Lc.prog(k->prN_enc_pub, k->mnA))) return rc;
            mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTP), D, k->cst(k->c_n76), D,
                        Lc.slot(SL_OUTP) + (size_t)D * L, D, L, cnt, out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
        } else if (k->padic_pub) {
            // P-adic kernel, P = n: plain r in IN0, raw digits (1, m) in C1; out = STOREP's < 6 n^2 mod n^2
            const int D = kPadicK;
            pack_rows(c->stream, rw, rwn, cnt, 0, Lc.slot(SL_IN0), S, L, Lc.B);
            Lc.fill(SL_C1, k->c_one_n2);
            m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_C1) + (size_t)D * L, D, L, Lc.B);
            if ((rc = Lc.prog(k->prP_enc_pub, k->mnP))) return rc;
            unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L, cnt, out + off * cw, cw, Lc.B);
        } else {
            pack_rows(c->stream, rw, rwn, cnt, 0,
                               Lc.slot(SL_IN0), S, L, Lc.B);
            if ((rc = Lc.prog(k->pr_enc_pub, k->mn2))) return rc;
            unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2),
                               S, L, cnt, out + off * cw, cw, Lc.B);
        }
        Lc.mm += L1.mm; L1.mm = 0;
        if (pipe && (rc = pipe->after(off, cnt))) return rc;
    }
    Lc.mm += Lq.mm;
    return end_call(c, Lc);
}

// Test hook (include/fthe.h): the exponent bases (y_p, y_q) the direct-y CRT encrypt draws for
// ciphertexts [index0, index0 + count) of a call with r == NULL and this rng_seed -- the same
// kernel, keys and per-index counters as encrypt_impl, so a test can rebuild each ciphertext's
// r = CRT(y_p^(q^-1 mod p-1) mod p, y_q^(p^-1 mod q-1) mod q) and check it against
// PowerMod(g, m, n^2) PowerMod(r, n, n^2) (paillier.cpp:134-137).
extern "C" int fthe_debug_direct_y(fthe_key *k, fthe_ctx *c, uint64_t rng_seed, uint64_t index0, size_t count,
                                   uint32_t *yp, uint32_t *yq) {
    if (!k || !c || !rng_seed || (count && (!yp || !yq))) return FTHE_ERR_ARG;
    if (k->device != c->device) return FTHE_ERR_ARG;
    if (!k->priv) return FTHE_ERR_NOPRIV;
    if (!count) return FTHE_OK;
    HIPOK(hipSetDevice(c->device));
    const RngKey rk = make_rng_key(rng_seed, 0);
    RngKey rq = rk; rq.nonce ^= kYqStream;
    const size_t words = count * (size_t)k->pq_w;
    DevBuf d;
    int rc = d.ensure(2 * words * 4);
    if (rc) return rc;
    uint32_t *dp = (uint32_t *)d.p, *dq = dp + words;
    const dim3 grid((unsigned)((count + 255) / 256));
    hipLaunchKernelGGL(k_rng_r, grid, dim3(256), 0, c->stream, k->d_pqwords, k->pq_w, (int)k->p.bits(), rk, index0,
                       count, dp);
    hipLaunchKernelGGL(k_rng_r, grid, dim3(256), 0, c->stream, k->d_pqwords + k->pq_w, k->pq_w, (int)k->q.bits(), rq,
                       index0, count, dq);
    HIPOK(hipGetLastError());
    HIPOK(hipMemcpyAsync(yp, dp, words * 4, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipMemcpyAsync(yq, dq, words * 4, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    return FTHE_OK;
}

// ---------------------------------------------------------------------------
// Fixed-base randomizer (FTHE_ENC_FIXED_BASE).
//
// The reference draws r uniform in Z_n^* and pays PowerMod(r, n, n^2) per
// ciphertext (paillier.cpp:127-136).  Here one random h per key gives
// hs = h^n mod n^2, and a ciphertext is (1 + m n) hs^alpha mod n^2 = g^m (h^alpha)^n:
// a Paillier encryption of m with r = h^alpha (the Damgard-Jurik-Nielsen
// fixed-base randomizer).  alpha is uniform over 8*nwin bits, 64 bits more than
// the order of hs (which divides lambda; p-1 for the CRT halves), so r^n is
// statistically uniform over <hs> (CRT: over <hs mod p^2> x <hs mod q^2>, with
// independent exponents).  With 8-bit windows and tables entry[j][d] = hs^(d 256^j)
// the exponentiation is nwin gathered products and no squarings.
namespace {

// entries[j][d] = store(base^(d 256^j) mod N), nwin windows, ew words each
std::vector<uint32_t> fb_table(const mpz_t base, const mpz_t N, int nwin, int ew,
                               const std::function<void(const mpz_t, uint32_t *)> &store) {
    std::vector<uint32_t> tab((size_t)nwin * 256 * ew, 0);
    std::vector<Mpz> b(nwin);
    mpz_mod(b[0], base, N);
    for (int j = 1; j < nwin; j++) mpz_powm_ui(b[j], b[j - 1], 256, N);
    int nt = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            Mpz acc, tmp;
            for (int j = t; j < nwin; j += nt) {
                mpz_set_ui(acc, 1);
                for (int d = 0; d < 256; d++) {
                    store(acc, &tab[((size_t)j * 256 + d) * ew]);
                    mpz_mul(tmp, acc, b[j]);
                    mpz_mod(acc, tmp, N);
                }
            }
        });
    for (auto &x : th) x.join();
    return tab;
}

int fb_upload(const std::vector<uint32_t> &v, uint32_t **d) {
    if (hipMalloc((void **)d, v.size() * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    HIPOK(hipMemcpy(*d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    return FTHE_OK;
}

// one-lane kernels: radix-2^B limbs of x R mod N, padded to ew words
std::function<void(const mpz_t, uint32_t *)> fb_store_limbs(const MontMod &M) {
    return [&M](const mpz_t x, uint32_t *dst) {
        std::vector<uint32_t> l = M.mont(x);
        std::copy(l.begin(), l.end(), dst);
    };
}

// Widen 8-bit-window tables to 16-bit windows on the device: entry (j, d) of the
// wide table = MontMul(entry (2j, d & 255), entry (2j+1, d >> 8)) of the narrow one
// (Montgomery forms multiply to the Montgomery form of the product), one launch of
// 65,536 lanes per wide window.  One-lane kernels: the product leaves in a slot and
// k_slot_to_entries transposes it into entries; the four-lane kernel writes the
// canonical rows itself (STOREW).
int fb_widen(fthe_key *k, fthe_ctx *c, const DevMod &mod, Shape sh, const uint32_t *tab8, int nwin16, int ew,
             bool rows_form, uint32_t **out) {
    const int Kd = mod.kernel_S > 1000 && mod.kernel_S < 2000 ? mod.kernel_S - 1000 : 0;   // P-adic: digit-form entries
    const size_t W16 = 65536;
    int rc;
    if (hipMalloc((void **)out, (size_t)nwin16 * W16 * ew * 4) != hipSuccess) return FTHE_ERR_NOMEM;
    Launch Lc;
    if ((rc = begin_call(c, k, W16, Lc, nslots_for(k), sh))) return rc;
    if ((size_t)Lc.L < W16) return FTHE_ERR_UNSUPPORTED;
    Lc.live = W16;
    // digits: row 0 = g & 255, row 1 = g >> 8 (u8, row stride L)
    if ((rc = c->hb[0].ensure(2 * (size_t)Lc.L))) return rc;
    std::vector<uint8_t> dg(2 * (size_t)Lc.L, 0);
    for (size_t g = 0; g < W16; g++) { dg[g] = (uint8_t)(g & 255); dg[Lc.L + g] = (uint8_t)(g >> 8); }
    HIPOK(hipMemcpy(c->hb[0].p, dg.data(), dg.size(), hipMemcpyHostToDevice));
    Prog pr;
    if (rows_form) { pr.loadgd(0); pr.mulgd(1); pr.storew(2); }
    else if (mod.kernel_S == kNadicS) { pr.loadgd(0); pr.mulgd(1); pr.canon(); pr.storex(SL_OUTP); }   // digits
    else { pr.loadgd(0); pr.mulgd(1); pr.storex(SL_OUTP); }
    pr.end();
    fthe_key::PH ph;
    if ((rc = upload_dyn_prog(c, pr, ph, c->io[3]))) return rc;
    const size_t eb = (size_t)ew * 4;
    for (int j = 0; j < nwin16; j++) {
        uint32_t *dst = *out + (size_t)j * W16 * ew;
        const void *rows[3] = {(const uint8_t *)tab8 + (size_t)(2 * j) * 256 * eb, c->hb[0].p, dst};
        if ((rc = launch_dyn(Lc, c->io[3].p, pr.montmuls, mod, rows, rows_form ? 3 : 2))) return rc;
        if (!rows_form)
        {
            if (Kd)
                hipLaunchKernelGGL(k_slot_to_digit_entries, dim3((unsigned)(W16 / 256)), dim3(256), 0, c->stream,
                                   Lc.slot(SL_OUTP), Kd, ew / 2, 2, Lc.L, W16, dst);
            else if (mod.kernel_S == kNadicS)          // n-adic: lane quarters of 19 limbs + a pad word
                hipLaunchKernelGGL(k_slot_to_digit_entries, dim3((unsigned)(W16 / 256)), dim3(256), 0, c->stream,
                                   Lc.slot(SL_OUTP), kNadicDigit.S / 4, ew / 8, 8, Lc.L, W16, dst);
            else
                hipLaunchKernelGGL(k_slot_to_entries, dim3((unsigned)(W16 / 256)), dim3(256), 0, c->stream,
                                   Lc.slot(SL_OUTP), Lc.S, Lc.L, W16, ew, dst);
        }
    }
    HIPOK(hipStreamSynchronize(c->stream));
    return end_call(c, Lc);
}

// Public-form (mod n^2) fixed-base tables for bases hs[0 .. nb), nwin16[b] 16-bit windows for base b,
// base after base: one-lane n^2 kernels store radix-2^B limb entries, the four-lane kernel
// canonical 2 n_words-word rows (k->sn2.lanes == 4).  wide = false keeps 8-bit windows.
int pub_tables(fthe_key *k, fthe_ctx *c, const Mpz *hs, int nb, const int *nwin16, bool wide, uint32_t **d_tab,
               int *ew, bool nadic = false) {
    const MontMod &M = k->mn2.m;
    const bool rows = k->sn2.lanes == 4 && !nadic;
    const int cw = 2 * k->n_words;
    const int D = kNadicDigit.S;
    const int Qd = D / 4, QP = Qd + 1;                   // gen_nadic.py: lane quarters of 19 limbs + a pad word
    *ew = nadic ? 8 * QP : rows ? cw : 4 * ((M.S + 3) / 4);
    std::vector<uint32_t> tab;
    for (int b = 0; b < nb; b++) {
        std::vector<uint32_t> tb;
        if (nadic)                                        // plain x as base-n digits (x mod n, x div n)
            tb = fb_table(hs[b], k->n2, 2 * nwin16[b], *ew, [k, D, Qd, QP](const mpz_t x, uint32_t *dst) {
                Mpz q, r; mpz_tdiv_qr(q, r, x, k->n);
                for (int h = 0; h < 2; h++) {
                    std::vector<uint32_t> l = to_limbs(h ? q : r, D, kNadicDigit.B);
                    for (int kq = 0; kq < 4; kq++)
                        std::copy(l.begin() + kq * Qd, l.begin() + (kq + 1) * Qd, dst + (h * 4 + kq) * QP);
                }
            });
        else if (rows)
            tb = fb_table(hs[b], k->n2, 2 * nwin16[b], cw, [&M, cw](const mpz_t x, uint32_t *dst) {
                Mpz t; mpz_mul(t, x, M.R); mpz_mod(t, t, M.N);
                mpz_to_words(t, dst, cw);
            });
        else
            tb = fb_table(hs[b], k->n2, 2 * nwin16[b], *ew, fb_store_limbs(M));
        if (nb == 1) tab.swap(tb);
        else tab.insert(tab.end(), tb.begin(), tb.end());
    }
    int rc;
    uint32_t *d8 = nullptr;
    if ((rc = fb_upload(tab, &d8))) return rc;
    if (!wide) { *d_tab = d8; return FTHE_OK; }
    int total = 0;
    for (int b = 0; b < nb; b++) total += nwin16[b];
    rc = fb_widen(k, c, nadic ? k->mnA : k->mn2, k->sn2, d8, total, *ew, rows, d_tab);
    (void)hipFree(d8);
    return rc;
}

// FTHE_FB_WINDOW=8 keeps the host-built 8-bit tables; the default widens them to 16 bits
// on the device (2x fewer products per encryption, 65536 entries per window).
int fb_window() {
    const char *e = getenv("FTHE_FB_WINDOW");
    return e && atoi(e) == 8 ? 8 : 16;
}

int fb_build(fthe_key *k, fthe_ctx *c, const mpz_t h) {
    fthe_key::FixedBase &F = k->fb;
    if (mpz_sgn(h) <= 0 || mpz_cmp(h, k->n) >= 0) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipStreamSynchronize(c->stream));
    for (uint32_t **p : {&F.d_tab_pub, &F.d_tab_p, &F.d_tab_q, &F.d_prog})
        if (*p) { (void)hipFree(*p); *p = nullptr; }
    F.ready = false;
    F.window = fb_window();
    const bool wide = F.window == 16;
    mpz_set(F.h, h);
    mpz_powm(F.hs, h, k->n, k->n2);
    std::vector<uint32_t> progs;
    auto add = [&](const Prog &p, size_t &off, double &mm) {
        off = progs.size(); mm = p.montmuls;
        progs.insert(progs.end(), p.w.begin(), p.w.end());
    };
    // the exponent program: X = entry(0); X <- X entry(j), j = 1 .. nwin-1
    auto expo = [&](Prog &e, int nwin) {
        if (wide) { e.loadgd16(0); for (int j = 1; j < nwin; j++) e.mulgd16(j); }
        else { e.loadgd(0); for (int j = 1; j < nwin; j++) e.mulgd(j); }
    };
    int rc;
    // public-key form: one-lane n^2 kernels, or the four-lane kernel's 128-word rows
    F.pub = k->pub_ok && (k->sn2.lanes == 1 || k->rowio);
    if (F.pub) {
        const int nwin16 = (k->n_bits + 64 + 15) / 16;          // alpha: n_bits + 64 bits
        F.nwin_pub = wide ? nwin16 : 2 * nwin16;
        F.pub_rows = k->sn2.lanes == 4;
        if ((rc = pub_tables(k, c, &F.hs, 1, &nwin16, wide, &F.d_tab_pub, &F.ew_pub))) return rc;
        Prog e;
        expo(e, F.nwin_pub);
        e.storex(SL_SAVED);
        e.loadx(SL_IN1); e.mul(SL_C1); e.addsmall(1); e.mul(SL_SAVED);   // (1 + m n) hs^alpha
        if (F.pub_rows) e.storew(2); else e.storex(SL_OUTP);
        e.end();
        add(e, F.off_pub, F.mm_pub);
    }
    if (k->priv) {
        const int nwin16 = (int)((std::max(k->p.bits(), k->q.bits()) + 64 + 15) / 16);
        F.nwin_crt = wide ? nwin16 : 2 * nwin16;
        F.ew_crt = 4 * ((k->spq.S + 3) / 4);
        for (int side = 0; side < 2; side++) {
            const DevMod &D = side ? k->mq2 : k->mp2;
            uint32_t **dt = side ? &F.d_tab_q : &F.d_tab_p;
            Mpz hsP; mpz_mod(hsP, F.hs, D.m.N);
            std::vector<uint32_t> tab = fb_table(hsP, D.m.N, 2 * nwin16, F.ew_crt, fb_store_limbs(D.m));
            if ((rc = fb_upload(tab, dt))) return rc;
            if (wide) {
                uint32_t *t16 = nullptr;
                rc = fb_widen(k, c, D, k->spq, *dt, nwin16, F.ew_crt, false, &t16);
                (void)hipFree(*dt);
                *dt = t16;
                if (rc) return rc;
            }
            Prog e;
            expo(e, F.nwin_crt);
            e.storex(SL_SAVED);
            e.loadx(SL_IN1); e.mul(side ? SL_C3 : SL_C1); e.addsmall(1); e.mul(SL_SAVED);
            if (side) e.storex(SL_OUTQ); else crt_tail(e);
            e.end();
            double mm;
            add(e, side ? F.off_q : F.off_p, mm);
            F.mm_crt = mm;
        }
    }
    if (progs.empty()) return FTHE_ERR_UNSUPPORTED;
    if ((rc = fb_upload(progs, &F.d_prog))) return rc;
    F.ready = true;
    return FTHE_OK;
}

int fb_ensure(fthe_key *k, fthe_ctx *c) {
    std::lock_guard<std::mutex> g(k->fb_mu);
    if (k->fb.ready) return FTHE_OK;
    HIPOK(hipSetDevice(c->device));
    // h uniform in [1, n) from /dev/urandom
    gmp_randstate_t st;
    gmp_randinit_default(st);
    seed_gmp_state(st, 0, 0);
    Mpz h, nm1; mpz_sub_ui(nm1, k->n, 1);
    mpz_urandomm(h, st, nm1); mpz_add_ui(h, h, 1);
    gmp_randclear(st);
    return fb_build(k, c, h);
}

}  // namespace

extern "C" int fthe_key_fixed_base(fthe_key *k, fthe_ctx *c, const uint32_t *h, int h_words) {
    if (!k || !c || k->device != c->device) return FTHE_ERR_ARG;
    if (!h) {
        { std::lock_guard<std::mutex> g(k->fb_mu); k->fb.ready = false; }
        return fb_ensure(k, c);
    }
    if (h_words <= 0 || h_words > k->n_words) return FTHE_ERR_ARG;
    std::lock_guard<std::mutex> g(k->fb_mu);
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipDeviceSynchronize());            // no call may still read the old tables
    Mpz hh; mpz_from_words(hh, h, h_words);
    return fb_build(k, c, hh);
}

extern "C" int fthe_key_fixed_base_info(fthe_key *k, int *alpha_bits_public, int *alpha_bits_crt, uint32_t *hs) {
    if (!k) return FTHE_ERR_ARG;
    std::lock_guard<std::mutex> g(k->fb_mu);
    if (!k->fb.ready) return FTHE_ERR_ARG;
    if (alpha_bits_public) *alpha_bits_public = k->fb.pub ? k->fb.window * k->fb.nwin_pub : 0;
    if (alpha_bits_crt) *alpha_bits_crt = k->priv ? k->fb.window * k->fb.nwin_crt : 0;
    if (hs) mpz_to_words(k->fb.hs, hs, 2 * k->n_words);
    return FTHE_OK;
}

static int encrypt_fb_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *alpha,
                           int a_words, uint64_t rng_seed, uint32_t *out, bool crt, HostPipe *pipe) {
    int rc = fb_ensure(k, c);
    if (rc) return rc;
    const fthe_key::FixedBase &F = k->fb;
    if (!crt && !F.pub) return FTHE_ERR_UNSUPPORTED;
    const int nwin = crt ? F.nwin_crt : F.nwin_pub, bpd = F.window / 8;   // bytes per digit
    if (alpha && (a_words <= 0 || a_words > (F.window * nwin + 31) / 32)) return FTHE_ERR_ARG;
    Launch Lc;
    if ((rc = begin_call(c, k, count, Lc, nslots_for(k), crt ? k->spq : k->sn2))) return rc;
    const int S = Lc.S, L = Lc.L, cw = 2 * k->n_words;
    const size_t dig_bytes = (size_t)nwin * L * bpd;           // [window][L] digits, per side
    if ((rc = c->scratch.ensure(2 * dig_bytes))) return rc;
    uint8_t *dig_p = (uint8_t *)c->scratch.p, *dig_q = dig_p + dig_bytes;
    RngKey rk{};
    if (!alpha) rk = make_rng_key(rng_seed, 0x6669786564626173ull);
    if (crt) {
        Lc.fill(SL_C1, k->c_nRp); Lc.fill(SL_C3, k->c_nRq);
        Lc.fill(SL_T1, k->c_qinvRp2);
    } else {
        Lc.fill(SL_C1, k->c_nRn2);
    }
    const uint32_t *prog = F.d_prog;
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt;
        if (pipe && (rc = pipe->before(off, L, count))) return rc;
        const int sides = crt && !alpha ? 2 : 1;
        if (alpha) {
            hipLaunchKernelGGL(k_alpha_digits, Lc.grid(), dim3(256), 0, c->stream, alpha + off * a_words, a_words,
                               a_words, cnt, nwin, L, bpd, dig_p);
        } else {
            for (int sd = 0; sd < sides; sd++)
                hipLaunchKernelGGL(k_rng_digits, Lc.grid(), dim3(256), 0, c->stream, rk, m.idx0 + off, cnt, nwin, L,
                                   bpd, sd, sd ? dig_q : dig_p);
        }
        m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_IN1), S, L, Lc.B);
        if (crt) {
            const void *rp[2] = {F.d_tab_p, dig_p};
            const void *rq[2] = {F.d_tab_q, sides == 2 ? dig_q : dig_p};
            if ((rc = Lc.prog_raw(prog + F.off_q, F.mm_crt, k->mq2, rq, 2))) return rc;
            hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTQ), k->cst(k->c_q2),
                               k->cst(k->c_2p2), Lc.slot(SL_T0), S, L, Lc.B);
            if ((rc = Lc.prog_raw(prog + F.off_p, F.mm_crt, k->mp2, rp, 2))) return rc;
            hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T2), k->cst(k->c_p2), S, L, Lc.B);
            mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTQ), S,
                        k->cst(k->c_q2), S, Lc.slot(SL_T2), S, L, cnt, out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
        } else if (F.pub_rows) {
            const void *rows[3] = {F.d_tab_pub, dig_p, out + off * cw};
            if ((rc = Lc.prog_raw(prog + F.off_pub, F.mm_pub, k->mn2, rows, 3))) return rc;
        } else {
            const void *rows[2] = {F.d_tab_pub, dig_p};
            if ((rc = Lc.prog_raw(prog + F.off_pub, F.mm_pub, k->mn2, rows, 2))) return rc;
            unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L, cnt, out + off * cw, cw, Lc.B);
        }
        if (pipe && (rc = pipe->after(off, cnt))) return rc;
    }
    return end_call(c, Lc);
}

// ---------------------------------------------------------------------------
// Exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT; key holder, CRT).
//
// The reference's r is uniform in Z_n^* (paillier.cpp:127-133), so r^n mod P^2
// (P = p, q) is uniform over G_P = {x^P mod P^2}, the cyclic subgroup of order
// P - 1 of Z_{P^2}^* (r -> (r^Q mod P)^P), independently for p and q.
// With bases gam_i = t_i^P mod P^2 such that <t_1, t_2, t_3> = Z_P^*, the map
// (y_1, y_2, y_3) -> prod gam_i^y_i is a homomorphism from Z_{P-1}^3 ONTO G_P, so
// uniform exponents (y_i uniform in [1, P), i.e. uniform mod P - 1) give an exactly
// uniform element of G_P: the reference's distribution, with precomputed tables
// (16-bit windows, 3 * ceil(bits(P)/16) gathered products, no squarings).
// <t_1, t_2, t_3> = Z_P^* iff no prime l | P - 1 has all three t_i l-th powers;
// every l < 2^24 is checked (bases redrawn until it holds).  A larger l escapes
// the check with probability l^-3 per l, at most 43 * 2^-72 < 2^-66 per key.
namespace {

const std::vector<uint32_t> &small_primes() {           // primes below 2^24
    static const std::vector<uint32_t> v = [] {
        const uint32_t L = 1u << 24;
        std::vector<uint8_t> comp(L, 0);
        std::vector<uint32_t> ps;
        for (uint32_t i = 2; i < L; i++) {
            if (comp[i]) continue;
            ps.push_back(i);
            for (uint64_t j = (uint64_t)i * i; j < L; j += i) comp[j] = 1;
        }
        return ps;
    }();
    return v;
}

// three t_i in [2, P - 1) generating Z_P^* at every prime l < 2^24 dividing P - 1
void xb_pick_bases(gmp_randstate_t st, const mpz_t P, Mpz t[3]) {
    Mpz Pm1, e, x, span;
    mpz_sub_ui(Pm1, P, 1);
    mpz_sub_ui(span, P, 3);
    std::vector<uint32_t> f;
    for (uint32_t l : small_primes())
        if (mpz_fdiv_ui(Pm1, l) == 0) f.push_back(l);
    for (;;) {
        for (int i = 0; i < 3; i++) { mpz_urandomm(t[i], st, span); mpz_add_ui(t[i], t[i], 2); }
        bool ok = true;
        for (uint32_t l : f) {
            mpz_divexact_ui(e, Pm1, l);
            bool all = true;
            for (int i = 0; i < 3 && all; i++) { mpz_powm(x, t[i], e, P); all = mpz_cmp_ui(x, 1) == 0; }
            if (all) { ok = false; break; }
        }
        if (ok) return;
    }
}

// P - 1 fully factored (factors = its distinct primes): a primitive root t mod P, so gam = t^P
// generates G_P by itself and one base with a uniform exponent is exactly uniform over G_P
void xb_pick_generator(gmp_randstate_t st, const mpz_t P, const std::vector<Mpz> &factors, Mpz &t) {
    Mpz Pm1, e, x, span;
    mpz_sub_ui(Pm1, P, 1);
    mpz_sub_ui(span, P, 3);
    for (;;) {
        mpz_urandomm(t, st, span); mpz_add_ui(t, t, 2);
        bool gen = true;
        for (const Mpz &l : factors) {
            mpz_divexact(e, Pm1, l);
            mpz_powm(x, t, e, P);
            if (mpz_cmp_ui(x, 1) == 0) { gen = false; break; }
        }
        if (gen) return;
    }
}

// gam_in (nb_in bases per prime, [side][base][2 pq_w words]): the generators of another key of the same primes
// (fthe_key_fixed_base_exact_info) instead of fresh ones -- a replica on another device draws the same r^n
int xb_build(fthe_key *k, fthe_ctx *c, uint64_t seed, const uint32_t *gam_in = nullptr, int nb_in = 0) {
    fthe_key::ExactBase &X = k->xb;
    if (!k->priv) return FTHE_ERR_NOPRIV;
    if (gam_in && nb_in != (k->order_known ? 1 : 3)) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipStreamSynchronize(c->stream));
    for (uint32_t **p : {&X.d_tab[0], &X.d_tab[1], &X.d_prog})
        if (*p) { (void)hipFree(*p); *p = nullptr; }
    X.ready = false;
    gmp_randstate_t st;
    gmp_randinit_default(st);
    if (seed) {
        Mpz sd;
        mpz_set_ui(sd, seed);
        mpz_mul_2exp(sd, sd, 64);
        mpz_add_ui(sd, sd, 0x5845584143544241ull);
        gmp_randseed(st, sd);
    } else {
        seed_gmp_state(st, 0, 0);       // 256 bits of /dev/urandom
    }
    X.nwin = (int)((std::max(k->p.bits(), k->q.bits()) + 15) / 16);
    // P-2048: the gathered products on the P-adic kernel, entries in its digit form (2 KB words)
    X.padic = k->padic && !k->padic_own_slots;
    const int Kd = X.padic ? k->mpA.kernel_S - 1000 : 0, KB = Kd + (Kd & 1);
    X.ew = X.padic ? 2 * KB : 4 * ((k->spq.S + 3) / 4);
    X.nb = k->order_known ? 1 : 3;
    std::vector<uint32_t> progs;
    int rc = FTHE_OK;
    for (int side = 0; side < 2 && rc == FTHE_OK; side++) {
        const Mpz &P = side ? k->q : k->p;
        const DevMod &D = side ? k->mq2 : k->mp2;
        const DevMod &A = side ? k->mqA : k->mpA;
        // digit form of x < P^2: x mod P at words 0.., x div P at KB..
        auto store_digits = [&P, Kd, KB](const mpz_t x, uint32_t *dst) {
            Mpz q, r; mpz_fdiv_qr(q, r, x, P);
            std::vector<uint32_t> a = to_limbs(r, Kd, 28), b = to_limbs(q, Kd, 28);
            std::copy(a.begin(), a.end(), dst);
            std::copy(b.begin(), b.end(), dst + KB);
        };
        Mpz t[3];
        if (!gam_in) {
            if (k->order_known) xb_pick_generator(st, P, side ? k->qm1_factors : k->pm1_factors, t[0]);
            else xb_pick_bases(st, P, t);
        }
        std::vector<uint32_t> tab;                        // 8-bit windows, base after base
        for (int b = 0; b < X.nb && rc == FTHE_OK; b++) {
            if (gam_in) {
                const size_t gw = 2 * (size_t)k->pq_w;
                mpz_from_words(X.gam[side][b], gam_in + ((size_t)side * X.nb + b) * gw, (int)gw);
                if (mpz_sgn(X.gam[side][b]) <= 0 || mpz_cmp(X.gam[side][b], D.m.N) >= 0) { rc = FTHE_ERR_ARG; break; }
            } else {
                mpz_powm(X.gam[side][b], t[b], P, D.m.N);
            }
            std::vector<uint32_t> tb = X.padic ? fb_table(X.gam[side][b], D.m.N, 2 * X.nwin, X.ew, store_digits)
                                               : fb_table(X.gam[side][b], D.m.N, 2 * X.nwin, X.ew, fb_store_limbs(D.m));
            tab.insert(tab.end(), tb.begin(), tb.end());
        }
        if (rc) break;
        uint32_t *d8 = nullptr;
        if ((rc = fb_upload(tab, &d8))) break;
        rc = fb_widen(k, c, X.padic ? A : D, k->spq, d8, X.nb * X.nwin, X.ew, false, &X.d_tab[side]);
        (void)hipFree(d8);
        if (rc) break;
        Prog e;                                           // X = prod_j entry(j, digit j), then (1 + m n) X
        e.loadgd16(0);
        for (int j = 1; j < X.nb * X.nwin; j++) e.mulgd16(j);
        if (X.padic) {
            e.storep(SL_SAVED);                           // the rest: k->prP_encB_* on s74
        } else {
            e.storex(SL_SAVED);
            e.loadx(SL_IN1); e.mul(side ? SL_C3 : SL_C1); e.addsmall(1); e.mul(SL_SAVED);
            if (side) e.storex(SL_OUTQ); else crt_tail(e);
        }
        e.end();
        X.off[side] = progs.size(); X.mm = std::max(X.mm, e.montmuls);
        progs.insert(progs.end(), e.w.begin(), e.w.end());
    }
    gmp_randclear(st);
    if (rc) return rc;
    if ((rc = fb_upload(progs, &X.d_prog))) return rc;
    X.ready = true;
    return FTHE_OK;
}

int xb_ensure(fthe_key *k, fthe_ctx *c) {
    std::lock_guard<std::mutex> g(k->fb_mu);
    return k->xb.ready ? FTHE_OK : xb_build(k, c, 0);
}

}  // namespace

extern "C" int fthe_key_fixed_base_exact(fthe_key *k, fthe_ctx *c, uint64_t seed) {
    if (!k || !c || k->device != c->device) return FTHE_ERR_ARG;
    std::lock_guard<std::mutex> g(k->fb_mu);
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipDeviceSynchronize());            // no call may still read the old tables
    return xb_build(k, c, seed);
}

extern "C" int fthe_key_fixed_base_exact_set(fthe_key *k, fthe_ctx *c, int nb, const uint32_t *gammas) {
    if (!k || !c || !gammas || k->device != c->device) return FTHE_ERR_ARG;
    std::lock_guard<std::mutex> g(k->fb_mu);
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipDeviceSynchronize());            // no call may still read the old tables
    return xb_build(k, c, 0, gammas, nb);
}

extern "C" int fthe_key_fixed_base_exact_info(fthe_key *k, int side, int base, uint32_t *gamma, int *exp_words) {
    if (!k || side < 0 || side > 1 || base < 0) return FTHE_ERR_ARG;
    std::lock_guard<std::mutex> g(k->fb_mu);
    if (!k->xb.ready || base >= k->xb.nb) return FTHE_ERR_ARG;
    if (gamma) mpz_to_words(k->xb.gam[side][base], gamma, 2 * k->pq_w);
    if (exp_words) *exp_words = k->pq_w;
    return FTHE_OK;
}

extern "C" int fthe_key_fixed_base_exact_bases(fthe_key *k) {
    if (!k) return 0;
    std::lock_guard<std::mutex> g(k->fb_mu);
    return k->xb.ready ? k->xb.nb : 0;
}

// ---------------------------------------------------------------------------
// Public exact fixed-base randomizer (FTHE_ENC_FIXED_BASE_EXACT, public form).
//
// Parties hold only n (party.h:181-185) and encrypt their histograms with the
// public formula (Party::encrypt_histogram, party.h:118-142), r uniform in Z_n^*.
// r -> r^n mod n^2 is a homomorphism of Z_n^* (r^n depends on r mod n only), so
// with published bases hs_i = t_i^n mod n^2 for t_1 .. t_nb generating Z_n^*, a
// uniform r^n is prod hs_i^y_i for y uniform modulo the group order.  The party
// does not know the order (it is phi(n)); it draws y_i uniform below 2^(16 nwin)
// >= n 2^64, which is within nb 2^-64 (statistical distance) of uniform modulo
// any order <= n.  The key holder picks and checks the t_i: Z_n^* = Z_p^* x Z_q^*
// needs, at every prime l | (p-1)(q-1), images spanning (Z_p^*/l-th powers) x
// (Z_q^*/l-th powers): one non-l-th power when l divides one of p-1, q-1, rank 2
// over GF(l) when it divides both (2 always does).  Checked exactly at every
// l < 2^24 (discrete logs in mu_l by baby-step giant-step), and at every l for
// FTHE_KEYGEN_KNOWN_ORDER keys (nb = 2); with 3 bases a larger l escapes with
// probability < 2^-65 per key (l^-3 per l dividing one side, as for the CRT mode).
namespace {

uint64_t mpz_low64(const mpz_t x) { return mpz_sgn(x) == 0 ? 0 : (uint64_t)mpz_getlimbn(x, 0); }

// d with z^d = a mod P, z of prime order l (< 2^24); -1 when a is not in <z>
long dlog_mu(const mpz_t z, const mpz_t a, uint32_t l, const mpz_t P) {
    const uint32_t m = (uint32_t)std::ceil(std::sqrt((double)l));
    std::unordered_map<uint64_t, uint32_t> baby;
    baby.reserve(2 * m);
    Mpz x(1), y, t, zm, chk;
    for (uint32_t j = 0; j < m; j++) {
        baby.emplace(mpz_low64(x), j);
        mpz_mul(t, x, z); mpz_mod(x, t, P);
    }
    mpz_powm_ui(zm, z, (unsigned long)(l - (m % l)) % l, P);     // z^-m (z has order l)
    mpz_set(y, a);
    for (uint32_t i = 0; i <= m; i++) {
        auto it = baby.find(mpz_low64(y));
        if (it != baby.end()) {
            const unsigned long d = ((unsigned long)i * m + it->second) % l;
            mpz_powm_ui(chk, z, d, P);
            if (mpz_cmp(chk, a) == 0) return (long)d;
        }
        mpz_mul(t, y, zm); mpz_mod(y, t, P);
    }
    return -1;
}

// do t[0 .. nb) generate Z_n^* at the primes l of `ls` (each dividing p-1 or q-1)?
bool pb_generates(const Mpz *t, int nb, const mpz_t p, const mpz_t q, const std::vector<Mpz> &ls) {
    Mpz pm1, qm1, e, a[3], b[3], bd;
    mpz_sub_ui(pm1, p, 1); mpz_sub_ui(qm1, q, 1);
    for (const Mpz &l : ls) {
        const bool inp = mpz_divisible_p(pm1, l), inq = mpz_divisible_p(qm1, l);
        if (inp) { mpz_divexact(e, pm1, l); for (int i = 0; i < nb; i++) mpz_powm(a[i], t[i], e, p); }
        if (inq) { mpz_divexact(e, qm1, l); for (int i = 0; i < nb; i++) mpz_powm(b[i], t[i], e, q); }
        int ia = -1, ib = -1;
        for (int i = 0; i < nb; i++) {
            if (inp && ia < 0 && mpz_cmp_ui(a[i], 1) != 0) ia = i;
            if (inq && ib < 0 && mpz_cmp_ui(b[i], 1) != 0) ib = i;
        }
        if ((inp && ia < 0) || (inq && ib < 0)) return false;
        if (!(inp && inq)) continue;
        if (mpz_sizeinbase(l, 2) > 24) continue;        // no small discrete logs: see the bound above
        // rank 2: some j with (log a_j, log b_j) not a multiple of (log a_ia, log b_ia) = (1, beta)
        const uint32_t lu = (uint32_t)mpz_get_ui(l);
        bool rank2 = false;
        for (int j = 0; j < nb && !rank2; j++) {
            if (j == ia) continue;
            const long d = dlog_mu(a[ia], a[j], lu, p);  // a_j = a_ia^d
            if (d < 0) return false;                     // cannot happen (mu_l is cyclic): refuse
            mpz_powm_ui(bd, b[ia], (unsigned long)d, q);
            rank2 = mpz_cmp(bd, b[j]) != 0;
        }
        if (!rank2) return false;
    }
    return true;
}

// the primes l to check: l < 2^24 dividing p-1 or q-1, plus the recorded factors of known-order keys
std::vector<Mpz> pb_primes(const fthe_key *k) {
    std::vector<Mpz> ls;
    if (k->order_known) {
        for (const std::vector<Mpz> *f : {&k->pm1_factors, &k->qm1_factors})
            for (const Mpz &l : *f) {
                bool dup = false;
                for (const Mpz &x : ls) dup = dup || mpz_cmp(x, l) == 0;
                if (!dup) ls.push_back(l);
            }
        return ls;
    }
    Mpz pm1, qm1;
    mpz_sub_ui(pm1, k->p, 1); mpz_sub_ui(qm1, k->q, 1);
    for (uint32_t l : small_primes())
        if (mpz_fdiv_ui(pm1, l) == 0 || mpz_fdiv_ui(qm1, l) == 0) ls.push_back(Mpz(l));
    return ls;
}

int pb_build(fthe_key *k, fthe_ctx *c, const Mpz *hs, int nb, const int *ebits) {
    fthe_key::PublicBase &B = k->pb;
    if (!k->pub_ok || (k->sn2.lanes == 4 && !k->rowio)) return FTHE_ERR_UNSUPPORTED;
    HIPOK(hipSetDevice(c->device));
    HIPOK(hipDeviceSynchronize());                       // no call may still read the old tables
    if (B.d_prog) { (void)hipFree(B.d_prog); B.d_prog = nullptr; }
    B.tab.reset();
    B.d_tab = nullptr;
    B.ready = false;
    B.nb = nb;
    B.wtot = 0;
    for (int i = 0; i < nb; i++) {
        B.nwin[i] = ebits ? ebits[i] / 16 : (k->n_bits + 64 + 15) / 16;
        B.wtot += B.nwin[i];
    }
    B.nadic = k->nadic && !getenv("FTHE_PB_MONT");     // FTHE_PB_MONT=1: Montgomery rows on s152 (A/B)
    B.rows = k->sn2.lanes == 4 && !B.nadic;
    for (int i = 0; i < nb; i++) mpz_set(B.hs[i], hs[i]);
    // process-wide cache: (device, n, hs_1 .. hs_nb) -> tables
    static std::mutex cache_mu;
    static std::map<std::string, std::weak_ptr<fthe_key::SharedTab>> cache;
    std::string id = std::to_string(c->device) + ":";
    {
        const int cw = 2 * k->n_words;
        std::vector<uint32_t> w((size_t)(nb + 1) * cw, 0);
        mpz_to_words(k->n, w.data(), cw);
        for (int i = 0; i < nb; i++) mpz_to_words(B.hs[i], w.data() + (size_t)(i + 1) * cw, cw);
        id.append((const char *)w.data(), w.size() * 4);
        id.append((const char *)B.nwin, sizeof(B.nwin));
        id.append(B.nadic ? "N" : "M");
    }
    int rc;
    {
        std::lock_guard<std::mutex> lk(cache_mu);
        auto it = cache.find(id);
        if (it != cache.end()) B.tab = it->second.lock();
        if (B.tab) {
            B.ew = B.nadic ? 8 * (kNadicDigit.S / 4 + 1) : B.rows ? 2 * k->n_words : 4 * ((k->mn2.m.S + 3) / 4);
        } else {
            auto t = std::make_shared<fthe_key::SharedTab>();
            if ((rc = pub_tables(k, c, B.hs, nb, B.nwin, true, &t->d, &B.ew, B.nadic))) return rc;
            B.tab = t;
            cache[id] = t;
            for (auto i = cache.begin(); i != cache.end();)      // drop entries whose tables are gone
                i = i->second.expired() ? cache.erase(i) : std::next(i);
        }
    }
    B.d_tab = B.tab->d;
    Prog e;                                              // X = prod_j entry(j, digit j), then (1 + m n) X
    e.loadgd16(0);
    for (int j = 1; j < B.wtot; j++) e.mulgd16(j);
    if (B.nadic) {                                       // digits: X (1, m) in C1, canonical digits out
        e.mul(SL_C1); e.canon(); e.storex(SL_OUTP);
    } else {
        e.storex(SL_SAVED);
        e.loadx(SL_IN1); e.mul(SL_C1); e.addsmall(1); e.mul(SL_SAVED);
        if (B.rows) e.storew(2); else e.storex(SL_OUTP);
    }
    e.end();
    B.mm = e.montmuls;
    if ((rc = fb_upload(e.w, &B.d_prog))) return rc;
    B.ready = true;
    return FTHE_OK;
}

}  // namespace

// Known-order keys, g = gcd(p-1, q-1) < 2^64: t_1 a primitive root mod p and mod q (order
// lambda = lcm(p-1, q-1), verified at every factor) and t_2 with t_2 mod p, q in different
// classes of Z_n^* / <t_1> = Z_g (rank 2 with t_1 at every l | g).  Then r = t_1^y_1 t_2^y_2
// is uniform once y_1 is uniform mod lambda and y_2 mod g: y_2 needs 128 bits, not n + 64.
static bool pb_pick_short(fthe_key *k, gmp_randstate_t st, Mpz t[2]) {
    Mpz gg, pm1, qm1, e, x, span, gc;
    mpz_sub_ui(pm1, k->p, 1); mpz_sub_ui(qm1, k->q, 1);
    mpz_gcd(gg, pm1, qm1);
    if (mpz_sizeinbase(gg, 2) > 64) return false;
    std::vector<Mpz> lg;                                  // primes dividing g (all recorded factors)
    for (const Mpz &l : k->pm1_factors)
        if (mpz_divisible_p(gg, l)) lg.push_back(l);
    mpz_sub_ui(span, k->n, 3);
    auto primitive = [&](const mpz_t t, const mpz_t P, const mpz_t Pm1, const std::vector<Mpz> &fs) {
        for (const Mpz &l : fs) {
            mpz_divexact(e, Pm1, l);
            mpz_powm(x, t, e, P);
            if (mpz_cmp_ui(x, 1) == 0) return false;
        }
        return true;
    };
    for (;;) {
        mpz_urandomm(t[0], st, span); mpz_add_ui(t[0], t[0], 2);
        mpz_gcd(gc, t[0], k->n);
        if (mpz_cmp_ui(gc, 1) == 0 && primitive(t[0], k->p, pm1, k->pm1_factors) &&
            primitive(t[0], k->q, qm1, k->qm1_factors)) break;
    }
    for (;;) {
        mpz_urandomm(t[1], st, span); mpz_add_ui(t[1], t[1], 2);
        mpz_gcd(gc, t[1], k->n);
        if (mpz_cmp_ui(gc, 1) == 0 && pb_generates(t, 2, k->p, k->q, lg)) return true;
    }
}

extern "C" int fthe_key_public_bases(fthe_key *k, uint64_t seed, uint32_t *hs, int *nb, int *exp_bits) {
    if (!k) return FTHE_ERR_ARG;
    if (!k->priv) return FTHE_ERR_NOPRIV;
    const int nbases = k->order_known ? 2 : 3;
    if (nb) *nb = nbases;
    if (!hs) return FTHE_OK;
    gmp_randstate_t st;
    gmp_randinit_default(st);
    if (seed) {
        Mpz sd;
        mpz_set_ui(sd, seed);
        mpz_mul_2exp(sd, sd, 64);
        mpz_add_ui(sd, sd, 0x5055424241534553ull);
        gmp_randseed(st, sd);
    } else {
        seed_gmp_state(st, 0, 0);       // 256 bits of /dev/urandom
    }
    Mpz t[3], span, g;
    const int full = 16 * ((k->n_bits + 64 + 15) / 16);
    int eb[3] = {full, full, full};
    if (k->order_known && pb_pick_short(k, st, t)) {
        eb[1] = 128;
    } else {
        const std::vector<Mpz> ls = pb_primes(k);
        mpz_sub_ui(span, k->n, 3);
        for (;;) {
            bool unit = true;
            for (int i = 0; i < nbases; i++) {
                mpz_urandomm(t[i], st, span); mpz_add_ui(t[i], t[i], 2);
                mpz_gcd(g, t[i], k->n);
                unit = unit && mpz_cmp_ui(g, 1) == 0;
            }
            if (unit && pb_generates(t, nbases, k->p, k->q, ls)) break;
        }
    }
    gmp_randclear(st);
    const int cw = 2 * k->n_words;
    for (int i = 0; i < nbases; i++) {
        mpz_powm(g, t[i], k->n, k->n2);
        mpz_to_words(g, hs + (size_t)i * cw, cw);
        if (exp_bits) exp_bits[i] = eb[i];
    }
    return FTHE_OK;
}

extern "C" int fthe_key_set_public_bases(fthe_key *k, fthe_ctx *c, const uint32_t *hs, int nb, const int *exp_bits) {
    if (!k || !c || !hs || k->device != c->device || nb < 1 || nb > 3) return FTHE_ERR_ARG;
    const int cw = 2 * k->n_words;
    Mpz h[3], g;
    for (int i = 0; i < nb; i++) {
        mpz_from_words(h[i], hs + (size_t)i * cw, cw);
        mpz_gcd(g, h[i], k->n);
        if (mpz_sgn(h[i]) <= 0 || mpz_cmp(h[i], k->n2) >= 0 || mpz_cmp_ui(g, 1) != 0) return FTHE_ERR_ARG;
        if (exp_bits && (exp_bits[i] < 16 || exp_bits[i] % 16 || exp_bits[i] > 16 * ((k->n_bits + 64 + 15) / 16)))
            return FTHE_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(k->fb_mu);
    return pb_build(k, c, h, nb, exp_bits);
}

extern "C" int fthe_key_public_bases_info(fthe_key *k, int *nb, int *exp_words) {
    if (!k) return FTHE_ERR_ARG;
    std::lock_guard<std::mutex> lk(k->fb_mu);
    if (!k->pb.ready) return FTHE_ERR_ARG;
    if (nb) *nb = k->pb.nb;
    if (exp_words)
        for (int i = 0; i < k->pb.nb; i++) exp_words[i] = (k->pb.nwin[i] + 1) / 2;
    return FTHE_OK;
}

static int encrypt_pb_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *y, int y_words,
                           uint64_t rng_seed, uint32_t *out, HostPipe *pipe) {
    const fthe_key::PublicBase &B = k->pb;
    const int nb = B.nb;
    int ewd[3], ewo[3], wo[3], ytot = 0, wsum = 0;        // words per injected exponent, their offsets
    for (int b = 0; b < nb; b++) {
        ewd[b] = (B.nwin[b] + 1) / 2; ewo[b] = ytot; ytot += ewd[b];
        wo[b] = wsum; wsum += B.nwin[b];                  // first window of base b
    }
    if (y && y_words != ytot) return FTHE_ERR_ARG;
    Launch Lc;
    int rc;
    if ((rc = begin_call(c, k, count, Lc, nslots_for(k), k->sn2))) return rc;
    const int S = Lc.S, L = Lc.L, cw = 2 * k->n_words;
    const size_t dig_bytes = (size_t)B.wtot * L * 2;     // u16 digits [window][L], base after base
    if ((rc = c->scratch.ensure(dig_bytes))) return rc;
    uint8_t *dig = (uint8_t *)c->scratch.p;
    RngKey rk{};
    if (!y) rk = make_rng_key(rng_seed, 0x7075626c69636273ull);
    Lc.fill(SL_C1, k->c_nRn2);
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt;
        if (pipe && (rc = pipe->before(off, L, count))) return rc;
        for (int b = 0; b < nb; b++) {
            uint8_t *dst = dig + (size_t)wo[b] * L * 2;
            if (y) {
                hipLaunchKernelGGL(k_alpha_digits, Lc.grid(), dim3(256), 0, c->stream, y + off * y_words + ewo[b],
                                   y_words, ewd[b], cnt, B.nwin[b], L, 2, dst);
            } else {
                RngKey kb = rk;
                kb.nonce += (uint64_t)(b + 1) << 56;                       // one stream per base
                hipLaunchKernelGGL(k_rng_digits, Lc.grid(), dim3(256), 0, c->stream, kb, m.idx0 + off, cnt, B.nwin[b],
                                   L, 2, 0, dst);
            }
        }
        if (B.nadic) {
            const int D = kNadicDigit.S;
            Lc.fill(SL_C1, k->c_one_n2);
            m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_C1) + (size_t)D * L, D, L, Lc.B);
            const void *rows[2] = {B.d_tab, dig};
            if ((rc = Lc.prog_raw(B.d_prog, B.mm, k->mnA, rows, 2))) return rc;
            mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTP), D, k->cst(k->c_n76), D,
                        Lc.slot(SL_OUTP) + (size_t)D * L, D, L, cnt, out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
            if (pipe && (rc = pipe->after(off, cnt))) return rc;
            continue;
        }
        m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_IN1), S, L, Lc.B);
        if (B.rows) {
            const void *rows[3] = {B.d_tab, dig, out + off * cw};
            if ((rc = Lc.prog_raw(B.d_prog, B.mm, k->mn2, rows, 3))) return rc;
        } else {
            const void *rows[2] = {B.d_tab, dig};
            if ((rc = Lc.prog_raw(B.d_prog, B.mm, k->mn2, rows, 2))) return rc;
            unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L, cnt, out + off * cw, cw, Lc.B);
        }
        if (pipe && (rc = pipe->after(off, cnt))) return rc;
    }
    return end_call(c, Lc);
}

static int encrypt_xb_impl(fthe_key *k, fthe_ctx *c, MsgSrc m, size_t count, const uint32_t *y,
                           int y_words, uint64_t rng_seed, uint32_t *out, HostPipe *pipe) {
    int rc = xb_ensure(k, c);
    if (rc) return rc;
    const fthe_key::ExactBase &X = k->xb;
    const int pw = k->pq_w;
    const int nb = X.nb;
    if (y && y_words != 2 * nb * pw) return FTHE_ERR_ARG;    // y_{p,1..nb}, y_{q,1..nb}, pq_w words each
    Launch Lc;
    if ((rc = begin_call(c, k, count, Lc, nslots_for(k), k->spq))) return rc;
    const int S = Lc.S, L = Lc.L, cw = 2 * k->n_words;
    const size_t dig_bytes = (size_t)nb * X.nwin * L * 2;   // per side: nb exponents x nwin u16 digit rows
    if ((rc = c->scratch.ensure(2 * dig_bytes + (size_t)L * pw * 4))) return rc;
    uint8_t *dig[2] = {(uint8_t *)c->scratch.p, (uint8_t *)c->scratch.p + dig_bytes};
    uint32_t *ytmp = (uint32_t *)((uint8_t *)c->scratch.p + 2 * dig_bytes);
    RngKey rk{};
    if (!y) rk = make_rng_key(rng_seed, 0x6578616374626173ull);
    Lc.fill(SL_C1, k->c_nRp); Lc.fill(SL_C3, k->c_nRq);
    Lc.fill(SL_T1, k->c_qinvRp2);
    if (X.padic) { Lc.fill(SL_C0, k->c_R2p); Lc.fill(SL_C2, k->c_R2q); }
    const size_t exp_bytes = (size_t)X.nwin * L * 2;
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt;
        if (pipe && (rc = pipe->before(off, L, count))) return rc;
        for (int side = 0; side < 2; side++)
            for (int b = 0; b < nb; b++) {
                uint8_t *dst = dig[side] + b * exp_bytes;
                if (y) {
                    hipLaunchKernelGGL(k_alpha_digits, Lc.grid(), dim3(256), 0, c->stream,
                                       y + off * y_words + (size_t)(nb * side + b) * pw, y_words, pw, cnt, X.nwin, L, 2,
                                       dst);
                } else {
                    RngKey kb = rk;
                    kb.nonce += (uint64_t)(3 * side + b + 1) << 56;           // one stream per (prime, base)
                    hipLaunchKernelGGL(k_rng_r, Lc.grid(), dim3(256), 0, c->stream, k->d_pqwords + side * pw, pw,
                                       (int)(side ? k->q : k->p).bits(), kb, m.idx0 + off, cnt, ytmp);
                    hipLaunchKernelGGL(k_alpha_digits, Lc.grid(), dim3(256), 0, c->stream, ytmp, pw, pw, cnt, X.nwin,
                                       L, 2, dst);
                }
            }
        m.pack(c->stream, Lc.grid(), off, cnt, Lc.slot(SL_IN1), S, L, Lc.B);
        const void *rp[2] = {X.d_tab[0], dig[0]};
        const void *rq[2] = {X.d_tab[1], dig[1]};
        if ((rc = Lc.prog_raw(X.d_prog + X.off[1], X.mm, X.padic ? k->mqA : k->mq2, rq, 2))) return rc;
        if (X.padic && (rc = Lc.prog(k->prP_encB_q, k->mq2))) return rc;
        hipLaunchKernelGGL(k_crt_prep_q, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTQ), k->cst(k->c_q2),
                           k->cst(k->c_2p2), Lc.slot(SL_T0), S, L, Lc.B);
        if ((rc = Lc.prog_raw(X.d_prog + X.off[0], X.mm, X.padic ? k->mpA : k->mp2, rp, 2))) return rc;
        if (X.padic && (rc = Lc.prog(k->prP_encB_p, k->mp2))) return rc;
        hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T2), k->cst(k->c_p2), S, L, Lc.B);
        mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTQ), S,
                    k->cst(k->c_q2), S, Lc.slot(SL_T2), S, L, cnt, out + off * cw, cw, (uint64_t *)nullptr, Lc.B);
        if (pipe && (rc = pipe->after(off, cnt))) return rc;
    }
    return end_call(c, Lc);
}

extern "C" int fthe_encrypt_u64_dev(fthe_key *k, fthe_ctx *c, const uint64_t *m, size_t count,
                                    const uint32_t *r, int r_words, uint64_t rng_seed,
                                    uint32_t *out, int flags) {
    MsgSrc ms; ms.m64 = m;
    return encrypt_impl(k, c, ms, count, r, r_words, rng_seed, out, flags, nullptr);
}

extern "C" int fthe_encrypt_u64_at_dev(fthe_key *k, fthe_ctx *c, const uint64_t *m, size_t count, const uint32_t *r,
                                       int r_words, uint64_t rng_seed, uint64_t index0, uint32_t *out, int flags) {
    MsgSrc ms; ms.m64 = m; ms.idx0 = index0;
    return encrypt_impl(k, c, ms, count, r, r_words, rng_seed, out, flags, nullptr);
}

extern "C" int fthe_encrypt_words_dev(fthe_key *k, fthe_ctx *c, const uint32_t *m, int m_words, size_t count,
                                      const uint32_t *r, int r_words, uint64_t rng_seed, uint32_t *out, int flags) {
    MsgSrc ms; ms.mw = m; ms.mww = m_words;
    return encrypt_impl(k, c, ms, count, r, r_words, rng_seed, out, flags, nullptr);
}

// ---------------------------------------------------------------------------
// Decrypt (CRT)
static int decrypt_impl(fthe_key *k, fthe_ctx *c, const uint32_t *ct, size_t count, uint64_t *m_low,
                        uint32_t *m_full, HostPipe *pipe, bool short_pt = false) {
    if (!k || !c || (!ct && count)) return FTHE_ERR_ARG;
    if (!k->priv) return FTHE_ERR_NOPRIV;
    // Batches that leave most of the chip idle (a GHPair from decrypt_gh, one tree node's sums) run the
    // c^(q-1) mod q^2 exponentiation on the side stream, in a second slot region, beside c^(p-1) mod p^2:
    // one exponentiation of latency instead of two.  Large batches fill the chip with one half at a time.
    // Smaller batches still (<= 16,384 ciphertexts) take both exponentiations on the four-lane s80 kernel,
    // each Montgomery product spread over a quad of lanes (~3x less latency per exponentiation), and
    // hand c^(P-1) mod P^2 back to the s74 layout for the unchanged L-function / CRT tail.
    const int vi = variant_index(k->spq.S);
    const bool quad = k->slat.S && count > 0 && count <= dec_quad_max() && count <= chunk_lanes();
    const bool small_split = !quad && !short_pt && vi >= 0 && count * (size_t)kVariants[vi].lanes <= dec_split_lanes();
    bool split = small_split || (!quad && !short_pt && vi >= 0 && split_all());
    const int nsl = nslots_for(k);
    Launch Lc;
    int rc = begin_call(c, k, count, Lc, split ? 2 * nsl : nsl, k->spq);
    if (rc == FTHE_ERR_NOMEM && split && !small_split) {     // one region when two do not fit (as encrypt_impl)
        split = false;
        rc = begin_call(c, k, count, Lc, nsl, k->spq);
    }
    if (rc) return rc;
    const int S = Lc.S, L = Lc.L, nw = k->n_words, cw = 2 * nw;
    Launch Lp4 = Lc, Lq4 = Lc;             // quad: s80 regions for the p and q halves (slots1)
    const int wl = (kLatShape.S * kLatShape.B + 31) / 32;   // u32 words of an s80 row
    uint32_t *rowp = nullptr, *rowq = nullptr;
    if (quad) {
        if (count > (size_t)L) return FTHE_ERR_ARG;        // one chunk by construction
        const size_t reg = (size_t)nsl * kLatShape.S * L * 4;
        if ((rc = c->slots1.ensure(2 * reg))) return rc;
        if ((rc = c->scratch.ensure((size_t)2 * L * wl * 4))) return rc;
        rowp = (uint32_t *)c->scratch.p; rowq = rowp + (size_t)L * wl;
        Lp4.S = kLatShape.S; Lp4.B = kLatShape.B; Lp4.base = c->slots1.p; Lp4.spread = !short_pt;
        Lq4 = Lp4; Lq4.base = (uint8_t *)c->slots1.p + reg; Lq4.st = c->side;
        Lp4.fill(SL_C0, k->cl_R2p); Lp4.fill(SL_C1, k->cl_R3p); Lp4.fill(SL_T5, k->cl_one);
        if (!short_pt) { Lq4.fill(SL_C2, k->cl_R2q); Lq4.fill(SL_C3, k->cl_R3q); Lq4.fill(SL_T5, k->cl_one); }
    }
    Launch Lq = Lc;                        // q half: region 2 of the slots, side stream
    if (split) {
        Lq.base = (uint8_t *)Lc.base + (size_t)nsl * S * L * 4;
        Lq.st = c->side;
        Lc.spread = Lq.spread = true;
        HIPOK(hipEventRecord(c->ev_fork, c->stream));
        HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
        Lq.fill(SL_C2, k->c_R2q); Lq.fill(SL_C3, k->c_R3q); Lq.fill(SL_T5, k->c_one);
    }
    Launch Lpa, Lpaq;                      // the P-adic kernel's own slots (Paillier-1024; else Lc's)
    if (!quad && (rc = padic_region(c, k, Lc, Lpa, split ? &Lpaq : nullptr))) return rc;
    Lc.fill(SL_C0, k->c_R2p); Lc.fill(SL_C1, k->c_R3p);
    Lc.fill(SL_C2, k->c_R2q); Lc.fill(SL_C3, k->c_R3q);
    Lc.fill(SL_T5, k->c_one);
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt; Lq.live = cnt;
        if (pipe && (rc = pipe->before(off, L, count))) return rc;
        const uint32_t *src = ct + off * cw;
        if (quad) {
            const int S4 = kLatShape.S, B4 = kLatShape.B;
            Lp4.live = cnt; Lq4.live = cnt;
            pack_rows(c->stream, src, cw, cnt, 0, Lp4.slot(SL_IN0), S4, L, B4);
            pack_rows(c->stream, src, cw, cnt, B4 * S4, Lp4.slot(SL_IN1), S4, L, B4);
            if (!short_pt) {
                pack_rows(c->stream, src, cw, cnt, 0, Lq4.slot(SL_IN0), S4, L, B4);
                pack_rows(c->stream, src, cw, cnt, B4 * S4, Lq4.slot(SL_IN1), S4, L, B4);
                HIPOK(hipEventRecord(c->ev_fork, c->stream));
                HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
                if ((rc = Lq4.prog(k->pr_dec_ql, k->mq2l))) return rc;
                HIPOK(hipEventRecord(c->ev_join, c->side));
            }
            if ((rc = Lp4.prog(k->pr_dec_pl, k->mp2l))) return rc;
            // canonical c^(P-1) mod P^2 rows -> the s74 slots the tail reads
            unpack_rows(c->stream, Lp4.slot(SL_OUTP), k->cst(k->cl_p2), S4, L, cnt, rowp, wl, B4);
            pack_rows(c->stream, rowp, wl, cnt, 0, Lc.slot(SL_OUTP), S, L, Lc.B);
            if (!short_pt) {
                HIPOK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
                unpack_rows(c->stream, Lq4.slot(SL_OUTQ), k->cst(k->cl_q2), S4, L, cnt, rowq, wl, B4);
                pack_rows(c->stream, rowq, wl, cnt, 0, Lc.slot(SL_OUTQ), S, L, Lc.B);
            }
            Lc.mm += Lp4.mm + Lq4.mm; Lp4.mm = Lq4.mm = 0;
        } else {
            pack_rows(c->stream, src, cw, cnt, 0, Lc.slot(SL_IN0), S, L, Lc.B);
            pack_rows(c->stream, src, cw, cnt, Lc.B * S, Lc.slot(SL_IN1), S, L, Lc.B);
            if (split) {
                pack_rows(c->stream, src, cw, cnt, 0, Lq.slot(SL_IN0), S, L, Lc.B);
                pack_rows(c->stream, src, cw, cnt, Lc.B * S, Lq.slot(SL_IN1), S, L, Lc.B);
                HIPOK(hipEventRecord(c->ev_fork, c->stream));
                HIPOK(hipStreamWaitEvent(c->side, c->ev_fork, 0));
                if ((rc = dec_pow(Lq, k, 1, &Lpaq))) return rc;
                HIPOK(hipEventRecord(c->ev_join, c->side));
            }
            if ((rc = dec_pow(Lc, k, 0, &Lpa))) return rc;
        }
        if (short_pt) {
            // plaintext < p: m = m_p = L_p(c^(p-1) mod p^2) h_p mod p, the q half and the CRT skipped
            hipLaunchKernelGGL(k_dec_lfunc, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTP), k->cst(k->c_p2), S,
                               k->cst(k->c_pinv), k->kp, Lc.slot(SL_T1), L, Lc.B);
            Lc.fill(SL_C0, k->c_hRp);
            if ((rc = Lc.prog(k->pr_dec_hp, k->mp))) return rc;
            hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTP), k->cst(k->c_p), S, L, Lc.B);
            hipLaunchKernelGGL(k_mul_add_out, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTP), k->kp,
                               k->cst(k->c_zero), 1, Lc.slot(SL_OUTP), k->kp, L, cnt,
                               m_full ? m_full + off * nw : (uint32_t *)nullptr, nw,
                               m_low ? m_low + off : (uint64_t *)nullptr, Lc.B);
            if (off + L < count) Lc.fill(SL_C0, k->c_R2p);
            if (pipe && (rc = pipe->after(off, cnt))) return rc;
            continue;
        }
        if (split) {
            HIPOK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
        } else if (!quad && (rc = dec_pow(Lc, k, 1, &Lpa))) {
            return rc;
        }
        hipLaunchKernelGGL(k_dec_lfunc, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTP), k->cst(k->c_p2), S,
                           k->cst(k->c_pinv), k->kp, Lc.slot(SL_T1), L, Lc.B);
        hipLaunchKernelGGL(k_dec_lfunc, Lc.grid(), dim3(256), 0, c->stream, (split ? Lq : Lc).slot(SL_OUTQ), k->cst(k->c_q2), S,
                           k->cst(k->c_qinv2), k->kq, Lc.slot(SL_T2), L, Lc.B);
        // slots C0/C1/C2 are reused for the mod-p / mod-q constants of the tail
        Lc.fill(SL_C0, k->c_hRp); Lc.fill(SL_C1, k->c_hRq); Lc.fill(SL_C2, k->c_qinvRp);
        if ((rc = Lc.prog(k->pr_dec_hp, k->mp))) return rc;
        if ((rc = Lc.prog(k->pr_dec_hq, k->mq))) return rc;
        hipLaunchKernelGGL(k_crt_dec_prep, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_OUTP), Lc.slot(SL_OUTQ),
                           k->cst(k->c_p), k->cst(k->c_q), k->cst(k->c_2p), Lc.slot(SL_T3), S, L, Lc.B);
        if ((rc = Lc.prog(k->pr_dec_t, k->mp))) return rc;
        hipLaunchKernelGGL(k_canon, Lc.grid(), dim3(256), 0, c->stream, Lc.slot(SL_T4), k->cst(k->c_p), S, L, Lc.B);
        // m = mq + q t   (< n)
        mul_add_out(c->stream, Lc.grid(), Lc.slot(SL_OUTQ), S, k->cst(k->c_q), k->kq, Lc.slot(SL_T4), k->kp, L, cnt,
                    m_full ? m_full + off * nw : (uint32_t *)nullptr, nw, m_low ? m_low + off : (uint64_t *)nullptr,
                    Lc.B);
        if (off + L < count) {   // restore the exponentiation constants for the next chunk
            Lc.fill(SL_C0, k->c_R2p); Lc.fill(SL_C1, k->c_R3p); Lc.fill(SL_C2, k->c_R2q);
        }
        if (pipe && (rc = pipe->after(off, cnt))) return rc;
    }
    Lc.mm += Lq.mm;
    return end_call(c, Lc);
}

extern "C" int fthe_decrypt_dev(fthe_key *k, fthe_ctx *c, const uint32_t *ct, size_t count,
                                uint64_t *m_low, uint32_t *m_full) {
    return decrypt_impl(k, c, ct, count, m_low, m_full, nullptr);
}

extern "C" int fthe_decrypt_short_dev(fthe_key *k, fthe_ctx *c, const uint32_t *ct, size_t count,
                                      uint64_t *m_low, uint32_t *m_full) {
    return decrypt_impl(k, c, ct, count, m_low, m_full, nullptr, true);
}

// ---------------------------------------------------------------------------
// Add / k-way product / scalar mul (mod n^2)

// out = x y mod n^2 for count rows on fthe_addb_q152 (gen_addb.py): 16 rows per wave, 12 waves per workgroup.
// xi / yi (device int64 lists of count entries, nullable): operand row g is row xi[g] of x (xi[g] < 0: the
// integer 1), the gathered products of the histogram scatter and segment sums.
static int launch_addb(fthe_ctx *c, const fthe_key *k, const uint32_t *x, const uint32_t *y, uint32_t *out,
                       size_t count, const int64_t *xi = nullptr, const int64_t *yi = nullptr) {
    // the kernel addresses rows by 32-bit byte offsets (row * 512 < 2^32): launches of at most 4M rows
    constexpr size_t kMaxRows = (size_t)1 << 22;
    const size_t cw = 2 * (size_t)k->n_words;
    while (count > kMaxRows) {
        int rc = launch_addb(c, k, x, y, out, kMaxRows, xi, yi);
        if (rc) return rc;
        if (xi) xi += kMaxRows; else x += kMaxRows * cw;
        if (yi) yi += kMaxRows; else y += kMaxRows * cw;
        out += kMaxRows * cw;
        count -= kMaxRows;
    }
    if (count == 0) return FTHE_OK;
    // persistent workgroups, one per CU at most: each wave sweeps batches of 16 rows across the grid
    const unsigned blocks = (unsigned)std::min<size_t>((count + kAddbPerWg - 1) / kAddbPerWg, (size_t)c->n_cu);
    struct { const void *x, *y; void *o; const void *kc; uint32_t count, nwg; const void *xi, *yi; } args = {
        x, y, out, k->d_addb, (uint32_t)count, blocks, xi, yi};
    static_assert(sizeof(args) == 56, "kernarg layout of gen_addb.py");
    size_t sz = sizeof(args);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    if (hipModuleLaunchKernel(c->fn_addb, blocks, 1, 1, 64 * kAddbWaves, 1, 1, 0, c->stream, nullptr, cfg) != hipSuccess)
        return FTHE_ERR_HIP;
    return FTHE_OK;
}

// Test hook (include/fthe.h): the per-key context bytes of fthe_addb_q152, host only.
extern "C" int fthe_debug_addb_image(const uint32_t *n, int n_words, uint8_t *out, size_t cap, size_t *len) {
    if (!n || n_words <= 0 || !len) return FTHE_ERR_ARG;
    mpz_t nn;
    mpz_init(nn);
    mpz_import(nn, (size_t)n_words, -1, 4, 0, 0, n);
    std::vector<uint8_t> img;
    const bool ok = addb::build(nn, img);
    mpz_clear(nn);
    if (!ok) return FTHE_ERR_UNSUPPORTED;
    *len = img.size();
    if (!out) return FTHE_OK;
    if (cap < img.size()) return FTHE_ERR_ARG;
    memcpy(out, img.data(), img.size());
    return FTHE_OK;
}

// Bring-up / test hook of fthe_nadic_b76: run an op program (uint32 pairs, gen_nadicb.py ops; prog_words words) on
// the key's matrix-core Barrett n-adic kernel over `count` ciphertexts whose slots 0 .. nslots-1 are given as
// host limbs (in: nslots x count x 152 limbs of 27 bits: digit x0 in limbs 0..75, x1 in 76..151); slot out_slot
// is returned the same way.  FTHE_ERR_UNSUPPORTED unless the key runs fthe_nadic_b76.
extern "C" int fthe_debug_nadicb_prog(fthe_key *k, fthe_ctx *c, const uint32_t *prog, int prog_words,
                                      const uint32_t *in, int nslots, size_t count, int out_slot, uint32_t *out) {
    if (!k || !c || !prog || prog_words < 2 || !in || nslots <= 0 || nslots > 16 || !count || !out ||
        out_slot < 0 || out_slot >= nslots)
        return FTHE_ERR_ARG;
    if (!k->nadic_b) return FTHE_ERR_UNSUPPORTED;
    Launch Lc;
    int rc = begin_call(c, k, count, Lc, nslots, k->sn2);
    if (rc) return rc;
    if (count > (size_t)Lc.L) return FTHE_ERR_ARG;
    const int S = Lc.S, L = Lc.L;
    std::vector<uint32_t> slab((size_t)nslots * S * L, 0u);
    for (int s = 0; s < nslots; s++)
        for (size_t g = 0; g < count; g++)
            for (int j = 0; j < S; j++) slab[((size_t)s * S + j) * L + g] = in[((size_t)s * count + g) * S + j];
    HIPOK(hipMemcpy(Lc.base, slab.data(), slab.size() * 4, hipMemcpyHostToDevice));
    Prog p;
    p.w.assign(prog, prog + prog_words);
    fthe_key::PH ph;
    if ((rc = upload_dyn_prog(c, p, ph, c->io[3]))) return rc;
    Lc.live = count;
    if ((rc = launch_dyn(Lc, c->io[3].p, 0, k->mnB))) return rc;
    HIPOK(hipStreamSynchronize(c->stream));
    HIPOK(hipMemcpy(slab.data(), Lc.slot(out_slot), (size_t)S * L * 4, hipMemcpyDeviceToHost));
    for (size_t g = 0; g < count; g++)
        for (int j = 0; j < S; j++) out[g * S + j] = slab[(size_t)j * L + g];
    return end_call(c, Lc);
}

extern "C" int fthe_debug_nadicb_image(const uint32_t *n, int n_words, uint8_t *out, size_t cap, size_t *len) {
    if (!n || n_words <= 0 || !len) return FTHE_ERR_ARG;
    mpz_t nn;
    mpz_init(nn);
    mpz_import(nn, (size_t)n_words, -1, 4, 0, 0, n);
    std::vector<uint8_t> img;
    const bool ok = nadicb::build(nn, img);
    mpz_clear(nn);
    if (!ok) return FTHE_ERR_UNSUPPORTED;
    *len = img.size();
    if (!out) return FTHE_OK;
    if (cap < img.size()) return FTHE_ERR_ARG;
    memcpy(out, img.data(), img.size());
    return FTHE_OK;
}

static int pair_impl(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out,
                     HostPipe *pipe, bool sub) {
    if (!k || !c || ((!a || !b || !out) && count)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    Launch Lc;
    // Row I/O reads and writes the AoS rows directly: the only slot is the R^2 constant, so
    // device-resident calls take 4x larger launches (fewer launch tails) at no memory cost.
    int rc = k->rowio ? begin_call(c, k, count, Lc, SL_C0 + 1, k->sn2, pipe ? 0 : rowio_chunk_lanes())
                      : begin_call(c, k, count, Lc, nslots_for(k), k->sn2);
    if (rc) return rc;
    const int S = Lc.S, L = Lc.L, cw = 2 * k->n_words;
    const bool addb = !sub && k->d_addb && c->fn_addb;
    if (addb && !pipe) {
        // device rows: one launch of persistent workgroups for the whole batch (no chunk tails)
        if ((rc = launch_addb(c, k, a, b, out, count))) return rc;
        Lc.mm += (double)count;
        return end_call(c, Lc);
    }
    if (sub || !k->rowio || !k->add_classical) Lc.fill(SL_C0, k->c_R2n2);    // the classical add needs no R^2
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt;
        if (pipe && (rc = pipe->before(off, L, count))) return rc;
        if (addb) {
            if ((rc = launch_addb(c, k, a + off * cw, b + off * cw, out + off * cw, cnt))) return rc;
            Lc.mm += (double)cnt;
        } else if (k->rowio) {
            const void *rows[3] = {a + off * cw, b + off * cw, out + off * cw};
            if ((rc = Lc.prog(sub ? k->pr_sub_w : k->pr_add_w, k->mn2, rows, 3))) return rc;
        } else {
            pack_rows(c->stream, a + off * cw, cw, cnt, 0, Lc.slot(SL_IN0), S, L, Lc.B);
            pack_rows(c->stream, b + off * cw, cw, cnt, 0, Lc.slot(SL_IN1), S, L, Lc.B);
            if ((rc = Lc.prog(sub ? k->pr_sub : k->pr_add, k->mn2))) return rc;
            unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L,
                               cnt, out + off * cw, cw, Lc.B);
        }
        if (pipe && (rc = pipe->after(off, cnt))) return rc;
    }
    return end_call(c, Lc);
}

extern "C" int fthe_add_dev(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out) {
    return pair_impl(k, c, a, b, count, out, nullptr, false);
}

// out = a * b^(2^64-1) mod n^2: the homomorphic a - b of GHPair::operator- (common.h:253-337,
// both operands encrypted), i.e. Paillier::add(a, Paillier::mul(b, (unsigned long)-1)).
extern "C" int fthe_sub_dev(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out) {
    return pair_impl(k, c, a, b, count, out, nullptr, true);
}

// Programs built per call (k-way product, scalar exponent) go through a
// per-context device buffer; the stream is drained before it is rewritten.

namespace {
// Launch with an explicit (dynamic) program pointer.
}  // namespace

// Row products with a closing constant: out[i] = prod_j xs[j][i] * K R^-kk mod n^2 (X = x_0;
// X <- x_j X R^-1; X <- X K R^-1), or without it (cst = nullptr): prod_j xs[j][i] R^-(kk-1).
//   k-way product:  K = R^kk mod n^2       -> prod x_j
//   to Montgomery:  kk = 1, K = R^2         -> x R
//   from Montgomery: kk = 1, K = 1          -> x R^-1
//   Montgomery add: kk = 2, no constant     -> (aR)(bR)R^-1 = (ab)R
static int rowprod_impl(fthe_key *k, fthe_ctx *c, const uint32_t *const *xs, int kk, size_t count, uint32_t *out,
                        const mpz_t cst, bool classical = false) {
    if (!k || !c || kk <= 0 || kk > 64 || (!out && count)) return FTHE_ERR_ARG;
    for (int j = 0; j < kk; j++)
        if (!xs[j] && count) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    const int base = nslots_for(k);               // inputs live after the standard slots
    const bool rowio = k->rowio && kk + 1 <= 16;
    Launch Lc;
    bool chain = classical && kk >= 2 && k->d_addb && c->fn_addb;
    for (int j = 0; j < kk && chain; j++) {       // out must not overlap an input still to be read
        const size_t bytes = count * 8 * (size_t)k->n_words;
        const char *o = (const char *)out, *x = (const char *)xs[j];
        // the first launch reads x_0, x_1 row by row before writing that row: out may be exactly one of them
        chain = o + bytes <= x || x + bytes <= o || (j < 2 && o == x);
    }
    if (chain) {
        // plain k-way products with a 2048-bit n: a chain of matrix-core Barrett adds over the whole batch,
        // out = x_0 x_1, then out = out x_j (rows are independent, so out may alias x_0 or x_1)
        int rc = begin_call(c, k, count, Lc, SL_C0 + 1, k->sn2, rowio_chunk_lanes());
        if (rc) return rc;
        for (int j = 1; j < kk; j++)
            if ((rc = launch_addb(c, k, j == 1 ? xs[0] : out, xs[j], out, count))) return rc;
        Lc.mm += (double)count * (kk - 1);
        return end_call(c, Lc);
    }
    int rc = rowio ? begin_call(c, k, count, Lc, SL_C0 + 1, k->sn2, rowio_chunk_lanes())   // constant slot only
                   : begin_call(c, k, count, Lc, base + kk, k->sn2);
    if (rc) return rc;
    const int S = Lc.S, L = Lc.L, cw = 2 * k->n_words;
    std::vector<uint32_t> rl;
    if (cst) rl = k->mn2.m.limbs(cst);
    else rl.assign(1, 0u);
    Prog p;
    // plain products (k-way, cst = R^kk) with a 2048-bit n: classical products, no R^kk correction
    classical = classical && rowio && kk >= 2 && k->mn2.m.classical_ok() && !getenv("FTHE_ADD_MONT");
    if (classical) {
        cst = nullptr;
        p.loadw(0); p.canon();
        for (int j = 1; j < kk; j++) p.mulwc(j, j + 1 < kk);
        p.storew(kk); p.end();
    } else if (rowio) {
        p.loadw(0);
        for (int j = 1; j < kk; j++) p.mulw(j);
        if (cst) p.mul(SL_C0);
        p.storew(kk); p.end();
    } else {
        p.loadx(base);
        for (int j = 1; j < kk; j++) p.mul(base + j);
        if (cst) p.mul(SL_C0);
        p.storex(SL_OUTP); p.end();
    }
    std::vector<uint32_t> blob(p.w);
    size_t prog_words = blob.size();
    blob.insert(blob.end(), rl.begin(), rl.end());      // constant after the program
    fthe_key::PH ph;
    Prog tmp; tmp.w = blob; tmp.montmuls = p.montmuls;
    if ((rc = upload_dyn_prog(c, tmp, ph, c->io[3]))) return rc;
    HIPOK(hipEventRecord(c->ev0, c->stream));
    const uint32_t *dconst = (const uint32_t *)c->io[3].p + prog_words;
    if (cst) hipLaunchKernelGGL(k_fill_const, Lc.grid(), dim3(256), 0, c->stream, dconst, Lc.slot(SL_C0), S, L);
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt;
        if (rowio) {
            const void *rows[16];
            for (int j = 0; j < kk; j++) rows[j] = xs[j] + off * cw;
            rows[kk] = out + off * cw;
            if ((rc = launch_dyn(Lc, c->io[3].p, p.montmuls, k->mn2, rows, kk + 1))) return rc;
            continue;
        }
        for (int j = 0; j < kk; j++)
            pack_rows(c->stream, xs[j] + off * cw, cw, cnt, 0, Lc.slot(base + j), S, L, Lc.B);
        if ((rc = launch_dyn(Lc, c->io[3].p, p.montmuls, k->mn2))) return rc;
        unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L,
                           cnt, out + off * cw, cw, Lc.B);
    }
    return end_call(c, Lc);
}

// out[i] = prod_j x[j*count + i] mod n^2.
extern "C" int fthe_reduce_kway_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, int kk, size_t count, uint32_t *out) {
    if (!k || kk <= 0 || kk > 64 || (!x && count)) return FTHE_ERR_ARG;
    std::vector<const uint32_t *> xs(kk);
    for (int j = 0; j < kk; j++) xs[j] = x + (size_t)j * count * 2 * k->n_words;
    Mpz Rk; mpz_powm_ui(Rk, k->mn2.m.R, (unsigned long)kk, k->n2);
    return rowprod_impl(k, c, xs.data(), kk, count, out, Rk, true);
}

// Montgomery-resident rows: x R mod n^2 in the same 2 n_words-word row layout.  Products of
// resident rows need one Montgomery product instead of two (fthe_add_mont_dev).
extern "C" int fthe_to_mont_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count, uint32_t *out) {
    if (!k) return FTHE_ERR_ARG;
    Mpz R2; mpz_mul(R2, k->mn2.m.R, k->mn2.m.R); mpz_mod(R2, R2, k->n2);
    return rowprod_impl(k, c, &x, 1, count, out, R2);
}

extern "C" int fthe_from_mont_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count, uint32_t *out) {
    if (!k) return FTHE_ERR_ARG;
    Mpz one(1);
    return rowprod_impl(k, c, &x, 1, count, out, one);
}

extern "C" int fthe_add_mont_dev(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count,
                                 uint32_t *out) {
    const uint32_t *xs[2] = {a, b};
    return rowprod_impl(k, c, xs, 2, count, out, nullptr);
}

// Gathered K-way products: out[g] = prod_{j<K} x[idx[j*G + g]] mod n^2 (idx < 0 -> 1),
// the building block of the segmented product and the segmented scan.  One
// launch per chunk: K gathered tile loads, then X = x_0; X <- x_j X R^-1;
// X <- X (R^K) R^-1.  idx is a host array, uploaded per pass.
namespace {
struct GatherProd {
    fthe_key *k; fthe_ctx *c;
    static constexpr int K = 8;
    Launch Lc; int base = 0; double mm = 0; size_t prog_words = 0;
    int init(size_t maxG) {
        base = nslots_for(k);
        int rc = begin_call(c, k, maxG, Lc, base + K, k->sn2);
        if (rc) return rc;
        Mpz Rk; mpz_powm_ui(Rk, k->mn2.m.R, (unsigned long)K, k->n2);
        std::vector<uint32_t> rl = k->mn2.m.limbs(Rk);
        Prog p;
        if (k->rowio && k->mn2.m.classical_ok() && !getenv("FTHE_ADD_MONT")) {
            p.loadwg(1); p.canon();       // classical products: no R^K correction
            for (int j = 1; j < K; j++) p.mulwgc(1 + j, j + 1 < K);
            p.storew(K + 1); p.end();
        } else if (k->rowio) {        // rows[0] = source, rows[1..K] = index lists, rows[K+1] = output
            p.loadwg(1);
            for (int j = 1; j < K; j++) p.mulwg(1 + j);
            p.mul(SL_C0);
            p.storew(K + 1); p.end();
        } else {
            p.loadx(base);
            for (int j = 1; j < K; j++) p.mul(base + j);
            p.mul(SL_C0);
            p.storex(SL_OUTP); p.end();
        }
        mm = p.montmuls;
        prog_words = p.w.size();
        Prog blob; blob.w = p.w; blob.w.insert(blob.w.end(), rl.begin(), rl.end());
        fthe_key::PH ph;
        if ((rc = upload_dyn_prog(c, blob, ph, c->io[3]))) return rc;
        HIPOK(hipEventRecord(c->ev0, c->stream));
        hipLaunchKernelGGL(k_fill_const, Lc.grid(), dim3(256), 0, c->stream,
                           (const uint32_t *)c->io[3].p + prog_words, Lc.slot(SL_C0), Lc.S, Lc.L);
        return FTHE_OK;
    }
    // idx: K x G host indices into src (rows of cw words; src holds src_rows rows)
    int run(const uint32_t *src, size_t src_rows, const std::vector<int64_t> &idx, size_t G, uint32_t *dst) {
        int rc;
        HIPOK(hipStreamSynchronize(c->stream));          // previous pass done with scratch
        if ((rc = c->scratch.ensure(std::max<size_t>(8, idx.size() * 8)))) return rc;
        if (!idx.empty()) HIPOK(hipMemcpy(c->scratch.p, idx.data(), idx.size() * 8, hipMemcpyHostToDevice));
        return run_dev(src, src_rows, (const int64_t *)c->scratch.p, G, dst);
    }
    // gidx: K x G device indices into src (src_rows rows)
    int run_dev(const uint32_t *src, size_t src_rows, const int64_t *gidx, size_t G, uint32_t *dst) {
        const int cw = 2 * k->n_words, S = Lc.S, L = Lc.L;
        int rc;
        // the chain of launches re-reads src after the first one has written dst: only for disjoint ranges
        const size_t rb = (size_t)cw * 4;
        const char *d0 = (const char *)dst, *s0 = (const char *)src;
        const bool disjoint = d0 + G * rb <= s0 || s0 + src_rows * rb <= d0;
        if (k->d_addb && c->fn_addb && disjoint) {
            // 2048-bit n: K - 1 matrix-core Barrett add launches over all G rows, gathered operands
            // (dst = src[i_0] src[i_1], then dst = dst src[i_j]; an index < 0 is the integer 1)
            if ((rc = launch_addb(c, k, src, src, dst, G, gidx, gidx + G))) return rc;
            for (int j = 2; j < K; j++)
                if ((rc = launch_addb(c, k, dst, src, dst, G, nullptr, gidx + (size_t)j * G))) return rc;
            Lc.mm += (double)G * (K - 1);
            return FTHE_OK;
        }
        for (size_t off = 0; off < G; off += L) {
            size_t cnt = std::min((size_t)L, G - off);
            Lc.live = cnt;
            if (k->rowio) {
                const void *rows[K + 2];
                rows[0] = src;
                for (int j = 0; j < K; j++) rows[1 + j] = gidx + (size_t)j * G + off;
                rows[K + 1] = dst + off * cw;
                if ((rc = launch_dyn(Lc, c->io[3].p, mm, k->mn2, rows, K + 2))) return rc;
                continue;
            }
            for (int j = 0; j < K; j++)
                pack_rows(c->stream, src, cw, cnt, 0, Lc.slot(base + j), S, L, Lc.B,
                          gidx + (size_t)j * G + off);
            if ((rc = launch_dyn(Lc, c->io[3].p, mm, k->mn2))) return rc;
            unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L, cnt, dst + off * cw, cw, Lc.B);
        }
        return FTHE_OK;
    }
};
}  // namespace

// Segmented product: out[s] = prod_{t in [seg_ptr[s], seg_ptr[s+1])} x[idx ? idx[t] : t]
// mod n^2 (an empty segment gives 1).  Histogram scatter by bin id
// (hist_tree_builder.cpp:565-595: hist[bin] = hist[bin] + gh[iid]), root sums
// (tree.cpp:20-34) and node sums.  Passes of K-way products over groups of <= K
// consecutive members of a segment, until one element per segment remains.
// seg_ptr / idx are host arrays; x and out device pointers.
extern "C" int fthe_reduce_segments_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count,
                                        const int64_t *seg_ptr, const int64_t *idx, size_t nseg, uint32_t *out) {
    if (!k || !c || !seg_ptr || (nseg && !out)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (seg_ptr[0] != 0) return FTHE_ERR_ARG;
    for (size_t s = 0; s < nseg; s++) if (seg_ptr[s + 1] < seg_ptr[s]) return FTHE_ERR_ARG;
    size_t total = (size_t)seg_ptr[nseg];
    if (idx) for (size_t t = 0; t < total; t++) if (idx[t] < 0 || (size_t)idx[t] >= count) return FTHE_ERR_ARG;
    if (!idx && total > count) return FTHE_ERR_ARG;
    if (!nseg) return FTHE_OK;
    const int K = GatherProd::K;
    std::vector<std::vector<int64_t>> members(nseg);
    for (size_t s = 0; s < nseg; s++)
        for (int64_t t = seg_ptr[s]; t < seg_ptr[s + 1]; t++) members[s].push_back(idx ? idx[t] : t);
    const int cw = 2 * k->n_words;
    size_t maxg = 0;
    for (auto &m : members) maxg += std::max<size_t>(1, (m.size() + K - 1) / K);
    int rc;
    if ((rc = c->io[2].ensure(maxg * cw * 4)) || (rc = c->io[1].ensure(maxg * cw * 4))) return rc;
    GatherProd gp{k, c};
    if ((rc = gp.init(maxg))) return rc;
    const uint32_t *src = x;
    size_t src_rows = count;
    int bufsel = 1;
    std::vector<int64_t> gidx;
    while (true) {
        size_t G = 0;
        for (auto &m : members) G += std::max<size_t>(1, (m.size() + K - 1) / K);
        gidx.assign((size_t)K * G, -1);
        std::vector<std::vector<int64_t>> next(nseg);
        size_t g = 0;
        bool done_after = true;
        for (size_t s = 0; s < nseg; s++) {
            size_t ng = std::max<size_t>(1, (members[s].size() + K - 1) / K);
            for (size_t q = 0; q < ng; q++, g++) {
                for (int j = 0; j < K; j++) {
                    size_t t = q * K + j;
                    if (t < members[s].size()) gidx[(size_t)j * G + g] = members[s][t];
                }
                next[s].push_back((int64_t)g);
            }
            if (ng > 1) done_after = false;
        }
        uint32_t *dst = done_after ? out : (uint32_t *)c->io[bufsel].p;
        if ((rc = gp.run(src, src_rows, gidx, G, dst))) return rc;
        if (done_after) break;
        members.swap(next);
        src = dst;
        src_rows = G;
        bufsel = 3 - bufsel;       // ping-pong io[1] / io[2]
    }
    return end_call(c, gp.Lc);
}

// Segmented product with the CSR on the device: the same passes as above, planned
// by k_group_counts / scan / k_plan_groups in HBM (one 8-byte read-back of the
// group count per pass).  seg_ptr (nseg+1) and idx (nullable: identity) are
// device arrays and are only read.
namespace {
int reduce_segments_csr(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t x_rows, const int64_t *seg_dev,
                        const int64_t *idx_dev, size_t nseg, int64_t total, uint32_t *out) {
    const int K = GatherProd::K;
    const int cw = 2 * k->n_words;
    const size_t maxg = (size_t)total / K + nseg;                // groups of the first (largest) pass
    int rc;
    if ((rc = c->io[2].ensure(maxg * cw * 4)) || (rc = c->io[1].ensure(maxg * cw * 4))) return rc;
    if ((rc = c->hb[2].ensure((nseg + 1) * 8)) || (rc = c->hb[3].ensure((maxg + 1) * 8)) ||
        (rc = c->hb[4].ensure((maxg + 1) * 8)) || (rc = c->hb[5].ensure((size_t)K * maxg * 8))) return rc;
    GatherProd gp{k, c};
    if ((rc = gp.init(maxg))) return rc;
    hipStream_t st = c->stream;
    const int64_t *seg = seg_dev, *members = idx_dev;
    const uint32_t *src = x;
    size_t src_rows = x_rows;
    int bufsel = 1, gsel = 3;
    size_t n = nseg;
    while (true) {
        int64_t *ng = (int64_t *)c->hb[2].p;
        int64_t *gptr = (int64_t *)c->hb[gsel].p;
        hipLaunchKernelGGL(k_group_counts, dim3((unsigned)((n + 256) / 256)), dim3(256), 0, st, seg, n, K, ng);
        if ((rc = exclusive_scan_i64(ng, gptr, n + 1, c->cub_tmp, c->cub_bytes, st))) return rc;
        int64_t G = 0;
        HIPOK(hipMemcpyAsync(&G, gptr + n, 8, hipMemcpyDeviceToHost, st));
        HIPOK(hipStreamSynchronize(st));
        if (G <= 0 || (size_t)G > maxg) return FTHE_ERR_ARG;
        int64_t *gidx = (int64_t *)c->hb[5].p;
        hipLaunchKernelGGL(k_plan_groups, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, st, seg, members, n, gptr,
                           (size_t)G, K, gidx);
        const bool last = (size_t)G == nseg;                      // one group per segment: final pass
        uint32_t *dst = last ? out : (uint32_t *)c->io[bufsel].p;
        if ((rc = gp.run_dev(src, src_rows, gidx, (size_t)G, dst))) return rc;
        if (last) break;
        // next pass: segment s owns groups [gptr[s], gptr[s+1]) of dst, members = identity
        seg = gptr; members = nullptr; src = dst; src_rows = (size_t)G;
        bufsel = 3 - bufsel; gsel = 7 - gsel;                      // ping-pong io[1]/io[2], hb[3]/hb[4]
        // n stays nseg: the segments are the same, only their members shrink
    }
    return end_call(c, gp.Lc);
}
}  // namespace

// out[s] <- out[s] * enc_zero[s] for every populated segment s (seg: device, nseg + 1): the Enc(0)
// the reference folds into a bin on its first add (Q10).  Empty segments keep the integer 1.
static int fold_zero_first(fthe_key *k, fthe_ctx *c, const int64_t *seg_dev, size_t nseg, const uint32_t *enc_zero,
                           uint32_t *out) {
    const int cw = 2 * k->n_words;
    int rc;
    if ((rc = c->ezm.ensure(nseg * (size_t)cw * 4))) return rc;
    hipLaunchKernelGGL(k_zero_first_rows, dim3((unsigned)((nseg * cw + 255) / 256)), dim3(256), 0, c->stream,
                       enc_zero, seg_dev, nseg, cw, (uint32_t *)c->ezm.p);
    const uint32_t *xs[2] = {out, (const uint32_t *)c->ezm.p};
    Mpz R2; mpz_powm_ui(R2, k->mn2.m.R, 2ul, k->n2);
    return rowprod_impl(k, c, xs, 2, nseg, out, R2, true);    // row-wise, alias-safe
}

extern "C" int fthe_reduce_segments_csr_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count,
                                            const int64_t *seg_ptr, const int64_t *idx, size_t nseg, uint32_t *out) {
    if (!k || !c || !seg_ptr || (nseg && !out)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (!nseg) return FTHE_OK;
    HIPOK(hipSetDevice(c->device));
    int64_t ends[1] = {0};
    HIPOK(hipMemcpyAsync(ends, seg_ptr + nseg, 8, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    if (ends[0] < 0 || (!idx && (size_t)ends[0] > count)) return FTHE_ERR_ARG;
    if (!x && ends[0]) return FTHE_ERR_ARG;
    (void)count;
    return reduce_segments_csr(k, c, x, count, seg_ptr, idx, nseg, ends[0], out);
}

// Histogram of a node on the device (hist_tree_builder.cpp:565-595 for the root,
// :640-664 for the smaller child of a sibling pair): the CSR of (plane, feature,
// bin) segments from dense_bin_id (atomic count, scan, atomic scatter), then the
// segmented K-way product.  out[p*n_bins + cut[f] + bid] = prod x[p*count + iid]
// over the selected iid with bin_ids[iid*n_col + f] == bid != max_num_bin.
static int histogram_impl(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count, int planes,
                          const uint8_t *bin_ids, int n_col, const int32_t *cut_col_ptr, int max_num_bin,
                          const int32_t *inst, size_t n_sel, const uint32_t *enc_zero, uint32_t *out) {
    if (!k || !c || !cut_col_ptr || n_col <= 0 || planes <= 0 || (!inst && n_sel > count)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (cut_col_ptr[0] != 0) return FTHE_ERR_ARG;
    for (int f = 0; f < n_col; f++) if (cut_col_ptr[f + 1] < cut_col_ptr[f]) return FTHE_ERR_ARG;
    const int64_t n_bins = cut_col_ptr[n_col];
    const size_t nseg = (size_t)planes * (size_t)n_bins;
    if (!nseg) return FTHE_OK;
    if (!out || (n_sel && (!x || !bin_ids))) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc;
    const size_t cells = n_sel * (size_t)n_col;
    // hb[0]: cut (int32) | counts (u64, nseg+1) ; hb[1]: seg (nseg+1) | cursor (nseg) ; io[0]: idx
    const size_t cut_b = ((size_t)(n_col + 1) * 4 + 255) / 256 * 256;
    if ((rc = c->hb[0].ensure(cut_b + (nseg + 1) * 8)) || (rc = c->hb[1].ensure((2 * nseg + 1) * 8))) return rc;
    int32_t *d_cut = (int32_t *)c->hb[0].p;
    unsigned long long *cnt = (unsigned long long *)((char *)c->hb[0].p + cut_b);
    int64_t *seg = (int64_t *)c->hb[1].p;
    unsigned long long *cursor = (unsigned long long *)(seg + nseg + 1);
    HIPOK(hipMemcpyAsync(d_cut, cut_col_ptr, (size_t)(n_col + 1) * 4, hipMemcpyHostToDevice, st));
    HIPOK(hipMemsetAsync(cnt, 0, (nseg + 1) * 8, st));
    HIPOK(hipMemsetAsync(cursor, 0, nseg * 8, st));
    const unsigned gb = (unsigned)std::max<size_t>(1, (cells + 255) / 256);
    if (cells)
        hipLaunchKernelGGL(k_hist_count, dim3(gb), dim3(256), 0, st, bin_ids, n_col, d_cut, max_num_bin, inst, n_sel,
                           planes, n_bins, cnt);
    // counts -> int64 in seg, exclusive scan in place through io[0] as temp
    if ((rc = c->io[0].ensure((nseg + 1) * 8))) return rc;
    int64_t *tmp = (int64_t *)c->io[0].p;
    hipLaunchKernelGGL(k_u64_to_i64, dim3((unsigned)((nseg + 256) / 256)), dim3(256), 0, st, cnt, tmp, nseg + 1);
    if ((rc = exclusive_scan_i64(tmp, seg, nseg + 1, c->cub_tmp, c->cub_bytes, st))) return rc;
    int64_t total = 0;
    HIPOK(hipMemcpyAsync(&total, seg + nseg, 8, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    if ((rc = c->io[0].ensure(std::max<int64_t>(1, total) * 8))) return rc;
    int64_t *idx = (int64_t *)c->io[0].p;
    if (cells)
        hipLaunchKernelGGL(k_hist_scatter, dim3(gb), dim3(256), 0, st, bin_ids, n_col, d_cut, max_num_bin, inst, n_sel,
                           planes, n_bins, count, seg, cursor, idx);
    // io[0] (idx) and hb[1] (seg) stay untouched by the product passes (io[1]/io[2], hb[2..5])
    if ((rc = reduce_segments_csr(k, c, x, (size_t)planes * count, seg, idx, nseg, total, out))) return rc;
    return enc_zero ? fold_zero_first(k, c, seg, nseg, enc_zero, out) : FTHE_OK;
}

extern "C" int fthe_histogram_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count, int planes,
                                  const uint8_t *bin_ids, int n_col, const int32_t *cut_col_ptr, int max_num_bin,
                                  const int32_t *inst, size_t n_sel, uint32_t *out) {
    return histogram_impl(k, c, x, count, planes, bin_ids, n_col, cut_col_ptr, max_num_bin, inst, n_sel, nullptr, out);
}

extern "C" int fthe_histogram_zero_first_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count, int planes,
                                             const uint8_t *bin_ids, int n_col, const int32_t *cut_col_ptr,
                                             int max_num_bin, const int32_t *inst, size_t n_sel,
                                             const uint32_t *enc_zero, uint32_t *out) {
    if (!enc_zero) return FTHE_ERR_ARG;
    return histogram_impl(k, c, x, count, planes, bin_ids, n_col, cut_col_ptr, max_num_bin, inst, n_sel, enc_zero,
                          out);
}

// Segmented inclusive scan: out[t] = prod_{t' in [seg_start(t), t]} x[t'] mod n^2, the
// inclusive_scan_by_key over (node, feature) of the histogram (hist_tree_builder.cpp:695-708;
// GHPair::operator+ as the binary op).  Hillis-Steele in radix K: pass p multiplies the K
// elements at stride K^p, so ceil(log_K(longest segment)) passes.  seg_ptr is a host
// array over the elements x[0 .. seg_ptr[nseg]).
extern "C" int fthe_scan_segments_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, const int64_t *seg_ptr,
                                      size_t nseg, uint32_t *out) {
    if (!k || !c || !seg_ptr) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (seg_ptr[0] != 0) return FTHE_ERR_ARG;
    size_t longest = 0;
    for (size_t s = 0; s < nseg; s++) {
        if (seg_ptr[s + 1] < seg_ptr[s]) return FTHE_ERR_ARG;
        longest = std::max(longest, (size_t)(seg_ptr[s + 1] - seg_ptr[s]));
    }
    const size_t N = (size_t)seg_ptr[nseg];
    if (!N) return FTHE_OK;
    if (!x || !out) return FTHE_ERR_ARG;
    const int K = GatherProd::K;
    const int cw = 2 * k->n_words;
    std::vector<int64_t> start(N);
    for (size_t s = 0; s < nseg; s++)
        for (int64_t t = seg_ptr[s]; t < seg_ptr[s + 1]; t++) start[t] = seg_ptr[s];
    int npass = 1;
    for (size_t span = K; span < longest; span *= K) npass++;
    int rc;
    if ((rc = c->io[2].ensure(N * cw * 4)) || (rc = c->io[1].ensure(N * cw * 4))) return rc;
    GatherProd gp{k, c};
    if ((rc = gp.init(N))) return rc;
    std::vector<int64_t> gidx((size_t)K * N);
    const uint32_t *src = x;
    int bufsel = 1;
    size_t stride = 1;
    for (int p = 0; p < npass; p++, stride *= K) {
        for (int j = 0; j < K; j++)
            for (size_t t = 0; t < N; t++) {
                int64_t from = (int64_t)t - (int64_t)(j * stride);
                gidx[(size_t)j * N + t] = from >= start[t] ? from : -1;
            }
        uint32_t *dst = p == npass - 1 ? out : (uint32_t *)c->io[bufsel].p;
        if ((rc = gp.run(src, N, gidx, N, dst))) return rc;
        src = dst;
        bufsel = 3 - bufsel;
    }
    return end_call(c, gp.Lc);
}

// Segmented product with the reference's Enc(0)-first semantics: out[s] = enc_zero[s] * prod(members)
// for a populated segment, 1 for an empty one.  seg_ptr / idx host arrays as fthe_reduce_segments_dev.
extern "C" int fthe_reduce_segments_zero_first_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count,
                                                   const int64_t *seg_ptr, const int64_t *idx, size_t nseg,
                                                   const uint32_t *enc_zero, uint32_t *out) {
    if (!enc_zero && nseg) return FTHE_ERR_ARG;
    int rc = fthe_reduce_segments_dev(k, c, x, count, seg_ptr, idx, nseg, out);
    if (rc || !nseg) return rc;
    if ((rc = c->hb[1].ensure((nseg + 1) * 8))) return rc;
    HIPOK(hipMemcpyAsync(c->hb[1].p, seg_ptr, (nseg + 1) * 8, hipMemcpyHostToDevice, c->stream));
    rc = fold_zero_first(k, c, (const int64_t *)c->hb[1].p, nseg, enc_zero, out);
    HIPOK(hipStreamSynchronize(c->stream));                 // seg_ptr is the caller's host array
    return rc;
}

extern "C" int fthe_reduce_segments(fthe_key *k, fthe_ctx *c, const uint32_t *x, size_t count,
                                    const int64_t *seg_ptr, const int64_t *idx, size_t nseg, uint32_t *out) {
    if (!k || !c || !seg_ptr) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    size_t cw = 2 * (size_t)k->n_words;
    int rc;
    // x staged in io[0], out in io[4]; io[1] / io[2] are the pass buffers, io[3] the program
    if ((rc = c->io[0].ensure(std::max<size_t>(1, count) * cw * 4))) return rc;
    if (count) HIPOK(hipMemcpyAsync(c->io[0].p, x, count * cw * 4, hipMemcpyHostToDevice, c->stream));
    if ((rc = c->io[4].ensure(std::max<size_t>(1, nseg) * cw * 4))) return rc;
    if ((rc = fthe_reduce_segments_dev(k, c, (const uint32_t *)c->io[0].p, count, seg_ptr, idx, nseg,
                                       (uint32_t *)c->io[4].p))) return rc;
    if (nseg) HIPOK(hipMemcpyAsync(out, c->io[4].p, nseg * cw * 4, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    return FTHE_OK;
}

extern "C" int fthe_scan_segments(fthe_key *k, fthe_ctx *c, const uint32_t *x, const int64_t *seg_ptr, size_t nseg,
                                  uint32_t *out) {
    if (!k || !c || !seg_ptr) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    const size_t N = (size_t)seg_ptr[nseg], bytes = N * 2 * (size_t)k->n_words * 4;
    int rc;
    if ((rc = c->io[0].ensure(std::max<size_t>(4, bytes))) || (rc = c->io[4].ensure(std::max<size_t>(4, bytes))))
        return rc;
    if (N) HIPOK(hipMemcpyAsync(c->io[0].p, x, bytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = fthe_scan_segments_dev(k, c, (const uint32_t *)c->io[0].p, seg_ptr, nseg, (uint32_t *)c->io[4].p)))
        return rc;
    if (N) HIPOK(hipMemcpyAsync(out, c->io[4].p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    return FTHE_OK;
}

// out[i] = x[i]^e mod n^2 (Paillier::mul, paillier.cpp:118), e uniform.
// x^e mod n^2 for one exponent e shared by the batch (Paillier::mul, paillier.cpp:107-120)
static int scalar_mul_impl(fthe_key *k, fthe_ctx *c, const uint32_t *x, const mpz_t ez, size_t count, uint32_t *out) {
    if (!k || !c || ((!x || !out) && count)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    Launch Lc;
    int rc = begin_call(c, k, count, Lc, nslots_for(k), k->sn2);
    if (rc) return rc;
    const int S = Lc.S, L = Lc.L, cw = 2 * k->n_words;
    const bool rowio = k->rowio;
    Prog p;
    p.lds_a = lds_prefetch(k->sn2);
    if (mpz_sgn(ez) == 0) {
        p.loadx(SL_C1);                 // x^0 = 1
    } else {
        if (rowio) p.loadw(0); else p.loadx(SL_IN0);
        p.mul(SL_C0);                    // Montgomery form
        p.pow(ez, SL_TAB, SL_SQ, std::min(best_window(mpz_sizeinbase(ez, 2)), 5));
        p.mul(SL_C1);                    // * 1 -> out of Montgomery
    }
    if (rowio) p.storew(1); else p.storex(SL_OUTP);
    p.end();
    fthe_key::PH ph;
    if ((rc = upload_dyn_prog(c, p, ph, c->io[3]))) return rc;
    HIPOK(hipEventRecord(c->ev0, c->stream));
    Lc.fill(SL_C0, k->c_R2n2); Lc.fill(SL_C1, k->c_one_n2);
    for (size_t off = 0; off < count; off += L) {
        size_t cnt = std::min((size_t)L, count - off);
        Lc.live = cnt;
        if (rowio) {
            const void *rows[2] = {x + off * cw, out + off * cw};
            if ((rc = launch_dyn(Lc, c->io[3].p, p.montmuls, k->mn2, rows, 2))) return rc;
            continue;
        }
        pack_rows(c->stream, x + off * cw, cw, cnt, 0, Lc.slot(SL_IN0), S, L, Lc.B);
        if ((rc = launch_dyn(Lc, c->io[3].p, p.montmuls, k->mn2))) return rc;
        unpack_rows(c->stream, Lc.slot(SL_OUTP), k->cst(k->c_n2), S, L,
                           cnt, out + off * cw, cw, Lc.B);
    }
    return end_call(c, Lc);
}

extern "C" int fthe_scalar_mul_u64_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, uint64_t e, size_t count, uint32_t *out) {
    Mpz ez; mpz_import(ez, 1, -1, 8, 0, 0, &e);
    return scalar_mul_impl(k, c, x, ez, count, out);
}

extern "C" int fthe_scalar_mul_words_dev(fthe_key *k, fthe_ctx *c, const uint32_t *x, const uint32_t *e, int e_words,
                                         size_t count, uint32_t *out) {
    if (!e || e_words <= 0) return FTHE_ERR_ARG;
    Mpz ez; mpz_from_words(ez, e, e_words);
    return scalar_mul_impl(k, c, x, ez, count, out);
}

// ---------------------------------------------------------------------------
// Host-resident variants: stage through device buffers, synchronous.
namespace {
struct HostIO {
    fthe_ctx *c;
    int in(int i, const void *h, size_t bytes, void **d) {
        int rc = c->io[i].ensure(bytes ? bytes : 4);
        if (rc) return rc;
        if (bytes) HIPOK(hipMemcpyAsync(c->io[i].p, h, bytes, hipMemcpyHostToDevice, c->stream));
        *d = c->io[i].p;
        return FTHE_OK;
    }
    int outbuf(int i, size_t bytes, void **d) {
        int rc = c->io[i].ensure(bytes ? bytes : 4);
        if (rc) return rc;
        *d = c->io[i].p;
        return FTHE_OK;
    }
    int back(void *h, const void *d, size_t bytes) {
        if (bytes) HIPOK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
        HIPOK(hipStreamSynchronize(c->stream));
        return FTHE_OK;
    }
};
}  // namespace

// Host-resident encrypt: inputs staged and outputs drained chunk by chunk through pinned buffers
// (HostPipe); m is either u64 codec values or general plaintexts of mww words.
static int encrypt_host(fthe_key *k, fthe_ctx *c, const void *m, int mww, size_t count, const uint32_t *r,
                        int r_words, uint64_t rng_seed, uint32_t *out, int flags, uint64_t index0 = 0) {
    if (!k || !c || (!m && count) || (!out && count)) return FTHE_ERR_ARG;
    if (mww && (mww < 0 || mww > k->n_words)) return FTHE_ERR_ARG;
    if (r && (r_words <= 0 || r_words > ((flags & FTHE_ENC_FIXED_BASE_EXACT) ? 3 * (k->n_words + 2)
                                         : k->n_words + ((flags & FTHE_ENC_FIXED_BASE) ? 4 : 0)))) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    size_t cw = 2 * (size_t)k->n_words, mb = mww ? (size_t)mww * 4 : 8;
    int rc;
    if ((rc = c->io[0].ensure(std::max<size_t>(4, count * mb))) || (rc = c->io[2].ensure(std::max<size_t>(4, count * cw * 4))))
        return rc;
    if (r && (rc = c->io[1].ensure(std::max<size_t>(4, count * r_words * 4)))) return rc;
    HostPipe pipe{c};
    pipe.add_in(m, c->io[0].p, mb);
    if (r) pipe.add_in(r, c->io[1].p, (size_t)r_words * 4);
    pipe.add_out(out, c->io[2].p, cw * 4);
    MsgSrc ms;
    if (mww) { ms.mw = (const uint32_t *)c->io[0].p; ms.mww = mww; } else ms.m64 = (const uint64_t *)c->io[0].p;
    ms.idx0 = index0;
    if ((rc = encrypt_impl(k, c, ms, count, r ? (const uint32_t *)c->io[1].p : nullptr, r_words,
                           rng_seed, (uint32_t *)c->io[2].p, flags, count ? &pipe : nullptr))) return rc;
    return pipe.finish();
}

extern "C" int fthe_encrypt_u64(fthe_key *k, fthe_ctx *c, const uint64_t *m, size_t count, const uint32_t *r,
                                int r_words, uint64_t rng_seed, uint32_t *out, int flags) {
    return encrypt_host(k, c, m, 0, count, r, r_words, rng_seed, out, flags);
}

extern "C" int fthe_encrypt_u64_at(fthe_key *k, fthe_ctx *c, const uint64_t *m, size_t count, const uint32_t *r,
                                   int r_words, uint64_t rng_seed, uint64_t index0, uint32_t *out, int flags) {
    return encrypt_host(k, c, m, 0, count, r, r_words, rng_seed, out, flags, index0);
}

extern "C" int fthe_encrypt_words(fthe_key *k, fthe_ctx *c, const uint32_t *m, int m_words, size_t count,
                                  const uint32_t *r, int r_words, uint64_t rng_seed, uint32_t *out, int flags) {
    if (m_words <= 0) return FTHE_ERR_ARG;
    return encrypt_host(k, c, m, m_words, count, r, r_words, rng_seed, out, flags);
}

static int decrypt_host(fthe_key *k, fthe_ctx *c, const uint32_t *ct, size_t count, uint64_t *m_low, uint32_t *m_full,
                        bool short_pt) {
    if (!k || !c || (!ct && count)) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    size_t cw = 2 * (size_t)k->n_words, nw = k->n_words;
    int rc;
    if ((rc = c->io[0].ensure(std::max<size_t>(4, count * cw * 4)))) return rc;
    if (m_low && (rc = c->io[1].ensure(std::max<size_t>(4, count * 8)))) return rc;
    if (m_full && (rc = c->io[2].ensure(std::max<size_t>(4, count * nw * 4)))) return rc;
    HostPipe pipe{c};
    pipe.add_in(ct, c->io[0].p, cw * 4);
    if (m_low) pipe.add_out(m_low, c->io[1].p, 8);
    if (m_full) pipe.add_out(m_full, c->io[2].p, nw * 4);
    if ((rc = decrypt_impl(k, c, (const uint32_t *)c->io[0].p, count, m_low ? (uint64_t *)c->io[1].p : nullptr,
                           m_full ? (uint32_t *)c->io[2].p : nullptr, count ? &pipe : nullptr, short_pt))) return rc;
    return pipe.finish();
}

extern "C" int fthe_decrypt(fthe_key *k, fthe_ctx *c, const uint32_t *ct, size_t count, uint64_t *m_low, uint32_t *m_full) {
    return decrypt_host(k, c, ct, count, m_low, m_full, false);
}

// Staging buffers of the shared queues above this many bytes are released after their batch
// (one large shared call must not pin a second copy of its ciphertexts for the key's lifetime).
constexpr size_t kCoalesceKeepBytes = (size_t)64 << 20;
template <class V> static void trim(V &v) {
    if (v.capacity() * sizeof(typename V::value_type) > kCoalesceKeepBytes) { V().swap(v); }
}

// One leader runs everything pending (its own request included) as at most two batched calls
// (full / short), then hands leadership to a caller still waiting.  A lone request runs straight
// on the caller's buffers (no staging copy).
static void coalesced_batch_impl(fthe_key *k, Coalescer *co, const std::vector<DecReq *> &batch) {
    const size_t cw = 2 * (size_t)k->n_words, nw = k->n_words;
    int rc0 = FTHE_OK;
    if (!co->ctx) rc0 = fthe_ctx_create(k->device, &co->ctx);
    if (batch.size() == 1) {
        DecReq *r = batch[0];
        r->rc = rc0 ? rc0 : decrypt_host(k, co->ctx, r->ct, r->count, r->m_low, r->m_full, r->short_pt);
        return;
    }
    for (int kind = 0; kind < 2; kind++) {
        size_t tot = 0;
        bool want_full = false;
        for (DecReq *r : batch)
            if (r->short_pt == (kind == 1)) { tot += r->count; want_full |= r->m_full != nullptr; }
        if (!tot) continue;
        int rc = rc0;
        if (!rc) {
            co->ct.resize(tot * cw); co->lo.resize(tot);
            if (want_full) co->full.resize(tot * nw);
            size_t at = 0;
            for (DecReq *r : batch)
                if (r->short_pt == (kind == 1)) { memcpy(&co->ct[at * cw], r->ct, r->count * cw * 4); at += r->count; }
            rc = decrypt_host(k, co->ctx, co->ct.data(), tot, co->lo.data(), want_full ? co->full.data() : nullptr,
                              kind == 1);
        }
        size_t at = 0;
        for (DecReq *r : batch) {
            if (r->short_pt != (kind == 1)) continue;
            r->rc = rc;
            if (!rc) {
                if (r->m_low) memcpy(r->m_low, &co->lo[at], r->count * 8);
                if (r->m_full) memcpy(r->m_full, &co->full[at * nw], r->count * nw * 4);
            }
            at += r->count;
        }
    }
    trim(co->ct); trim(co->lo); trim(co->full);
}

// Nothing may leave the C ABI by exception, and the leader must always mark its batch done and
// hand over (fthe_decrypt_shared): allocation failures (staging vectors, copy threads) become
// FTHE_ERR_NOMEM for every request of the batch.
static void coalesced_batch(fthe_key *k, Coalescer *co, const std::vector<DecReq *> &batch) {
    try {
        coalesced_batch_impl(k, co, batch);
    } catch (...) {
        for (DecReq *r : batch) r->rc = FTHE_ERR_NOMEM;
        try { trim(co->ct); trim(co->lo); trim(co->full); } catch (...) {}
    }
}

// Encrypt side of the queue: requests grouped by flags, fresh device randomness per batch.
static void coalesced_encrypt_impl(fthe_key *k, Coalescer *co, const std::vector<EncReq *> &batch) {
    const size_t cw = 2 * (size_t)k->n_words;
    int rc0 = FTHE_OK;
    if (!co->ectx) rc0 = fthe_ctx_create(k->device, &co->ectx);
    if (batch.size() == 1) {
        EncReq *r = batch[0];
        r->rc = rc0 ? rc0 : encrypt_host(k, co->ectx, r->m, 0, r->count, nullptr, 0, 0, r->out, r->flags);
        return;
    }
    std::vector<int> kinds;
    for (EncReq *r : batch)
        if (std::find(kinds.begin(), kinds.end(), r->flags) == kinds.end()) kinds.push_back(r->flags);
    for (int fl : kinds) {
        size_t tot = 0;
        for (EncReq *r : batch) if (r->flags == fl) tot += r->count;
        int rc = rc0;
        if (!rc) {
            co->em.resize(tot); co->eout.resize(tot * cw);
            size_t at = 0;
            for (EncReq *r : batch)
                if (r->flags == fl) { memcpy(&co->em[at], r->m, r->count * 8); at += r->count; }
            rc = encrypt_host(k, co->ectx, co->em.data(), 0, tot, nullptr, 0, 0, co->eout.data(), fl);
        }
        size_t at = 0;
        for (EncReq *r : batch) {
            if (r->flags != fl) continue;
            r->rc = rc;
            if (!rc) memcpy(r->out, &co->eout[at * cw], r->count * cw * 4);
            at += r->count;
        }
    }
    trim(co->em); trim(co->eout);
}

static void coalesced_encrypt(fthe_key *k, Coalescer *co, const std::vector<EncReq *> &batch) {
    try {
        coalesced_encrypt_impl(k, co, batch);
    } catch (...) {
        for (EncReq *r : batch) r->rc = FTHE_ERR_NOMEM;
        try { trim(co->em); trim(co->eout); } catch (...) {}
    }
}

static Coalescer *key_coalescer(fthe_key *k) {
    std::lock_guard<std::mutex> g(k->co_mu);
    if (!k->co) k->co.reset(new (std::nothrow) Coalescer);
    return k->co.get();
}

// Group commit with a linger.  The callers of a finished batch come back one at a time (each wakes from
// notify_all, re-takes the mutex, returns, issues its next call), so a new leader that took the queue at
// once would run a batch of one and leave the others to the round trip after: FedTree's OpenMP loops of
// single-element calls (hist_tree_builder.cpp:574-591 through GHPair's operators; decrypt_gh per node,
// FLtrainer.cpp:758-764) ran two launches per round.  A new leader waits until as many requests are pending
// as there were callers in the previous round (its batch plus the requests that arrived while it ran), at
// most FTHE_LINGER_US (default 200 us; 0: off) or a quarter of the previous batch's duration if that is
// longer (a merged decrypt takes ~10 ms), the latter capped at kLingerCapUs so one huge batch (a bulk
// add_shared of millions of rows) cannot make the next leader wait for callers that never come back; a lone
// caller never waits.  Arrivals wake it when the count is reached.
static constexpr int64_t kLingerCapUs = 3000;
static int linger_us() {
    static const int v = [] {
        const char *e = getenv("FTHE_LINGER_US");
        return e ? std::max(0, atoi(e)) : 200;
    }();
    return v;
}
template <class Req>
static void linger(Coalescer *co, std::unique_lock<std::mutex> &lk, const std::vector<Req *> &pend, size_t last,
                   bool &lingering, int64_t last_us) {
    if (last <= 1 || pend.size() >= last || linger_us() <= 0) return;
    lingering = true;
    // a quarter of a long batch (decrypts), capped: one huge batch must not make the next lone caller wait long
    const int64_t bound = std::max<int64_t>(linger_us(), std::min<int64_t>(last_us / 4, kLingerCapUs));
    co->lcv.wait_for(lk, std::chrono::microseconds(bound), [&] { return pend.size() >= last; });
    lingering = false;
}
static int64_t us_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
}
template <class Req>
static void arrived(Coalescer *co, const std::vector<Req *> &pend, size_t last, bool lingering) {
    if (lingering && pend.size() >= last) co->lcv.notify_all();
}

extern "C" int fthe_decrypt_shared(fthe_key *k, const uint32_t *ct, size_t count, uint64_t *m_low, uint32_t *m_full,
                                   int short_pt) {
    if (!k || (!ct && count)) return FTHE_ERR_ARG;
    if (!k->priv) return FTHE_ERR_NOPRIV;
    if (!count) return FTHE_OK;
    Coalescer *co = key_coalescer(k);
    if (!co) return FTHE_ERR_NOMEM;
    DecReq r{ct, count, m_low, m_full, short_pt != 0};
    std::unique_lock<std::mutex> lk(co->mu);
    try { co->pending.push_back(&r); } catch (...) { return FTHE_ERR_NOMEM; }
    arrived(co, co->pending, co->last, co->lingering);
    for (;;) {
        if (r.done) return r.rc;
        if (!co->leader) {
            co->leader = true;
            linger(co, lk, co->pending, co->last, co->lingering, co->last_us);
            std::vector<DecReq *> batch;
            batch.swap(co->pending);                 // includes r
            lk.unlock();
            const auto t_batch = std::chrono::steady_clock::now();
            coalesced_batch(k, co, batch);
            co->last_us = us_since(t_batch);
            lk.lock();
            for (DecReq *q : batch) q->done = true;
            co->last = batch.size() + co->pending.size();   // callers active in this round
            co->leader = false;
            co->cv.notify_all();
            return r.rc;
        }
        co->cv.wait(lk);
    }
}

extern "C" int fthe_decrypt_short(fthe_key *k, fthe_ctx *c, const uint32_t *ct, size_t count, uint64_t *m_low,
                                  uint32_t *m_full) {
    return decrypt_host(k, c, ct, count, m_low, m_full, true);
}

// Host-resident pair ops of at most this many rows take the single-stream path (FTHE_SMALL_HOST; 0: never).
static size_t small_host_rows() {
    static const size_t v = [] {
        const char *e = getenv("FTHE_SMALL_HOST");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)4096;
    }();
    return v;
}
static int pair_host(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out,
                     bool sub) {
    if (!k || !c || ((!a || !b || !out) && count)) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    size_t row = 2 * (size_t)k->n_words * 4;
    int rc;
    if (count <= small_host_rows()) {
        // small batches (GHPair operators through fthe_add_shared): one stream, no staging pipeline --
        // the pipe's copy-stream / compute-stream event hand-offs cost more than its overlap saves here
        HostIO io{c}; void *da, *db, *dout;
        if ((rc = io.in(0, a, count * row, &da)) || (rc = io.in(1, b, count * row, &db)) ||
            (rc = io.outbuf(2, count * row, &dout)))
            return rc;
        if ((rc = pair_impl(k, c, (const uint32_t *)da, (const uint32_t *)db, count, (uint32_t *)dout, nullptr, sub)))
            return rc;
        return io.back(out, dout, count * row);
    }
    for (int i = 0; i < 3; i++) if ((rc = c->io[i].ensure(std::max<size_t>(4, count * row)))) return rc;
    HostPipe pipe{c};
    pipe.input_first = false;                    // PCIe-bound: keep the DMA engine busy during host copies
    pipe.add_in(a, c->io[0].p, row);
    pipe.add_in(b, c->io[1].p, row);
    pipe.add_out(out, c->io[2].p, row);
    if ((rc = pair_impl(k, c, (const uint32_t *)c->io[0].p, (const uint32_t *)c->io[1].p, count, (uint32_t *)c->io[2].p,
                        count ? &pipe : nullptr, sub))) return rc;
    return pipe.finish();
}

extern "C" int fthe_add(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out) {
    return pair_host(k, c, a, b, count, out, false);
}

extern "C" int fthe_sub(fthe_key *k, fthe_ctx *c, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out) {
    return pair_host(k, c, a, b, count, out, true);
}

extern "C" int fthe_reduce_kway(fthe_key *k, fthe_ctx *c, const uint32_t *x, int kk, size_t count, uint32_t *out) {
    if (!k || !c || kk <= 0) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HostIO io{c}; void *dx, *dout; int rc;
    size_t bytes = count * 2 * (size_t)k->n_words * 4;
    if ((rc = io.in(0, x, bytes * kk, &dx))) return rc;
    if ((rc = io.outbuf(2, bytes, &dout))) return rc;
    if ((rc = fthe_reduce_kway_dev(k, c, (const uint32_t *)dx, kk, count, (uint32_t *)dout))) return rc;
    return io.back(out, dout, bytes);
}

extern "C" int fthe_scalar_mul_u64(fthe_key *k, fthe_ctx *c, const uint32_t *x, uint64_t e, size_t count, uint32_t *out) {
    if (!k || !c) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HostIO io{c}; void *dx, *dout; int rc;
    size_t bytes = count * 2 * (size_t)k->n_words * 4;
    if ((rc = io.in(0, x, bytes, &dx))) return rc;
    if ((rc = io.outbuf(2, bytes, &dout))) return rc;
    if ((rc = fthe_scalar_mul_u64_dev(k, c, (const uint32_t *)dx, e, count, (uint32_t *)dout))) return rc;
    return io.back(out, dout, bytes);
}

extern "C" int fthe_scalar_mul_words(fthe_key *k, fthe_ctx *c, const uint32_t *x, const uint32_t *e, int e_words,
                                     size_t count, uint32_t *out) {
    if (!k || !c) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    HostIO io{c}; void *dx, *dout; int rc;
    size_t bytes = count * 2 * (size_t)k->n_words * 4;
    if ((rc = io.in(0, x, bytes, &dx))) return rc;
    if ((rc = io.outbuf(2, bytes, &dout))) return rc;
    if ((rc = fthe_scalar_mul_words_dev(k, c, (const uint32_t *)dx, e, e_words, count, (uint32_t *)dout))) return rc;
    return io.back(out, dout, bytes);
}

// ---------------------------------------------------------------------------
// Codec
// ---------------------------------------------------------------------------
// Decimal wire strings on the device (fthe_dec.hip): the bytes of fthe_ct_to_decimal
// (mpz_get_str, the reference's GHEncBatch text) without the host round trip.
extern "C" int fthe_ct_to_decimal_dev(fthe_ctx *c, const uint32_t *ct, int words, size_t count, char *buf,
                                      size_t buf_len, size_t *offsets) {
    if (!c || (!ct && count) || words <= 0 || words > 128 || !offsets) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    const int nch = (int)((fthe_decimal_max_len(words) + 8) / 9);
    int rc;
    if ((rc = c->dec[0].ensure(std::max<size_t>(4, (size_t)nch * count * 4))) ||
        (rc = c->dec[1].ensure((count + 1) * 8)) || (rc = c->dec[2].ensure(std::max<size_t>(4, count * 4))))
        return rc;
    hipStream_t st = c->stream;
    HIPOK(hipEventRecord(c->ev0, st));
    uint32_t *chunks = (uint32_t *)c->dec[0].p;
    int64_t *len = (int64_t *)c->dec[1].p, *off = (int64_t *)offsets;
    int32_t *top = (int32_t *)c->dec[2].p;
    if (count && dec_launch_chunks(ct, words, count, nch, chunks, st)) return FTHE_ERR_UNSUPPORTED;
    dec_launch_len_write(chunks, count, nch, len, top, 0, nullptr, nullptr, st);
    if ((rc = exclusive_scan_i64(len, off, count + 1, c->cub_tmp, c->cub_bytes, st))) return FTHE_ERR_HIP;
    int64_t total = 0;
    HIPOK(hipMemcpyAsync(&total, off + count, 8, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    if ((size_t)total > buf_len || (!buf && total)) return FTHE_ERR_ARG;   // offsets[count]: bytes needed
    if (count) dec_launch_len_write(chunks, count, nch, len, top, 1, off, buf, st);
    HIPOK(hipEventRecord(c->ev1, st));
    c->timed = true;
    return hipGetLastError() == hipSuccess ? FTHE_OK : FTHE_ERR_HIP;
}

extern "C" int fthe_ct_from_decimal_dev(fthe_ctx *c, const char *buf, const size_t *offsets, size_t count, int words,
                                        uint32_t *ct) {
    if (!c || (!buf && count) || !offsets || words <= 0 || words > 128 || (!ct && count)) return FTHE_ERR_ARG;
    HIPOK(hipSetDevice(c->device));
    int rc;
    if ((rc = c->dec[2].ensure(4))) return rc;
    hipStream_t st = c->stream;
    int *err = (int *)c->dec[2].p;
    HIPOK(hipEventRecord(c->ev0, st));
    HIPOK(hipMemsetAsync(err, 0, 4, st));
    if (count && dec_launch_parse(buf, (const int64_t *)offsets, count, words, (int)fthe_decimal_max_len(words), ct,
                                  err, st)) return FTHE_ERR_UNSUPPORTED;
    HIPOK(hipEventRecord(c->ev1, st));
    c->timed = true;
    int h = 0;
    HIPOK(hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    return h ? FTHE_ERR_ARG : FTHE_OK;
}

extern "C" int fthe_encode_fixed_dev(fthe_ctx *c, const float *x, size_t count, uint64_t *m) {
    if (!c) return FTHE_ERR_ARG;
    if (!count) return FTHE_OK;
    HIPOK(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_encode_fixed, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, c->stream, x, count, m);
    return hipGetLastError() == hipSuccess ? FTHE_OK : FTHE_ERR_HIP;
}
extern "C" int fthe_decode_fixed_dev(fthe_ctx *c, const uint64_t *m, size_t count, float *x) {
    if (!c) return FTHE_ERR_ARG;
    if (!count) return FTHE_OK;
    HIPOK(hipSetDevice(c->device));
    hipLaunchKernelGGL(k_decode_fixed, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, c->stream, m, count, x);
    return hipGetLastError() == hipSuccess ? FTHE_OK : FTHE_ERR_HIP;
}

extern "C" int fthe_encrypt_shared(fthe_key *k, const uint64_t *m, size_t count, uint32_t *out, int flags) {
    if (!k || ((!m || !out) && count)) return FTHE_ERR_ARG;
    if (!count) return FTHE_OK;
    Coalescer *co = key_coalescer(k);
    if (!co) return FTHE_ERR_NOMEM;
    EncReq r{m, count, out, flags};
    std::unique_lock<std::mutex> lk(co->mu);
    try { co->epending.push_back(&r); } catch (...) { return FTHE_ERR_NOMEM; }
    arrived(co, co->epending, co->elast, co->elingering);
    for (;;) {
        if (r.done) return r.rc;
        if (!co->eleader) {
            co->eleader = true;
            linger(co, lk, co->epending, co->elast, co->elingering, co->elast_us);
            std::vector<EncReq *> batch;
            batch.swap(co->epending);                // includes r
            lk.unlock();
            const auto t_batch = std::chrono::steady_clock::now();
            coalesced_encrypt(k, co, batch);
            co->elast_us = us_since(t_batch);
            lk.lock();
            for (EncReq *q : batch) q->done = true;
            co->elast = batch.size() + co->epending.size();   // callers active in this round
            co->eleader = false;
            co->cv.notify_all();
            return r.rc;
        }
        co->cv.wait(lk);
    }
}

// ---------------------------------------------------------------------------
// Shared ciphertext add / scalar mul: GHPair::operator+, +=, - of the USE_HIP build
// (common.h:150-337) call these once per GHPair from FedTree's OpenMP workers
// (hist_tree_builder.cpp:574-591, 1031-1047); the key's third queue merges the concurrent
// calls into one launch per operation kind (adds together, muls per exponent).  Inputs are
// staged before any output is written, so out may alias a or b (fixes SURVEY Q11).
static void coalesced_ops_impl(fthe_key *k, Coalescer *co, const std::vector<OpReq *> &batch) {
    const size_t cw = 2 * (size_t)k->n_words;
    int rc0 = FTHE_OK;
    if (!co->octx) rc0 = fthe_ctx_create(k->device, &co->octx);
    // kinds: adds (mul == false), then one group per distinct exponent
    std::vector<std::pair<bool, uint64_t>> kinds;
    for (OpReq *r : batch) {
        std::pair<bool, uint64_t> kd{r->mul, r->mul ? r->k : 0};
        if (std::find(kinds.begin(), kinds.end(), kd) == kinds.end()) kinds.push_back(kd);
    }
    for (const auto &kd : kinds) {
        size_t tot = 0;
        for (OpReq *r : batch) if (r->mul == kd.first && (!kd.first || r->k == kd.second)) tot += r->count;
        int rc = rc0;
        if (!rc) {
            co->oa.resize(tot * cw); co->oout.resize(tot * cw);
            if (!kd.first) co->ob.resize(tot * cw);
            size_t at = 0;
            for (OpReq *r : batch) {
                if (r->mul != kd.first || (kd.first && r->k != kd.second)) continue;
                memcpy(&co->oa[at * cw], r->a, r->count * cw * 4);
                if (!kd.first) memcpy(&co->ob[at * cw], r->b, r->count * cw * 4);
                at += r->count;
            }
            rc = kd.first ? fthe_scalar_mul_u64(k, co->octx, co->oa.data(), kd.second, tot, co->oout.data())
                          : fthe_add(k, co->octx, co->oa.data(), co->ob.data(), tot, co->oout.data());
        }
        size_t at = 0;
        for (OpReq *r : batch) {
            if (r->mul != kd.first || (kd.first && r->k != kd.second)) continue;
            r->rc = rc;
            if (!rc) memcpy(r->out, &co->oout[at * cw], r->count * cw * 4);
            at += r->count;
        }
    }
    trim(co->oa); trim(co->ob); trim(co->oout);
}

static int op_shared(fthe_key *k, OpReq &r) {
    Coalescer *co = key_coalescer(k);
    if (!co) return FTHE_ERR_NOMEM;
    std::unique_lock<std::mutex> lk(co->mu);
    try { co->opending.push_back(&r); } catch (...) { return FTHE_ERR_NOMEM; }
    arrived(co, co->opending, co->olast, co->olingering);
    for (;;) {
        if (r.done) return r.rc;
        if (!co->oleader) {
            co->oleader = true;
            linger(co, lk, co->opending, co->olast, co->olingering, co->olast_us);
            std::vector<OpReq *> batch;
            batch.swap(co->opending);                // includes r
            lk.unlock();
            try {
                const auto t_batch = std::chrono::steady_clock::now();
                coalesced_ops_impl(k, co, batch);
                co->olast_us = us_since(t_batch);
            } catch (...) {
                for (OpReq *q : batch) q->rc = FTHE_ERR_NOMEM;
            }
            lk.lock();
            for (OpReq *q : batch) q->done = true;
            co->olast = batch.size() + co->opending.size();   // callers active in this round
            co->oleader = false;
            co->cv.notify_all();
            return r.rc;
        }
        co->cv.wait(lk);
    }
}

extern "C" int fthe_add_shared(fthe_key *k, const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out) {
    if (!k || ((!a || !b || !out) && count)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (!count) return FTHE_OK;
    OpReq r{false, a, b, 0, count, out};
    return op_shared(k, r);
}

extern "C" int fthe_scalar_mul_u64_shared(fthe_key *k, const uint32_t *x, uint64_t e, size_t count, uint32_t *out) {
    if (!k || ((!x || !out) && count)) return FTHE_ERR_ARG;
    if (!k->pub_ok) return FTHE_ERR_UNSUPPORTED;
    if (!count) return FTHE_OK;
    OpReq r{true, x, nullptr, e, count, out};
    return op_shared(k, r);
}
