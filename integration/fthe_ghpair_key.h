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
// assignment.  Where each runs is chosen for FedTree's per-element call sites (one operator per
// histogram member from OpenMP threads, hist_tree_builder.cpp:586-591, 1030-1036):
//   add     -> the host, one product x y mod n^2 (as Paillier_GPU::add, paillier_gpu.cu:57-61); a GPU
//              round trip per element cannot compete with ~3 us of host work.  Alias-safe.
//   encrypt -> (1 + m n) rho mod n^2 on the host, rho = r^n mod n^2 drawn from the key's randomizer
//              pool; the engine refills the pool in bulk (Enc(0) batches, fresh uniform r per row,
//              the key holder's CRT path or the public formula) on a background thread, so a
//              promotion (common.h:156-160) costs one host product instead of an
//              exponentiation.  Every pooled rho is used exactly once.
//   mul     -> a host mpz_powm for exponents of at most 64 bits (operator-'s 2^64 - 1), as the reference GPU
//              build's Paillier_GPU::mul (paillier_gpu.cu:65-67); FTHE_SHIM_MUL_ENGINE=1 sends them to
//              fthe_scalar_mul_u64_shared instead (A/B); fthe_scalar_mul_words for exponents above 64 bits.
// The batch call sites go to the engine directly (Paillier_HIP's helpers, include/fthe.h).
//
// Copies are free of atomics: a key is an interned, immutable host cell (n, n^2, g limbs; the pool),
// looked up by n once at bind time, and every Paillier_HIP_Pub holds a plain pointer to it.  The
// public fields are read-only GMP views (mpz_roinit_n) of the cell's limbs, so GHPair's key copies
// (common.h:170, 190, 384) copy three structs instead of three big integers.  Cells live for the
// process; their pools are freed when the last Paillier_HIP owning the key goes away.
//
// The maintainer's change to common.h is the member type and the branch condition:
//     #if defined(USE_HIP)
//         #include "fthe_ghpair_key.h"
//         typedef Paillier_HIP_Pub GHPairKey;
//     #elif defined(USE_CUDA) ... typedef Paillier_GMP GHPairKey;
//     struct GHPair { ... GHPairKey paillier; ... }   and `#ifdef USE_CUDA` -> `#if defined(USE_CUDA) || defined(USE_HIP)`
// so the operator bodies compile unchanged.
#pragma once
#include <gmp.h>
// The key fields are read-only views (mpz_roinit_n, alloc 0) of the cell's limbs.  A caller that writes one
// relies on GMP allocating afresh for an alloc-0 destination, which GMP guarantees from 6.2 on; older
// releases realloc the view's pointer (the cell's std::vector storage) and corrupt the heap.
#if (__GNU_MP_VERSION * 100 + __GNU_MP_VERSION_MINOR) < 602
#error "fthe_ghpair_key.h needs GMP >= 6.2 (writes to mpz_roinit_n views)"
#endif
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
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
// The devices the drop-in's batch calls shard over (integration/paillier_hip.h): FTHE_DEVICES, a comma list
// ("0,1,2,3"; a device may repeat -- "0,0" runs two shards on device 0, the tests' two-context configuration),
// else FTHE_DEVICE alone, else every visible device (fthe_device_count).  The first is the primary device: the
// keys of keygen / operator=, the GHPair operators' engine work and the randomizer pool live there.
inline std::vector<int> parse_devices(const char *e) {
    std::vector<int> d;
    for (const char *p = e; p && *p;) {
        char *end = nullptr;
        const long x = std::strtol(p, &end, 10);
        if (end == p) throw std::runtime_error(std::string("FTHE_DEVICES: not a device list: ") + e);
        d.push_back((int)x);
        p = end;
        while (*p == ',' || *p == ' ') p++;
    }
    return d;
}
inline const std::vector<int> &shard_devices() {
    static const std::vector<int> v = [] {
        std::vector<int> d = parse_devices(std::getenv("FTHE_DEVICES"));
        if (d.empty()) {
            if (const char *e = std::getenv("FTHE_DEVICE")) d.push_back(std::atoi(e));
            else for (int i = 0, n = fthe_device_count(); i < n; i++) d.push_back(i);
        }
        if (d.empty()) d.push_back(0);          // no device: the first context creation fails loudly
        return d;
    }();
    return v;
}
inline int primary_device() { return shard_devices()[0]; }
// The calling thread's engine context on device d, one per (thread, device), created on first use (the boundary
// is entered from OpenMP regions, FLtrainer.cpp:275-306; a context serves one host thread at a time).
inline fthe_ctx *ctx_on(int d) {
    static thread_local std::vector<std::pair<int, fthe_ctx *>> cs;
    for (auto &x : cs) if (x.first == d) return x.second;
    fthe_ctx *c = nullptr;
    check(fthe_ctx_create(d, &c), "fthe_ctx_create");
    cs.emplace_back(d, c);
    return c;
}
// ... on the primary device.
inline fthe_ctx *thread_ctx() { return ctx_on(primary_device()); }
// mpz <-> little-endian u32 words (paillier_gpu.cu:7,18 order: mpz_export / mpz_import with order -1, size 4).
// On a little-endian host with 64-bit limbs and no nails those words ARE the limbs' bytes, so the batch
// marshalling copies limbs directly (memcpy + size) instead of GMP's generic word loop, which runs ~1.2M
// ciphertexts/s per core at 4096 bits -- short of feeding 8 GPUs from one host (integration/marshal_rate.cpp,
// DESIGN 6).  Same values either way (tests: integration/host_ops_test.cpp round trips).
#if defined(__BYTE_ORDER__) && __BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__ && GMP_LIMB_BITS == 64 && GMP_NAIL_BITS == 0
#define FTHE_SHIM_LIMB_COPY 1
#endif
inline void to_words(const mpz_t x, uint32_t *w, int nw) {
    if (mpz_sgn(x) < 0) throw std::runtime_error("negative operand");
    if (mpz_sizeinbase(x, 2) > (size_t)nw * 32) throw std::runtime_error("operand does not fit");
#ifdef FTHE_SHIM_LIMB_COPY
    const size_t nb = mpz_size(x) * sizeof(mp_limb_t), cap = (size_t)nw * 4;
    const size_t cp = std::min(nb, cap);                 // the top limb may hold only the row's last word
    if (cp) std::memcpy(w, mpz_limbs_read(x), cp);
    if (cp < cap) std::memset(reinterpret_cast<char *>(w) + cp, 0, cap - cp);
#else
    size_t cnt = 0;
    for (int i = 0; i < nw; i++) w[i] = 0;
    mpz_export(w, &cnt, -1, 4, 0, 0, x);
#endif
}
inline void from_words(mpz_t x, const uint32_t *w, int nw) {
#ifdef FTHE_SHIM_LIMB_COPY
    int top = nw;
    while (top > 0 && w[top - 1] == 0) top--;
    const mp_size_t nl = (top + 1) / 2;
    if (nl == 0) { mpz_set_ui(x, 0); return; }
    mp_limb_t *d = mpz_limbs_write(x, nl);
    d[nl - 1] = 0;                                      // an odd word count leaves the top limb's high half 0
    std::memcpy(d, w, (size_t)top * 4);
    mpz_limbs_finish(x, nl);
#else
    mpz_import(x, (size_t)nw, -1, 4, 0, 0, w);
#endif
}
inline size_t words_of(const mpz_t x) { return (mpz_sizeinbase(x, 2) + 31) / 32; }

// Scratch integers of the calling thread (the operators run from OpenMP workers).
struct Scratch {
    mpz_t t, u, v;
    Scratch() { mpz_init2(t, 8448); mpz_init2(u, 4352); mpz_init2(v, 4352); }
    ~Scratch() { mpz_clear(t); mpz_clear(u); mpz_clear(v); }
};
inline Scratch &scratch() { static thread_local Scratch s; return s; }

class KeyCell;
void schedule_refill(KeyCell *c);

// The host side of one public key n, shared by every Paillier_HIP_Pub bound to it: immutable limbs of
// n, n^2 and g = n + 1 with read-only GMP views of them, the engine keys that can draw randomizers
// for it, and the randomizer pool.
class KeyCell {
public:
    explicit KeyCell(const mpz_t nn) {
        mpz_t t;
        mpz_init(t);
        set(nl_, n, nn);
        mpz_mul(t, nn, nn);
        set(n2l_, n2, t);
        mpz_add_ui(t, nn, 1);
        set(gl_, g, t);
        mpz_clear(t);
        nw = (int)words_of(n);
    }
    mpz_t n, n2, g;       // read-only views (mpz_roinit_n): never written, never cleared
    int nw = 0;           // u32 words of n; ciphertext rows have 2 nw

    // -- engine keys able to draw r^n mod n^2 for this n (weak: the Paillier_HIP objects own them) --
    void attach(const std::shared_ptr<fthe_key> &k) {
        std::lock_guard<std::mutex> g_(emu_);
        if (fthe_key_has_private(k.get())) priv_ = k; else pub_ = k;
    }
    // The key the pool and engine-side operators use: the private one (CRT) while any holder lives,
    // else a public one, else a public-only key made from n on first need (kept for the process).
    std::shared_ptr<fthe_key> engine() {
        std::lock_guard<std::mutex> g_(emu_);
        if (auto k = priv_.lock()) return k;
        if (auto k = pub_.lock()) return k;
        if (!own_) {
            std::vector<uint32_t> w(nw);
            to_words(n, w.data(), nw);
            fthe_key *k = nullptr;
            check(fthe_key_from_n(thread_ctx(), w.data(), nw, &k), "key_from_n");
            own_.reset(k, [](fthe_key *p) { fthe_key_destroy(p); });
        }
        return own_;
    }

    // -- owners: Paillier_HIP objects holding this key; the pool is released with the last one --
    void retain() {
        if (owners_.fetch_add(1) == 0) prefill();
    }
    void release() {
        if (owners_.fetch_sub(1) != 1) return;
        std::lock_guard<std::mutex> lk(pm_);
        batches_.clear();
        avail_ = 0;
    }

    // -- randomizer pool: rows rho = r^n mod n^2 (Enc(0) under a fresh uniform r), FIFO --
    // Copies the next unused row into `row` (2 nw words).  trace (tests): the batch's rng seed and
    // the row's index in that batch.
    void draw(uint32_t *row, uint64_t *seed = nullptr, uint64_t *index = nullptr) {
        std::unique_lock<std::mutex> lk(pm_);
        bool waited = false;
        while (avail_ == 0) {
            if (err_) { auto e = err_; err_ = nullptr; std::rethrow_exception(e); }
            if (!refilling_) { refilling_ = true; schedule_refill(this); }
            waited = true;
            waiters_++;
            pcv_.wait(lk);
            waiters_--;
        }
        if (waited && !fixed_batch_ && batch_ < kMaxBatch) batch_ *= 2;   // ran dry: refill in larger batches
        Batch &b = batches_.front();
        std::memcpy(row, &b.rows[b.used * 2 * (size_t)nw], 2 * (size_t)nw * sizeof(uint32_t));
        if (seed) *seed = b.seed;
        if (index) *index = b.used;
        b.used++;
        avail_--;
        if (b.used == b.count) batches_.pop_front();
        if (avail_ <= batch_ / 2 && !refilling_) { refilling_ = true; schedule_refill(this); }
    }
    // Test hook: deterministic batches (seed0 + k for the k-th batch from now on) of a fixed size.
    // Drops what the pool holds and waits for an in-flight refill first.
    void set_test_seed(uint64_t seed0, size_t batch) {
        std::unique_lock<std::mutex> lk(pm_);
        pcv_.wait(lk, [&] { return !refilling_; });
        batches_.clear();
        avail_ = 0;
        test_seed_ = seed0;
        test_batches_ = 0;
        batch_ = std::max<size_t>(1, batch);
        fixed_batch_ = true;
    }
    size_t pooled() { std::lock_guard<std::mutex> lk(pm_); return avail_; }

    // Runs on the refill worker: one engine batch of Enc(0), then hands it to the waiting drawers.
    void refill() {
        size_t cnt;
        uint64_t seed = 0;
        {
            std::lock_guard<std::mutex> lk(pm_);
            cnt = (owners_.load() > 0 || fixed_batch_) ? batch_ : std::min<size_t>(batch_, 1024);
            if (test_seed_) seed = test_seed_ + test_batches_++;
        }
        Batch b;
        b.count = cnt;
        b.seed = seed;
        try {
            auto k = engine();
            b.rows.resize(cnt * 2 * (size_t)nw);
            std::vector<uint64_t> zero(cnt, 0);
            check(fthe_encrypt_u64(k.get(), thread_ctx(), zero.data(), cnt, nullptr, 0, seed, b.rows.data(),
                                   FTHE_ENC_DEFAULT), "randomizer pool");
        } catch (...) {
            std::lock_guard<std::mutex> lk(pm_);
            err_ = std::current_exception();
            refilling_ = false;
            pcv_.notify_all();
            return;
        }
        std::lock_guard<std::mutex> lk(pm_);
        refilling_ = false;
        if (owners_.load() > 0 || waiters_ > 0 || fixed_batch_) {   // an ownerless cell keeps a batch for a waiter only
            avail_ += cnt;
            batches_.push_back(std::move(b));
        }
        pcv_.notify_all();
    }

private:
    struct Batch {
        std::vector<uint32_t> rows;
        size_t count = 0, used = 0;
        uint64_t seed = 0;
    };
    static constexpr size_t kMaxBatch = 1 << 18;
    static void set(std::vector<mp_limb_t> &l, mpz_t view, const mpz_t x) {
        l.assign(std::max<size_t>(1, mpz_size(x)), 0);
        mpz_export(l.data(), nullptr, -1, sizeof(mp_limb_t), 0, 0, x);
        mpz_roinit_n(view, l.data(), (mp_size_t)mpz_size(x));
    }
    void prefill() {
        std::lock_guard<std::mutex> lk(pm_);
        if (avail_ == 0 && !refilling_) { refilling_ = true; schedule_refill(this); }
    }
    std::vector<mp_limb_t> nl_, n2l_, gl_;
    std::mutex emu_;
    std::weak_ptr<fthe_key> priv_, pub_;
    std::shared_ptr<fthe_key> own_;
    std::atomic<int> owners_{0};
    std::mutex pm_;
    std::condition_variable pcv_;
    std::deque<Batch> batches_;
    size_t avail_ = 0, batch_ = 1 << 14;
    int waiters_ = 0;
    bool refilling_ = false, fixed_batch_ = false;
    uint64_t test_seed_ = 0, test_batches_ = 0;
    std::exception_ptr err_;
};

// Cells by n (one per distinct public key in the process; looked up at bind time only).
inline KeyCell *intern(const mpz_t n) {
    static std::mutex m;
    static std::map<std::vector<mp_limb_t>, KeyCell *> *cells = new std::map<std::vector<mp_limb_t>, KeyCell *>();
    std::vector<mp_limb_t> id(std::max<size_t>(1, mpz_size(n)), 0);
    mpz_export(id.data(), nullptr, -1, sizeof(mp_limb_t), 0, 0, n);
    std::lock_guard<std::mutex> lk(m);
    KeyCell *&c = (*cells)[id];
    if (!c) c = new KeyCell(n);
    return c;
}

// The process's pool refill worker: one thread, one engine context, jobs in arrival order.  Joined at
// exit (a refill in flight finishes first) before the HIP runtime tears down.
class RefillWorker {
public:
    static RefillWorker &get() {
        static RefillWorker *w = [] {
            auto *p = new RefillWorker();
            std::atexit([] { get().stop(); });
            return p;
        }();
        return *w;
    }
    void push(KeyCell *c) {
        std::lock_guard<std::mutex> lk(m_);
        if (stopped_) return;
        q_.push_back(c);
        if (!th_.joinable()) th_ = std::thread([this] { loop(); });
        cv_.notify_one();
    }
    void stop() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stopped_ = true;
            cv_.notify_one();
        }
        if (th_.joinable()) th_.join();
    }

private:
    void loop() {
        for (;;) {
            KeyCell *c;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stopped_ || !q_.empty(); });
                if (stopped_) return;
                c = q_.front();
                q_.pop_front();
            }
            c->refill();
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<KeyCell *> q_;
    std::thread th_;
    bool stopped_ = false;
};
inline void schedule_refill(KeyCell *c) { RefillWorker::get().push(c); }
}  // namespace fthe_shim

// The engine key shared by the Paillier_HIP objects that own it.  Keys are immutable in the engine and
// usable from any thread.
using fthe_key_ref = std::shared_ptr<fthe_key>;
inline fthe_key_ref fthe_key_adopt(fthe_key *k) { return fthe_key_ref(k, [](fthe_key *p) { fthe_key_destroy(p); }); }

class Paillier_HIP_Pub {
public:
    Paillier_HIP_Pub() { mpz_init(n); mpz_init(n_square); mpz_init(generator); }
    Paillier_HIP_Pub(const Paillier_HIP_Pub &o) : Paillier_HIP_Pub() { *this = o; }
    ~Paillier_HIP_Pub() { clear_owned(); }
    // Paillier_GMP::operator= (paillier_gmp.h:12-21): the public part only -- here a pointer to the
    // shared cell and views of its limbs, no big-integer copies and no reference counting.
    Paillier_HIP_Pub &operator=(const Paillier_HIP_Pub &o) {
        if (this == &o) return *this;
        if (cell_ != o.cell_ || owns_fields()) {
            drop_fields();
            if (o.cell_) view_fields(o.cell_);
            else { mpz_init(n); mpz_init(n_square); mpz_init(generator); }
        }
        cell_ = o.cell_;
        key_length = o.key_length;
#ifdef FTHE_REFERENCE_SHARED_R
        shared_r_ = o.shared_r_;
#endif
        return *this;
    }

    // Bind to an engine key (Paillier_HIP::keygen / key_from_primes / operator=).
    void bind(const fthe_key_ref &k, uint32_t keyLength) {
        const int nw = fthe_key_n_words(k.get());
        std::vector<uint32_t> w(nw);
        fthe_shim::check(fthe_key_export(k.get(), w.data(), nullptr, nullptr, nullptr, nullptr), "export");
        mpz_t nn;
        mpz_init(nn);
        fthe_shim::from_words(nn, w.data(), nw);
        bind_n(nn, keyLength);
        mpz_clear(nn);
        cell_->attach(k);
    }
    // Host-only binding to a public n (no engine key yet: add works at once; encrypt / mul make a
    // public engine key from n on first use).
    void bind_n(const mpz_t nn, uint32_t keyLength) {
        if (mpz_sgn(nn) <= 0) throw std::runtime_error("bind_n: n must be positive");
        drop_fields();
        cell_ = fthe_shim::intern(nn);
        view_fields(cell_);
        key_length = keyLength;
    }
    fthe_shim::KeyCell *cell() const { return cell_; }
    int n_words() const { return need()->nw; }

    // Paillier_GMP::encrypt (paillier_gmp.cpp:37-73): r <- g^m r'^n mod n^2 with a fresh uniform r'.
    // GHPair::homo_encrypt passes the codec value (common.h:81-88): m < 2^64, computed on the host as
    // (1 + m n) rho = rho + n ((m rho) mod n)  (mod n^2) with rho = r'^n mod n^2 from the key's pool.
    // r must be initialised, as every GHPair operand is.
    void encrypt(mpz_t &r, const mpz_t &message) const {
        fthe_shim::KeyCell *c = need();
        if (mpz_sgn(message) < 0) throw std::runtime_error("encrypt: negative plaintext");
        const int cw = 2 * c->nw;
#ifdef FTHE_REFERENCE_SHARED_R
        if (!shared_r_.empty()) {                 // reference GMP / GPU semantics: one fixed r
            const int mw = std::max<int>(1, (int)fthe_shim::words_of(message));
            std::vector<uint32_t> m(mw), ct(cw);
            fthe_shim::to_words(message, m.data(), mw);
            auto k = c->engine();
            fthe_shim::check(fthe_encrypt_words(k.get(), fthe_shim::thread_ctx(), m.data(), mw, 1, shared_r_.data(),
                                                c->nw, 0, ct.data(), FTHE_ENC_PUBLIC), "encrypt");
            fthe_shim::from_words(r, ct.data(), cw);
            return;
        }
#endif
        if (mpz_sizeinbase(message, 2) > 64) {    // Paillier::encrypt(ZZ) of any size (paillier.cpp:122)
            const int mw = (int)fthe_shim::words_of(message);
            std::vector<uint32_t> m(mw), ct(cw);
            fthe_shim::to_words(message, m.data(), mw);
            auto k = c->engine();
            fthe_shim::check(fthe_encrypt_words(k.get(), fthe_shim::thread_ctx(), m.data(), mw, 1, nullptr, 0, 0,
                                                ct.data(), FTHE_ENC_DEFAULT), "encrypt");
            fthe_shim::from_words(r, ct.data(), cw);
            return;
        }
        encrypt_pooled(r, message, nullptr, nullptr);
    }
    // encrypt() of a plaintext below 2^64 from the pool, reporting which pooled row it used (tests).
    void encrypt_pooled(mpz_t &r, const mpz_t &message, uint64_t *seed, uint64_t *index) const {
        fthe_shim::KeyCell *c = need();
        uint32_t stack[256];
        std::vector<uint32_t> heap;
        uint32_t *row = stack;
        if (2 * c->nw > 256) { heap.resize(2 * (size_t)c->nw); row = heap.data(); }
        c->draw(row, seed, index);
        fthe_shim::Scratch &s = fthe_shim::scratch();
        fthe_shim::from_words(s.t, row, 2 * c->nw);                 // rho
        if (mpz_sgn(message) == 0) { mpz_set(r, s.t); return; }    // Enc(0) = rho (every Q10 promotion of 0)
        mpz_mul(s.u, s.t, message);                                 // m rho
        mpz_tdiv_r(s.u, s.u, c->n);
        mpz_mul(s.u, s.u, c->n);                                    // n ((m rho) mod n) < n^2
        mpz_add(r, s.t, s.u);
        if (mpz_cmp(r, c->n2) >= 0) mpz_sub(r, r, c->n2);
    }

    // Paillier_GMP::add (paillier_gmp.cpp:16-21): r <- x y mod n^2, on the host.  Alias-safe: the product
    // is formed in thread scratch before r is written, so add(s, s, c) (common.h:207, 221, 229) gives
    // s c, not 0.  r must be initialised, as every GHPair operand is (common.h:347-386).
    void add(mpz_t &r, const mpz_t &x, const mpz_t &y) const {
        fthe_shim::KeyCell *c = need();
        fthe_shim::Scratch &s = fthe_shim::scratch();
        mpz_mul(s.t, x, y);
        mpz_mod(r, s.t, c->n2);
    }

    // Paillier_GMP::mul (paillier_gmp.cpp:24-28): r <- x^y mod n^2.  Like the reference it
    // initialises r: operator- passes an uninitialised mpz_t (common.h:270-272).  Alias-safe.
    void mul(mpz_t &r, const mpz_t &x, const mpz_t &y) const {
        mpz_init(r);
        mul_into(r, x, y);
    }
    // The same into an initialised r (Paillier_GPU::mul's contract, paillier_gpu.cu:65-67).  One element with
    // an exponent of at most 64 bits -- operator-'s 2^64 - 1 (common.h:253-337) from the sibling subtraction
    // and missing_gh loops (hist_tree_builder.cpp:672-680, 715-726) -- is a host mpz_powm, as in the
    // reference's GPU build: 64 squarings of 4096 bits take ~0.2 ms on one core, and a GPU queue round trip per
    // element costs more than that and serialises the OpenMP callers (bench
    // secondary.histogram_loop_unchanged_callers.*.sub).  FTHE_SHIM_MUL_ENGINE=1 sends them to the engine's
    // coalescing queue instead (the round-3 behaviour, kept for the A/B).  Batches of subtractions go to the
    // engine through Paillier_HIP::subtract (fthe_sub).  Larger exponents run on the engine.
    void mul_into(mpz_ptr r, const mpz_t &x, const mpz_t &y) const {
        fthe_shim::KeyCell *c = need();
        const int cw = 2 * c->nw;
        if (mpz_sgn(y) < 0) throw std::runtime_error("mul: negative exponent");
        static const bool on_engine = [] { const char *e = std::getenv("FTHE_SHIM_MUL_ENGINE"); return e && *e == '1'; }();
        fthe_shim::Scratch &s = fthe_shim::scratch();
        if (!on_engine && mpz_sizeinbase(y, 2) <= 64) {
            mpz_powm(s.v, x, y, c->n2);                             // x reduced mod n^2 first, as the reference's
            mpz_set(r, s.v);
            return;
        }
        std::vector<uint32_t> a(cw), o(cw);
        mpz_mod(s.v, x, c->n2);                                     // the reference's powm reduces x first
        fthe_shim::to_words(s.v, a.data(), cw);
        auto k = c->engine();
        if (mpz_sizeinbase(y, 2) <= 64) {
            uint64_t e = 0;
            mpz_export(&e, nullptr, -1, 8, 0, 0, y);
            fthe_shim::check(fthe_scalar_mul_u64_shared(k.get(), a.data(), e, 1, o.data()), "mul");
        } else {
            std::vector<uint32_t> e(fthe_shim::words_of(y));
            fthe_shim::to_words(y, e.data(), (int)e.size());
            fthe_shim::check(fthe_scalar_mul_words(k.get(), fthe_shim::thread_ctx(), a.data(), e.data(), (int)e.size(),
                                                   1, o.data()), "mul");
        }
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
    fthe_shim::KeyCell *cell_ = nullptr;
#ifdef FTHE_REFERENCE_SHARED_R
    std::vector<uint32_t> shared_r_;
#endif
    fthe_shim::KeyCell *need() const {
        if (!cell_) throw std::runtime_error("Paillier_HIP_Pub: no key (keygen / assignment from a keyed object first)");
        return cell_;
    }
    // A field written by a caller (mpz_set on a view) holds its own allocation: GMP allocates afresh
    // for a view (alloc 0), so the cell's limbs are never touched; such a field is cleared here.
    bool owns_fields() const { return n->_mp_alloc || n_square->_mp_alloc || generator->_mp_alloc; }
    void clear_owned() {
        for (mpz_ptr f : {n, n_square, generator})
            if (f->_mp_alloc) mpz_clear(f);
    }
    void drop_fields() {
        clear_owned();
        mpz_init(n); mpz_init(n_square); mpz_init(generator);
    }
    void view_fields(fthe_shim::KeyCell *c) {
        *n = *c->n;
        *n_square = *c->n2;
        *generator = *c->g;
    }
};
