// paillier_hip.h -- drop-in HE engine class for a FedTree build with USE_HIP.
//
// Copy to include/FedTree/Encryption/paillier_hip.h in a FedTree tree and select
// it where the reference selects Paillier_GPU (server.h:47-51, party.h:181-185,
// common.h:43-61 use USE_CUDA; add the same branches for USE_HIP).  The class has
// the member functions and fields of Paillier_GPU (paillier_gpu.h:28-94), so the
// callers -- Server::{homo_init, encrypt_gh_pairs, decrypt_gh_pairs, decrypt_gh}
// (server.h:58-135), Party::encrypt_histogram (party.h:118-142) and GHPair's
// operators through paillier_cpu (common.h:150-337) -- compile unchanged.
//
// Everything is computed by libfthe.so through the C ABI (include/fthe.h).
// Differences from Paillier_GPU, all deliberate:
//   * a fresh uniform r per ciphertext (device ChaCha20) instead of one shared,
//     unseeded-MT r per batch (paillier_gpu.cu:262-272);
//   * any key size up to Paillier-2048 with CRT on the key holder, instead of a
//     fixed 512-bit n (BITS=1024, paillier_gpu.h:13);
//   * add() is alias-safe; errors throw std::runtime_error instead of
//     exit(1) / CHECK aborts.
#pragma once
#include <gmp.h>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fthe.h"
#include "fthe_ghpair_key.h"
#include "FedTree/syncarray.h"
#include "FedTree/common.h"

namespace fthe_shim {
// The per-element mpz marshalling of a large batch on several host threads (a few hundred ns
// per ciphertext; at the engine's rates it would otherwise dominate a batch call).  Small batches
// stay on the calling thread, which may itself be one of FedTree's OpenMP workers.
template <class F>
inline void parallel_for(size_t n, F f, unsigned cap = 16) {
    const size_t grain = 1 << 16;
    unsigned nt = std::min<unsigned>(std::max(1u, cap), std::max(1u, std::thread::hardware_concurrency()));
    if (n < 2 * grain || nt < 2) { f(0, n); return; }
    nt = (unsigned)std::min<size_t>(nt, n / grain);
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(nt);                // a worker's exception resurfaces here
    const size_t per = (n + nt - 1) / nt;
    for (unsigned t = 1; t < nt; t++) {
        const size_t b = t * per, e = std::min(n, b + per);
        if (b < e) th.emplace_back([=, &f, &err] { try { f(b, e); } catch (...) { err[t] = std::current_exception(); } });
    }
    try { f(0, std::min(n, per)); } catch (...) { err[0] = std::current_exception(); }
    for (auto &x : th) x.join();
    for (auto &e : err) if (e) std::rethrow_exception(e);
}
// Page-locked row buffers (fthe_host_alloc) for the batch calls, which then DMA straight from / into them (no
// pinned staging copy, no page faults on a fresh multi-GB vector).  A process-wide pool, not per thread: a
// lease takes the smallest free buffer that fits (or pins a new one) and returns it when the call ends; free
// buffers beyond FTHE_SHIM_PINNED_CACHE_MB (default 4096) are unpinned at once, so many OpenMP or server
// threads cannot accumulate page-locked memory, and pinning is still paid once for a steady batch size.  The
// pool is emptied by an atexit handler registered at the first pin -- after the HIP runtime's own
// initialisation, so it runs before the runtime tears down.
class PinnedPool {
public:
    static PinnedPool &get() {
        static PinnedPool *p = new PinnedPool();          // never destroyed: the atexit handler empties it
        return *p;
    }
    void *acquire(size_t bytes) {
        {
            std::lock_guard<std::mutex> lk(m_);
            auto best = free_.end();
            for (auto it = free_.begin(); it != free_.end(); ++it)
                if (it->second >= bytes && (best == free_.end() || it->second < best->second)) best = it;
            if (best != free_.end()) {
                void *q = best->first;
                cached_ -= best->second;
                size_[q] = best->second;
                free_.erase(best);
                return q;
            }
        }
        void *q = nullptr;
        check(fthe_host_alloc(bytes, &q), "host_alloc");
        std::lock_guard<std::mutex> lk(m_);
        if (!hooked_) { hooked_ = true; std::atexit([] { PinnedPool::get().drain(0); }); }
        size_[q] = bytes;
        return q;
    }
    void release(void *q) {
        if (!q) return;
        std::vector<void *> unpin;
        {
            std::lock_guard<std::mutex> lk(m_);
            auto it = size_.find(q);
            if (it == size_.end()) return;
            free_.emplace_back(q, it->second);
            cached_ += it->second;
            size_.erase(it);
            unpin = trim(cap_);
        }
        unpin_all(unpin);
    }
    void drain(size_t keep) {
        std::vector<void *> unpin;
        { std::lock_guard<std::mutex> lk(m_); unpin = trim(keep); }
        unpin_all(unpin);
    }
    size_t cached_bytes() { std::lock_guard<std::mutex> lk(m_); return cached_; }

private:
    PinnedPool() {
        const char *e = std::getenv("FTHE_SHIM_PINNED_CACHE_MB");
        cap_ = (size_t)(e ? std::atoll(e) : 4096) << 20;
    }
    // Takes the largest free buffers out of the pool until at most `keep` bytes stay cached (under m_) and
    // returns them; the caller unpins them after releasing m_ -- hipHostFree synchronises the device, and
    // other threads' acquire / release must not wait behind it.
    std::vector<void *> trim(size_t keep) {
        std::vector<void *> out;
        while (cached_ > keep && !free_.empty()) {
            auto big = std::max_element(free_.begin(), free_.end(),
                                        [](const auto &a, const auto &b) { return a.second < b.second; });
            out.push_back(big->first);
            cached_ -= big->second;
            free_.erase(big);
        }
        return out;
    }
    static void unpin_all(const std::vector<void *> &v) { for (void *p : v) fthe_host_free(p); }
    std::mutex m_;
    std::vector<std::pair<void *, size_t>> free_;
    std::map<void *, size_t> size_;
    size_t cached_ = 0, cap_ = 0;
    bool hooked_ = false;
};
// One call's page-locked buffer of count T (returned to the pool when the lease ends).
template <class T>
struct Pinned {
    explicit Pinned(size_t count) : p(static_cast<T *>(PinnedPool::get().acquire(std::max<size_t>(1, count) * sizeof(T)))) {}
    ~Pinned() { PinnedPool::get().release(p); }
    Pinned(const Pinned &) = delete;
    Pinned &operator=(const Pinned &) = delete;
    T *get() const { return p; }
    T *p;
};
// codec of common.h:81-86 and paillier_gpu.cu:487
inline uint64_t encode(float_type v) { long l = (long)(v * 1e6); return (uint64_t)l; }
inline float_type decode(uint64_t m) { long l = (long)m; return (float_type)l / 1e6; }

// ---- multi-device sharding of the batch calls ----------------------------------------------------------------
// Ciphertexts are independent, so a batch of rows splits into contiguous shards, one per entry of
// shard_devices() (north_star: batches "shard trivially across the 8 GPUs", per-GPU streams, no collective).
// shard_plan: [lo, hi) of each shard for `rows` rows over at most `slots` shards of at least `min_rows` rows
// (fewer shards for a small batch; balanced to +-1 row).  FTHE_SHARD_ROWS sets min_rows (default 8192).
inline size_t shard_min_rows() {
    static const size_t v = [] {
        const char *e = std::getenv("FTHE_SHARD_ROWS");
        const long long x = e ? std::atoll(e) : 8192;
        return (size_t)std::max(1LL, x);
    }();
    return v;
}
inline std::vector<std::pair<size_t, size_t>> shard_plan(size_t rows, size_t slots, size_t min_rows) {
    const size_t ns = std::max<size_t>(1, std::min(slots, rows / std::max<size_t>(1, min_rows)));
    std::vector<std::pair<size_t, size_t>> v;
    for (size_t i = 0; i < ns; i++) v.emplace_back(rows / ns * i + std::min(i, rows % ns),
                                                     rows / ns * (i + 1) + std::min(i + 1, rows % ns));
    return v;
}
// The same for segmented products: contiguous segment ranges of about equal member counts (ptr: nseg + 1 CSR
// offsets), so each shard does about the same number of products.
inline std::vector<std::pair<size_t, size_t>> shard_plan_segments(const int64_t *ptr, size_t nseg, size_t slots,
                                                                  size_t min_members) {
    const size_t tot = (size_t)(ptr[nseg] - ptr[0]);
    const size_t ns = std::max<size_t>(1, std::min({slots, nseg, tot / std::max<size_t>(1, min_members)}));
    std::vector<std::pair<size_t, size_t>> v;
    size_t s = 0;
    for (size_t i = 0; i < ns; i++) {
        size_t e = s;
        if (i + 1 == ns) e = nseg;
        else {
            const int64_t goal = ptr[0] + (int64_t)(tot * (i + 1) / ns);
            while (e < nseg && ptr[e] < goal) e++;          // first boundary at or past the goal
            e = std::max(e, s + 1);
            e = std::min(e, nseg - (ns - 1 - i));             // leave a segment for every later shard
        }
        v.emplace_back(s, e);
        s = e;
    }
    return v;
}
// One worker thread per shard slot beyond the first, each with its own engine context on its device (the
// calling thread runs slot 0 on its own context on the primary device).  Jobs of one slot run in arrival order;
// concurrent callers (FedTree's OpenMP threads) queue on the workers.  Joined at exit before the HIP runtime
// tears down (the pool starts after it), like the randomizer pool's worker.
class ShardPool {
public:
    static ShardPool &get() {
        static ShardPool *p = [] {
            auto *q = new ShardPool();
            std::atexit([] { get().stop(); });
            return q;
        }();
        return *p;
    }
    // f(slot, ctx) for slots 0 .. n-1 concurrently; returns when all are done, rethrowing the first error.
    void run(size_t n, const std::function<void(size_t, fthe_ctx *)> &f) {
        const std::vector<int> &devs = shard_devices();
        if (n > devs.size()) throw std::runtime_error("ShardPool: more shards than devices");
        struct Join { std::mutex m; std::condition_variable cv; size_t left; std::vector<std::exception_ptr> err; } j;
        j.left = n - 1;
        j.err.resize(n);
        size_t queued = 1;
        try {
            for (; queued < n; queued++)
                worker(queued).push([&j, &f, i = queued, d = devs[queued]] {
                    try { f(i, ctx_on(d)); } catch (...) { j.err[i] = std::current_exception(); }
                    std::lock_guard<std::mutex> lk(j.m);
                    if (--j.left == 0) j.cv.notify_all();
                });
        } catch (...) {
            // a push failed (the pool is stopping at exit): the jobs already queued still reference j and f, so
            // wait for them before this frame unwinds; the shards never queued report the error
            j.err[0] = std::current_exception();
            std::unique_lock<std::mutex> lk(j.m);
            j.left -= n - queued;
            j.cv.wait(lk, [&] { return j.left == 0; });
            std::rethrow_exception(j.err[0]);
        }
        try { f(0, ctx_on(devs[0])); } catch (...) { j.err[0] = std::current_exception(); }
        {
            std::unique_lock<std::mutex> lk(j.m);
            j.cv.wait(lk, [&] { return j.left == 0; });
        }
        for (auto &e : j.err) if (e) std::rethrow_exception(e);
    }

private:
    struct Worker {
        std::mutex m;
        std::condition_variable cv;
        std::deque<std::function<void()>> q;
        bool stopped = false;
        std::thread th;
        void push(std::function<void()> job) {
            std::lock_guard<std::mutex> lk(m);
            if (stopped) throw std::runtime_error("ShardPool: stopped");
            q.push_back(std::move(job));
            cv.notify_one();
        }
        void loop() {
            for (;;) {
                std::function<void()> job;
                {
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [&] { return stopped || !q.empty(); });
                    if (q.empty()) return;                 // stopped and drained
                    job = std::move(q.front());
                    q.pop_front();
                }
                job();
            }
        }
    };
    Worker &worker(size_t i) {
        std::lock_guard<std::mutex> lk(m_);
        if (w_.size() <= i) w_.resize(i + 1);
        if (!w_[i]) {
            w_[i].reset(new Worker());
            Worker *w = w_[i].get();
            w->th = std::thread([w] { w->loop(); });
        }
        return *w_[i];
    }
    void stop() {
        std::lock_guard<std::mutex> lk(m_);
        for (auto &w : w_) {
            if (!w) continue;
            { std::lock_guard<std::mutex> wl(w->m); w->stopped = true; w->cv.notify_one(); }
            if (w->th.joinable()) w->th.join();
        }
    }
    std::mutex m_;
    std::vector<std::unique_ptr<Worker>> w_;
};
// The slot a single-shard call of this thread runs on: consecutive threads take consecutive devices, so
// FedTree's OpenMP callers with small batches (Party::encrypt_histogram per party, FLtrainer.cpp:275-306)
// spread over the node's GPUs instead of all landing on the primary one.
inline size_t home_slot() {
    static std::atomic<size_t> next{0};
    static thread_local size_t mine = next.fetch_add(1);
    return mine % shard_devices().size();
}
}  // namespace fthe_shim

class Paillier_HIP {
public:
    // Encryption mode of encrypt().  The modes give the reference's ciphertext distribution
    // (paillier.cpp:127-137: r uniform in Z_n^*); the build must opt in (FTHE_ENABLE_NONREFERENCE_MODES)
    // before a mode that does not can even be named.
    enum class EncMode {
        Default,              // one exponentiation per ciphertext
        FixedBaseExact,       // precomputed generator tables, the same distribution, ~4x the rate on the key
                              // holder; parties with published bases (publish_bases) ~5.6x (include/fthe.h)
#ifdef FTHE_ENABLE_NONREFERENCE_MODES
        FixedBaseSubgroup,    // r = h^alpha for one h per key: NOT the reference's distribution (r^n ranges
                              // over a subgroup of the n-th residues; FTHE_ENC_FIXED_BASE)
#endif
    };
    EncMode enc_mode = EncMode::Default;
    // Key generation of keygen().
    enum class KeygenMode {
        Reference,            // unconstrained random primes of keyLength / 2 bits (paillier.cpp:43-62)
#ifdef FTHE_ENABLE_NONREFERENCE_MODES
        KnownOrder,           // p - 1, q - 1 factored (FTHE_KEYGEN_KNOWN_ORDER): NOT the reference's prime
                              // distribution; one generator per prime in FixedBaseExact (~2.6x faster again)
#endif
    };
    KeygenMode keygen_mode = KeygenMode::Reference;
    // decrypt() with plaintexts known to be < p -- every GHPair codec value and any sum of fewer
    // than 2^900 of them at P-2048 -- takes the p half of the CRT only (fthe_decrypt_short,
    // ~2x the decrypts/s, the same low 64 bits).  Not in the reference; off by default.
    bool dec_short = false;
    // key_length = bits of n (the NTL meaning).  The default is a 2048-bit n.  The reference
    // GPU build's keygen() is paillier_cpu.keyGen(BITS = 1024), GMP semantics, a 512-bit n
    // (paillier_gpu.cu:119-121, paillier_gpu.h:13) -- factorable, so it is only the default when the
    // build asks for the reference's weak key explicitly (-DFTHE_REFERENCE_GPU_KEYLEN).  keygen(keylength)
    // honours FLParam.key_length.
#ifdef FTHE_REFERENCE_GPU_KEYLEN
    static constexpr uint32_t kDefaultKeyLength = 512;
#else
    static constexpr uint32_t kDefaultKeyLength = 2048;
#endif
    Paillier_HIP() : key_length(kDefaultKeyLength) {}
    Paillier_HIP(const Paillier_HIP &o) : key_length(o.key_length) { copy_public(o); }
    ~Paillier_HIP() { disown(); }

    // Paillier_GPU::operator= (paillier_gpu.h:32-37): public part, re-uploaded.
    Paillier_HIP &operator=(const Paillier_HIP &source) {
        if (this != &source) { key_length = source.key_length; copy_public(source); }
        return *this;
    }

    // Key holder: publish checked fixed-base bases with the public key (fthe_key_public_bases).
    // Parties that receive this key by operator= build their tables from them, and their
    // encrypt() with enc_mode = FixedBaseExact (Party::encrypt_histogram) then draws r^n from the
    // tables (within 3 * 2^-64 of the reference's distribution).  Not in the reference.
    // seed 0 (production): the bases' generators from /dev/urandom; nonzero: deterministic (tests).
    void publish_bases(uint64_t seed = 0) {
        int nb = 0;
        fthe_shim::check(fthe_key_public_bases(key(), seed, nullptr, &nb, nullptr), "public_bases");
        bases_.assign((size_t)nb * 2 * fthe_key_n_words(key()), 0);
        base_bits_.assign(nb, 0);
        fthe_shim::check(fthe_key_public_bases(key(), seed, bases_.data(), &nb, base_bits_.data()), "public_bases");
        nbases_ = nb;
    }

    // Paillier_GPU::keygen (paillier_gpu.cu:119-121) with this object's key_length (bits of n).
    void keygen() { keygen((int)key_length); }
    void keygen(int keyLength) {
        key_length = (uint32_t)keyLength;
        reset_bases();
        fthe_key *k = nullptr;
        fthe_shim::check(fthe_key_generate_ex(fthe_shim::thread_ctx(), keyLength, 0, keygen_flags(), &k), "keygen");
        adopt(fthe_key_adopt(k));
    }
    // Injected primes (the key of a reference run, test fixtures): fthe_key_from_primes.
    void key_from_primes(const mpz_t p, const mpz_t q) {
        const int w = (int)std::max(fthe_shim::words_of(p), fthe_shim::words_of(q));
        std::vector<uint32_t> pw(w), qw(w);
        fthe_shim::to_words(p, pw.data(), w);
        fthe_shim::to_words(q, qw.data(), w);
        reset_bases();
        fthe_key *k = nullptr;
        fthe_shim::check(fthe_key_from_primes(fthe_shim::thread_ctx(), pw.data(), qw.data(), w, &k), "key_from_primes");
        adopt(fthe_key_adopt(k));
        key_length = (uint32_t)mpz_sizeinbase(paillier_cpu.n, 2);
        paillier_cpu.key_length = key_length;
    }
    // Paillier_GPU::parameters_cpu_to_gpu (paillier_gpu.cu:77-117): engine keys live on the device from
    // creation (keygen, key_from_primes, operator=), so there is nothing left to upload.
    void parameters_cpu_to_gpu() {}

    // ---- batch calls: sharded over shard_devices() ----------------------------------------------------------
    // A batch of rows splits into contiguous shards (fthe_shim::shard_plan), one per device of FTHE_DEVICES (else
    // every visible GPU): the calling thread runs the first, one worker thread per further device the others,
    // each on its own engine context with this key's replica on that device (key_on), no collective.  Batches
    // below two shards of FTHE_SHARD_ROWS run whole on the calling thread's home device (fthe_shim::home_slot).
    // Results do not depend on the sharding: decrypt / add / products are deterministic, and a seeded encrypt
    // (rng_seed) draws row i's randomness at position i of the whole batch (fthe_encrypt_u64_at).
    // Deterministic device randomness for the batch encrypts (tests, benchmarks); 0: fresh keys from
    // /dev/urandom per call and shard, the production setting.
    uint64_t rng_seed = 0;

    // Paillier_GPU::encrypt(SyncArray<GHPair>&) (paillier_gpu.cu:211-313): rows 0..n-1 are the pairs' g,
    // rows n..2n-1 their h; each shard marshals, encrypts and unmarshals its own rows.
    void encrypt(SyncArray<GHPair> &message) {
        auto *d = message.host_data();
        size_t n = message.size();
        if (n == 0) return;
        const int cw = 2 * fthe_key_n_words(key()), flags = eff_flags();
        prepare_exact();
        fthe_shim::Pinned<uint64_t> mb(2 * n);
        fthe_shim::Pinned<uint32_t> cb(2 * n * (size_t)cw);
        uint64_t *m = mb.get();
        uint32_t *c = cb.get();
        for_shards(2 * n, [&](fthe_ctx *ctx, fthe_key *k, size_t lo, size_t hi, unsigned nt) {
            encode_rows(d, n, lo, hi, m, nt);
            fthe_shim::check(fthe_encrypt_u64_at(k, ctx, m + lo, hi - lo, nullptr, 0, rng_seed, lo,
                                                 c + lo * (size_t)cw, flags), "encrypt");
            rows_to_fields(d, n, lo, hi, c, cw, nt);
        });
    }

    // The host marshalling of the batch calls (integration/marshal_rate.cpp times it alone, for 1..8 concurrent
    // shards: the host side of a multi-GPU server), over rows [lo, hi) of the 2n:
    // encrypt: the codec of common.h:81-86 into plaintext words; result rows into the pairs' mpz fields
    // (mpz_import, as paillier_gpu.cu:18).
    static void encode_rows(const GHPair *d, size_t n, size_t lo, size_t hi, uint64_t *m, unsigned nt = 16) {
        fthe_shim::parallel_for(hi - lo, [&](size_t b, size_t e) {
            for (size_t r = lo + b; r < lo + e; r++) m[r] = fthe_shim::encode(r < n ? d[r].g : d[r - n].h);
        }, nt);
    }
    static void rows_to_fields(GHPair *d, size_t n, size_t lo, size_t hi, const uint32_t *c, int cw, unsigned nt = 16) {
        fthe_shim::parallel_for(hi - lo, [&](size_t b, size_t e) {
            for (size_t r = lo + b; r < lo + e; r++)
                fthe_shim::from_words(r < n ? d[r].g_enc : d[r - n].h_enc, &c[r * (size_t)cw], cw);
        }, nt);
    }
    // decrypt: the pairs' mpz fields into rows (mpz_export, paillier_gpu.cu:7; unencrypted pairs: zero rows),
    // then the plaintexts' codec back into g, h
    static void fields_to_rows(const GHPair *d, size_t n, size_t lo, size_t hi, uint32_t *c, int cw, unsigned nt = 16) {
        fthe_shim::parallel_for(hi - lo, [&](size_t b, size_t e) {  // to_words throws only on oversize input
            for (size_t r = lo + b; r < lo + e; r++) {
                const GHPair &p = d[r < n ? r : r - n];
                if (!p.encrypted) std::fill(&c[r * (size_t)cw], &c[(r + 1) * (size_t)cw], 0u);
                else fthe_shim::to_words(r < n ? p.g_enc : p.h_enc, &c[r * (size_t)cw], cw);
            }
        }, nt);
    }
    static void decode_rows(GHPair *d, size_t n, size_t lo, size_t hi, const uint64_t *m, unsigned nt = 16) {
        fthe_shim::parallel_for(hi - lo, [&](size_t b, size_t e) {
            for (size_t r = lo + b; r < lo + e; r++) {
                GHPair &p = d[r < n ? r : r - n];
                if (p.encrypted) (r < n ? p.g : p.h) = fthe_shim::decode(m[r]);
            }
        }, nt);
    }
    // whole-batch forms (marshal_rate.cpp)
    static void encode_pairs(const GHPair *d, size_t n, uint64_t *m) { encode_rows(d, n, 0, 2 * n, m); }
    static void rows_to_pairs(GHPair *d, size_t n, const uint32_t *c, int cw) { rows_to_fields(d, n, 0, 2 * n, c, cw); }
    static void pairs_to_rows(const GHPair *d, size_t n, uint32_t *c, int cw) { fields_to_rows(d, n, 0, 2 * n, c, cw); }
    static void decode_pairs(GHPair *d, size_t n, const uint64_t *m) { decode_rows(d, n, 0, 2 * n, m); }

    // Paillier_GPU::decrypt(SyncArray<GHPair>&) (paillier_gpu.cu:448-494)
    void decrypt(SyncArray<GHPair> &message) {
        auto *d = message.host_data();
        size_t n = message.size();
        if (n == 0) return;
        const int cw = 2 * fthe_key_n_words(key());
        fthe_shim::Pinned<uint32_t> cb(2 * n * (size_t)cw);
        fthe_shim::Pinned<uint64_t> mb(2 * n);
        uint32_t *c = cb.get();
        uint64_t *m = mb.get();
        for_shards(2 * n, [&](fthe_ctx *ctx, fthe_key *k, size_t lo, size_t hi, unsigned nt) {
            fields_to_rows(d, n, lo, hi, c, cw, nt);
            fthe_shim::check((dec_short ? fthe_decrypt_short : fthe_decrypt)(k, ctx, c + lo * (size_t)cw, hi - lo,
                                                                             m + lo, nullptr), "decrypt");
            decode_rows(d, n, lo, hi, m, nt);
        });
    }

    // Paillier_GPU::decrypt(GHPair&) (paillier_gpu.cu:497-542)
    void decrypt(GHPair &message) {
        if (!message.encrypted) return;
        int cw = 2 * fthe_key_n_words(key());
        std::vector<uint32_t> c(2 * (size_t)cw);
        fthe_shim::to_words(message.g_enc, &c[0], cw);
        fthe_shim::to_words(message.h_enc, &c[cw], cw);
        uint64_t m[2];
        // Server::decrypt_gh runs this per tree node from OpenMP threads (FLtrainer.cpp:758-764):
        // the key's coalescing queue merges the concurrent pairs into one launch
        fthe_shim::check(fthe_decrypt_shared(key(), c.data(), 2, m, nullptr, dec_short ? 1 : 0), "decrypt");
        message.g = fthe_shim::decode(m[0]);
        message.h = fthe_shim::decode(m[1]);
    }

    // Paillier_GPU::add / mul (paillier_gpu.cu:57-68): single values, alias-safe, into an initialised
    // result -- both on the host (one product, and a 64-bit-exponent mpz_powm, as the reference GPU build).
    // Batch callers should use the helpers below or fthe_add / fthe_reduce_kway directly.
    void add(mpz_t &result, mpz_t &x, mpz_t &y) { paillier_cpu.add(result, x, y); }
    void mul(mpz_t result, mpz_t &x, mpz_t &y) { paillier_cpu.mul_into(result, x, y); }

    // ---- batch helpers for FedTree's HE call sites (not Paillier_GPU members) ----
    // Each replaces a loop of per-pair GHPair operators (CPU GMP, ~11.5 us per add) with one sharded engine call.
    // Unencrypted operands are encrypted first, as the operators promote them (common.h:156-160).

    // Histogram of one node (hist_tree_builder.cpp:565-595): hist[cut_col_ptr[f] + b] accumulates gh[i]
    // for each instance i whose feature f has bin b = dense_bin_id[i * n_col + f] (b == max_num_bin: a
    // missing value, skipped), in instance order: one segmented product over g and h
    // (fthe_reduce_segments), sharded by bins of about equal member counts.  hist holds cut_col_ptr[n_col]
    // entries; bins without instances are left untouched (unencrypted zero, like the reference's).  A
    // populated bin is the product of its members; zero_first also folds a fresh Enc(0) into every populated
    // bin, the reference's exact sequence (its first += promotes the unencrypted zero accumulator,
    // common.h:156-160).
    void histogram(SyncArray<GHPair> &gh, const unsigned char *dense_bin_id, const int *cut_col_ptr, int n_col,
                   int max_num_bin, SyncArray<GHPair> &hist, bool zero_first = false) {
        const size_t n = gh.size(), nb = (size_t)cut_col_ptr[n_col];
        if (hist.size() < nb) throw std::runtime_error("histogram: hist smaller than cut_col_ptr[n_col]");
        std::vector<int64_t> ptr(2 * nb + 1, 0);                 // CSR: g segments, then h segments
        for (size_t i = 0; i < n; i++)
            for (int f = 0; f < n_col; f++) {
                const int b = dense_bin_id[i * n_col + f];
                if (b != max_num_bin) ptr[cut_col_ptr[f] + b + 1]++;
            }
        for (size_t s = 0; s < nb; s++) ptr[s + 1] += ptr[s];
        const int64_t tot = ptr[nb];
        std::vector<int64_t> idx(2 * (size_t)tot), cur(ptr.begin(), ptr.begin() + nb);
        for (size_t i = 0; i < n; i++)
            for (int f = 0; f < n_col; f++) {
                const int b = dense_bin_id[i * n_col + f];
                if (b != max_num_bin) idx[cur[cut_col_ptr[f] + b]++] = (int64_t)i;
            }
        for (size_t s = 0; s < nb; s++) ptr[nb + s + 1] = tot + ptr[s + 1];    // h rows are n .. 2n-1
        for (int64_t t = 0; t < tot; t++) idx[tot + t] = idx[t] + (int64_t)n;
        const int cw = 2 * fthe_key_n_words(key());
        std::vector<uint32_t> x = rows(gh), out(2 * nb * (size_t)cw);
        segments_rows(x.data(), 2 * n, ptr.data(), idx.data(), 2 * nb, out.data());
        if (zero_first) {                                        // Enc(0) * prod, populated bins only
            std::vector<size_t> pop;
            for (size_t s = 0; s < nb; s++) if (ptr[s + 1] > ptr[s]) pop.push_back(s);
            const size_t np = pop.size();
            std::vector<uint64_t> zero(2 * np, 0);
            std::vector<uint32_t> ez(2 * np * (size_t)cw), a(2 * np * (size_t)cw);
            encrypt_rows(zero.data(), 2 * np, ez.data());
            for (size_t j = 0; j < np; j++)
                for (int pl = 0; pl < 2; pl++)
                    std::copy(&out[(pl * nb + pop[j]) * cw], &out[(pl * nb + pop[j] + 1) * cw], &a[(pl * np + j) * cw]);
            add_rows(a.data(), ez.data(), 2 * np, a.data());
            for (size_t j = 0; j < np; j++)
                for (int pl = 0; pl < 2; pl++)
                    std::copy(&a[(pl * np + j) * cw], &a[(pl * np + j + 1) * cw], &out[(pl * nb + pop[j]) * cw]);
        }
        auto *hd = hist.host_data();
        fthe_shim::parallel_for(nb, [&](size_t b, size_t e) {
            for (size_t s = b; s < e; s++)
                if (ptr[s + 1] > ptr[s]) set_enc(hd[s], &out[s * cw], &out[(nb + s) * cw], cw);
        });
    }

    // k-party merge (hist_tree_builder.cpp:1015-1058): out[b] = prod_j parties[j][b] as one k-way product
    // (fthe_reduce_kway), sharded by bins.  zero_first: Enc(0) * prod_j ..., the reference's exact sequence
    // (its zero accumulator's first += encrypts 0) at the price of one fresh encryption per entry;
    // without it the plaintexts are the same and only the randomness differs.
    void merge(const std::vector<SyncArray<GHPair> *> &parties, SyncArray<GHPair> &out, bool zero_first = false) {
        const size_t z = zero_first ? 1 : 0, k = parties.size() + z, nb = out.size();
        if (k > 64 || parties.empty()) throw std::runtime_error("merge: 1 to 63 parties per call");
        for (auto *pt : parties)
            if (pt->size() != nb) throw std::runtime_error("merge: histogram sizes differ");
        const int cw = 2 * fthe_key_n_words(key());
        std::vector<uint32_t> x(k * 2 * nb * (size_t)cw), o(2 * nb * (size_t)cw);
        if (zero_first) {
            std::vector<uint64_t> zero(2 * nb, 0);
            encrypt_rows(zero.data(), 2 * nb, x.data());
        }
        for (size_t j = z; j < k; j++) {
            std::vector<uint32_t> r = rows(*parties[j - z]);
            std::copy(r.begin(), r.end(), x.begin() + j * 2 * nb * (size_t)cw);
        }
        kway_rows(x.data(), k, 2 * nb, o.data());
        auto *d = out.host_data();
        fthe_shim::parallel_for(nb, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; i++) set_enc(d[i], &o[i * cw], &o[(nb + i) * cw], cw);
        });
    }

    // Per-feature prefix sums of a histogram (inclusive_scan_by_key, hist_tree_builder.cpp:695-708), in
    // place: hist[t] = sum of hist[cut_col_ptr[f] .. t] within feature f, one segmented scan (g and h
    // planes as segments of their own, fthe_scan_segments), sharded by features.
    void prefix(SyncArray<GHPair> &hist, const int *cut_col_ptr, int n_col) {
        const size_t nb = (size_t)cut_col_ptr[n_col];
        if (hist.size() < nb) throw std::runtime_error("prefix: hist smaller than cut_col_ptr[n_col]");
        const int cw = 2 * fthe_key_n_words(key());
        std::vector<int64_t> seg(2 * (size_t)n_col + 1);
        for (int f = 0; f <= n_col; f++) seg[f] = cut_col_ptr[f];
        for (int f = 1; f <= n_col; f++) seg[n_col + f] = (int64_t)nb + cut_col_ptr[f];
        std::vector<uint32_t> x = rows_n(hist, nb), o(2 * nb * (size_t)cw);
        const size_t ns = 2 * (size_t)n_col;
        auto plan = fthe_shim::shard_plan_segments(seg.data(), ns, fthe_shim::shard_devices().size(),
                                                   fthe_shim::shard_min_rows());
        run_plan(plan, [&](fthe_ctx *ctx, fthe_key *kk, size_t s0, size_t s1, unsigned) {
            std::vector<int64_t> ls(seg.begin() + s0, seg.begin() + s1 + 1);
            for (auto &v : ls) v -= seg[s0];
            fthe_shim::check(fthe_scan_segments(kk, ctx, x.data() + seg[s0] * cw, ls.data(), s1 - s0,
                                                o.data() + seg[s0] * cw), "prefix");
        });
        auto *d = hist.host_data();
        fthe_shim::parallel_for(nb, [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; i++) set_enc(d[i], &o[i * cw], &o[(nb + i) * cw], cw);
        });
    }

    // Sibling histogram (hist_tree_builder.cpp:678) and missing_gh (:724): out = a - b, exactly the ciphertext
    // GHPair::operator- produces (a * b^(2^64-1), common.h:253-337), as one fused batch (fthe_sub).
    void subtract(SyncArray<GHPair> &a, SyncArray<GHPair> &b, SyncArray<GHPair> &out) {
        const size_t n = a.size();
        if (b.size() != n || out.size() != n) throw std::runtime_error("subtract: sizes differ");
        const int cw = 2 * fthe_key_n_words(key());
        std::vector<uint32_t> xa = rows(a), xb = rows(b), o(2 * n * (size_t)cw);
        for_shards(2 * n, [&](fthe_ctx *ctx, fthe_key *k, size_t lo, size_t hi, unsigned) {
            fthe_shim::check(fthe_sub(k, ctx, xa.data() + lo * cw, xb.data() + lo * cw, hi - lo, o.data() + lo * cw),
                             "subtract");
        });
        auto *d = out.host_data();
        fthe_shim::parallel_for(n, [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; i++) set_enc(d[i], &o[i * cw], &o[(n + i) * cw], cw);
        });
    }

    // The N-to-1 root sum of Tree::init_CPU (tree.cpp:20-34: thrust::reduce of the gradients with GHPair::operator+):
    // sum_gh = prod_i gh[i] for g and h.  Sharded over the devices by instance ranges: each shard's
    // partial products of its g rows and h rows on its device (fthe_reduce_segments, one segment each), the <= 7
    // partials combined on the host (x y mod n^2, the reference's own add).  zero_first: Enc(0) * prod, the
    // reference's exact sequence (thrust's GHPair() initial value is an unencrypted zero, whose first + encrypts 0,
    // SURVEY Q10).  Unencrypted entries are encrypted first, as the operators promote them.
    GHPair sum(SyncArray<GHPair> &gh, bool zero_first = false) {
        const size_t n = gh.size();
        GHPair out;
        if (n == 0) return out;                                  // the reference's GHPair(): an unencrypted zero
        const size_t cw = 2 * (size_t)fthe_key_n_words(key());
        std::vector<uint32_t> x = rows(gh);
        auto plan = fthe_shim::shard_plan(n, fthe_shim::shard_devices().size(), fthe_shim::shard_min_rows());
        std::vector<uint32_t> part(plan.size() * 2 * cw);
        run_plan(plan, [&](fthe_ctx *ctx, fthe_key *kk, size_t lo, size_t hi, unsigned) {
            const size_t i = (size_t)(std::find(plan.begin(), plan.end(), std::make_pair(lo, hi)) - plan.begin());
            const int64_t ptr[2] = {0, (int64_t)(hi - lo)};
            for (int pl = 0; pl < 2; pl++)                       // the g rows, then the h rows of [lo, hi)
                fthe_shim::check(fthe_reduce_segments(kk, ctx, x.data() + (pl * n + lo) * cw, hi - lo, ptr, nullptr,
                                                      1, part.data() + (2 * i + pl) * cw), "sum");
        });
        mpz_t acc[2], t;
        for (int pl = 0; pl < 2; pl++) {
            mpz_init(acc[pl]);
            fthe_shim::from_words(acc[pl], part.data() + pl * cw, (int)cw);
        }
        mpz_init(t);
        for (size_t i = 1; i < plan.size(); i++)
            for (int pl = 0; pl < 2; pl++) {
                fthe_shim::from_words(t, part.data() + (2 * i + pl) * cw, (int)cw);
                paillier_cpu.add(acc[pl], acc[pl], t);
            }
        if (zero_first) {
            uint64_t zero[2] = {0, 0};
            std::vector<uint32_t> ez(2 * cw);
            encrypt_rows(zero, 2, ez.data());
            for (int pl = 0; pl < 2; pl++) {
                fthe_shim::from_words(t, ez.data() + pl * cw, (int)cw);
                paillier_cpu.add(acc[pl], t, acc[pl]);
            }
        }
        std::vector<uint32_t> gw(cw), hw(cw);
        fthe_shim::to_words(acc[0], gw.data(), (int)cw);
        fthe_shim::to_words(acc[1], hw.data(), (int)cw);
        set_enc(out, gw.data(), hw.data(), (int)cw);
        mpz_clear(acc[0]); mpz_clear(acc[1]); mpz_clear(t);
        return out;
    }

    // ---- sharded engine calls on host rows (the helpers above; public for callers with rows in hand) ----
    // c[i] = Enc(m[i]) (fthe_encrypt_u64_at with this object's enc_mode and rng_seed)
    void encrypt_rows(const uint64_t *m, size_t count, uint32_t *c) {
        const int cw = 2 * fthe_key_n_words(key()), flags = eff_flags();
        prepare_exact();
        for_shards(count, [&](fthe_ctx *ctx, fthe_key *k, size_t lo, size_t hi, unsigned) {
            fthe_shim::check(fthe_encrypt_u64_at(k, ctx, m + lo, hi - lo, nullptr, 0, rng_seed, lo, c + lo * cw, flags),
                             "encrypt");
        });
    }
    // out[i] = a[i] b[i] mod n^2 (fthe_add; alias-safe)
    void add_rows(const uint32_t *a, const uint32_t *b, size_t count, uint32_t *out) {
        const int cw = 2 * fthe_key_n_words(key());
        for_shards(count, [&](fthe_ctx *ctx, fthe_key *k, size_t lo, size_t hi, unsigned) {
            fthe_shim::check(fthe_add(k, ctx, a + lo * cw, b + lo * cw, hi - lo, out + lo * cw), "add");
        });
    }
    // out[i] = prod_j x[j * count + i] mod n^2 (fthe_reduce_kway); each shard gathers its k column blocks
    void kway_rows(const uint32_t *x, size_t k, size_t count, uint32_t *out) {
        const size_t cw = 2 * (size_t)fthe_key_n_words(key());
        auto plan = fthe_shim::shard_plan(count, fthe_shim::shard_devices().size(), fthe_shim::shard_min_rows());
        run_plan(plan, [&](fthe_ctx *ctx, fthe_key *kk, size_t lo, size_t hi, unsigned) {
            const size_t cnt = hi - lo;
            const uint32_t *src = x;
            std::vector<uint32_t> local;
            if (cnt != count) {                                  // this shard's rows of every party
                local.resize(k * cnt * cw);
                for (size_t j = 0; j < k; j++)
                    std::copy(x + (j * count + lo) * cw, x + (j * count + hi) * cw, local.begin() + j * cnt * cw);
                src = local.data();
            }
            fthe_shim::check(fthe_reduce_kway(kk, ctx, src, (int)k, cnt, out + lo * cw), "merge");
        });
    }
    // out[s] = prod_{t in [ptr[s], ptr[s+1])} x[idx[t]] mod n^2 (fthe_reduce_segments; ptr[0] == 0): each shard
    // takes a range of segments of about equal member counts, with all of x (the members are gathered by idx)
    void segments_rows(const uint32_t *x, size_t count, const int64_t *ptr, const int64_t *idx, size_t nseg,
                       uint32_t *out) {
        const size_t cw = 2 * (size_t)fthe_key_n_words(key());
        if (!nseg) return;
        auto plan = fthe_shim::shard_plan_segments(ptr, nseg, fthe_shim::shard_devices().size(),
                                                   fthe_shim::shard_min_rows());
        run_plan(plan, [&](fthe_ctx *ctx, fthe_key *kk, size_t s0, size_t s1, unsigned) {
            std::vector<int64_t> lp(ptr + s0, ptr + s1 + 1);
            for (auto &v : lp) v -= ptr[s0];
            fthe_shim::check(fthe_reduce_segments(kk, ctx, x, count, lp.data(), idx + ptr[s0], s1 - s0, out + s0 * cw),
                             "histogram");
        });
    }

    // This key on the device of context c: the key itself on the primary device, else its replica there, made on
    // first use from p, q (key holder) or n and the published bases (public key) -- the same n, the same results.
    // FTHE_SHIM_REPLICATE=1 (tests): replicas on the primary device too, so a one-GPU box runs the replica path.
    // A key holder's replica in FixedBaseExact mode also takes the key's own table generators
    // (fthe_key_fixed_base_exact_set), so its r^n are the key's for the same exponents (exact_tables).
    fthe_key *key_on(fthe_ctx *c) {
        static const bool force = [] { const char *e = std::getenv("FTHE_SHIM_REPLICATE"); return e && *e == '1'; }();
        const int dv = fthe_ctx_device(c);
        fthe_key *k0 = key();
        if (dv == fthe_shim::primary_device() && !force) return k0;
        std::lock_guard<std::mutex> lk(rep_mu_);
        for (auto &r : replicas_)
            if (r.first == dv) { sync_exact(k0, r.second.get(), c); return r.second.get(); }
        fthe_key *k = new_replica(k0, c);
        sync_exact(k0, k, c);
        return k;
    }

    // Key holder, FixedBaseExact: (re)build this key's exact tables (fthe_key_fixed_base_exact; seed 0: fresh
    // generators from /dev/urandom, nonzero: deterministic, for tests) -- the replicas on other devices follow on
    // their next use.  Built on the first FixedBaseExact batch otherwise.
    void exact_tables(uint64_t seed = 0) {
        std::lock_guard<std::mutex> lk(rep_mu_);
        fthe_shim::check(fthe_key_fixed_base_exact(key(), fthe_shim::thread_ctx(), seed), "fixed_base_exact");
    }

private:
    // the replica's exact tables from k0's generators, when k0 has tables and the replica's differ
    void sync_exact(fthe_key *k0, fthe_key *k, fthe_ctx *c) {
        if (enc_mode != EncMode::FixedBaseExact || !fthe_key_has_private(k0)) return;
        const int nb = fthe_key_fixed_base_exact_bases(k0);
        if (!nb) return;
        const size_t gw = (size_t)fthe_key_n_words(k0);
        std::vector<uint32_t> g0(2 * nb * gw), g1(2 * nb * gw);
        for (int s = 0; s < 2; s++)
            for (int b = 0; b < nb; b++)
                fthe_shim::check(fthe_key_fixed_base_exact_info(k0, s, b, &g0[(s * nb + b) * gw], nullptr), "exact_info");
        if (fthe_key_fixed_base_exact_bases(k) == nb) {
            for (int s = 0; s < 2; s++)
                for (int b = 0; b < nb; b++)
                    fthe_shim::check(fthe_key_fixed_base_exact_info(k, s, b, &g1[(s * nb + b) * gw], nullptr),
                                     "exact_info");
            if (g0 == g1) return;
        }
        fthe_shim::check(fthe_key_fixed_base_exact_set(k, c, nb, g0.data()), "exact_set");
    }
    // Key holder, FixedBaseExact: the key's own tables exist before the shards start, so no shard builds
    // fresh ones beside another's use of them (run on the calling thread, before run_plan)
    void prepare_exact() {
        if (enc_mode != EncMode::FixedBaseExact || !fthe_key_has_private(key())) return;
        std::lock_guard<std::mutex> lk(rep_mu_);
        if (!fthe_key_fixed_base_exact_bases(key()))
            fthe_shim::check(fthe_key_fixed_base_exact(key(), fthe_shim::thread_ctx(), 0), "fixed_base_exact");
    }
    fthe_key *new_replica(fthe_key *k0, fthe_ctx *c) {
        const int dv = fthe_ctx_device(c);
        const int nw = fthe_key_n_words(k0);
        fthe_key *k = nullptr;
        if (fthe_key_has_private(k0)) {
            const int hw = (nw + 1) / 2;
            std::vector<uint32_t> p(hw), q(hw);
            fthe_shim::check(fthe_key_export(k0, nullptr, nullptr, nullptr, p.data(), q.data()), "export");
            fthe_shim::check(fthe_key_from_primes(c, p.data(), q.data(), hw, &k), "key replica");
        } else {
            std::vector<uint32_t> n(nw);
            fthe_shim::check(fthe_key_export(k0, n.data(), nullptr, nullptr, nullptr, nullptr), "export");
            fthe_shim::check(fthe_key_from_n(c, n.data(), nw, &k), "key replica");
        }
        fthe_key_ref ref = fthe_key_adopt(k);
        if (nbases_ && !fthe_key_has_private(k0))              // a party's published-bases tables (operator=)
            fthe_shim::check(fthe_key_set_public_bases(k, c, bases_.data(), nbases_, base_bits_.data()),
                             "set_public_bases");
        replicas_.emplace_back(dv, ref);
        return k;
    }

public:
    uint32_t key_length;
    // The GHPair key (common.h:72; server.h:119 and party.h:124 assign it to every encrypted GHPair):
    // the public part of this object's engine key, whose add / mul / encrypt run on the engine.
    Paillier_HIP_Pub paillier_cpu;
    fthe_key *key() const {
        if (!key_) throw std::runtime_error("Paillier_HIP: no key (keygen() first)");
        return key_.get();
    }

private:
    fthe_key_ref key_;
    std::mutex rep_mu_;
    std::vector<std::pair<int, fthe_key_ref>> replicas_;   // (device, key) beyond the primary device
    std::vector<uint32_t> bases_;          // published fixed-base bases (nbases_ x 2 n_words words)
    std::vector<int> base_bits_;           // and the bits of each base's exponent
    int nbases_ = 0;
    int keygen_flags() const {
#ifdef FTHE_ENABLE_NONREFERENCE_MODES
        if (keygen_mode == KeygenMode::KnownOrder) return FTHE_KEYGEN_KNOWN_ORDER;
#endif
        return 0;
    }
    int eff_flags() const {             // exact fixed-base: p, q (key holder) or published bases (party)
        switch (enc_mode) {
            case EncMode::Default: return FTHE_ENC_DEFAULT;
            case EncMode::FixedBaseExact:
                return (fthe_key_has_private(key()) || nbases_) ? FTHE_ENC_FIXED_BASE_EXACT : FTHE_ENC_DEFAULT;
#ifdef FTHE_ENABLE_NONREFERENCE_MODES
            case EncMode::FixedBaseSubgroup: return FTHE_ENC_FIXED_BASE;
#endif
        }
        return FTHE_ENC_DEFAULT;
    }
    // f(ctx, key, lo, hi, marshalling threads) for each range of a plan: one range on the calling thread's home
    // device, several on the shard pool (each range on its slot's device, with this key's replica there)
    template <class F>
    void run_plan(const std::vector<std::pair<size_t, size_t>> &plan, F f) {
        if (plan.empty()) return;
        const std::vector<int> &devs = fthe_shim::shard_devices();
        if (plan.size() == 1) {
            fthe_ctx *c = fthe_shim::ctx_on(devs[fthe_shim::home_slot()]);
            f(c, key_on(c), plan[0].first, plan[0].second, 16u);
            return;
        }
        const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
        const unsigned nt = std::max(1u, std::min(16u, hc / (unsigned)plan.size()));
        fthe_shim::ShardPool::get().run(plan.size(), [&](size_t i, fthe_ctx *c) {
            f(c, key_on(c), plan[i].first, plan[i].second, nt);
        });
    }
    template <class F>
    void for_shards(size_t rows, F f) {
        run_plan(fthe_shim::shard_plan(rows, fthe_shim::shard_devices().size(), fthe_shim::shard_min_rows()), f);
    }
    void reset_bases() { bases_.clear(); base_bits_.clear(); nbases_ = 0; }
    void reset_replicas() { std::lock_guard<std::mutex> lk(rep_mu_); replicas_.clear(); }
    fthe_shim::KeyCell *owned_cell_ = nullptr;   // the cell whose randomizer pool this object keeps alive
    void disown() {
        if (owned_cell_) owned_cell_->release();
        owned_cell_ = nullptr;
    }
    void adopt(const fthe_key_ref &k) {
        reset_replicas();
        key_ = k;
        paillier_cpu.bind(k, key_length);
        fthe_shim::KeyCell *c = paillier_cpu.cell();
        if (c != owned_cell_) {
            c->retain();                          // first owner: the pool starts filling in the background
            disown();
            owned_cell_ = c;
        }
    }
    void set_enc(GHPair &p, const uint32_t *g, const uint32_t *h, int cw) const {
        fthe_shim::from_words(p.g_enc, g, cw);
        fthe_shim::from_words(p.h_enc, h, cw);
        p.g = 0;
        p.h = 0;
        p.encrypted = true;
        p.paillier = paillier_cpu;      // the public key rides along, as after GHPair::operator+
    }
    // g rows then h rows of a batch (2 n_words words each); unencrypted entries are encrypted here
    std::vector<uint32_t> rows(SyncArray<GHPair> &a) { return rows_n(a, a.size()); }
    std::vector<uint32_t> rows_n(SyncArray<GHPair> &a, size_t n) {       // the first n entries
        auto *d = a.host_data();
        const int cw = 2 * fthe_key_n_words(key());
        std::vector<uint32_t> x(2 * n * (size_t)cw, 0);
        std::vector<size_t> plain;
        for (size_t i = 0; i < n; i++)
            if (!d[i].encrypted) plain.push_back(i);
        if (!plain.empty()) {
            const size_t np = plain.size();
            std::vector<uint64_t> m(2 * np);
            for (size_t j = 0; j < np; j++) {
                m[j] = fthe_shim::encode(d[plain[j]].g);
                m[np + j] = fthe_shim::encode(d[plain[j]].h);
            }
            std::vector<uint32_t> c(2 * np * (size_t)cw);
            encrypt_rows(m.data(), 2 * np, c.data());
            for (size_t j = 0; j < np; j++) {
                std::copy(&c[j * cw], &c[(j + 1) * cw], &x[plain[j] * cw]);
                std::copy(&c[(np + j) * cw], &c[(np + j + 1) * cw], &x[(n + plain[j]) * cw]);
            }
        }
        fthe_shim::parallel_for(n, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; i++) {
                if (!d[i].encrypted) continue;
                fthe_shim::to_words(d[i].g_enc, &x[i * cw], cw);
                fthe_shim::to_words(d[i].h_enc, &x[(n + i) * cw], cw);
            }
        });
        return x;
    }
    // operator= / copy: a public-only engine key of the source's n (Paillier_GPU::operator= keeps the
    // public part of paillier_cpu and re-uploads it, paillier_gpu.h:32-37) and the published bases.
    void copy_public(const Paillier_HIP &o) {
        reset_bases();
        reset_replicas();
        key_.reset();
        paillier_cpu = Paillier_HIP_Pub();
        if (!o.key_) { disown(); return; }
        const int nw = fthe_key_n_words(o.key_.get());
        std::vector<uint32_t> w(nw);
        fthe_shim::to_words(o.paillier_cpu.n, w.data(), nw);
        fthe_key *k = nullptr;
        fthe_shim::check(fthe_key_from_n(fthe_shim::thread_ctx(), w.data(), nw, &k), "key_from_n");
        adopt(fthe_key_adopt(k));
        bases_ = o.bases_;                                                // published with n (publish_bases)
        base_bits_ = o.base_bits_;
        nbases_ = o.nbases_;
        if (nbases_)
            fthe_shim::check(fthe_key_set_public_bases(key(), fthe_shim::thread_ctx(), bases_.data(), nbases_,
                                                       base_bits_.data()), "set_public_bases");
    }
};
