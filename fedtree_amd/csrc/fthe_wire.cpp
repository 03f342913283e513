// fthe_wire.cpp -- ciphertext wire formats (host side of the C ABI).
//
// The reference ships ciphertexts between server and parties as decimal strings
// (fedtree.proto:82-99 GHEncBatch { repeated string g_enc, h_enc }): written with
// `stream << g_enc` (distributed_server.cpp:37-54, distributed_party.cpp:1285-1300)
// and parsed with NTL::to_ZZ(str) (distributed_party.cpp:1267-1273,
// distributed_server.cpp:1427-1433).  Two codecs here:
//
//  * decimal: byte-identical to those strings (canonical base-10, no sign, no
//    leading zeros, "0" for zero) in both directions, so an engine-side peer
//    interoperates with an unmodified one;  GMP's subquadratic radix
//    conversion, threaded over the batch;
//  * binary ("FTHW" frame): the little-endian u32 words the engine already
//    holds, behind a 24-byte header -- the raw-limb replacement of SURVEY
//    8(f) rank 1 (a `bytes` field in place of the repeated strings).
//
// Frame layout (all little-endian):
//   0  char[4] "FTHW"      4  u16 version (1)      6  u16 flags (bit 0: h present)
//   8  u32 words per ciphertext                    12 u32 reserved (0)
//   16 u64 count           24 count*words u32 of g, then (flags&1) count*words of h
#include <gmp.h>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/fthe.h"

namespace {

int pick_threads(int threads, size_t count) {
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    threads = std::min(threads, 64);
    return (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, count / 64 + 1));
}

template <class F>
void parallel_for(size_t count, int threads, F f) {
    int nt = pick_threads(threads, count);
    if (nt <= 1) { f(0, count); return; }
    std::vector<std::thread> th;
    size_t per = (count + nt - 1) / nt;
    for (int t = 0; t < nt; t++) {
        size_t b = t * per, e = std::min(count, b + per);
        if (b >= e) break;
        th.emplace_back([=] { f(b, e); });
    }
    for (auto &x : th) x.join();
}

// significant words (little-endian)
int sig_words(const uint32_t *w, int nw) {
    while (nw > 0 && w[nw - 1] == 0) nw--;
    return nw;
}

}  // namespace

extern "C" size_t fthe_decimal_max_len(int words) {
    // digits of 2^(32 words) - 1, plus one of slack
    return words <= 0 ? 2 : (size_t)((double)words * 32 * 0.30102999566398120) + 2;
}

extern "C" int fthe_ct_to_decimal(const uint32_t *ct, int words, size_t count, char *buf, size_t buf_len,
                                  size_t *offsets, int threads) {
    if ((!ct && count) || words <= 0 || !offsets || (!buf && buf_len)) return FTHE_ERR_ARG;
    const size_t slot = fthe_decimal_max_len(words) + 1;       // + GMP's terminating NUL
    std::vector<char> tmp(count * slot);
    std::vector<size_t> len(count);
    parallel_for(count, threads, [&](size_t b, size_t e) {
        mpz_t z;
        mpz_init2(z, (mp_bitcnt_t)words * 32);
        for (size_t i = b; i < e; i++) {
            const uint32_t *w = ct + i * (size_t)words;
            mpz_import(z, (size_t)sig_words(w, words), -1, 4, 0, 0, w);
            char *p = tmp.data() + i * slot;
            mpz_get_str(p, 10, z);
            len[i] = strlen(p);
        }
        mpz_clear(z);
    });
    size_t total = 0;
    offsets[0] = 0;
    for (size_t i = 0; i < count; i++) offsets[i + 1] = (total += len[i]);
    if (total > buf_len) return FTHE_ERR_ARG;                 // offsets[count] = bytes needed
    parallel_for(count, threads, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) memcpy(buf + offsets[i], tmp.data() + i * slot, len[i]);
    });
    return FTHE_OK;
}

extern "C" int fthe_ct_from_decimal(const char *buf, const size_t *offsets, size_t count, int words, uint32_t *ct,
                                    int threads) {
    if ((!buf && count) || !offsets || words <= 0 || (!ct && count)) return FTHE_ERR_ARG;
    for (size_t i = 0; i < count; i++)
        if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > fthe_decimal_max_len(words)) return FTHE_ERR_ARG;
    std::vector<int> bad(std::max<size_t>(1, pick_threads(threads, count)), 0);
    const size_t maxd = fthe_decimal_max_len(words);
    int nt = pick_threads(threads, count);
    size_t per = (count + nt - 1) / std::max(1, nt);
    parallel_for(count, threads, [&](size_t b, size_t e) {
        mpz_t z;
        mpz_init2(z, (mp_bitcnt_t)words * 32);
        std::vector<char> s(maxd + 1);
        int flag = 0;
        for (size_t i = b; i < e && !flag; i++) {
            size_t n = offsets[i + 1] - offsets[i];
            const char *p = buf + offsets[i];
            if (n == 0) { flag = 1; break; }
            for (size_t j = 0; j < n; j++)
                if (p[j] < '0' || p[j] > '9') { flag = 1; break; }
            if (flag) break;
            memcpy(s.data(), p, n);
            s[n] = 0;
            if (mpz_set_str(z, s.data(), 10) != 0) { flag = 1; break; }
            if (mpz_sizeinbase(z, 2) > (size_t)words * 32) { flag = 1; break; }
            uint32_t *w = ct + i * (size_t)words;
            size_t got = 0;
            memset(w, 0, (size_t)words * 4);
            if (mpz_sgn(z)) mpz_export(w, &got, -1, 4, 0, 0, z);
        }
        mpz_clear(z);
        if (flag) bad[per ? b / per : 0] = 1;
    });
    for (int f : bad) if (f) return FTHE_ERR_ARG;
    return FTHE_OK;
}

namespace {
constexpr size_t kHdr = 24;
void put16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }
void put32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
void put64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
}  // namespace

extern "C" size_t fthe_wire_size(size_t count, int words, int with_h) {
    return kHdr + count * (size_t)words * 4 * (with_h ? 2 : 1);
}

extern "C" int fthe_wire_encode(const uint32_t *g, const uint32_t *h, size_t count, int words, uint8_t *out,
                                size_t cap, size_t *len) {
    if (words <= 0 || !out || !len || (!g && count)) return FTHE_ERR_ARG;
    const size_t need = fthe_wire_size(count, words, h != nullptr);
    *len = need;
    if (cap < need) return FTHE_ERR_ARG;
    memcpy(out, "FTHW", 4);
    put16(out + 4, 1);
    put16(out + 6, h ? 1 : 0);
    put32(out + 8, (uint32_t)words);
    put32(out + 12, 0);
    put64(out + 16, (uint64_t)count);
    const size_t bytes = count * (size_t)words * 4;
    if (bytes) memcpy(out + kHdr, g, bytes);
    if (h && bytes) memcpy(out + kHdr + bytes, h, bytes);
    return FTHE_OK;
}

extern "C" int fthe_wire_decode(const uint8_t *in, size_t len, int words, uint32_t *g, uint32_t *h, size_t cap,
                                size_t *count) {
    if (!in || !count || words <= 0) return FTHE_ERR_ARG;
    if (len < kHdr || memcmp(in, "FTHW", 4) != 0) return FTHE_ERR_ARG;
    uint16_t ver, flags; uint32_t w; uint64_t n;
    memcpy(&ver, in + 4, 2); memcpy(&flags, in + 6, 2); memcpy(&w, in + 8, 4); memcpy(&n, in + 16, 8);
    if (ver != 1 || (int)w != words) return FTHE_ERR_ARG;
    const int with_h = flags & 1;
    if (n > (len - kHdr) / ((size_t)words * 4) || len != fthe_wire_size((size_t)n, words, with_h)) return FTHE_ERR_ARG;
    *count = (size_t)n;
    if (n > cap) return FTHE_ERR_ARG;
    const size_t bytes = (size_t)n * words * 4;
    if (bytes && !g) return FTHE_ERR_ARG;
    if (bytes) memcpy(g, in + kHdr, bytes);
    if (with_h && h && bytes) memcpy(h, in + kHdr + bytes, bytes);
    if (with_h && !h && bytes) return FTHE_ERR_ARG;
    return FTHE_OK;
}
