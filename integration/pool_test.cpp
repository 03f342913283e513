// The randomizer pool behind GHPair's promotions (integration/fthe_ghpair_key.h): homo_encrypt of a plain
// operand (common.h:75-97, 156-160) takes rho = r^n mod n^2 from the key's pool (engine Enc(0) batches)
// and computes (1 + m n) rho mod n^2 on the host.
//   pool_test trace <p hex> <q hex> <seed0> <batch> m_1 .. m_k
//       deterministic batches: prints "m seed index c" per plaintext (hex c); the Python test rebuilds the
//       r of (seed, index) from the engine's direct-y draws and compares c with the oracle's
//       encrypt(m, r) = PowerMod(g, m, n^2) PowerMod(r, n, n^2) % n^2 (paillier.cpp:134-137)
//   pool_test threads <p hex> <q hex> <threads> <per_thread>
//       concurrent GHPair promotions from OpenMP threads: every promoted pair decrypts to its codec
//       values and no pooled row is used twice                                    -> "pool OK"
#include <omp.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#include "paillier_hip.h"

static void set_hex(mpz_t x, const char *s) {
    if (mpz_set_str(x, s, 16) != 0) { std::fprintf(stderr, "bad hex\n"); std::exit(2); }
}

int main(int argc, char **argv) {
    if (argc < 6) return 2;
    const std::string mode = argv[1];
    mpz_t p, q;
    mpz_inits(p, q, nullptr);
    set_hex(p, argv[2]);
    set_hex(q, argv[3]);
    Paillier_HIP server;
    server.key_from_primes(p, q);
    GHPairKey key = server.paillier_cpu;
    if (mode == "trace") {
        key.cell()->set_test_seed(std::strtoull(argv[4], nullptr, 10), (size_t)std::atoi(argv[5]));
        mpz_t m, c;
        mpz_inits(m, c, nullptr);
        for (int i = 6; i < argc; i++) {
            mpz_set_str(m, argv[i], 10);
            uint64_t seed = 0, idx = 0;
            key.encrypt_pooled(c, m, &seed, &idx);
            gmp_printf("%s %llu %llu %Zx\n", argv[i], (unsigned long long)seed, (unsigned long long)idx, c);
        }
        mpz_clears(m, c, nullptr);
        return 0;
    }
    if (mode != "threads") return 2;
    const int T = std::atoi(argv[4]), per = std::atoi(argv[5]);
    std::vector<GHPair> out(2 * (size_t)T * per);           // [promoted plain pairs | promoted zeros]
    auto gv = [](int t, int i) { return (float)(0.001 * ((t * 31 + i) % 997) - 0.3); };
    auto hv = [](int t, int i) { return (float)(0.25 + 0.0001 * i); };
#pragma omp parallel for num_threads(T) schedule(static)
    for (int t = 0; t < T; t++)
        for (int i = 0; i < per; i++) {
            GHPair plain(gv(t, i), hv(t, i)), zero;               // zero: the histogram's unencrypted 0
            plain.homo_encrypt(key);                              // codec value (negative g wraps mod 2^64)
            zero.homo_encrypt(key);                               // Enc(0) = rho itself
            out[(size_t)t * per + i] = plain;
            out[(size_t)(T + t) * per + i] = zero;
        }
    // decrypt everything; check the codec values and that no randomizer repeats (all ciphertexts distinct)
    SyncArray<GHPair> arr(out.size());
    for (size_t i = 0; i < out.size(); i++) arr.host_data()[i] = out[i];
    server.decrypt(arr);
    int bad = 0;
    std::set<std::string> seen;
    for (size_t k = 0; k < out.size(); k++) {
        const bool z = k >= (size_t)T * per;
        const int t = (int)((k % ((size_t)T * per)) / per), i = (int)(k % per);
        const float wg = z ? 0.f : fthe_shim::decode(fthe_shim::encode(gv(t, i)));
        const float wh = z ? 0.f : fthe_shim::decode(fthe_shim::encode(hv(t, i)));
        if (arr.host_data()[k].g != wg || arr.host_data()[k].h != wh) bad++;
        for (mpz_ptr e : {out[k].g_enc, out[k].h_enc}) {
            char *s = mpz_get_str(nullptr, 16, e);
            if (!seen.insert(s).second) bad++;
            std::free(s);
        }
    }
    std::printf("%d threads x %d promotions, %d bad -> pool %s\n", T, per, bad, bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
