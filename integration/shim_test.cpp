// Compile/run test of integration/paillier_hip.h against the mock FedTree types:
// the Server/Party call sequence of server.h:58-135 and party.h:118-142.
#include <cstdio>
#include <cmath>
#include "paillier_hip.h"

#include <cstdlib>
#include <string>
int main(int argc, char **argv) {
    int bits = argc > 1 ? std::atoi(argv[1]) : 1024;
    Paillier_HIP server;                 // Server::paillier
    if (argc > 2 && std::string(argv[2]) == "exact_known_order") server.keygen_flags = FTHE_KEYGEN_KNOWN_ORDER;
    server.keygen(bits);                 // homo_init (NTL semantics: n of `bits` bits)
    const std::string mode = argc > 2 ? argv[2] : "default";
    if (mode == "public_exact") server.publish_bases();          // bases travel with the public key
    Paillier_HIP party;                  // Party::paillier
    party = server;                      // Server::send_key: public part only
    if (mode.rfind("exact", 0) == 0 || mode == "public_exact")  // table-driven randomizer; the party (no p, q)
        server.enc_flags = party.enc_flags = FTHE_ENC_FIXED_BASE_EXACT;   // uses published bases, else the default
    const float g[5] = {0.4f, 1.2f, 0.1f, 0.8f, -0.7f}, h[5] = {0.6f, 1.4f, 0.2f, 1.0f, 0.8f};
    SyncArray<GHPair> gh(5), hist(5);
    for (int i = 0; i < 5; i++) { gh.host_data()[i] = GHPair(g[i], h[i]); hist.host_data()[i] = GHPair(g[i], h[i]); }
    server.encrypt(gh);                                          // encrypt_gh_pairs
    for (int i = 0; i < 5; i++) gh.host_data()[i].encrypted = true;
    party.encrypt(hist);                                         // encrypt_histogram (public key)
    for (int i = 0; i < 5; i++) {
        hist.host_data()[i].encrypted = true;
        // party-side homomorphic add (GHPair::operator+ through paillier.add)
        party.add(hist.host_data()[i].g_enc, hist.host_data()[i].g_enc, gh.host_data()[i].g_enc);
        party.add(hist.host_data()[i].h_enc, hist.host_data()[i].h_enc, gh.host_data()[i].h_enc);
    }
    if (mode == "short") server.dec_short = true;                // p half of the CRT only
    server.decrypt(hist);                                        // decrypt_gh_pairs
    int bad = 0;
    for (int i = 0; i < 5; i++) {
        auto &p = hist.host_data()[i];
        if (std::fabs(p.g - 2 * g[i]) > 3e-6 || std::fabs(p.h - 2 * h[i]) > 3e-6) bad++;
        printf("%d: g %.6f (want %.6f)  h %.6f (want %.6f)\n", i, p.g, 2 * g[i], p.h, 2 * h[i]);
    }
    if (argc > 2 && std::string(argv[2]) == "big") {            // the multi-threaded marshalling path
        const size_t N = 300000;
        SyncArray<GHPair> big(N);
        for (size_t i = 0; i < N; i++) big.host_data()[i] = GHPair(1e-6f * (float)(i % 100000), -0.5f);
        server.encrypt(big);
        for (size_t i = 0; i < N; i++) big.host_data()[i].encrypted = true;
        server.decrypt(big);
        for (size_t i = 0; i < N; i += 997) {
            const auto &p = big.host_data()[i];
            if (std::fabs(p.g - 1e-6f * (float)(i % 100000)) > 2e-6 || std::fabs(p.h + 0.5f) > 2e-6) bad++;
        }
        printf("big batch of %zu checked\n", N);
    }
    GHPair one = gh.host_data()[0];
    server.decrypt(one);                                         // decrypt_gh
    if (std::fabs(one.g - g[0]) > 2e-6) bad++;
    printf("shim %s\n", bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
