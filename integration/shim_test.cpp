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
#ifdef FTHE_ENABLE_NONREFERENCE_MODES
    if (argc > 2 && std::string(argv[2]) == "exact_known_order") server.keygen_mode = Paillier_HIP::KeygenMode::KnownOrder;
#endif
    server.keygen(bits);                 // homo_init (NTL semantics: n of `bits` bits)
    const std::string mode = argc > 2 ? argv[2] : "default";
    if (mode == "public_exact") server.publish_bases();          // bases travel with the public key
    Paillier_HIP party;                  // Party::paillier
    party = server;                      // Server::send_key: public part only
    if (mode.rfind("exact", 0) == 0 || mode == "public_exact")  // table-driven randomizer; the party (no p, q)
        server.enc_mode = party.enc_mode = Paillier_HIP::EncMode::FixedBaseExact;   // published bases, else default
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
    if (mode == "helpers") {                                     // histogram / merge / sibling subtract
        const int n = 40, n_col = 2, cut[3] = {0, 4, 7}, missing = 255;
        std::vector<unsigned char> bins(n * n_col);
        SyncArray<GHPair> ggh(n);
        double want_g[7] = {0}, want_h[7] = {0};
        for (int i = 0; i < n; i++) {
            const float gi = 0.01f * (float)(i % 13) - 0.05f, hi = 0.02f * (float)(i % 7) + 0.1f;
            ggh.host_data()[i] = GHPair(gi, hi);
            bins[i * n_col] = (unsigned char)(i % 4);
            bins[i * n_col + 1] = (unsigned char)(i % 5 == 4 ? missing : i % 3);
            for (int f = 0; f < n_col; f++) {
                const int b = bins[i * n_col + f];
                if (b == missing) continue;
                want_g[cut[f] + b] += (double)(long)(gi * 1e6) / 1e6;
                want_h[cut[f] + b] += (double)(long)(hi * 1e6) / 1e6;
            }
        }
        server.encrypt(ggh);
        for (int i = 0; i < n; i++) ggh.host_data()[i].encrypted = true;
        SyncArray<GHPair> h1(7), merged(7), sib(7);
        party.histogram(ggh, bins.data(), cut, n_col, missing, h1);   // party side, public key
        SyncArray<GHPair> hz(7);
        party.histogram(ggh, bins.data(), cut, n_col, missing, hz, true);   // Enc(0) first (Q10)
        server.decrypt(hz);
        for (int s = 0; s < 7; s++)
            if (std::fabs(hz.host_data()[s].g - want_g[s]) > 1e-5 || std::fabs(hz.host_data()[s].h - want_h[s]) > 1e-5) bad++;
        SyncArray<GHPair> h2(7), h3(7);
        for (int s = 0; s < 7; s++) { h2.host_data()[s] = h1.host_data()[s]; h3.host_data()[s] = h1.host_data()[s]; }
        h3.host_data()[6] = GHPair(0.5f, 0.25f);                        // an unencrypted operand is promoted
        party.merge({&h1, &h2, &h3}, merged, true);
        party.subtract(merged, h1, sib);
        SyncArray<GHPair> pre(7);
        for (int s = 0; s < 7; s++) pre.host_data()[s] = h1.host_data()[s];
        party.prefix(pre, cut, n_col);                                  // per-feature inclusive scan
        server.decrypt(pre);
        double acc = 0;
        for (int s = 0; s < 7; s++) {
            acc = (s == cut[0] || s == cut[1]) ? want_g[s] : acc + want_g[s];
            if (std::fabs(pre.host_data()[s].g - acc) > 2e-5) bad++;
            printf("bin %d: prefix g %.6f (want %.6f)\n", s, pre.host_data()[s].g, acc);
        }
        server.decrypt(h1);
        server.decrypt(merged);
        server.decrypt(sib);
        for (int s = 0; s < 7; s++) {
            const double g3 = s == 6 ? 2 * want_g[s] + 0.5 : 3 * want_g[s], h3v = s == 6 ? 2 * want_h[s] + 0.25 : 3 * want_h[s];
            if (std::fabs(h1.host_data()[s].g - want_g[s]) > 1e-5 || std::fabs(h1.host_data()[s].h - want_h[s]) > 1e-5) bad++;
            if (std::fabs(merged.host_data()[s].g - g3) > 1e-5 || std::fabs(merged.host_data()[s].h - h3v) > 1e-5) bad++;
            if (std::fabs(sib.host_data()[s].g - (g3 - want_g[s])) > 1e-5) bad++;
            printf("bin %d: hist g %.6f (want %.6f)  merged g %.6f (want %.6f)  sibling g %.6f\n", s,
                   h1.host_data()[s].g, want_g[s], merged.host_data()[s].g, g3, sib.host_data()[s].g);
        }
    }
    GHPair one = gh.host_data()[0];
    server.decrypt(one);                                         // decrypt_gh
    if (std::fabs(one.g - g[0]) > 2e-6) bad++;
    printf("shim %s\n", bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
