// Rate of FedTree's party histogram loop with its callers unchanged (hist_tree_builder.cpp:572-591): an
// OpenMP loop over features, each thread running `dest = dest + src` per instance through GHPair's
// operator+ (integration/mock/FedTree/common.h, the common.h:150-195 text) on the USE_HIP key.  Each
// operator issues two fthe_add_shared calls (g, h), merged across the threads by the key's queue; the
// first add into an empty bin promotes it with homo_encrypt (two fthe_encrypt_shared calls, Q10).
// Checked: every populated bin decrypts to the codec sum of its members.
//   ghpair_rate [bits] [threads = features] [instances] [bins]      -> one JSON line
#include <omp.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "paillier_hip.h"

int main(int argc, char **argv) {
    const int bits = argc > 1 ? std::atoi(argv[1]) : 2048;
    const int F = argc > 2 ? std::atoi(argv[2]) : 32;
    const int N = argc > 3 ? std::atoi(argv[3]) : 512;
    const int B = argc > 4 ? std::atoi(argv[4]) : 16;
    if (bits <= 0 || F <= 0 || N <= 0 || B <= 0) return 2;
    Paillier_HIP server;
    server.keygen(bits);
    SyncArray<GHPair> gh(N);
    std::vector<float> g0(N), h0(N);
    for (int i = 0; i < N; i++) {
        g0[i] = 0.001f * (float)(i % 100) - 0.05f;
        h0[i] = 0.25f + 0.001f * (float)(i % 50);
        gh.host_data()[i] = GHPair(g0[i], h0[i]);
    }
    server.encrypt(gh);
    for (int i = 0; i < N; i++) {                     // encrypt_gh_pairs marks the pairs (server.h:113-121)
        gh.host_data()[i].encrypted = true;
        gh.host_data()[i].paillier = server.paillier_cpu;
    }
    auto bin_of = [&](int iid, int fid) { return (iid * 7 + fid * 3) % B; };
    {   // first use of the key's queue (its context) outside the timed loop
        GHPair a = gh.host_data()[0], b = gh.host_data()[1];
        GHPair s = a + b;
        (void)s;
    }
    std::vector<GHPair> hist((size_t)F * B);          // GHPair(): plain zeros, as the histogram starts
    const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(F) schedule(static)
    for (int fid = 0; fid < F; fid++) {
        for (int iid = 0; iid < N; iid++) {
            const GHPair src = gh.host_data()[iid];
            GHPair &dest = hist[(size_t)fid * B + bin_of(iid, fid)];
            dest = dest + src;
        }
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // check: the codec sums (long)(x * 1e6) of each bin's members
    std::vector<int64_t> wg(hist.size(), 0), wh(hist.size(), 0);
    for (int fid = 0; fid < F; fid++)
        for (int iid = 0; iid < N; iid++) {
            const size_t b = (size_t)fid * B + bin_of(iid, fid);
            wg[b] += (long)(g0[iid] * 1e6);
            wh[b] += (long)(h0[iid] * 1e6);
        }
    SyncArray<GHPair> out(hist.size());
    int populated = 0;
    for (size_t b = 0; b < hist.size(); b++) {
        out.host_data()[b] = hist[b];
        populated += hist[b].encrypted;
    }
    server.decrypt(out);
    int bad = 0;
    for (size_t b = 0; b < hist.size(); b++) {
        if (!hist[b].encrypted) continue;
        const double eg = (double)wg[b] / 1e6, eh = (double)wh[b] / 1e6;
        if (std::fabs(out.host_data()[b].g - eg) > 1e-5 + 1e-6 * std::fabs(eg) ||
            std::fabs(out.host_data()[b].h - eh) > 1e-5 + 1e-6 * std::fabs(eh))
            bad++;
    }
    const double ops = (double)F * N;
    std::printf("{\"bits\": %d, \"threads\": %d, \"instances\": %d, \"bins\": %d, \"operators\": %.0f, "
                "\"ciphertext_adds\": %.0f, \"promotions\": %d, \"s\": %.4f, \"operators_per_s\": %.0f, "
                "\"ciphertext_adds_per_s\": %.0f, \"bad_bins\": %d, \"ok\": %s}\n",
                bits, F, N, B, ops, 2 * ops, populated, s, ops / s, 2 * ops / s, bad, bad ? "false" : "true");
    return bad ? 1 : 0;
}
