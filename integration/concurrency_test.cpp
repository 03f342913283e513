// Reentrancy of the boundary through integration/paillier_hip.h.  FedTree enters the
// HE interface from OpenMP regions (encrypt_histogram per party, FLtrainer.cpp:275-306;
// decrypt_gh per node, :758-764; the distributed decode loops, distributed_server.cpp:1427):
// T host threads share ONE key object, each on its own engine context (thread_ctx),
// issuing small batch and single-element calls concurrently.  Every result is checked.
//   concurrency_test [bits] [threads] [iters] [default|exact|public_exact]
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "paillier_hip.h"

int main(int argc, char **argv) {
    int bits = argc > 1 ? std::atoi(argv[1]) : 1024;
    int T = argc > 2 ? std::atoi(argv[2]) : 16;
    int iters = argc > 3 ? std::atoi(argv[3]) : 24;
    Paillier_HIP server;
    server.keygen(bits);
    const std::string mode = argc > 4 ? argv[4] : "default";
    if (mode == "exact") server.enc_mode = Paillier_HIP::EncMode::FixedBaseExact;
    if (mode == "public_exact") server.publish_bases();  // the party encrypts from the published bases
    Paillier_HIP party;
    party = server;                                   // public part, shared by the party threads
    if (mode == "public_exact") party.enc_mode = Paillier_HIP::EncMode::FixedBaseExact;
    std::atomic<int> bad{0}, done{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            try {
                for (int it = 0; it < iters; it++) {
                    const float g0 = 0.001f * (float)(t * iters + it), g1 = -0.25f + 0.01f * (float)t;
                    SyncArray<GHPair> a(3);
                    a.host_data()[0] = GHPair(g0, 1.0f);
                    a.host_data()[1] = GHPair(g1, 0.5f);
                    a.host_data()[2] = GHPair(-g0, 2.0f);
                    ((t + it) % 2 ? party : server).encrypt(a);          // server or party side
                    for (int i = 0; i < 3; i++) a.host_data()[i].encrypted = true;
                    GHPair &x = a.host_data()[0], &y = a.host_data()[1];
                    party.add(x.g_enc, x.g_enc, y.g_enc);                // aliased in-place add
                    party.add(x.h_enc, x.h_enc, y.h_enc);
                    GHPair one = x;                                      // decrypt_gh: one element
                    server.decrypt(one);
                    if (std::fabs(one.g - (g0 + g1)) > 3e-6 || std::fabs(one.h - 1.5f) > 3e-6) bad++;
                    server.decrypt(a);                                   // decrypt_gh_pairs: the batch
                    if (std::fabs(a.host_data()[2].g + g0) > 2e-6 || std::fabs(a.host_data()[2].h - 2.0f) > 2e-6) bad++;
                    done++;
                }
            } catch (const std::exception &e) {
                std::fprintf(stderr, "thread %d: %s\n", t, e.what());
                bad++;
            }
        });
    for (auto &x : th) x.join();
    std::printf("threads %d x iters %d: %d done, %d bad -> concurrency %s\n", T, iters, done.load(), bad.load(),
                bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
