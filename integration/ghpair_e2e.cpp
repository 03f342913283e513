// End-to-end rate of the drop-in's batch boundary at FedTree's own types: Server::encrypt_gh_pairs /
// decrypt_gh_pairs (server.h:105-135) call Paillier_HIP::encrypt / decrypt(SyncArray<GHPair>&)
// (integration/paillier_hip.h; Paillier_GPU::encrypt / decrypt, paillier_gpu.cu:211-313, 448-494), which
// marshal every ciphertext between mpz_t and engine rows (mpz_import / mpz_export, as the reference does
// at paillier_gpu.cu:240-258, 299-310) around one engine call with host buffers (PCIe both ways).
//   ghpair_e2e [bits] [pairs] [reps]      -> one JSON line (best of reps; every plaintext checked)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "paillier_hip.h"

int main(int argc, char **argv) {
    const int bits = argc > 1 ? std::atoi(argv[1]) : 2048;
    const size_t N = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 2000000;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 2;
    if (bits <= 0 || N == 0 || reps <= 0) return 2;
    Paillier_HIP server;
    server.keygen(bits);
    std::vector<float> g0(N), h0(N);
    for (size_t i = 0; i < N; i++) {
        g0[i] = 0.0001f * (float)((i * 7919) % 20001) - 1.0f;     // logistic-loss range gradients
        h0[i] = 0.00001f * (float)((i * 104729) % 25001);
    }
    SyncArray<GHPair> gh(N);
    {   // engine warm-up (context, programs) outside the timed calls
        SyncArray<GHPair> w(1024);
        server.encrypt(w);
        server.decrypt(w);
    }
    double enc_best = 1e30, dec_best = 1e30;
    int bad = 0;
    for (int rep = 0; rep < reps; rep++) {
        auto *d = gh.host_data();
        for (size_t i = 0; i < N; i++) { d[i].g = g0[i]; d[i].h = h0[i]; d[i].encrypted = false; }
        auto t0 = std::chrono::steady_clock::now();
        server.encrypt(gh);                                       // encrypt_gh_pairs (server.h:105-121)
        const double te = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (size_t i = 0; i < N; i++) d[i].encrypted = true;     // server.h:116-119 marks them
        t0 = std::chrono::steady_clock::now();
        server.decrypt(gh);                                       // decrypt_gh_pairs (server.h:123-135)
        const double td = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        enc_best = std::min(enc_best, te);
        dec_best = std::min(dec_best, td);
        for (size_t i = 0; i < N; i++)
            if (d[i].g != fthe_shim::decode(fthe_shim::encode(g0[i])) || d[i].h != fthe_shim::decode(fthe_shim::encode(h0[i])))
                bad++;
    }
    std::printf("{\"bits\": %d, \"pairs\": %zu, \"ciphertexts\": %zu, \"reps\": %d, \"encrypt_s\": %.4f, "
                "\"decrypt_s\": %.4f, \"encrypts_per_s\": %.0f, \"decrypts_per_s\": %.0f, \"bad\": %d, \"ok\": %s}\n",
                bits, N, 2 * N, reps, enc_best, dec_best, 2.0 * N / enc_best, 2.0 * N / dec_best, bad,
                bad ? "false" : "true");
    return bad ? 1 : 0;
}
