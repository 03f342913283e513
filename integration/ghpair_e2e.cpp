// End-to-end rate of the drop-in's batch boundary at FedTree's own types: Server::encrypt_gh_pairs /
// decrypt_gh_pairs (server.h:105-135) call Paillier_HIP::encrypt / decrypt(SyncArray<GHPair>&)
// (integration/paillier_hip.h; Paillier_GPU::encrypt / decrypt, paillier_gpu.cu:211-313, 448-494), which
// marshal every ciphertext between mpz_t and engine rows (mpz_import / mpz_export, as the reference does
// at paillier_gpu.cu:240-258, 299-310) around one engine call with host buffers (PCIe both ways).
//   ghpair_e2e [bits] [pairs] [reps] [devices] -> one JSON line (best of reps; every plaintext checked)
// devices: the FTHE_DEVICES list the batch calls shard over ("0,1,2,3"; "0,0" = two contexts on device 0), or a
// count k for devices 0 .. k-1; default: the environment's (FTHE_DEVICES, else every visible GPU).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "paillier_hip.h"

int main(int argc, char **argv) {
    const int bits = argc > 1 ? std::atoi(argv[1]) : 2048;
    const size_t N = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 2000000;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 2;
    if (bits <= 0 || N == 0 || reps <= 0) return 2;
    if (argc > 4) {                                   // before the first engine call reads the device list
        std::string dl = argv[4];
        if (dl.find(',') == std::string::npos) {
            const int k = std::atoi(argv[4]);
            if (k <= 0) return 2;
            dl.clear();
            for (int i = 0; i < k; i++) dl += (i ? "," : "") + std::to_string(i);
        }
        setenv("FTHE_DEVICES", dl.c_str(), 1);
    }
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
    std::printf("{\"bits\": %d, \"pairs\": %zu, \"ciphertexts\": %zu, \"reps\": %d, \"shards\": %zu, "
                "\"encrypt_s\": %.4f, \"decrypt_s\": %.4f, \"encrypts_per_s\": %.0f, \"decrypts_per_s\": %.0f, "
                "\"bad\": %d, \"ok\": %s}\n",
                bits, N, 2 * N, reps, fthe_shim::shard_plan(2 * N, fthe_shim::shard_devices().size(),
                                                             fthe_shim::shard_min_rows()).size(),
                enc_best, dec_best, 2.0 * N / enc_best, 2.0 * N / dec_best, bad, bad ? "false" : "true");
    return bad ? 1 : 0;
}
