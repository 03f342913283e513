// Host side of a multi-GPU server: the mpz_t <-> row marshalling of
// Paillier_HIP::encrypt / decrypt(SyncArray<GHPair>&) (integration/paillier_hip.h: encode_pairs,
// rows_to_pairs, pairs_to_rows, decode_pairs -- the code those calls run around the engine, the reference's
// to_mpz / from_mpz loops of paillier_gpu.cu:6-21, 240-258, 299-310) for S concurrent shards, one host
// thread per shard as a server driving S GPUs would (fedtree_amd/multi.py's layout), each shard's loops on
// up to 16 threads as in the class.  No engine call and no kernel: rows are synthetic ciphertext-sized words.
//   marshal_rate [bits] [pairs per shard] [reps] [shard counts, comma list]   -> one JSON line
// Per shard count: ciphertexts per second through each direction (encrypt: codec + rows -> mpz_import;
// decrypt: mpz_export -> rows + codec), aggregated over the shards, and the host CPUs the process may use.
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "paillier_hip.h"

int main(int argc, char **argv) {
    const int bits = argc > 1 ? std::atoi(argv[1]) : 2048;
    const size_t N = argc > 2 ? (size_t)std::atoll(argv[2]) : 250000;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
    std::vector<int> shards;
    {
        std::stringstream ss(argc > 4 ? argv[4] : "1,2,4,8");
        std::string t;
        while (std::getline(ss, t, ',')) shards.push_back(std::atoi(t.c_str()));
    }
    if (bits <= 0 || bits % 32 || N == 0 || reps <= 0 || shards.empty()) return 2;
    const int cw = 2 * bits / 32;                       // u32 words of one ciphertext row (n^2)
    {   // the limb-copy marshalling (fthe_ghpair_key.h) against GMP's own import / export on edge rows:
        // zero, one word, every top-word position (odd and even), all ones
        int bad = 0;
        std::vector<uint32_t> w(cw), back(cw), ref(cw);
        mpz_t a, b;
        mpz_init(a);
        mpz_init(b);
        std::mt19937 rng(7);
        for (int top = -1; top < cw; top++)
            for (int pat = 0; pat < 3; pat++) {
                for (int i = 0; i < cw; i++) w[i] = i <= top ? (pat == 0 ? 0xffffffffu : pat == 1 ? 1u : rng()) : 0u;
                if (top >= 0 && w[top] == 0) w[top] = 1;
                fthe_shim::from_words(a, w.data(), cw);
                mpz_import(b, (size_t)cw, -1, 4, 0, 0, w.data());
                bad += mpz_cmp(a, b) != 0;
                fthe_shim::to_words(a, back.data(), cw);
                std::fill(ref.begin(), ref.end(), 0u);
                mpz_export(ref.data(), nullptr, -1, 4, 0, 0, b);
                bad += back != ref || back != w;
            }
        mpz_clear(a);
        mpz_clear(b);
        if (bad) { std::fprintf(stderr, "limb-copy marshalling differs from mpz_import/export (%d)\n", bad); return 1; }
    }
    cpu_set_t cs;
    CPU_ZERO(&cs);
    const int cpus = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : -1;
    const int smax = *std::max_element(shards.begin(), shards.end());
    // per shard: the pairs, their ciphertext rows (full-size random words below 2^(2 bits - 1)), plaintexts
    std::vector<SyncArray<GHPair>> pairs;
    std::vector<std::vector<uint32_t>> rows(smax);
    std::vector<std::vector<uint64_t>> msg(smax);
    pairs.reserve(smax);
    for (int s = 0; s < smax; s++) {
        pairs.emplace_back(N);
        std::mt19937 rng(1234 + s);
        rows[s].resize(2 * N * (size_t)cw);
        for (auto &w : rows[s]) w = rng();
        for (size_t i = 0; i < 2 * N; i++) rows[s][i * cw + cw - 1] &= 0x7fffffffu;
        msg[s].resize(2 * N);
        GHPair *d = pairs[s].host_data();
        for (size_t i = 0; i < N; i++) {
            d[i].g = 0.001f * (float)(i % 1000) - 0.5f;
            d[i].h = 0.25f;
            d[i].encrypted = true;
        }
        Paillier_HIP::rows_to_pairs(d, N, rows[s].data(), cw);   // every pair holds full-size mpz fields
    }
    auto run = [&](int S, bool enc) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int s = 0; s < S; s++)
            th.emplace_back([&, s] {
                GHPair *d = pairs[s].host_data();
                if (enc) {
                    Paillier_HIP::encode_pairs(d, N, msg[s].data());
                    Paillier_HIP::rows_to_pairs(d, N, rows[s].data(), cw);
                } else {
                    Paillier_HIP::pairs_to_rows(d, N, rows[s].data(), cw);
                    Paillier_HIP::decode_pairs(d, N, msg[s].data());
                }
            });
        for (auto &t : th) t.join();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    std::printf("{\"bits\": %d, \"pairs_per_shard\": %zu, \"host_cpus\": %d, \"threads_per_shard_max\": 16, "
                "\"reps\": %d, \"shards\": [", bits, N, cpus, reps);
    for (size_t k = 0; k < shards.size(); k++) {
        const int S = shards[k];
        double te = 1e30, td = 1e30;
        for (int r = 0; r < reps; r++) {
            te = std::min(te, run(S, true));
            td = std::min(td, run(S, false));
        }
        const double cts = 2.0 * N * S;
        std::printf("%s{\"shards\": %d, \"ciphertexts\": %.0f, \"encrypt_side_s\": %.4f, \"decrypt_side_s\": %.4f, "
                    "\"encrypt_side_per_s\": %.0f, \"decrypt_side_per_s\": %.0f}",
                    k ? ", " : "", S, cts, te, td, cts / te, cts / td);
    }
    // a round trip leaves the rows as they were: the marshalling is lossless
    int bad = 0;
    for (int s = 0; s < smax && !bad; s++) {
        std::vector<uint32_t> back(rows[s].size());
        Paillier_HIP::pairs_to_rows(pairs[s].host_data(), N, back.data(), cw);
        bad = back != rows[s];
    }
    std::printf("], \"round_trip_ok\": %s}\n", bad ? "false" : "true");
    return bad ? 1 : 0;
}
