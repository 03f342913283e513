// Rate of FedTree's party histogram loop with its callers unchanged (hist_tree_builder.cpp:572-591): an
// OpenMP loop over features, each thread running `dest = dest + src` per instance through GHPair's
// operator+ (integration/mock/FedTree/common.h, the common.h:150-195 text) on the USE_HIP key.  Each
// operator makes two host adds (g, h: x y mod n^2, integration/fthe_ghpair_key.h); the first add into an
// empty bin promotes it with homo_encrypt (two pooled encryptions, Q10).  Checked: every populated bin
// decrypts to the codec sum of its members.  The same run times the reference's own per-element add
// (Paillier_GMP::add = mpz_mul + mpz_mod, paillier_gmp.cpp:16-21) on the same threads and operands.
// Then the sibling subtraction (hist_tree_builder.cpp:672-680, and missing_gh :715-726): an OpenMP loop over
// bins, `dest[i] = father[i] - child[i]` through GHPair::operator- (common.h:253-337: two mul(x, 2^64 - 1)
// and two adds per operator), timed beside the reference GPU build's own per-element work on the same threads
// and operands (Paillier_GPU::mul = mpz_powm(x, 2^64 - 1, n^2), paillier_gpu.cu:65-67, then
// Paillier_GPU::add = mpz_mul + mpz_mod, :57-61).  Checked: every difference decrypts to the codec difference.
// Both legs run interleaved for `rounds` rounds (default 7) and the comparison is the median over rounds of the
// per-round ratio reference time / operator time: a shared host's drift hits both legs of a round alike.
//   ghpair_rate [bits] [threads = features] [instances] [bins] [sub_bins] [rounds]    -> one JSON line
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "paillier_hip.h"

int main(int argc, char **argv) {
    const int bits = argc > 1 ? std::atoi(argv[1]) : 2048;
    const int F = argc > 2 ? std::atoi(argv[2]) : 32;
    const int N = argc > 3 ? std::atoi(argv[3]) : 512;
    const int B = argc > 4 ? std::atoi(argv[4]) : 16;
    const int SB = argc > 5 ? std::atoi(argv[5]) : 4096;
    const int R = argc > 6 ? std::atoi(argv[6]) : 7;
    if (bits <= 0 || F <= 0 || N <= 0 || B <= 0 || SB < 0 || R < 1) return 2;
    auto median = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        const size_t h = v.size() / 2;
        return v.size() % 2 ? v[h] : 0.5 * (v[h - 1] + v[h]);
    };
    auto ratios = [](const std::vector<double> &num, const std::vector<double> &den) {
        std::vector<double> r;
        for (size_t i = 0; i < num.size() && i < den.size(); i++) r.push_back(num[i] / den[i]);
        return r;
    };
    auto arr = [](const std::vector<double> &v) {
        std::string o = "[";
        char b[32];
        for (size_t i = 0; i < v.size(); i++) {
            std::snprintf(b, sizeof b, "%s%.4f", i ? ", " : "", v[i]);
            o += b;
        }
        return o + "]";
    };
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
    {   // the key's randomizer pool fills in the background from keygen on (as it has long before
        // FedTree's first histogram); wait for its first batch outside the timed loop
        const auto w0 = std::chrono::steady_clock::now();
        while (server.paillier_cpu.cell()->pooled() == 0 &&
               std::chrono::steady_clock::now() - w0 < std::chrono::seconds(20))
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        GHPair a = gh.host_data()[0], b = gh.host_data()[1];
        GHPair s = a + b;
        (void)s;
    }
    // the reference's add on the same threads and operands (one mpz_mul + mpz_mod per ciphertext add),
    // alternated with the operator loop, R rounds each, medians reported (short runs on a shared host are
    // noisy; every round of the operator loop starts from a fresh, unencrypted histogram)
    auto ref_round = [&]() {
        const auto r0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(F) schedule(static)
        for (int fid = 0; fid < F; fid++) {
            mpz_t r;
            mpz_init(r);
            for (int iid = 0; iid < N; iid++) {
                const GHPair &x = gh.host_data()[iid], &y = gh.host_data()[(iid * 7 + fid) % N];
                mpz_mul(r, x.g_enc, y.g_enc);
                mpz_mod(r, r, server.paillier_cpu.n_square);
                mpz_mul(r, x.h_enc, y.h_enc);
                mpz_mod(r, r, server.paillier_cpu.n_square);
            }
            mpz_clear(r);
        }
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - r0).count();
    };
    std::vector<GHPair> hist;
    auto op_round = [&]() {
        hist.assign((size_t)F * B, GHPair());            // GHPair(): plain zeros, as the histogram starts
        const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(F) schedule(static)
        for (int fid = 0; fid < F; fid++) {
            for (int iid = 0; iid < N; iid++) {
                const GHPair src = gh.host_data()[iid];
                GHPair &dest = hist[(size_t)fid * B + bin_of(iid, fid)];
                dest = dest + src;
            }
        }
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    std::vector<double> ref_all, op_all;
    for (int rep = 0; rep < R; rep++) {
        ref_all.push_back(ref_round());
        op_all.push_back(op_round());
    }
    const double ref_s = median(ref_all), s = median(op_all), vs_add = median(ratios(ref_all, op_all));
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
    // -- sibling subtraction: father - child per bin (both encrypted: the encrypted-rhs branch) --
    double sub_s = 0, sub_ref_s = 0, vs_sub = 0;
    std::vector<double> sub_all, sub_ref_all;
    int sub_bad = 0;
    if (SB > 0) {
        std::vector<GHPair> father(SB), child(SB), diff(SB);
        std::vector<float> fg(SB), fh(SB), cg(SB), ch(SB);
        {
            SyncArray<GHPair> fc(2 * (size_t)SB);
            for (int i = 0; i < SB; i++) {
                fg[i] = 0.002f * (float)(i % 97) - 0.09f;   fh[i] = 1.5f + 0.003f * (float)(i % 41);
                cg[i] = 0.001f * (float)(i % 89) - 0.04f;   ch[i] = 0.5f + 0.002f * (float)(i % 37);
                fc.host_data()[i] = GHPair(fg[i], fh[i]);
                fc.host_data()[SB + i] = GHPair(cg[i], ch[i]);
            }
            server.encrypt(fc);
            for (int i = 0; i < 2 * SB; i++) {
                fc.host_data()[i].encrypted = true;
                fc.host_data()[i].paillier = server.paillier_cpu;
            }
            for (int i = 0; i < SB; i++) { father[i] = fc.host_data()[i]; child[i] = fc.host_data()[SB + i]; }
        }
        const int T = F;
        auto sub_round = [&]() {
            const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(T) schedule(static)
            for (int i = 0; i < SB; i++) diff[i] = father[i] - child[i];
            return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        };
        // the reference GPU build's per-element work for one operator-: mpz_powm(x, 2^64 - 1, n^2) and a
        // product mod n^2, for g and h
        auto sub_ref_round = [&]() {
            const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel num_threads(T)
            {
                mpz_t mo, r, t;
                mpz_init(r); mpz_init(t); mpz_init(mo);
                const long m1 = -1;
                mpz_import(mo, 1, -1, sizeof(m1), 0, 0, &m1);
#pragma omp for schedule(static)
                for (int i = 0; i < SB; i++) {
                    mpz_powm(t, child[i].g_enc, mo, server.paillier_cpu.n_square);
                    mpz_mul(r, father[i].g_enc, t);
                    mpz_mod(r, r, server.paillier_cpu.n_square);
                    mpz_powm(t, child[i].h_enc, mo, server.paillier_cpu.n_square);
                    mpz_mul(r, father[i].h_enc, t);
                    mpz_mod(r, r, server.paillier_cpu.n_square);
                }
                mpz_clear(r); mpz_clear(t); mpz_clear(mo);
            }
            return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        };
        for (int rep = 0; rep < R; rep++) {
            sub_ref_all.push_back(sub_ref_round());
            sub_all.push_back(sub_round());
        }
        sub_s = median(sub_all);
        sub_ref_s = median(sub_ref_all);
        vs_sub = median(ratios(sub_ref_all, sub_all));
        SyncArray<GHPair> dd(SB);
        for (int i = 0; i < SB; i++) dd.host_data()[i] = diff[i];
        server.decrypt(dd);
        for (int i = 0; i < SB; i++) {
            // decrypt_gh_pairs decodes the low 64 bits as a signed fixed-point value (Q6, Q9)
            const double eg = (double)((long)(fg[i] * 1e6) - (long)(cg[i] * 1e6)) / 1e6;
            const double eh = (double)((long)(fh[i] * 1e6) - (long)(ch[i] * 1e6)) / 1e6;
            if (!diff[i].encrypted || std::fabs(dd.host_data()[i].g - eg) > 1e-5 + 1e-6 * std::fabs(eg) ||
                std::fabs(dd.host_data()[i].h - eh) > 1e-5 + 1e-6 * std::fabs(eh))
                sub_bad++;
        }
    }
    const double sops = 2.0 * SB;   // ciphertext subtractions (g and h)
    const double ops = (double)F * N;
    std::printf("{\"bits\": %d, \"threads\": %d, \"instances\": %d, \"bins\": %d, \"operators\": %.0f, "
                "\"ciphertext_adds\": %.0f, \"promotions\": %d, \"s\": %.4f, \"operators_per_s\": %.0f, "
                "\"ciphertext_adds_per_s\": %.0f, \"reference_add_same_threads_per_s\": %.0f, "
                "\"vs_reference_add\": %.3f, \"rounds\": %d, \"rounds_s\": %s, \"reference_rounds_s\": %s, "
                "\"bad_bins\": %d, \"sub\": {\"bins\": %d, \"ciphertext_subs\": %.0f, \"s\": %.5f, "
                "\"ciphertext_subs_per_s\": %.0f, \"reference_sub_same_threads_per_s\": %.0f, \"vs_reference_sub\": %.3f, "
                "\"rounds_s\": %s, \"reference_rounds_s\": %s, \"bad_bins\": %d}, \"ok\": %s}\n",
                bits, F, N, B, ops, 2 * ops, 2 * populated, s, ops / s, 2 * ops / s, 2 * ops / ref_s,
                vs_add, R, arr(op_all).c_str(), arr(ref_all).c_str(),
                bad, SB, sops, SB ? sub_s : 0.0, SB ? sops / sub_s : 0.0, SB ? sops / sub_ref_s : 0.0,
                vs_sub, arr(sub_all).c_str(), arr(sub_ref_all).c_str(), sub_bad,
                (bad || sub_bad) ? "false" : "true");
    return (bad || sub_bad) ? 1 : 0;
}
