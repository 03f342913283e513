// The USE_HIP GHPair key's host-side operators without a GPU: Paillier_HIP_Pub bound to a public n only
// (bind_n) adds on the host, so GHPair's operator+ / += (common.h:150-237) and add(s, s, c) reproduce the
// reference's golden adds (tests/golden, Paillier_GMP::add = x y mod n^2, paillier_gmp.cpp:16-21).
//   host_ops_test check <fixture>      fixture: n, then (x y want) triples, hex     -> "host ops OK"
//   host_ops_test rate <fixture> <threads> <ops_per_thread>
//       per-element rates on this host: bare mpz x y mod n^2 (the reference's add) and
//       `dest = dest + src` through GHPair::operator+ (2 adds per operator)            -> one JSON line
#include <omp.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "fthe_ghpair_key.h"
#include "FedTree/common.h"

static void set_hex(mpz_t x, const std::string &s) {
    if (mpz_set_str(x, s.c_str(), 16) != 0) { std::fprintf(stderr, "bad hex token\n"); std::exit(2); }
}

int main(int argc, char **argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: host_ops_test check|rate <fixture> [threads ops]\n"); return 2; }
    const std::string mode = argv[1];
    std::ifstream in(argv[2]);
    std::string tok;
    mpz_t n;
    mpz_init(n);
    in >> tok;
    set_hex(n, tok);
    Paillier_HIP_Pub key;
    key.bind_n(n, (uint32_t)mpz_sizeinbase(n, 2));
    std::vector<GHPair> xs, ys;
    std::vector<std::string> want;
    std::string a, b, w;
    while (in >> a >> b >> w) {
        GHPair x, y;
        set_hex(x.g_enc, a); set_hex(x.h_enc, b);
        set_hex(y.g_enc, b); set_hex(y.h_enc, a);
        x.encrypted = y.encrypted = true;
        x.paillier = key; y.paillier = key;
        xs.push_back(x); ys.push_back(y);
        want.push_back(w);
    }
    if (xs.empty()) { std::fprintf(stderr, "empty fixture\n"); return 2; }
    if (mode == "check") {
        int bad = 0;
        mpz_t wv, t;
        mpz_inits(wv, t, nullptr);
        for (size_t i = 0; i < xs.size(); i++) {
            set_hex(wv, want[i]);
            GHPair s = xs[i] + ys[i];                       // g: x y, h: y x
            bad += mpz_cmp(s.g_enc, wv) != 0 || mpz_cmp(s.h_enc, wv) != 0;
            GHPair d = xs[i];
            d += ys[i];                                     // the aliased add(g_enc, g_enc, rhs.g_enc)
            bad += mpz_cmp(d.g_enc, wv) != 0 || mpz_cmp(d.h_enc, wv) != 0;
            mpz_set(t, xs[i].g_enc);
            key.add(t, t, ys[i].g_enc);                     // add(s, s, c): the product, not 0 (Q11)
            bad += mpz_cmp(t, wv) != 0;
            // unreduced operands (the reference reduces the product whatever its inputs)
            mpz_add(t, xs[i].g_enc, key.n_square);
            key.add(t, t, ys[i].g_enc);
            bad += mpz_cmp(t, wv) != 0;
        }
        // copies share the cell, views read n, n^2, g = n + 1; a caller's write to a view stays private
        Paillier_HIP_Pub k2 = key, k3;
        k3 = k2;
        bad += k3.cell() != key.cell() || mpz_cmp(k3.n, n) != 0;
        mpz_mul(t, n, n);
        bad += mpz_cmp(k3.n_square, t) != 0;
        mpz_add_ui(t, n, 1);
        bad += mpz_cmp(k3.generator, t) != 0;
        mpz_set_ui(k3.generator, 7);
        bad += mpz_cmp(key.generator, t) != 0 || mpz_cmp_ui(k3.generator, 7) != 0;
        k3 = key;
        bad += mpz_cmp(k3.generator, t) != 0;
        mpz_clears(wv, t, nullptr);
        std::printf("%zu adds, %d mismatches -> host ops %s\n", xs.size(), bad, bad ? "FAIL" : "OK");
        return bad ? 1 : 0;
    }
    if (mode != "rate" || argc < 5) return 2;
    const int T = std::atoi(argv[3]), per = std::atoi(argv[4]);
    const size_t K = xs.size();
    // the reference's add: mpz_mul + mpz_mod into the result (paillier_gmp.cpp:16-21, minus its mpz_init leak)
    auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel num_threads(T)
    {
        mpz_t r;
        mpz_init(r);
        const int id = omp_get_thread_num();
        for (int i = 0; i < per; i++) {
            mpz_mul(r, xs[(id + i) % K].g_enc, ys[(id + 3 * i) % K].g_enc);
            mpz_mod(r, r, key.n_square);
        }
        mpz_clear(r);
    }
    const double bare = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<GHPair> acc(T);
    for (int id = 0; id < T; id++) acc[id] = xs[id % K];
    t0 = std::chrono::steady_clock::now();
#pragma omp parallel num_threads(T)
    {
        const int id = omp_get_thread_num();
        GHPair &dest = acc[id];
        for (int i = 0; i < per / 2; i++) dest = dest + ys[(id + i) % K];    // 2 adds per operator
    }
    const double ops = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double nadd = (double)T * per, nop_adds = (double)T * (per / 2) * 2;
    std::printf("{\"threads\": %d, \"bare_adds_per_s\": %.0f, \"operator_adds_per_s\": %.0f, \"ratio\": %.3f}\n", T,
                nadd / bare, nop_adds / ops, (nop_adds / ops) / (nadd / bare));
    return 0;
}
