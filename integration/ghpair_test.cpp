// GHPair's operators (common.h:150-337 call shapes, integration/mock/FedTree/common.h) on the USE_HIP
// key (integration/fthe_ghpair_key.h), checked bit for bit against the reference's own outputs.
// Built with -DFTHE_REFERENCE_SHARED_R so that promotions of unencrypted operands use the
// reference's fixed r (Paillier_GMP::encrypt draws the same r on every call) and reproduce
// its ciphertexts.  Input (tests/test_integration_shim.py writes it from tests/golden/): whitespace-
// separated hex / decimal tokens
//   p q r                                  primes and the reference's shared r
//   ncase  c_0 .. c_{ncase-1}              golden ciphertexts
//   nadd   (i j want) x nadd               golden adds c_i c_j mod n^2
//   parties bins  ct[party][bin] ..  merged[bin] ..   golden 8-party merge, Enc(0) first (Q10)
//   nsub   (i j want) x nsub               c_i c_j^(2^64-1) mod n^2
//   g h j want_g want_h                    GHPair(g, h) - enc(c_j, c_j): plain lhs promoted (common.h:268-283)
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "paillier_hip.h"

static std::string next(std::istream &in) {
    std::string t;
    if (!(in >> t)) { std::fprintf(stderr, "input ended early\n"); std::exit(2); }
    return t;
}
static void set_hex(mpz_t x, const std::string &s) {
    if (mpz_set_str(x, s.c_str(), 16) != 0 || mpz_sgn(x) == 0) {   // every token here is a nonzero residue
        std::fprintf(stderr, "bad hex token '%.20s'\n", s.c_str());
        std::exit(2);
    }
}
static bool eq_hex(const mpz_t x, const std::string &s) {
    mpz_t w; mpz_init(w); set_hex(w, s);
    bool ok = mpz_cmp(x, w) == 0;
    mpz_clear(w);
    return ok;
}

int main(int argc, char **argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ghpair_test <fixture>\n"); return 2; }
    FILE *f = std::fopen(argv[1], "r");
    if (!f) return 2;
    std::string all;
    char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) all.append(buf, got);
    std::fclose(f);
    std::istringstream in(all);
    mpz_t p, q, r;
    mpz_inits(p, q, r, nullptr);
    set_hex(p, next(in)); set_hex(q, next(in)); set_hex(r, next(in));
    Paillier_HIP server;
    server.key_from_primes(p, q);
    GHPairKey key = server.paillier_cpu;                 // what encrypt_gh_pairs hangs on every GHPair (server.h:119)
    key.set_shared_r(r);
    const int ncase = std::atoi(next(in).c_str());
    std::vector<GHPair> ct(ncase);
    for (auto &x : ct) {                                  // g and h carry the same ciphertext
        std::string s = next(in);
        set_hex(x.g_enc, s); set_hex(x.h_enc, s);
        x.encrypted = true; x.paillier = key;
    }
    int bad = 0, checks = 0;
    auto expect = [&](bool ok, const char *what, int a, int b) {
        checks++;
        if (!ok) { bad++; std::printf("MISMATCH %s (%d, %d)\n", what, a, b); }
    };
    const int nadd = std::atoi(next(in).c_str());
    for (int t = 0; t < nadd; t++) {
        int i = std::atoi(next(in).c_str()), j = std::atoi(next(in).c_str());
        std::string want = next(in);
        GHPair s = ct[i] + ct[j];                         // dest = dest + src (hist_tree_builder.cpp:591)
        expect(eq_hex(s.g_enc, want) && eq_hex(s.h_enc, want), "operator+", i, j);
        GHPair d = ct[i];
        d += ct[j];                                       // key.add(g_enc, g_enc, rhs.g_enc): aliased
        expect(eq_hex(d.g_enc, want) && eq_hex(d.h_enc, want), "operator+=", i, j);
        mpz_t a; mpz_init_set(a, ct[i].g_enc);
        key.add(a, a, ct[j].g_enc);                       // add(s, s, c): the product, not 0 (Q11)
        expect(eq_hex(a, want) && mpz_sgn(a) != 0, "add(s, s, c)", i, j);
        mpz_clear(a);
    }
    const int parties = std::atoi(next(in).c_str()), bins = std::atoi(next(in).c_str());
    std::vector<std::vector<GHPair>> ph(parties, std::vector<GHPair>(bins));
    for (auto &row : ph)
        for (auto &x : row) {
            std::string s = next(in);
            set_hex(x.g_enc, s); set_hex(x.h_enc, s);
            x.encrypted = true; x.paillier = key;
        }
    for (int b = 0; b < bins; b++) {
        std::string want = next(in);
        GHPair acc;                                       // merged_hist entry: an unencrypted zero
        GHPair acc2;
        for (int pi = 0; pi < parties; pi++) {
            acc = acc + ph[pi][b];                        // hist_tree_builder.cpp:1035; the first + encrypts 0
            acc2 += ph[pi][b];                            // the += form: promote, then the aliased add
        }
        expect(eq_hex(acc.g_enc, want) && eq_hex(acc.h_enc, want), "merge via operator+", b, parties);
        expect(eq_hex(acc2.g_enc, want) && eq_hex(acc2.h_enc, want), "merge via operator+=", b, parties);
    }
    const int nsub = std::atoi(next(in).c_str());
    for (int t = 0; t < nsub; t++) {
        int i = std::atoi(next(in).c_str()), j = std::atoi(next(in).c_str());
        std::string want = next(in);
        GHPair d = ct[i] - ct[j];                         // father - child (hist_tree_builder.cpp:678)
        expect(eq_hex(d.g_enc, want) && eq_hex(d.h_enc, want), "operator-", i, j);
    }
    {
        float g = std::strtof(next(in).c_str(), nullptr), h = std::strtof(next(in).c_str(), nullptr);
        int j = std::atoi(next(in).c_str());
        std::string wg = next(in), wh = next(in);
        GHPair lhs(g, h);
        GHPair d = lhs - ct[j];                           // plain lhs promoted with rhs.paillier
        expect(eq_hex(d.g_enc, wg) && eq_hex(d.h_enc, wh), "plain - encrypted", j, -1);
    }
    mpz_clears(p, q, r, nullptr);
    std::printf("%d checks, %d mismatches -> ghpair %s\n", checks, bad, bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
