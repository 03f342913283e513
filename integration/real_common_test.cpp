// FedTree's own GHPair -- the reference's include/FedTree/common.h with integration/common_h_use_hip.patch
// applied, compiled with -DUSE_HIP against integration/fthe_ghpair_key.h -- running
// its unchanged operator bodies (common.h:150-237) on the USE_HIP key bound to a public n, no GPU:
// operator+, the aliased operator+= and dest = dest + src reproduce the reference's golden adds.
// tests/test_integration_shim.py builds it in a temporary tree where /root/reference exists (the
// reference's header is never copied into this repository and never travels to a GPU box).
//   real_common_test <fixture>        fixture: n, then (x y want) triples, hex      -> "real common.h OK"
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "FedTree/common.h"

static void set_hex(mpz_t x, const std::string &s) { mpz_set_str(x, s.c_str(), 16); }

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    std::ifstream in(argv[1]);
    std::string tok, a, b, w;
    mpz_t n, wv;
    mpz_inits(n, wv, nullptr);
    in >> tok;
    set_hex(n, tok);
    GHPairKey key;                                         // common.h's member type under USE_HIP
    key.bind_n(n, (uint32_t)mpz_sizeinbase(n, 2));
    int bad = 0, cnt = 0;
    while (in >> a >> b >> w) {
        GHPair x, y;
        set_hex(x.g_enc, a); set_hex(x.h_enc, b);
        set_hex(y.g_enc, b); set_hex(y.h_enc, a);
        x.encrypted = y.encrypted = true;
        x.paillier = key;
        y.paillier = key;
        set_hex(wv, w);
        GHPair s = x + y;                                  // common.h:150-195
        bad += mpz_cmp(s.g_enc, wv) != 0 || mpz_cmp(s.h_enc, wv) != 0 || !s.encrypted;
        GHPair d(x);
        d += y;                                            // common.h:197-238: add(g_enc, g_enc, rhs.g_enc)
        bad += mpz_cmp(d.g_enc, wv) != 0 || mpz_cmp(d.h_enc, wv) != 0;
        GHPair e(x);
        e = e + y;                                         // hist_tree_builder.cpp:591's form
        bad += mpz_cmp(e.g_enc, wv) != 0 || mpz_cmp(e.h_enc, wv) != 0;
        GHPair p(0.5f, 0.25f), q(0.125f, 1.f);
        GHPair r = p + q;                                  // plain + plain stays plain
        bad += r.encrypted || r.g != 0.625f || r.h != 1.25f;
        cnt++;
    }
    mpz_clears(n, wv, nullptr);
    std::printf("%d adds, %d mismatches -> real common.h %s\n", cnt, bad, (bad || !cnt) ? "FAIL" : "OK");
    return (bad || !cnt) ? 1 : 0;
}
