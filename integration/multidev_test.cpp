// The drop-in's multi-device sharding (integration/paillier_hip.h, FTHE_DEVICES).
//   multidev_test plan                      -> checks fthe_shim::shard_plan / shard_plan_segments (no GPU):
//                                              configs[4]'s 80M pairs (160M rows) over 8 devices, ragged sizes,
//                                              segment plans of skewed CSRs; prints one JSON line
//   multidev_test run <p hex> <q hex> <N>   -> the Server / Party call sequence (server.h:58-135,
//                                              party.h:118-142) plus the batch helpers on N pairs with a seeded
//                                              key holder and party; prints one digest line per call.  Run under
//                                              FTHE_DEVICES=0 and FTHE_DEVICES=0,0 (two contexts on device 0,
//                                              FTHE_SHARD_ROWS small) the digests must be equal: sharding does not
//                                              change a ciphertext (tests/test_integration_shim.py); on a node with
//                                              several GPUs also under FTHE_DEVICES=0,1,..,k-1 (one shard, context
//                                              and key replica per physical device: configs[4]'s path).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "paillier_hip.h"

static uint64_t fnv(uint64_t h, const std::string &s) {
    for (unsigned char ch : s) { h ^= ch; h *= 1099511628211ull; }
    return h ^ 0xff;
}
static std::string hex(const mpz_t x) {
    char *p = mpz_get_str(nullptr, 16, x);
    std::string s(p);
    void (*fr)(void *, size_t);
    mp_get_memory_functions(nullptr, nullptr, &fr);
    fr(p, s.size() + 1);
    return s;
}
static uint64_t digest(SyncArray<GHPair> &a) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < a.size(); i++) {
        const GHPair &p = a.host_data()[i];
        h = fnv(h, p.encrypted ? hex(p.g_enc) + ":" + hex(p.h_enc) : "plain");
    }
    return h;
}

static int plan_checks() {
    int bad = 0;
    // configs[4]: 80M pairs = 160M rows over 8 GPUs -> 8 contiguous shards of 20M rows (10M pairs each)
    auto p8 = fthe_shim::shard_plan(160000000ull, 8, 8192);
    if (p8.size() != 8) bad++;
    for (size_t i = 0; i < p8.size(); i++)
        if (p8[i].first != i * 20000000ull || p8[i].second != (i + 1) * 20000000ull) bad++;
    // every size: contiguous, covering, balanced to +-1, at least min_rows per shard unless only one
    std::mt19937_64 rng(7);
    for (int t = 0; t < 20000; t++) {
        const size_t rows = rng() % 200000, slots = 1 + rng() % 9, mn = 1 + rng() % 5000;
        auto p = fthe_shim::shard_plan(rows, slots, mn);
        if (p.empty() || p.size() > slots || p.front().first != 0 || p.back().second != rows) { bad++; continue; }
        size_t mx = 0, mi = (size_t)-1;
        for (size_t i = 0; i < p.size(); i++) {
            if (i && p[i].first != p[i - 1].second) bad++;
            mx = std::max(mx, p[i].second - p[i].first);
            mi = std::min(mi, p[i].second - p[i].first);
        }
        if (mx - mi > 1) bad++;
        if (p.size() > 1 && mi < mn) bad++;
        if (p.size() < std::min(slots, rows / mn)) bad++;
    }
    // segment plans: contiguous non-empty segment ranges, member counts near tot / shards for even CSRs
    for (int t = 0; t < 3000; t++) {
        const size_t nseg = 1 + rng() % 3000, slots = 1 + rng() % 8;
        std::vector<int64_t> ptr(nseg + 1, 0);
        const bool skew = rng() % 2;
        for (size_t s = 0; s < nseg; s++) ptr[s + 1] = ptr[s] + (int64_t)(skew && s % 97 == 0 ? rng() % 5000 : rng() % 40);
        auto p = fthe_shim::shard_plan_segments(ptr.data(), nseg, slots, 64);
        if (p.empty() || p.size() > slots || p.front().first != 0 || p.back().second != nseg) { bad++; continue; }
        for (size_t i = 0; i < p.size(); i++) {
            if (p[i].second <= p[i].first) bad++;
            if (i && p[i].first != p[i - 1].second) bad++;
        }
        if (!skew && p.size() > 1) {
            const double tot = (double)ptr[nseg], per = tot / p.size();
            for (auto &r : p)
                if (std::fabs((double)(ptr[r.second] - ptr[r.first]) - per) > 0.05 * tot + 80) bad++;
        }
    }
    std::printf("{\"plan_ok\": %s, \"bad\": %d, \"config4_shard_rows\": %llu}\n", bad ? "false" : "true", bad,
                (unsigned long long)(p8[0].second - p8[0].first));
    return bad ? 1 : 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "plan") return plan_checks();
    if (argc < 5 || std::string(argv[1]) != "run") {
        std::fprintf(stderr, "usage: multidev_test plan | run <p hex> <q hex> <pairs>\n");
        return 2;
    }
    const size_t N = std::strtoull(argv[4], nullptr, 10);
    mpz_t p, q;
    mpz_init_set_str(p, argv[2], 16);
    mpz_init_set_str(q, argv[3], 16);
    Paillier_HIP server;                                     // Server::paillier, the key holder
    server.key_from_primes(p, q);
    server.rng_seed = 1234;
    server.publish_bases(77);                               // deterministic bases: runs comparable
    Paillier_HIP party;                                      // Party::paillier (Server::send_key, operator=)
    party = server;
    party.rng_seed = 5678;
    int bad = 0;
    auto val = [](size_t i, int w) { return (float)(0.001 * (double)((i * (w ? 7919 : 104729)) % 20001) - 10.0); };
    auto expect = [](float v) { return fthe_shim::decode(fthe_shim::encode(v)); };

    SyncArray<GHPair> gh(N);                                 // Server::encrypt_gh_pairs (server.h:105-121)
    for (size_t i = 0; i < N; i++) gh.host_data()[i] = GHPair(val(i, 0), val(i, 1));
    server.encrypt(gh);
    for (size_t i = 0; i < N; i++) gh.host_data()[i].encrypted = true;
    std::printf("encrypt %016llx\n", (unsigned long long)digest(gh));

    SyncArray<GHPair> hist(N);                               // Party::encrypt_histogram (party.h:118-142)
    for (size_t i = 0; i < N; i++) hist.host_data()[i] = GHPair(val(i + 3, 1), val(i + 5, 0));
    party.encrypt(hist);
    for (size_t i = 0; i < N; i++) hist.host_data()[i].encrypted = true;
    std::printf("party_encrypt %016llx\n", (unsigned long long)digest(hist));
    party.enc_mode = Paillier_HIP::EncMode::FixedBaseExact;  // published bases: a replica per device builds tables
    SyncArray<GHPair> hx(N);
    for (size_t i = 0; i < N; i++) hx.host_data()[i] = GHPair(val(i + 11, 0), val(i + 13, 1));
    party.encrypt(hx);
    for (size_t i = 0; i < N; i++) hx.host_data()[i].encrypted = true;
    std::printf("party_encrypt_exact %016llx\n", (unsigned long long)digest(hx));
    party.enc_mode = Paillier_HIP::EncMode::Default;
    // the key holder's exact fixed-base mode: tables from deterministic generators on the primary key; every
    // replica takes the same generators (fthe_key_fixed_base_exact_set), so the digest does not depend on sharding
    server.enc_mode = Paillier_HIP::EncMode::FixedBaseExact;
    server.exact_tables(99);
    SyncArray<GHPair> sx(N);
    for (size_t i = 0; i < N; i++) sx.host_data()[i] = GHPair(val(i + 17, 1), val(i + 19, 0));
    server.encrypt(sx);
    for (size_t i = 0; i < N; i++) sx.host_data()[i].encrypted = true;
    std::printf("server_encrypt_exact %016llx\n", (unsigned long long)digest(sx));
    server.enc_mode = Paillier_HIP::EncMode::Default;

    // node histogram (zero first), the 3-party merge (zero first), sibling subtraction, prefix sums
    const int n_col = 3, missing = 255;
    const int cut[4] = {0, 5, 12, 16};
    std::vector<unsigned char> bins(N * n_col);
    for (size_t i = 0; i < N; i++)
        for (int f = 0; f < n_col; f++) {
            const int nb = cut[f + 1] - cut[f];
            bins[i * n_col + f] = (unsigned char)((i * (f + 3)) % 11 == 0 ? missing : (i * (2 * f + 1) / 3) % nb);
        }
    SyncArray<GHPair> h1(16), h2(16), h3(16), merged(16), sib(16);
    party.histogram(gh, bins.data(), cut, n_col, missing, h1, true);
    std::printf("histogram %016llx\n", (unsigned long long)digest(h1));
    party.histogram(hist, bins.data(), cut, n_col, missing, h2);
    party.histogram(hx, bins.data(), cut, n_col, missing, h3);
    h3.host_data()[7] = GHPair(0.5f, 0.25f);                 // an unencrypted operand is promoted
    party.merge({&h1, &h2, &h3}, merged, true);
    std::printf("merge %016llx\n", (unsigned long long)digest(merged));
    party.subtract(merged, h1, sib);
    std::printf("subtract %016llx\n", (unsigned long long)digest(sib));
    SyncArray<GHPair> pre(16);
    for (int s = 0; s < 16; s++) pre.host_data()[s] = merged.host_data()[s];
    party.prefix(pre, cut, n_col);
    std::printf("prefix %016llx\n", (unsigned long long)digest(pre));
    // a batch large enough for several shards of the merge / subtract paths
    SyncArray<GHPair> a(N), b(N), d(N);
    for (size_t i = 0; i < N; i++) { a.host_data()[i] = gh.host_data()[i]; b.host_data()[i] = hist.host_data()[i]; }
    party.merge({&a, &b}, d);
    std::printf("merge_big %016llx\n", (unsigned long long)digest(d));
    party.subtract(d, b, a);
    std::printf("subtract_big %016llx\n", (unsigned long long)digest(a));

    // the root sum of Tree::init_CPU (tree.cpp:20-34), plain product and the reference's Enc(0)-first sequence
    GHPair root = party.sum(gh), root0 = party.sum(gh, true);
    std::printf("sum %016llx\n", (unsigned long long)fnv(fnv(1469598103934665603ull, hex(root.g_enc) + ":" + hex(root.h_enc)),
                                                         hex(root0.g_enc) + ":" + hex(root0.h_enc)));
    SyncArray<GHPair> rs(2);
    rs.host_data()[0] = root;
    rs.host_data()[1] = root0;

    // Server::decrypt_gh_pairs (server.h:123-135) of everything: the plaintexts
    server.decrypt(a);                                       // (gh + hist) - hist = gh
    for (size_t i = 0; i < N; i++)
        if (a.host_data()[i].g != expect(val(i, 0)) || a.host_data()[i].h != expect(val(i, 1))) bad++;
    server.decrypt(hx);
    for (size_t i = 0; i < N; i++)
        if (hx.host_data()[i].g != expect(val(i + 11, 0)) || hx.host_data()[i].h != expect(val(i + 13, 1))) bad++;
    server.decrypt(sx);
    for (size_t i = 0; i < N; i++)
        if (sx.host_data()[i].g != expect(val(i + 17, 1)) || sx.host_data()[i].h != expect(val(i + 19, 0))) bad++;
    double want[16] = {0};
    for (size_t i = 0; i < N; i++)
        for (int f = 0; f < n_col; f++) {
            const int bn = bins[i * n_col + f];
            if (bn != missing) want[cut[f] + bn] += (double)(long)(val(i, 0) * 1e6) / 1e6;
        }
    server.decrypt(h1);
    for (int s = 0; s < 16; s++)
        if (std::fabs(h1.host_data()[s].g - want[s]) > 1e-3 * (1 + std::fabs(want[s]))) bad++;
    server.dec_short = true;                                 // the p half of the CRT only
    server.decrypt(d);
    for (size_t i = 0; i < N; i++)
        if (std::fabs(d.host_data()[i].g - (expect(val(i, 0)) + expect(val(i + 3, 1)))) > 2e-5) bad++;
    server.dec_short = false;
    server.decrypt(rs);                                      // the root sums: sum of the codec values mod 2^64
    {
        int64_t sg = 0, sh = 0;
        for (size_t i = 0; i < N; i++) {
            sg += (int64_t)fthe_shim::encode(val(i, 0));
            sh += (int64_t)fthe_shim::encode(val(i, 1));
        }
        for (int r = 0; r < 2; r++)
            if (rs.host_data()[r].g != fthe_shim::decode((uint64_t)sg) || rs.host_data()[r].h != fthe_shim::decode((uint64_t)sh))
                bad++;
    }
    std::printf("decrypt_checks bad=%d\n", bad);
    std::printf("devices %zu\n", fthe_shim::shard_devices().size());
    std::printf("multidev %s\n", bad ? "FAIL" : "OK");
    mpz_clear(p);
    mpz_clear(q);
    return bad ? 1 : 0;
}
