// Standalone bring-up test + timing of the P-adic exponentiation kernel (fedtree_amd/csrc/gen_padic.py).
// Build: hipcc --offload-arch=gfx950 -O2 -idirafter /opt/conda/include tools/test_padic.cpp -l:libgmp.so.10 -o tools/bin/test_padic
// Run:   [M37_BLOCK=512] tools/bin/test_padic <hsaco> [lanes] [mode] [kernel]   mode 0: y^P, y < P (encrypt); 1: c^(P-1), c < P^2;
//        bring-up programs: 2: LOADP; STOREP (c < P^2), 3: LOADP; SQR 1; STOREP, 4: LOADP; SQR 1; MUL IN; STOREP
//        kernel: fthe_padic_k37 (default) or fthe_padic_m37 (gen_padic_mfma.py: ctx carries the LDS tile image)
// Checks sampled lanes against GMP's mpz_powm and prints the launch time and products per second.
#include <hip/hip_runtime.h>
#include <gmp.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>
#include <cstring>
#include <string>
#include "../fedtree_amd/csrc/padic_tiles.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static const int K = 37, B = 28, S = 2 * K;
static const uint32_t MASK = (1u << B) - 1;

static void to_limbs(const mpz_t x, uint32_t *l, int n) {
    mpz_t t; mpz_init_set(t, x);
    for (int k = 0; k < n; k++) { l[k] = (uint32_t)(mpz_get_ui(t) & MASK); mpz_fdiv_q_2exp(t, t, B); }
    if (mpz_sgn(t)) { printf("to_limbs: value does not fit\n"); exit(1); }
    mpz_clear(t);
}
static void from_limbs(mpz_t x, const uint32_t *l, int n) {
    mpz_set_ui(x, 0);
    for (int k = n - 1; k >= 0; k--) { mpz_mul_2exp(x, x, B); mpz_add_ui(x, x, l[k]); }
}

struct Prog {
    std::vector<uint32_t> w;
    int products = 0;
    void op(uint32_t o, uint32_t a) { w.push_back(o); w.push_back(a); }
    void sqr(int n) { if (n > 0) { op(3, n); products += n; } }
    void mul(int s) { op(4, s); products++; }
    // left-to-right sliding window (the engine's Prog::pow, bn_host.hpp)
    void pow(const mpz_t e, int tbl0, int sq_slot, int w_) {
        long nb = (long)mpz_sizeinbase(e, 2);
        int ntab = 1 << (w_ - 1);
        op(2, tbl0); sqr(1); op(2, sq_slot); op(1, tbl0);
        for (int k = 1; k < ntab; k++) { mul(sq_slot); op(2, tbl0 + k); }
        auto bit = [&](long b) { return mpz_tstbit(e, (mp_bitcnt_t)b); };
        auto window = [&](long top, long &low, unsigned &val) {
            low = top - w_ + 1; if (low < 0) low = 0;
            while (!bit(low)) low++;
            val = 0;
            for (long b = top; b >= low; b--) val = (val << 1) | (unsigned)bit(b);
        };
        long i = nb - 1, low; unsigned v;
        window(i, low, v);
        op(1, tbl0 + (int)((v - 1) / 2));
        i = low - 1;
        int pend = 0;
        while (i >= 0) {
            if (!bit(i)) { pend++; i--; continue; }
            window(i, low, v);
            pend += (int)(i - low + 1);
            sqr(pend); mul(tbl0 + (int)((v - 1) / 2)); pend = 0;
            i = low - 1;
        }
        sqr(pend);
    }
};

int main(int argc, char **argv) {
    const char *path = argc > 1 ? argv[1] : "padic.hsaco";
    int L = argc > 2 ? atoi(argv[2]) : 65536;
    int mode = argc > 3 ? atoi(argv[3]) : 0;
    std::string kname = argc > 4 ? argv[4] : "fthe_padic_k37";
    const int BLK = getenv("M37_BLOCK") ? atoi(getenv("M37_BLOCK")) : 256;   // 512: ping-pong m37 variants
    if (BLK <= 0 || BLK % 256 || L % BLK) { printf("lanes must be a multiple of the block (%d)\n", BLK); return 2; }
    std::ifstream f(path, std::ios::binary);
    std::vector<char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (blob.empty()) { printf("no code object at %s\n", path); return 2; }
    hipModule_t mod; hipFunction_t fn;
    CHECK(hipModuleLoadData(&mod, blob.data()));
    CHECK(hipModuleGetFunction(&fn, mod, kname.c_str()));

    gmp_randstate_t rs; gmp_randinit_mt(rs); gmp_randseed_ui(rs, 20261016 + mode);
    mpz_t P, P2, mu, t, x, e, got, want;
    mpz_inits(P, P2, mu, t, x, e, got, want, NULL);
    mpz_urandomb(P, rs, 1024); mpz_setbit(P, 1023); mpz_setbit(P, 1022); mpz_setbit(P, 0);
    mpz_mul(P2, P, P);
    mpz_set_ui(t, 1); mpz_mul_2exp(t, t, 2 * B * K); mpz_fdiv_q(mu, t, P);
    std::vector<uint32_t> ctx(128 + padic_tiles::kImageBytes / 4, 0), pl(K);
    to_limbs(P, pl.data(), K);
    for (int j = 0; j < K; j++) ctx[j] = (uint32_t)(-(int32_t)pl[j]);
    to_limbs(mu, ctx.data() + K + 3, K + 1);
    {
        std::vector<uint8_t> img = padic_tiles::build(P);
        if (img.empty()) { printf("tile image failed\n"); return 2; }
        memcpy(ctx.data() + 128, img.data(), img.size());
    }
    if (mode == 0) mpz_set(e, P); else if (mode == 1) mpz_sub_ui(e, P, 1);
    else mpz_set_ui(e, mode == 2 ? 1 : mode == 3 ? 2 : 3);

    const int W = 6, TAB = 2, SQ = 1, IN = 0, OUT = TAB + (1 << (W - 1));
    const int NSLOTS = OUT + 1;
    Prog p;
    if (mode == 2) { p.op(22, IN); p.op(23, OUT); }
    else if (mode == 5) { p.op(22, IN); p.op(2, OUT); }          // raw digits x0 | x1 (dumped)
    else if (mode == 3) { p.op(22, IN); p.op(3, 1); p.op(23, OUT); }
    else if (mode == 4) { p.op(22, IN); p.op(2, TAB); p.op(3, 1); p.op(4, TAB); p.op(23, OUT); }
    else { p.op(22, IN); p.pow(e, TAB, SQ, W); p.op(23, OUT); }
    p.op(0, 0);

    size_t slot_words = (size_t)S * L;
    std::vector<uint32_t> in(slot_words), out(slot_words);
    std::vector<uint32_t> lb(S);
    std::vector<int> sample;
    for (int g = 0; g < 8; g++) sample.push_back(g);
    for (int g = 8; g < L; g += L / 256) sample.push_back(g);
    sample.push_back(L - 1);
    std::vector<std::vector<uint32_t>> xs(L);
    for (int g = 0; g < L; g++) {
        if (g == 0) mpz_set_ui(x, 1);
        else if (g == 1) { if (mode == 0) mpz_sub_ui(x, P, 1); else mpz_sub_ui(x, P2, 1); }
        else if (g == 2) mpz_set_ui(x, 2);
        else if (g == 3 && mode >= 2) mpz_sub_ui(x, P2, 1);
        else if (mode == 0) mpz_urandomm(x, rs, P);
        else mpz_urandomm(x, rs, P2);
        to_limbs(x, lb.data(), S);
        for (int k = 0; k < S; k++) in[(size_t)k * L + g] = lb[k];
    }
    uint32_t *d_slots, *d_prog, *d_ctx;
    CHECK(hipMalloc(&d_slots, NSLOTS * slot_words * 4));
    CHECK(hipMalloc(&d_prog, p.w.size() * 4));
    CHECK(hipMalloc(&d_ctx, ctx.size() * 4));
    CHECK(hipMemset(d_slots, 0, NSLOTS * slot_words * 4));
    CHECK(hipMemcpy(d_slots + IN * slot_words, in.data(), slot_words * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_prog, p.w.data(), p.w.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_ctx, ctx.data(), ctx.size() * 4, hipMemcpyHostToDevice));
    struct {
        void *s; const void *p; const void *cx; uint32_t ls, ss, live, pad; const void *rows[16];
    } args = {d_slots, d_prog, d_ctx, (uint32_t)L * 4, (uint32_t)(S * L * 4), (uint32_t)L, 0, {}};
    size_t sz = sizeof(args);
    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CHECK(hipEventRecord(e0));
        CHECK(hipModuleLaunchKernel(fn, L / BLK, 1, 1, BLK, 1, 1, 0, 0, nullptr, cfg));
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    CHECK(hipMemcpy(out.data(), d_slots + OUT * slot_words, slot_words * 4, hipMemcpyDeviceToHost));
    if (mode == 5) {                                            // lanes 0..7: P, input, raw output limbs
        FILE *fo = fopen("gpurun_out/padic_dump.txt", "w");
        gmp_fprintf(fo, "P %Zx\n", P);
        for (int g = 0; g < 8; g++) {
            fprintf(fo, "in %d", g);
            for (int k = 0; k < S; k++) fprintf(fo, " %x", in[(size_t)k * L + g]);
            fprintf(fo, "\nout %d", g);
            for (int k = 0; k < S; k++) fprintf(fo, " %x", out[(size_t)k * L + g]);
            fprintf(fo, "\n");
        }
        fclose(fo);
        return 0;
    }
    int bad = 0;
    for (int g : sample) {
        for (int k = 0; k < S; k++) lb[k] = out[(size_t)k * L + g];
        from_limbs(got, lb.data(), S);
        for (int k = 0; k < S; k++) lb[k] = in[(size_t)k * L + g];
        from_limbs(x, lb.data(), S);
        mpz_powm(want, x, e, P2);
        mpz_mod(t, got, P2);
        if (mpz_cmp(t, want) != 0 || mpz_cmp(got, P2) >= 0 && mpz_sizeinbase(got, 2) > 2051) {
            if (bad < 5) gmp_printf("lane %d: got %Zx\n   want %Zx\n", g, t, want);
            bad++;
        }
    }
    double prods = (double)p.products + 1.0;   // + the LOADP Barrett, about one product
    printf("{\"lanes\": %d, \"mode\": %d, \"checked\": %zu, \"bad\": %d, \"ms\": %.3f, \"products_per_lane\": %.0f, "
           "\"products_per_s\": %.4g, \"exps_per_s\": %.4g}\n",
           L, mode, sample.size(), bad, best, prods, prods * L / (best * 1e-3), L / (best * 1e-3));
    return bad ? 1 : 0;
}
