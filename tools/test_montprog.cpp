// Standalone bring-up test + timing for the generated montprog code object.
// Build: hipcc --offload-arch=gfx950 -O2 -I/opt/conda/include tools/test_montprog.cpp
//        -L/opt/conda/lib -Wl,-rpath,/opt/conda/lib -lgmp -o tools/bin/test_montprog
// Run:   tools/bin/test_montprog <hsaco> [lanes] [sqr_count]
#include <hip/hip_runtime.h>
#include <gmp.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <fstream>
#include <random>

#define CHECK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP error %s @%d\n",hipGetErrorString(e_),__LINE__); exit(1);} }while(0)

static const int S = 74, B = 28;
static const uint32_t MASK = (1u << B) - 1;

static void to_limbs(const mpz_t x, uint32_t* l) {
    mpz_t t; mpz_init_set(t, x);
    for (int k = 0; k < S; k++) { l[k] = (uint32_t)(mpz_get_ui(t) & MASK); mpz_fdiv_q_2exp(t, t, B); }
    mpz_clear(t);
}
static void from_limbs(mpz_t x, const uint32_t* l) {
    mpz_set_ui(x, 0);
    for (int k = S - 1; k >= 0; k--) { mpz_mul_2exp(x, x, B); mpz_add_ui(x, x, l[k]); }
}

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "montprog_s74.hsaco";
    int L = argc > 2 ? atoi(argv[2]) : 131072;
    int nsq = argc > 3 ? atoi(argv[3]) : 200;
    std::ifstream f(path, std::ios::binary);
    std::vector<char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    hipModule_t mod; hipFunction_t fn;
    CHECK(hipModuleLoadData(&mod, blob.data()));
    CHECK(hipModuleGetFunction(&fn, mod, "fthe_montprog_s74"));

    gmp_randstate_t rs; gmp_randinit_mt(rs); gmp_randseed_ui(rs, 12345);
    mpz_t N, R, R2, x, y, e;
    mpz_inits(N, R, R2, x, y, e, NULL);
    mpz_urandomb(N, rs, 2048); mpz_setbit(N, 2047); mpz_setbit(N, 0);
    mpz_set_ui(R, 1); mpz_mul_2exp(R, R, B * S);
    mpz_powm_ui(R2, R, 2, N);
    // nprime = -N^-1 mod 2^B
    mpz_t m2b, inv; mpz_inits(m2b, inv, NULL);
    mpz_set_ui(m2b, 1); mpz_mul_2exp(m2b, m2b, B);
    mpz_invert(inv, N, m2b); mpz_sub(inv, m2b, inv);
    uint32_t nprime = (uint32_t)mpz_get_ui(inv);

    std::vector<uint32_t> ctx(S + 1);
    to_limbs(N, ctx.data()); ctx[S] = nprime;

    const int NSLOTS = 4;   // 0 x, 1 R2, 2 one, 3 out
    size_t slot_words = (size_t)S * L;
    std::vector<uint32_t> slots(NSLOTS * slot_words, 0);
    std::vector<uint32_t> lb(S);
    std::vector<std::vector<uint32_t>> xs(L, std::vector<uint32_t>(S));
    for (int g = 0; g < L; g++) {
        mpz_urandomm(x, rs, N);
        if (g == 0) mpz_set_ui(x, 1);
        if (g == 1) mpz_sub_ui(x, N, 1);
        to_limbs(x, xs[g].data());
        for (int k = 0; k < S; k++) slots[0 * slot_words + (size_t)k * L + g] = xs[g][k];
    }
    to_limbs(R2, lb.data());
    for (int g = 0; g < L; g++) for (int k = 0; k < S; k++) slots[1 * slot_words + (size_t)k * L + g] = lb[k];
    for (int g = 0; g < L; g++) slots[2 * slot_words + g] = 1;

    auto run = [&](const std::vector<uint32_t>& prog, float* ms) {
        uint32_t *d_slots, *d_prog, *d_ctx;
        CHECK(hipMalloc(&d_slots, slots.size() * 4));
        CHECK(hipMalloc(&d_prog, prog.size() * 4));
        CHECK(hipMalloc(&d_ctx, ctx.size() * 4));
        CHECK(hipMemcpy(d_slots, slots.data(), slots.size() * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(d_prog, prog.data(), prog.size() * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(d_ctx, ctx.data(), ctx.size() * 4, hipMemcpyHostToDevice));
        struct { void* s; void* p; void* c; uint32_t ls; uint32_t ss; } args = {
            d_slots, d_prog, d_ctx, (uint32_t)L * 4, (uint32_t)(S * L * 4)};
        size_t sz = sizeof(args);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
        CHECK(hipEventRecord(a, 0));
        CHECK(hipModuleLaunchKernel(fn, L / 256, 1, 1, 256, 1, 1, 0, 0, nullptr, cfg));
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(ms, a, b));
        CHECK(hipMemcpy(slots.data(), d_slots, slots.size() * 4, hipMemcpyDeviceToHost));
        CHECK(hipFree(d_slots)); CHECK(hipFree(d_prog)); CHECK(hipFree(d_ctx));
    };
    // correctness: x -> xR -> (xR)^(2^5) R^.. -> x^32 R -> x^32
    std::vector<uint32_t> prog = {1, 0, 4, 1, 3, 5, 4, 2, 2, 3, 0, 0};
    float ms;
    run(prog, &ms);
    int bad = 0;
    for (int g = 0; g < L; g++) {
        std::vector<uint32_t> o(S);
        for (int k = 0; k < S; k++) o[k] = slots[3 * slot_words + (size_t)k * L + g];
        from_limbs(y, o.data());
        mpz_mod(y, y, N);
        from_limbs(x, xs[g].data());
        mpz_powm_ui(e, x, 32, N);
        if (mpz_cmp(e, y) != 0) { if (bad < 5) gmp_printf("mismatch lane %d\n got %Zx\n exp %Zx\n", g, y, e); bad++; }
        if (g >= 4096 && bad == 0) break;   // host check of a prefix is enough
    }
    printf("correctness: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);
    // timing: nsq squarings
    std::vector<uint32_t> prog2 = {1, 0, 3, (uint32_t)nsq, 2, 3, 0, 0};
    run(prog2, &ms);   // warm
    run(prog2, &ms);
    double mm = (double)L * nsq;
    double macs = mm * 2.0 * S * S;
    printf("L=%d sqr=%d  %.3f ms  %.3e MontMul/s  %.3e MAC(v_mad_u64_u32)/s\n", L, nsq, ms, mm / (ms * 1e-3), macs / (ms * 1e-3));
    return bad ? 1 : 0;
}
