// Minimal stand-in for the USE_CUDA/USE_HIP GHPair of FedTree's common.h:65-412
// (fields + deep copy) for the shim test.  NOT the reference file.
#pragma once
#include <gmp.h>
#include "FedTree/Encryption/paillier_gmp.h"
typedef float float_type;
struct GHPair {
    float_type g = 0, h = 0;
    bool encrypted = false;
    mpz_t g_enc, h_enc;
    Paillier_GMP paillier;
    GHPair() { mpz_init(g_enc); mpz_init(h_enc); }
    GHPair(float_type g_, float_type h_) : GHPair() { g = g_; h = h_; }
    GHPair(const GHPair &o) : GHPair() { *this = o; }
    GHPair &operator=(const GHPair &o) {
        g = o.g; h = o.h; encrypted = o.encrypted;
        mpz_set(g_enc, o.g_enc); mpz_set(h_enc, o.h_enc);
        paillier = o.paillier;
        return *this;
    }
    ~GHPair() { mpz_clear(g_enc); mpz_clear(h_enc); }
};
