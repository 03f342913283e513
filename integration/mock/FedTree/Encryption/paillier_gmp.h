// Minimal stand-in for FedTree's Paillier_GMP fields (paillier_gmp.h:8-49) used by
// the shim test; the GHPair below only needs the key fields.  NOT the reference file.
#pragma once
#include <gmp.h>
#include <cstdint>
class Paillier_GMP {
public:
    Paillier_GMP() { mpz_inits(n, n_square, generator, p, q, lambda, mu, nullptr); }
    Paillier_GMP(const Paillier_GMP &o) : Paillier_GMP() { *this = o; }
    ~Paillier_GMP() { mpz_clears(n, n_square, generator, p, q, lambda, mu, nullptr); }
    Paillier_GMP &operator=(const Paillier_GMP &o) {   // public part, as paillier_gmp.h:12-20
        mpz_set(n, o.n); mpz_set(n_square, o.n_square); mpz_set(generator, o.generator);
        key_length = o.key_length;
        return *this;
    }
    mpz_t n, n_square, generator;
    uint32_t key_length = 0;
    mpz_t p, q, lambda, mu;
};
