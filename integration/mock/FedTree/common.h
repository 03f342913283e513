// Stand-in for the GHPair of FedTree's common.h:65-412 as a USE_HIP build compiles it -- for the
// shim tests only; NOT the reference file (written for this repository).
//
// What matters for the drop-in is how the operators call the key they carry, and those calls are
// the reference's, call for call (the `#ifdef USE_CUDA` branches, taken by USE_HIP too):
//   operator+  (common.h:150-195): plain + plain adds the floats; otherwise the plain side is
//              promoted with homo_encrypt(other.paillier) and res.g_enc / res.h_enc come from
//              key.add(res.x_enc, lhs.x_enc, rhs.x_enc); res.paillier = the key used.
//   operator+= (common.h:197-238): the same into *this, with the ALIASED call
//              key.add(g_enc, g_enc, rhs.g_enc) -- the call that zeroes the sum under
//              Paillier_GMP::add.
//   operator-  (common.h:253-337): mpz minus_one = (long)-1 imported as 64 bits; encrypted rhs:
//              key.mul(minus, rhs.x_enc, minus_one) then key.add(res.x_enc, lhs.x_enc, minus)
//              (in the !encrypted branch `minus` is passed to mul uninitialised); plain rhs:
//              negate the floats, promote, add.
//   homo_encrypt (common.h:75-97): long v = (long)(x * 1e6) imported as one 64-bit word,
//              pl.encrypt(x_enc, v); paillier = pl; g = h = 0; encrypted = true.
// tests/test_integration_shim.py checks, where /root/reference exists, that every key call in the
// reference's operator bodies appears here with the same arguments.
#pragma once
#include <gmp.h>
#include "fthe_ghpair_key.h"
typedef float float_type;
typedef Paillier_HIP_Pub GHPairKey;          // common.h:72 in the USE_HIP build

struct GHPair {
    float_type g = 0, h = 0;
    bool encrypted = false;
    mpz_t g_enc, h_enc;
    GHPairKey paillier;

    GHPair() { mpz_init(g_enc); mpz_init(h_enc); }
    GHPair(float_type v) : GHPair() { g = h = v; }
    GHPair(float_type g_, float_type h_) : GHPair() { g = g_; h = h_; }
    GHPair(const GHPair &o) : GHPair() {
        g = o.g; h = o.h;
        if (o.encrypted) { mpz_set(g_enc, o.g_enc); mpz_set(h_enc, o.h_enc); }
        paillier = o.paillier;
        encrypted = o.encrypted;
    }
    // (the reference has no copy assignment, so its implicit one copies the mpz_t structs
    //  shallowly; a deep copy here keeps the test free of double frees)
    GHPair &operator=(const GHPair &o) {
        g = o.g; h = o.h; encrypted = o.encrypted;
        mpz_set(g_enc, o.g_enc); mpz_set(h_enc, o.h_enc);
        paillier = o.paillier;
        return *this;
    }
    ~GHPair() { mpz_clear(g_enc); mpz_clear(h_enc); }

    void homo_encrypt(const GHPairKey &pl) {
        if (encrypted) return;
        mpz_t gm, hm;
        mpz_init(gm); mpz_init(hm);
        long gl = (long)(g * 1e6), hl = (long)(h * 1e6);
        mpz_import(gm, 1, -1, sizeof(gl), 0, 0, &gl);
        mpz_import(hm, 1, -1, sizeof(hl), 0, 0, &hl);
        pl.encrypt(g_enc, gm);
        pl.encrypt(h_enc, hm);
        paillier = pl;
        g = 0; h = 0;
        encrypted = true;
        mpz_clear(gm); mpz_clear(hm);
    }

    GHPair operator+(const GHPair &rhs) const {
        GHPair res;
        if (!encrypted && !rhs.encrypted) {
            res.g = g + rhs.g; res.h = h + rhs.h;
            return res;
        }
        if (!encrypted) {
            GHPair tmp_lhs = *this;
            tmp_lhs.homo_encrypt(rhs.paillier);
            rhs.paillier.add(res.g_enc, tmp_lhs.g_enc, rhs.g_enc);
            rhs.paillier.add(res.h_enc, tmp_lhs.h_enc, rhs.h_enc);
            res.paillier = rhs.paillier;
        } else if (!rhs.encrypted) {
            GHPair tmp_rhs = rhs;
            tmp_rhs.homo_encrypt(paillier);
            paillier.add(res.g_enc, g_enc, tmp_rhs.g_enc);
            paillier.add(res.h_enc, h_enc, tmp_rhs.h_enc);
            res.paillier = paillier;
        } else {
            paillier.add(res.g_enc, g_enc, rhs.g_enc);
            paillier.add(res.h_enc, h_enc, rhs.h_enc);
            res.paillier = paillier;
        }
        res.encrypted = true;
        return res;
    }

    void operator+=(const GHPair &rhs) {
        if (!encrypted && !rhs.encrypted) {
            g += rhs.g; h += rhs.h;
            return;
        }
        if (!encrypted) {
            homo_encrypt(rhs.paillier);
            rhs.paillier.add(g_enc, g_enc, rhs.g_enc);
            rhs.paillier.add(h_enc, h_enc, rhs.h_enc);
            paillier = rhs.paillier;
        } else if (!rhs.encrypted) {
            GHPair tmp_rhs = rhs;
            tmp_rhs.homo_encrypt(paillier);
            paillier.add(g_enc, g_enc, tmp_rhs.g_enc);
            paillier.add(h_enc, h_enc, tmp_rhs.h_enc);
        } else {
            paillier.add(g_enc, g_enc, rhs.g_enc);
            paillier.add(h_enc, h_enc, rhs.h_enc);
        }
        encrypted = true;
    }

    GHPair operator-(const GHPair &rhs) const {
        GHPair res;
        if (!encrypted && !rhs.encrypted) {
            res.g = g - rhs.g; res.h = h - rhs.h;
            return res;
        }
        GHPair tmp_lhs = *this;
        GHPair tmp_rhs = rhs;
        mpz_t minus_one;
        mpz_init(minus_one);
        long mo = (long)-1;
        mpz_import(minus_one, 1, -1, sizeof(mo), 0, 0, &mo);
        if (!encrypted) {
            tmp_lhs.homo_encrypt(rhs.paillier);
            mpz_t minus_g_enc, minus_h_enc;                  // not initialised: mul initialises them
            rhs.paillier.mul(minus_g_enc, tmp_rhs.g_enc, minus_one);
            rhs.paillier.mul(minus_h_enc, tmp_rhs.h_enc, minus_one);
            rhs.paillier.add(res.g_enc, tmp_lhs.g_enc, minus_g_enc);
            rhs.paillier.add(res.h_enc, tmp_lhs.h_enc, minus_h_enc);
            mpz_clear(minus_g_enc);
            mpz_clear(minus_h_enc);
            res.paillier = rhs.paillier;
        } else if (!rhs.encrypted) {
            tmp_rhs.g *= -1;
            tmp_rhs.h *= -1;
            tmp_rhs.homo_encrypt(paillier);
            paillier.add(res.g_enc, g_enc, tmp_rhs.g_enc);
            paillier.add(res.h_enc, h_enc, tmp_rhs.h_enc);
            res.paillier = paillier;
        } else {
            mpz_t minus_g_enc, minus_h_enc;
            mpz_init(minus_g_enc);
            mpz_init(minus_h_enc);
            paillier.mul(minus_g_enc, tmp_rhs.g_enc, minus_one);
            paillier.mul(minus_h_enc, tmp_rhs.h_enc, minus_one);
            paillier.add(res.g_enc, g_enc, minus_g_enc);
            paillier.add(res.h_enc, h_enc, minus_h_enc);
            mpz_clear(minus_g_enc);
            mpz_clear(minus_h_enc);
            res.paillier = paillier;
        }
        mpz_clear(minus_one);
        res.encrypted = true;
        return res;
    }
};
