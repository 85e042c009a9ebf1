// ezrs_field.hpp -- host-side GF(2^m) / RS(N,K) codec construction for the MI355X engine.
//
// Builds, once per codec, everything the device kernels read: the log/antilog tables, the
// generator polynomial and the CCSDS dual-basis maps.  Same definitions as the reference
// (c++/ezpwd/rs_base:537-557 gfpoly, 599-635 reed_solomon_tabs, 1248-1286 genpoly), written for
// runtime (m, poly, fcr, prim, nroots) instead of template parameters.
#pragma once

#include <cstdint>
#include <vector>

namespace ezrs {

struct Field {
    unsigned mm = 0, nn = 0, poly = 0;
    std::vector<uint16_t> alpha_to;  // nn+1 entries, alpha_to[nn] = 0
    std::vector<uint16_t> index_of;  // nn+1 entries, index_of[0] = nn ("log 0")

    // Returns false if poly does not generate the multiplicative group the way the reference's
    // primitivity test requires (rs_base:622-625: alpha^NN must come back to 1).
    bool build(unsigned m, unsigned p) {
        mm = m; nn = (1u << m) - 1; poly = p;
        alpha_to.assign(nn + 1, 0);
        index_of.assign(nn + 1, 0);
        index_of[0] = (uint16_t)nn;
        unsigned sr = 1;
        for (unsigned i = 0; i < nn; ++i) {
            index_of[sr] = (uint16_t)i;
            alpha_to[i] = (uint16_t)sr;
            sr <<= 1;
            if (sr & (1u << m)) sr ^= p;
            sr &= nn;
        }
        return sr == alpha_to[0];
    }
    unsigned mod(unsigned x) const { return x % nn; }
    // Polynomial-basis product of two field elements.
    unsigned mul(unsigned a, unsigned b) const {
        if (!a || !b) return 0;
        return alpha_to[mod(index_of[a] + index_of[b])];
    }
    unsigned pow_alpha(unsigned e) const { return alpha_to[mod(e)]; }
};

// CCSDS Berlekamp dual basis (rs_base:109-146): GF(2)-linear byte maps, generated from the images
// of the eight basis bytes (CCSDS 131.0-B Annex F transform).
inline void dual_maps(uint8_t into[256], uint8_t from[256]) {
    static const uint8_t col[8] = {0x7b, 0xaf, 0x99, 0xfa, 0x86, 0xec, 0xef, 0x8d};
    for (unsigned x = 0; x < 256; ++x) {
        uint8_t y = 0;
        for (unsigned b = 0; b < 8; ++b)
            if (x >> b & 1) y ^= col[b];
        into[x] = y;
    }
    for (unsigned x = 0; x < 256; ++x) from[into[x]] = (uint8_t)x;
}

struct CodecSpec {
    unsigned mm, poly, fcr, prim, nroots;
    int dual;
};

struct CodecMath {
    CodecSpec spec{};
    Field gf;
    unsigned nn = 0, load = 0, iprim = 0;
    std::vector<uint16_t> genpoly;      // index form, nroots+1 (rs_base:1263-1285)
    std::vector<uint16_t> genpoly_poly; // polynomial form, genpoly_poly[nroots] == 1
    uint8_t into_dual[256]{}, from_dual[256]{};

    bool build(const CodecSpec &s) {
        spec = s;
        if (s.mm < 2 || s.mm > 16 || s.prim == 0) return false;
        if (!gf.build(s.mm, s.poly)) return false;
        nn = gf.nn;
        if (s.nroots == 0 || s.nroots >= nn) return false;
        if (s.dual && s.mm != 8) return false;
        load = nn - s.nroots;
        unsigned ip = 1;
        while (ip % s.prim != 0) ip += nn;
        iprim = ip / s.prim;
        // g(x) = prod_{i<nroots} (x - alpha^((fcr+i)*prim)), coefficients low to high
        std::vector<uint16_t> tp(s.nroots + 1, 0);
        tp[0] = 1;
        for (unsigned i = 0, root = s.fcr * s.prim; i < s.nroots; ++i, root += s.prim) {
            tp[i + 1] = 1;
            for (unsigned j = i; j > 0; --j)
                tp[j] = tp[j] ? (uint16_t)(tp[j - 1] ^ gf.alpha_to[gf.mod(gf.index_of[tp[j]] + root)])
                              : tp[j - 1];
            tp[0] = gf.alpha_to[gf.mod(gf.index_of[tp[0]] + root)];
        }
        genpoly_poly = tp;
        genpoly.resize(s.nroots + 1);
        for (unsigned i = 0; i <= s.nroots; ++i) genpoly[i] = gf.index_of[tp[i]];
        dual_maps(into_dual, from_dual);
        return true;
    }
};

} // namespace ezrs
