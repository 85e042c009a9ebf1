/*
 * ref_driver.C -- C-ABI shim over the REFERENCE codec (TEST INFRASTRUCTURE ONLY).
 *
 * Compiled by oracle/Makefile against the unmodified reference headers where they lie
 * (/root/reference/c++/ezpwd/{rs,rs_base,rs_definitions}); the output goes to oracle/_ref/ only and
 * is never committed.  This file contains no reference code: it instantiates the reference's own
 * ezpwd::RS<N,K> / RS_CCSDS / RS_CCSDS_CONV templates (rs:74-104) and exposes their lowest-level
 * public entry points, encode<INP>(data,len,parity) (rs_base:868-904) and
 * decode<INP>(data,len,parity,eras_pos,no_eras,corr) (rs_base:1170-1242), through extern "C" so the
 * Python tests can cross-check the restatement (oracle/ezrs_oracle.c) and generate golden fixtures.
 *
 * Built with -DEZPWD_NO_EXCEPTS so parameter errors come back as -1 instead of C++ exceptions.
 */
#include <cstdint>
#include <cstring>

#include <ezpwd/rs>
#include <ezpwd/rs_definitions>

namespace {

typedef int (*enc_fn)(const void *, unsigned, void *);
typedef int (*dec_fn)(void *, unsigned, void *, unsigned *, unsigned, void *);

struct entry {
    const char *name;
    unsigned mm, poly, fcr, prim, nroots;
    int dual;
    enc_fn enc;
    dec_fn dec;
};

template <class C> struct shim {
    typedef typename C::symbol_t T;
    static const C &rs() { static const C c; return c; }
    static int enc(const void *d, unsigned len, void *p) {
        return rs().encode(static_cast<const T *>(d), len, static_cast<T *>(p));
    }
    static int dec(void *d, unsigned len, void *p, unsigned *e, unsigned ne, void *corr) {
        return rs().decode(static_cast<T *>(d), len, static_cast<T *>(p), e, ne,
                           static_cast<T *>(corr));
    }
};

#define STD(N, K, M, P) {"RS(" #N "," #K ")", M, P, 1, 1, (N) - (K), 0, \
        &shim<ezpwd::RS<N, K>>::enc, &shim<ezpwd::RS<N, K>>::dec}
#define CCSDS(K, D, T) {D ? "RS_CCSDS(255," #K ")" : "RS_CCSDS_CONV(255," #K ")", 8, 0x187, \
        128 - (255 - (K)) / 2, 11, 255 - (K), D, &shim<ezpwd::T<255, K>>::enc, \
        &shim<ezpwd::T<255, K>>::dec}

const entry table[] = {
    STD(3, 1, 2, 0x7),
    STD(7, 5, 3, 0xb),
    STD(15, 11, 4, 0x13),
    STD(31, 29, 5, 0x25),
    STD(31, 26, 5, 0x25),
    STD(63, 60, 6, 0x43),
    STD(63, 55, 6, 0x43),
    STD(127, 111, 7, 0x89),
    STD(255, 254, 8, 0x11d),
    STD(255, 253, 8, 0x11d),
    STD(255, 251, 8, 0x11d),
    STD(255, 249, 8, 0x11d),
    STD(255, 247, 8, 0x11d),
    STD(255, 243, 8, 0x11d),
    STD(255, 239, 8, 0x11d),
    STD(255, 238, 8, 0x11d),
    STD(255, 228, 8, 0x11d),
    STD(255, 223, 8, 0x11d),
    STD(255, 209, 8, 0x11d),
    STD(255, 191, 8, 0x11d),
    STD(255, 178, 8, 0x11d),
    STD(255, 156, 8, 0x11d),
    STD(255, 128, 8, 0x11d),
    STD(255, 127, 8, 0x11d),
    STD(255, 126, 8, 0x11d),
    STD(255, 56, 8, 0x11d),
    CCSDS(223, 1, RS_CCSDS),
    CCSDS(239, 1, RS_CCSDS),
    CCSDS(223, 0, RS_CCSDS_CONV),
    CCSDS(239, 0, RS_CCSDS_CONV),
    STD(511, 479, 9, 0x211),
    STD(1023, 991, 10, 0x409),
    STD(4095, 4063, 12, 0x1053),
    STD(65535, 65503, 16, 0x1100b),
    STD(65535, 65279, 16, 0x1100b),
};
const unsigned ntable = sizeof table / sizeof table[0];

} // namespace

extern "C" {

unsigned ezref_count(void) { return ntable; }

/* Describe codec i: name and the (mm, poly, fcr, prim, nroots, dual) parameters it maps to. */
const char *ezref_describe(unsigned i, unsigned *params) {
    if (i >= ntable) return nullptr;
    const entry &e = table[i];
    params[0] = e.mm; params[1] = e.poly; params[2] = e.fcr;
    params[3] = e.prim; params[4] = e.nroots; params[5] = (unsigned)e.dual;
    return e.name;
}

int ezref_encode(unsigned i, const void *data, unsigned len, void *parity) {
    return i < ntable ? table[i].enc(data, len, parity) : -2;
}

int ezref_decode(unsigned i, void *data, unsigned len, void *parity, unsigned *eras_pos,
                 unsigned no_eras, void *corr) {
    return i < ntable ? table[i].dec(data, len, parity, eras_pos, no_eras, corr) : -2;
}

/* Batch forms for speed (same per-codeword calls, strides in elements). */
int ezref_encode_batch(unsigned i, const void *data, size_t dstride, unsigned len, void *parity,
                       size_t pstride, size_t ncw, unsigned width) {
    if (i >= ntable) return -2;
    int bad = 0;
    for (size_t k = 0; k < ncw; ++k) {
        const char *d = static_cast<const char *>(data) + k * dstride * width;
        char *p = static_cast<char *>(parity) + k * pstride * width;
        bad |= table[i].enc(d, len, p) < 0;
    }
    return bad ? -1 : 0;
}

int ezref_decode_batch(unsigned i, void *data, size_t dstride, unsigned len, void *parity,
                       size_t pstride, const uint32_t *eras, size_t estride,
                       const uint32_t *neras, int32_t *result, uint32_t *positions,
                       size_t posstride, size_t ncw, unsigned width) {
    if (i >= ntable) return -2;
    static thread_local unsigned pos[65536];
    for (size_t k = 0; k < ncw; ++k) {
        char *d = static_cast<char *>(data) + k * dstride * width;
        char *p = static_cast<char *>(parity) + k * pstride * width;
        unsigned ne = neras ? neras[k] : 0;
        for (unsigned j = 0; j < ne; ++j) pos[j] = eras[k * estride + j];
        int r = table[i].dec(d, len, p, pos, ne, nullptr);
        result[k] = r;
        if (positions)
            for (int j = 0; j < r; ++j) positions[k * posstride + j] = pos[j];
    }
    return 0;
}

/* The reference's own dual-basis tables (rs_base:109-146), for the restatement's table test. */
void ezref_dual_tables(uint8_t *into, uint8_t *from) {
    for (unsigned x = 0; x < 256; ++x) {
        into[x] = ezpwd::reed_solomon_base::into_dual[x];
        from[x] = ezpwd::reed_solomon_base::from_dual[x];
    }
}

} // extern "C"
