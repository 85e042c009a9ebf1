/* karn_shim.c -- batch entry points over Phil Karn's libfec RS codecs (TEST INFRASTRUCTURE ONLY).
 *
 * Linked with encode_rs_char.c, decode_rs_char.c, init_rs_char.c, encode_rs_8.c, decode_rs_8.c,
 * encode_rs_ccsds.c, decode_rs_ccsds.c and the tables their own generators emit, compiled in place
 * from phil-karn/fec-3.0.1.tar.gz by oracle/Makefile (target `karn`).  Used by
 * tests/golden/make_karn_fixtures.py to produce the Karn-side golden vectors for BASELINE config C2
 * ("bit-exact vs phil-karn rstest.c": the Tab row {8,0x11d,1,1,32}, phil-karn/rstest.c:36) and the
 * CCSDS rows (rstest.c:37-42, fec-3.0.1/encode_rs_ccsds.c).  Nothing here is on a product path.
 */
#include <stdint.h>
#include <string.h>
#include "fec.h"

/* General-purpose int codec (fec.h as patched by phil-karn/fec-3.0.1-int.patch): unsigned int
 * symbols, symsize up to 16.  Rows here are uint16 arrays (the engine's container for m > 8). */
void *karn_init_int(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad) {
    return init_rs_int(symsize, gfpoly, fcr, prim, nroots, pad);
}

void karn_free_int(void *rs) { free_rs_int(rs); }

void karn_encode_int_batch(void *rs, const uint16_t *data, long stride, uint16_t *parity, long pstride,
                           long ncw, int len, int nroots) {
    unsigned int buf[65536], par[65536];
    for (long i = 0; i < ncw; ++i) {
        for (int j = 0; j < len; ++j) buf[j] = data[i * stride + j];
        encode_rs_int(rs, buf, par);
        for (int j = 0; j < nroots; ++j) parity[i * pstride + j] = (uint16_t)par[j];
    }
}

void karn_decode_int_batch(void *rs, uint16_t *rows, long stride, long ncw, int nroots, int rowlen, int *eras,
                           const int *neras, int *result) {
    static unsigned int buf[65536];
    for (long i = 0; i < ncw; ++i) {
        for (int j = 0; j < rowlen; ++j) buf[j] = rows[i * stride + j];
        result[i] = decode_rs_int(rs, buf, eras + i * nroots, neras ? neras[i] : 0);
        for (int j = 0; j < rowlen; ++j) rows[i * stride + j] = (uint16_t)buf[j];
    }
}

/* General-purpose char codec (fec.h: init_rs_char / encode_rs_char / decode_rs_char). */
void *karn_init_char(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad) {
    return init_rs_char(symsize, gfpoly, fcr, prim, nroots, pad);
}

void karn_free_char(void *rs) { free_rs_char(rs); }

/* ncw rows of `len` data bytes at `stride`; parity (nroots bytes) to `parity` at `pstride`. */
void karn_encode_char_batch(void *rs, const uint8_t *data, long stride, uint8_t *parity, long pstride,
                            long ncw, int len) {
    unsigned char buf[256];
    for (long i = 0; i < ncw; ++i) {
        memcpy(buf, data + i * stride, (size_t)len);
        encode_rs_char(rs, buf, parity + i * pstride);
    }
}

/* In place on rows of (len data + nroots parity) bytes at `stride`.  eras[i * nroots ..] holds
 * neras[i] erasure positions (in, Karn convention) and receives the corrected positions (out);
 * result[i] = the decoder's return value. */
void karn_decode_char_batch(void *rs, uint8_t *rows, long stride, long ncw, int nroots, int *eras,
                            const int *neras, int *result) {
    for (long i = 0; i < ncw; ++i)
        result[i] = decode_rs_char(rs, rows + i * stride, eras + i * nroots, neras ? neras[i] : 0);
}

/* Fixed CCSDS-polynomial codec (0x187, fcr 112, prim 11) in the conventional basis, and the
 * dual-basis CCSDS wrapper around it. */
void karn_encode_8_batch(const uint8_t *data, long stride, uint8_t *parity, long pstride, long ncw, int pad) {
    unsigned char buf[256];
    for (long i = 0; i < ncw; ++i) {
        memcpy(buf, data + i * stride, (size_t)(223 - pad));
        encode_rs_8(buf, parity + i * pstride, pad);
    }
}

void karn_encode_ccsds_batch(const uint8_t *data, long stride, uint8_t *parity, long pstride, long ncw, int pad) {
    unsigned char buf[256];
    for (long i = 0; i < ncw; ++i) {
        memcpy(buf, data + i * stride, (size_t)(223 - pad));
        encode_rs_ccsds(buf, parity + i * pstride, pad);
    }
}

void karn_decode_8_batch(uint8_t *rows, long stride, long ncw, int *eras, const int *neras, int *result, int pad) {
    for (long i = 0; i < ncw; ++i)
        result[i] = decode_rs_8(rows + i * stride, eras + i * 32, neras ? neras[i] : 0, pad);
}

void karn_decode_ccsds_batch(uint8_t *rows, long stride, long ncw, int *eras, const int *neras, int *result, int pad) {
    for (long i = 0; i < ncw; ++i)
        result[i] = decode_rs_ccsds(rows + i * stride, eras + i * 32, neras ? neras[i] : 0, pad);
}
