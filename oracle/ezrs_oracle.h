/*
 * ezrs_oracle.h -- CPU restatement of the ezpwd Reed-Solomon codec (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X engine.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path (libezrs_hip.so) never links it.
 *
 * Parity status: PINNED.  The restatement is checked bit-exact against (1) the reference itself,
 * compiled from /root/reference/c++/ezpwd/{rs,rs_base} by oracle/Makefile into oracle/_ref/, and
 * (2) golden fixtures generated from that build and committed under tests/golden/.
 *
 * Semantics follow c++/ezpwd/rs_base (reference VERSION 2.2.0) built with EZPWD_NO_EXCEPTS:
 * every EZPWD_RAISE_OR_RETURN becomes a plain -1 return.
 */
#ifndef EZRS_ORACLE_H
#define EZRS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ezo_codec ezo_codec;

/* Build a codec: symbol bits mm (2..16), field polynomial, first consecutive root, primitive
 * element, number of roots, Berlekamp dual basis (mm == 8 only).  NULL if the parameters are
 * invalid (rs_base:599-635 primitivity check, rs_base:1254-1256 nroots check). */
ezo_codec *ezo_create(unsigned mm, unsigned poly, unsigned fcr, unsigned prim, unsigned nroots,
                      int dual);
void ezo_destroy(ezo_codec *c);

/* Codec geometry: NN (symbols per block), LOAD = NN-NROOTS, datum bytes (1 for mm<=8, else 2). */
unsigned ezo_size(const ezo_codec *c);
unsigned ezo_nroots(const ezo_codec *c);
unsigned ezo_load(const ezo_codec *c);
unsigned ezo_datum_bytes(const ezo_codec *c);
unsigned ezo_iprim(const ezo_codec *c);
/* Tables, exposed for the tests: alpha_to / index_of (NN+1 entries), genpoly (NROOTS+1). */
void ezo_tables(const ezo_codec *c, uint16_t *alpha_to, uint16_t *index_of, uint16_t *genpoly);

/* encode<TYP>(data, len, parity) -- rs_base:868-904 (+ encode_symbols 1296-1332).
 * data/parity are arrays of the codec's datum type (uint8_t or uint16_t). Returns NROOTS or -1. */
int ezo_encode(const ezo_codec *c, const void *data, unsigned len, void *parity);

/* decode<TYP>(data, len, parity, eras_pos, no_eras, corr) -- rs_base:1170-1242
 * (+ decode_symbols 1335-1718). len counts data symbols only; parity != NULL.
 * eras_pos must hold max(NROOTS, no_eras) entries; on return its first `count` entries are the
 * corrected positions (relative to data[0]).  corr (nullable) holds NROOTS datums.
 * Returns the count of corrected symbols, 0 for a valid codeword, or -1. */
int ezo_decode(const ezo_codec *c, void *data, unsigned len, void *parity, unsigned *eras_pos,
               unsigned no_eras, void *corr);

/* Batch wrappers (strides in elements).  parity == NULL means "parity follows the data in the
 * same row" (parity row = data row + len).  Decode: eras (nullable) rows of eras_stride entries,
 * neras (nullable) per-codeword erasure counts, result[ncw], positions (nullable) rows of
 * pos_stride >= NROOTS entries, corr (nullable) rows of corr_stride >= NROOTS datums. */
int ezo_encode_batch(const ezo_codec *c, const void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, size_t ncw, int nthreads);
/* Decode with Phil Karn's libfec semantics instead (fec-3.0.1/decode_rs.h:71-298): erasures and
 * positions in the full NN frame, no failure for deg lambda = 0, den = 0 or a root in the pad. */
void ezo_set_karn(ezo_codec *c, int karn);
int ezo_decode_batch(const ezo_codec *c, void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                     const uint32_t *neras, int32_t *result, uint32_t *positions,
                     size_t pos_stride, void *corr, size_t corr_stride, size_t ncw, int nthreads);

/* Berlekamp dual-basis maps (rs_base:109-146), exposed for the tests. */
const uint8_t *ezo_into_dual(void);
const uint8_t *ezo_from_dual(void);

#ifdef __cplusplus
}
#endif
#endif
