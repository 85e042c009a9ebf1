/*
 * ezbch_oracle.h -- TEST INFRASTRUCTURE ONLY (see ezbch_oracle.c): the CPU restatement of the binary
 * BCH codec the reference wraps (ezpwd::bch_base, c++/ezpwd/bch:48-463).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline use it, as the checker.
 *
 * Parity status: pinned by the reference's BCH fixtures only (README vector, Itron SCM captures,
 * BCH(255,k,t) shape table); the Djelic sources are absent from the reference.
 */
#ifndef EZBCH_ORACLE_H
#define EZBCH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

typedef struct ezb ezb_t;

/* init_bch(m, t, prim_poly) (bch_base:49-69): NULL unless 5 <= m <= 15, t >= 1, m*t < 2^m-1 and
 * the polynomial (0 = default for m) is primitive of degree m. */
ezb_t *ezb_create(int m, int t, unsigned prim_poly);
void ezb_destroy(ezb_t *b);
/* out6 = { m, n, t, ecc_bits, ecc_bytes, prim_poly } (bch_base:30-47) */
void ezb_info(const ezb_t *b, unsigned *out6);
/* generator coefficients, x^0 first: ecc_bits + 1 bytes of 0/1 */
void ezb_genpoly(const ezb_t *b, uint8_t *coef);

/* encode_bch on a zeroed ECC (bch:196-205) */
void ezb_encode(const ezb_t *b, const uint8_t *data, unsigned len, uint8_t *ecc);
/* decode_bch(data, len, recv_ecc, NULL, NULL, errloc) (bch_base:86-127): the number of bit errors,
 * -74 (EBADMSG) or -22 (EINVAL); errloc[0..count) ascending. */
/* S_1..S_2t (syn[0..2t)) of a received codeword; decode from syndromes alone (decode_bch's
 * hardware-syndrome form) */
int ezb_syndromes(const ezb_t *b, const uint8_t *data, unsigned len, const uint8_t *recv_ecc,
                  unsigned *syn);
int ezb_decode_syn(const ezb_t *b, unsigned len, const unsigned *syn, unsigned *errloc);
int ezb_decode(const ezb_t *b, const uint8_t *data, unsigned len, const uint8_t *recv_ecc,
               unsigned *errloc);
/* correct_bch (bch_base:168-199): decode, then flip the reported bits of data and ECC. */
int ezb_correct(const ezb_t *b, uint8_t *data, unsigned len, uint8_t *ecc, unsigned *errloc);

/* Batch forms over rows (ecc == NULL: the ECC follows the data in the row); OpenMP threads. */
void ezb_encode_batch(const ezb_t *b, const uint8_t *data, size_t dstride, unsigned len,
                      uint8_t *ecc, size_t estride, size_t ncw, int nthreads);
void ezb_decode_batch(const ezb_t *b, uint8_t *data, size_t dstride, unsigned len, uint8_t *ecc,
                      size_t estride, int32_t *result, uint32_t *errloc, size_t lstride,
                      size_t ncw, int nthreads);

#endif /* EZBCH_ORACLE_H */
