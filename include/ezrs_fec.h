/* ezrs_fec.h -- Phil Karn's libfec Reed-Solomon ABI over the MI355X engine (libezrs_fec.so).
 *
 * Drop-in for the RS entry points of fec-3.0.1/fec.h:229-257 (with the reference's int-symbol
 * patch, phil-karn/fec-3.0.1-int.patch) and phil-karn/rs.h:22-23 / pad_rs.c, which ezpwd's Karn
 * callers bind (phil-karn/rstest.c:98-114 and exercise.c:169-224, rsspeed.C:75-109):
 *
 *   init_rs_char / init_rs_int      fec-3.0.1/init_rs.h:48-101       (codec; pad fixed at init)
 *   encode_rs_char / encode_rs_int  fec-3.0.1/encode_rs.h:37-58      (NN-NROOTS-PAD data symbols)
 *   decode_rs_char / decode_rs_int  fec-3.0.1/decode_rs.h:71-298     (NN-PAD symbols in place)
 *   free_rs_char / free_rs_int
 *   encode_rs_8 / decode_rs_8       fec-3.0.1/encode_rs_8.c, decode_rs_8.c (CCSDS polynomial
 *                                   0x187, fcr 112, prim 11, 32 roots, conventional basis)
 *   encode_rs_ccsds / decode_rs_ccsds  fec-3.0.1/encode_rs_ccsds.c, decode_rs_ccsds.c (the same
 *                                   codec on Berlekamp dual-basis symbols)
 *   pad_rs_char / pad_rs_int        phil-karn/pad_rs.c (change a codec's pad)
 *
 * Karn's semantics, not ezpwd's (the engine's EZRS_SEM_KARN mode, include/ezrs.h): erasure and
 * corrected positions are in the full NN frame (position p >= pad is data[p - pad]); a decode never
 * fails for deg lambda = 0, a zero Forney denominator or a root in the pad (decode_rs.h:232-289).
 *
 * Every call runs on the GPU (device 0, or EZRS_FEC_DEVICE): the single-codeword calls pay a PCIe
 * round trip, the *_batch forms move whole arrays.  init_* returns NULL when the parameters are
 * invalid or no GPU is usable; an engine failure inside a void call aborts with a message (there
 * is no CPU fallback and no silent failure).
 *
 * The codec handle points at a `struct rs` laid out as fec-3.0.1/rs-common.h:7-19 (mm, nn,
 * alpha_to, index_of, genpoly, nroots, fcr, prim, iprim, pad): callers that read rs->nn, rs->nroots
 * or rs->pad (exercise.c:49, 169-172) work unchanged.  The table pointers are NULL: the field
 * tables live on the device.
 */
#ifndef EZRS_FEC_H
#define EZRS_FEC_H

#include <stddef.h>

#include "ezrs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* General-purpose codec, 8-bit symbol containers (symsize 2..8). */
void *init_rs_char(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad);
void encode_rs_char(void *rs, unsigned char *data, unsigned char *parity);
int decode_rs_char(void *rs, unsigned char *data, int *eras_pos, int no_eras);
void free_rs_char(void *rs);

/* General-purpose codec, int symbol containers (symsize 2..16; fec.h as patched by
 * phil-karn/fec-3.0.1-int.patch). */
void *init_rs_int(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad);
void encode_rs_int(void *rs, unsigned int *data, unsigned int *parity);
int decode_rs_int(void *rs, unsigned int *data, int *eras_pos, int no_eras);
void free_rs_int(void *rs);

/* CCSDS (255,223), conventional basis (fixed.h) and dual basis (ccsds.h); pad per call. */
void encode_rs_8(unsigned char *data, unsigned char *parity, int pad);
int decode_rs_8(unsigned char *data, int *eras_pos, int no_eras, int pad);
void encode_rs_ccsds(unsigned char *data, unsigned char *parity, int pad);
int decode_rs_ccsds(unsigned char *data, int *eras_pos, int no_eras, int pad);

/* phil-karn/pad_rs.c: set a codec's pad; NULL (codec unchanged) unless 0 <= pad < NN - NROOTS. */
void *pad_rs_char(void *p, int pad);
void *pad_rs_int(void *p, int pad);

/* Batch forms (host arrays; one engine call for the whole batch).  Row k of `data` holds the
 * NN-NROOTS-PAD data symbols of codeword k at data + k*stride; encode writes its NROOTS parity
 * symbols at parity + k*parity_stride.  Decode works in place on rows of NN-PAD symbols (data then
 * parity, Karn's data[] array) at data + k*stride: eras_pos + k*eras_stride holds no_eras[k]
 * full-frame erasure positions (no_eras may be NULL: none) and receives the corrected positions,
 * result[k] = decode_rs_char's return value.  0 on success, -errno on an engine failure. */
int encode_rs_char_batch(void *rs, const unsigned char *data, size_t stride, unsigned char *parity,
                         size_t parity_stride, size_t ncw);
int decode_rs_char_batch(void *rs, unsigned char *data, size_t stride, int *eras_pos,
                         size_t eras_stride, const int *no_eras, int *result, size_t ncw);
int encode_rs_int_batch(void *rs, const unsigned int *data, size_t stride, unsigned int *parity,
                        size_t parity_stride, size_t ncw);
int decode_rs_int_batch(void *rs, unsigned int *data, size_t stride, int *eras_pos,
                        size_t eras_stride, const int *no_eras, int *result, size_t ncw);

/* The engine codec behind a Karn handle (EZRS_SEM_KARN decode semantics): device-resident batches
 * go through ezrs_encode / ezrs_decode on it, with len = NN - NROOTS - PAD. */
ezrs_codec *ezrs_fec_codec(void *rs);

#ifdef __cplusplus
}
#endif

#endif /* EZRS_FEC_H */
