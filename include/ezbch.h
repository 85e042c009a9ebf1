/*
 * ezbch.h -- C ABI of the MI355X binary BCH engine (part of libezrs_hip.so).
 *
 * Drop-in boundary for the BCH sibling of the reference's hot path: the Djelic (Linux lib/bch.c)
 * codec wrapped by
 *
 *   ezpwd::bch_base(m, t, prim_poly)            -> init_bch                 c++/ezpwd/bch:54-61
 *   ezpwd::BCH<N,K,T>                           (shape-checked)             c++/ezpwd/bch:423-443
 *   bch_base::encode(data, len, parity)         -> encode_bch, zeroed ECC   c++/ezpwd/bch:196-205
 *   bch_base::decode(data, len, parity, &pos)   -> correct_bch              c++/ezpwd/bch:316-331,
 *                                                                           c++/ezpwd/bch_base:168-199
 *
 * applied independently to every codeword of a batch.  Conventions follow ezrs.h: compute entry
 * points take DEVICE pointers and a hipStream_t passed as void*, are asynchronous and never
 * allocate; the *_host forms take host pointers and block.  Every function returns 0 or a negative
 * errno (-EINVAL bad arguments / parameters init_bch rejects, -ENODEV no usable HIP device, -ENOMEM, -EIO a HIP error).
 *
 * Bit conventions (bch_base:119-123): data bits enter MSB first; the ECC is the remainder
 * left-justified and big-endian in ecc_bytes bytes; an error location e addresses data[e/8] bit
 * (e%8) for e < 8*len and ECC byte e/8-len bit (e%8) beyond.  Every init_bch-valid codec runs on the
 * device: t <= 64 and ecc_bits <= 1024 one lane per codeword, larger ones one wavefront per codeword.
 */
#ifndef EZBCH_H
#define EZBCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ezbch_codec ezbch_codec;

typedef struct ezbch_info {
    unsigned m;          /* Galois field order                      (bch_base:32 m)         */
    unsigned n;          /* codeword bits 2^m - 1                   (bch_base:33 n)         */
    unsigned t;          /* correction capability in bits           (bch_base:34 t)         */
    unsigned ecc_bits;   /* generator degree                        (bch_base:35 ecc_bits)  */
    unsigned ecc_bytes;  /* ceil(m*t / 8)                           (bch_base:36 ecc_bytes) */
    unsigned prim_poly;  /* field polynomial in use                                         */
    int device;
} ezbch_info;

/* init_bch(m, t, prim_poly) (bch_base:49-69; prim_poly 0 = the default for m): -EINVAL unless
 * 5 <= m <= 15, t >= 1, m*t < 2^m - 1 and the polynomial is primitive of degree m. */
int ezbch_create(ezbch_codec **out, unsigned m, unsigned t, unsigned prim_poly, int device);
/* ezpwd::BCH<N,K,T>: as ezbch_create(log2(N+1), T, 0), and -EINVAL unless the codec init_bch builds
 * has exactly N - ecc_bits == K (the constructor's check, bch:436-442). */
int ezbch_create_nkt(ezbch_codec **out, unsigned n, unsigned k, unsigned t, int device);
int ezbch_destroy(ezbch_codec *codec);
int ezbch_get_info(const ezbch_codec *codec, ezbch_info *info);

/* Batch encode -- for every codeword k < ncw: ecc_k = encode_bch(data_k, len) with a zeroed ECC
 * (bch:196-205).  The data rows are only read; ecc is required (-EINVAL if NULL). */
int ezbch_encode(const ezbch_codec *codec, const uint8_t *data, size_t data_stride, unsigned len,
                 uint8_t *ecc, size_t ecc_stride, size_t ncw, void *stream);
/* Row form: each row carries its ECC after its data (rows + len), as in bch:184-195. */
int ezbch_encode_rows(const ezbch_codec *codec, uint8_t *rows, size_t stride, unsigned len,
                      size_t ncw, void *stream);

/* Batch decode, in place -- for every codeword k < ncw:
 *   result[k] = correct_bch(data_k, len, ecc_k, errloc_k)
 * i.e. the number of corrected bits (0 for a valid codeword), -74 (EBADMSG) if uncorrectable,
 * -22 (EINVAL) if 8*len > n - ecc_bits; the reported bits are flipped in data and ECC.
 * errloc (nullable): uint32 rows of errloc_stride >= t entries; entries 0..result[k]-1 receive the
 * error locations in ascending order.  ecc == NULL: the ECC follows the data in the row. */
int ezbch_decode(const ezbch_codec *codec, uint8_t *data, size_t data_stride, unsigned len,
                 uint8_t *ecc, size_t ecc_stride, int32_t *result, uint32_t *errloc,
                 size_t errloc_stride, size_t ncw, void *stream);

/* decode_bch's "ecc = recv_ecc XOR calc_ecc" form (bch_base:96-111, Djelic's decode without the
 * data): for every codeword k < ncw, result[k] = the number of errors the ECC difference ecc_k
 * reveals for a codeword of len data bytes (or -EBADMSG / -EINVAL), with the error locations in
 * errloc; nothing is corrected and no data is read.  Device pointers. */
int ezbch_decode_ecc(const ezbch_codec *codec, const uint8_t *ecc, size_t ecc_stride, unsigned len,
                     int32_t *result, uint32_t *errloc, size_t errloc_stride, size_t ncw,
                     void *stream);

/* decode_bch's syndrome form (bch_base:112-114, "by providing syndrome results @syn"): syn rows
 * hold S_1..S_2t (2t uint32 each, e.g. computed by hardware); result[k] = the number of errors
 * those syndromes locate in a codeword of len data bytes (or -EBADMSG / -EINVAL), locations in
 * errloc as ezbch_decode reports them; nothing is read or corrected.  Device pointers. */
int ezbch_decode_syn(const ezbch_codec *codec, const uint32_t *syn, size_t syn_stride, unsigned len,
                     int32_t *result, uint32_t *errloc, size_t errloc_stride, size_t ncw,
                     void *stream);

/* Host-memory forms (blocking), streamed through the device in chunks of `chunk` codewords
 * (0 = library default).  Encode moves only the data bytes in and a compact ECC block out; the
 * caller's data bytes are never written. */
int ezbch_encode_host(ezbch_codec *codec, const uint8_t *data, size_t data_stride, unsigned len,
                      uint8_t *ecc, size_t ecc_stride, size_t ncw, size_t chunk);
int ezbch_encode_rows_host(ezbch_codec *codec, uint8_t *rows, size_t stride, unsigned len,
                           size_t ncw, size_t chunk);
int ezbch_decode_host(ezbch_codec *codec, uint8_t *data, size_t data_stride, unsigned len,
                      uint8_t *ecc, size_t ecc_stride, int32_t *result, uint32_t *errloc,
                      size_t errloc_stride, size_t ncw, size_t chunk);
int ezbch_decode_syn_host(ezbch_codec *codec, const uint32_t *syn, size_t syn_stride, unsigned len,
                          int32_t *result, uint32_t *errloc, size_t errloc_stride, size_t ncw);

/* Human-readable text of the last BCH error seen by this thread ("" if none). */
const char *ezbch_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* EZBCH_H */
