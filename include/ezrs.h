/*
 * ezrs.h -- C ABI of the MI355X Reed-Solomon engine (libezrs_hip.so).
 *
 * Drop-in boundary for the hot path of pjkundert/ezpwd-reed-solomon: batched RS(N,K) encode and
 * errors+erasures decode over GF(2^m), m = 2..16, bit-exact with the reference's
 *
 *   ezpwd::reed_solomon<...>::encode<INP>(data, len, parity)                 c++/ezpwd/rs_base:868-904
 *   ezpwd::reed_solomon<...>::decode<INP>(data, len, parity, eras_pos,
 *                                         no_eras, corr)                     c++/ezpwd/rs_base:1170-1242
 *
 * applied independently to every codeword of a batch.  The reference has no batch or C ABI for
 * RS; each entry point below replaces a loop of those per-codeword calls (the loops in
 * rsencode.C:93-163, exercise.H:121-199, rsvalidate.C:97-289).  Codec construction replaces the
 * template instantiations ezpwd::RS<N,K>, RS_CCSDS<255,K>, RS_CCSDS_CONV<255,K> (c++/ezpwd/rs:74-104).
 *
 * Conventions
 *   - All compute entry points take DEVICE pointers (hipMalloc'd, on the codec's device) and a
 *     hipStream_t passed as void*; they are asynchronous and never synchronise.  A codec is const
 *     after creation and may be shared by threads and streams, like the reference's codec objects
 *     (rs_base:602-605): each stream gets its own device workspace (grown on demand, never freed
 *     before ezrs_destroy), so calls on different streams never share scratch memory.  The *_ws
 *     forms take a caller-owned workspace of ezrs_workspace_bytes() instead (no allocation at all:
 *     the form to capture into a hipGraph); ezrs_reserve_stream pre-sizes a stream's workspace.
 *     ezrs_*_host take host pointers and run a chunked, double-buffered H2D/kernel/D2H pipeline.
 *   - A codeword's symbols are stored as its datum type: uint8_t for m <= 8, uint16_t for m > 8
 *     (the reference's TYP, rs:75-89).  Strides are in ELEMENTS of the respective array.
 *   - `len` is the number of data (non-parity) symbols per codeword, 1..N-NROOTS; shorter codewords
 *     are shortened codes with implicit leading zeros (rs_base:1302-1304, 1378).
 *   - Encode reads `data` and writes `parity` (encode(data, len, parity), rs_base:868-904); rows that
 *     carry their own parity after the data (the reference's pair/container forms, rs_base:778-790)
 *     go through ezrs_encode_rows.  Decode with parity == NULL: the parity follows the data in the
 *     row, at data + len (the reference's decode(data, len+NROOTS) form, rs_base:1183-1186).
 *   - Symbols narrower than their datum (e.g. RS(31,K) in uint8_t) follow the reference's masked
 *     path: data bits above the symbol are ignored on encode and preserved on decode; a parity datum
 *     with bits above the symbol fails that codeword's decode with -1 (rs_base:1194-1235).
 *   - Return value of every function: 0 on success or a negative errno (-EINVAL bad arguments,
 *     -ENODEV no usable HIP device, -ENOMEM, -EIO a HIP runtime error).  No C++ exception ever
 *     crosses this ABI.  Per-codeword decode outcomes go to `result` (see ezrs_decode).
 */
#ifndef EZRS_H
#define EZRS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EZRS_ABI_VERSION 5

typedef struct ezrs_codec ezrs_codec;

typedef struct ezrs_info {
    unsigned symbol_bits;  /* m                                    (rs_base:570 SYMBOL/MM) */
    unsigned size;         /* N = 2^m - 1                          (rs_base:571 SIZE/NN)   */
    unsigned nroots;       /* N - K parity symbols                 (rs_base:723 NROOTS)    */
    unsigned load;         /* K = N - NROOTS max data symbols      (rs_base:724 LOAD)      */
    unsigned poly;         /* field polynomial                     (rs_base:756 poly())    */
    unsigned fcr;          /* first consecutive root               (rs_base:762 fcr())     */
    unsigned prim;         /* primitive element                    (rs_base:767 prim())    */
    unsigned datum_bytes;  /* 1 (uint8_t) or 2 (uint16_t)          (rs_base:568 DATUM/8)   */
    int dual;              /* CCSDS Berlekamp dual basis           (rs_base:772 dual())    */
    int device;            /* HIP device the codec lives on */
} ezrs_info;

/* Library / device probe: returns the number of visible HIP devices (>= 0) or a negative errno. */
int ezrs_device_count(void);
/* ABI version of the loaded library (EZRS_ABI_VERSION). */
int ezrs_abi_version(void);

/* Generic codec over GF(2^m): replaces ezpwd::reed_solomon<TYP,SYM,RTS,FCR,PRM,gfpoly<SYM,PLY>,DUAL>
 * (rs_base:702-1719).  Fails with -EINVAL where the reference's constructor would raise:
 * non-primitive poly (rs_base:623-625), nroots == 0 or >= N (rs_base:1254-1256), dual with m != 8
 * (rs_base:1188-1190); -ENOTSUP for m > 8 with more than 256 parity symbols (engine limit). */
int ezrs_create(ezrs_codec **out, unsigned symbol_bits, unsigned poly, unsigned fcr,
                unsigned prim, unsigned nroots, int dual, int device);
/* ezpwd::RS<N,K> -- the standard polynomial per N, FCR = 1, PRIM = 1 (rs:74-89). */
int ezrs_create_rs(ezrs_codec **out, unsigned n, unsigned k, int device);
/* ezpwd::RS_CCSDS<255,K> (dual = 1) / RS_CCSDS_CONV<255,K> (dual = 0): poly 0x187,
 * FCR = 128 - (255-K)/2, PRIM = 11 (rs:101-104). */
int ezrs_create_ccsds(ezrs_codec **out, unsigned k, int dual, int device);
int ezrs_destroy(ezrs_codec *codec);
/* Which kernel family serves the codec's full-length batches: EZRS_PATH_* (diagnostics; every
 * family is bit-exact with the reference). */
#define EZRS_PATH_GENERIC 0     /* per-codeword kernels (lane or 32-lane group per codeword)        */
#define EZRS_PATH_BITSLICE 1    /* bit-sliced GF(2^8) kernels (CCSDS dual basis)                     */
#define EZRS_PATH_PLANESLICE 2  /* plane-sliced GF(2^8) tile kernels (RS(255,K), NROOTS <= 32)       */
#define EZRS_PATH_WIDE 3        /* GF(2^16) remainder-network kernels (RS(65535,65503/65519))        */
int ezrs_kernel_path(const ezrs_codec *codec);
/* Decode semantics of a codec (encode is the same under both):
 *   EZRS_SEM_EZPWD (default) -- decode_symbols of c++/ezpwd/rs_base:1335-1718: erasures and
 *     positions relative to the first supplied symbol; -1 for deg lambda = 0, a zero Forney
 *     denominator or a root in the pad (rs_base:1589-1648).
 *   EZRS_SEM_KARN -- decode_rs_char / decode_rs_int of Phil Karn's libfec
 *     (fec-3.0.1/decode_rs.h:71-298): erasures and positions in the full NN frame (a position
 *     p >= pad is row symbol p - pad), none of those three checks (a zero denominator applies
 *     num1 * num2, a root in the pad is counted and reported but not corrected), the datum is the
 *     symbol.  The Karn ABI (include/ezrs_fec.h) creates its codecs in this mode.  As in libfec,
 *     the syndromes are checked before the erasures: a word with zero syndromes returns 0 even
 *     with an erasure position >= NN (otherwise -1, where libfec's result is undefined); a root in
 *     the pad gets correction value 0 in `corr`.
 * Set the semantics once, after create and before the codec's first decode: the setter takes the
 * codec's lock (it waits for a host-memory call in progress), but a device decode already enqueued
 * on a stream runs with the semantics it was launched with, and decodes issued concurrently from
 * other threads may see either. */
#define EZRS_SEM_EZPWD 0
#define EZRS_SEM_KARN 1
int ezrs_set_semantics(ezrs_codec *codec, int semantics);
int ezrs_get_semantics(const ezrs_codec *codec);
/* Test hook: cap the codewords one plane-sliced kernel launch of `codec` takes (0 restores the
 * default, the largest batch whose 32-bit buffer offsets fit).  Results never depend on it:
 * lowering it only splits a batch over more launches (mid-tile for shard batches), which the tests
 * use to exercise those splits at small sizes.  Per codec; takes the codec's lock, so it waits for
 * a host-memory call in progress, but a device call already enqueued keeps the cap it was
 * launched with. */
int ezrs_set_launch_rows(ezrs_codec *codec, size_t rows);
int ezrs_get_info(const ezrs_codec *codec, ezrs_info *info);

/* Pre-size the workspace of `stream` (NULL: the null stream) for batches of up to `ncw` codewords,
 * so that later calls of that size on that stream do not allocate. */
int ezrs_reserve(ezrs_codec *codec, size_t ncw);
int ezrs_reserve_stream(const ezrs_codec *codec, size_t ncw, void *stream);
/* Device workspace bytes a batch of ncw codewords needs (encode and decode alike; may be 0). */
size_t ezrs_workspace_bytes(const ezrs_codec *codec, size_t ncw);

/* Batch encode -- for every codeword k < ncw:
 *   encode<TYP>(data + k*data_stride, len, parity + k*parity_stride)          rs_base:868-904
 * data and parity are device arrays of the datum type; data is only read, parity is required. */
int ezrs_encode(const ezrs_codec *codec, const void *data, size_t data_stride, unsigned len,
                void *parity, size_t parity_stride, size_t ncw, void *stream);
/* Row form: row k holds len data symbols followed by its NROOTS parity symbols (written):
 *   encode(std::pair(rows_k, rows_k + len + NROOTS))                          rs_base:778-790 */
int ezrs_encode_rows(const ezrs_codec *codec, void *rows, size_t stride, unsigned len, size_t ncw,
                     void *stream);
/* The same with a caller-owned device workspace of >= ezrs_workspace_bytes(codec, ncw) bytes. */
int ezrs_encode_ws(const ezrs_codec *codec, const void *data, size_t data_stride, unsigned len,
                   void *parity, size_t parity_stride, size_t ncw, void *ws, size_t ws_bytes,
                   void *stream);
int ezrs_encode_rows_ws(const ezrs_codec *codec, void *rows, size_t stride, unsigned len,
                        size_t ncw, void *ws, size_t ws_bytes, void *stream);

/* Batch decode -- for every codeword k < ncw, in place:
 *   result[k] = decode<TYP>(data + k*data_stride, len, parity + k*parity_stride,
 *                           eras_pos_k, neras[k], corr + k*corr_stride)      rs_base:1170-1242
 * eras       (nullable) uint32 rows of eras_stride entries: erasure positions relative to data[0]
 *            (parity positions follow at len..len+NROOTS-1); neras (nullable) their counts.
 * result     int32[ncw]: number of corrected symbols (erasures included, even when the erased
 *            symbol was already right), 0 for a valid codeword, -1 if uncorrectable or invalid
 *            (rs_base:1335-1718).  On -1 the direct (unmasked) path may leave partial
 *            corrections applied, exactly as the reference does (rs_base:1610-1690, 1238-1241).
 * positions  (nullable) uint32 rows of pos_stride >= NROOTS: entries 0..result[k]-1 receive the
 *            corrected positions relative to data[0], in the reference's Chien-search order
 *            (rs_base:1557-1576, 1713-1716); other entries are left untouched.
 * corr       (nullable) datum rows of corr_stride >= NROOTS: corr[j] receives the correction
 *            pattern of position j, for the j the reference writes (rs_base:1658-1687). */
int ezrs_decode(const ezrs_codec *codec, void *data, size_t data_stride, unsigned len,
                void *parity, size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                const uint32_t *neras, int32_t *result, uint32_t *positions, size_t pos_stride,
                void *corr, size_t corr_stride, size_t ncw, void *stream);
int ezrs_decode_ws(const ezrs_codec *codec, void *data, size_t data_stride, unsigned len,
                   void *parity, size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                   const uint32_t *neras, int32_t *result, uint32_t *positions, size_t pos_stride,
                   void *corr, size_t corr_stride, size_t ncw, void *ws, size_t ws_bytes,
                   void *stream);

/* Shard batches (device-resident).  A shard of `shard_len` data symbols is stored as the rsencode
 * wire format lays it out (rsencode.C:93-163, one encode/decode per chunk): R = ceil(shard_len /
 * chunk) codewords back to back, each `chunk` data symbols followed by its NROOTS parity symbols,
 * except the last, which carries the remaining shard_len - (R-1)*chunk data symbols (a shortened
 * codeword, rs_base:1302-1304) and its parity.  Shard i starts at shards + i*shard_pitch (elements,
 * >= ezrs_shard_encoded_len).  Codewords are numbered shard-major, k = i*R + j: result[k],
 * erasure / position / correction rows k are codeword j of shard i, positions relative to that
 * codeword's first data symbol.  The whole batch is one launch of the codec's kernels. */
size_t ezrs_shard_codewords(const ezrs_codec *codec, size_t shard_len, unsigned chunk);
size_t ezrs_shard_encoded_len(const ezrs_codec *codec, size_t shard_len, unsigned chunk);
/* Writes every codeword's parity (its data is only read). */
int ezrs_encode_shards(const ezrs_codec *codec, void *shards, size_t shard_pitch, size_t shard_len,
                       unsigned chunk, size_t nshards, void *stream);
/* Decodes every codeword in place: result[k] etc. as ezrs_decode, for nshards * R codewords. */
int ezrs_decode_shards(const ezrs_codec *codec, void *shards, size_t shard_pitch, size_t shard_len,
                       unsigned chunk, size_t nshards, const uint32_t *eras, size_t eras_stride,
                       const uint32_t *neras, int32_t *result, uint32_t *positions,
                       size_t pos_stride, void *corr, size_t corr_stride, void *stream);

/* Host-memory forms: the same contracts with HOST pointers.  The batch is streamed through the
 * device in chunks of `chunk` codewords (0 = library default) over two HIP streams with
 * asynchronous copies; pinned host memory (ezrs_host_alloc) gets full PCIe overlap.  Blocking:
 * they return when the results are back in host memory.
 * Encode sends each chunk's rows to the device (one linear copy of the rows' span when the row
 * pitch is at most about twice the row; otherwise the rows are gathered into pinned staging first)
 * and brings back only the parity, as one compact block that is then scattered into place: the
 * caller's data symbols are never written.  Decode sends inline-parity rows as one linear span;
 * back come the results and only the rows whose result is nonzero (compacted on the device, then
 * scattered into place): a clean codeword's row is never written. */
int ezrs_encode_host(ezrs_codec *codec, const void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, size_t ncw, size_t chunk);
int ezrs_encode_rows_host(ezrs_codec *codec, void *rows, size_t stride, unsigned len, size_t ncw,
                          size_t chunk);
int ezrs_decode_host(ezrs_codec *codec, void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, const uint32_t *eras,
                     size_t eras_stride, const uint32_t *neras, int32_t *result,
                     uint32_t *positions, size_t pos_stride, void *corr, size_t corr_stride,
                     size_t ncw, size_t chunk);

/* rsencode wire format (replaces the per-chunk loop of rsencode.C:93-163, whose encode/decode
 * helpers call RS_t::encode / RS_t::decode once per chunk).  The input is cut into chunks of
 * `chunk` data symbols (the last may be shorter); each chunk is written followed by its NROOTS
 * parity symbols; symbols wider than 8 bits are big-endian on the wire (rsencode.C:52-85).  All
 * chunks of a call are one batch on the device.
 *  - ezrs_stream_encode: out receives at most ezrs_stream_encoded_bound(in_bytes) bytes.
 *  - ezrs_stream_decode: out receives the corrected data without parity (<= in_bytes bytes); a
 *    chunk the decoder cannot correct is passed on as the decoder left it, as rsencode does, and
 *    counted in *n_failed (nullable).
 * A trailing piece that cannot form a chunk (an odd byte for 16-bit symbols; for decode, fewer
 * than NROOTS + 1 symbols -- rsencode.C:110-111, 140-141) returns -EMSGSIZE after the whole
 * chunks before it were written (*out_bytes counts them).  -EINVAL: chunk 0 or above the codec's
 * load; -ENOSPC: out_cap too small. */
size_t ezrs_stream_encoded_bound(const ezrs_codec *codec, size_t in_bytes, unsigned chunk);
int ezrs_stream_encode(ezrs_codec *codec, const void *in, size_t in_bytes, unsigned chunk,
                       void *out, size_t out_cap, size_t *out_bytes);
int ezrs_stream_decode(ezrs_codec *codec, const void *in, size_t in_bytes, unsigned chunk,
                       void *out, size_t out_cap, size_t *out_bytes, size_t *n_failed);

/* Pinned host memory for the host-memory forms (hipHostMalloc / hipHostFree). */
int ezrs_host_alloc(void **ptr, size_t bytes);
int ezrs_host_free(void *ptr);

/* Human-readable text of the last HIP error seen by this thread ("" if none). */
const char *ezrs_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* EZRS_H */
