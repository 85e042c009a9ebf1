// ezrs_internal.hpp -- shared declarations of the MI355X RS engine (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <type_traits>
#include <vector>

#include "ezrs_field.hpp"

namespace ezrs {

// hipMemcpy2DAsync moves each row separately; when both pitches equal the row width the region
// is contiguous and goes as one linear copy.
inline hipError_t copy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                         size_t height, hipMemcpyKind kind, hipStream_t st) {
    if (height == 1 || (dpitch == width && spitch == width))
        return hipMemcpyAsync(dst, src, width * height, kind, st);
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, kind, st);
}

// Everything a kernel needs to know about a codec, passed by value at launch.
struct DevCodec {
    unsigned mm, nn, nroots, load, fcr, prim, iprim, poly;
    int dual;
    int masked;                   // symbol narrower than its datum (rs_base:1194)
    int ncu;                      // compute units of the device (persistent grids)
    size_t launch_rows;           // test hook (ezrs_set_launch_rows): codewords per plane-sliced
                                  // launch, 0 = the largest batch whose 32-bit offsets fit
    int karn;                     // decode with Phil Karn's libfec semantics (ezrs_set_semantics):
                                  // erasures and positions in the full NN frame, none of ezpwd's
                                  // extra failure checks (fec-3.0.1/decode_rs.h:71-298)
    const uint16_t *alpha_to;     // device, nn+1
    const uint16_t *index_of;     // device, nn+1
    const uint16_t *genpoly;      // device, nroots+1 (index form)
    const uint8_t *into_dual;     // device, 256
    const uint8_t *from_dual;     // device, 256
};

// Shard batches (ezrs_encode_shards / ezrs_decode_shards): codeword k is row j = k mod rows of
// shard s = k / rows, at element offset s * pitch + j * stride; every row holds `len` data symbols
// and its parity, except the shard's last row, which holds `tail` data symbols (a shortened
// codeword) and its parity.  rows == 0: a plain batch (row k at k * stride).
struct Shards {
    uint32_t rows = 0;
    uint32_t tail = 0;
    size_t pitch = 0;
};

// Element offset and data length of row k.
__host__ __device__ __forceinline__ size_t shard_row(const Shards &g, size_t k, size_t stride, unsigned len,
                                                     unsigned &rlen) {
    if (!g.rows) {
        rlen = len;
        return k * stride;
    }
    size_t s, j;
    if ((k >> 32) == 0) {                           // 32-bit division (the device's 64-bit one is a
        const uint32_t k32 = (uint32_t)k, s32 = k32 / g.rows;     // long software sequence)
        s = s32;
        j = k32 - s32 * g.rows;
    } else {
        s = k / g.rows;
        j = k - s * g.rows;
    }
    rlen = j + 1 == g.rows ? g.tail : len;
    return s * g.pitch + j * stride;
}

// Arguments of one batch decode (strides in elements).
struct DecodeArgs {
    void *data;
    size_t data_stride;
    unsigned len;
    void *parity;                 // never null here: the C ABI resolves parity == NULL
    size_t parity_stride;
    const uint32_t *eras;
    size_t eras_stride;
    const uint32_t *neras;
    int32_t *result;
    uint32_t *positions;
    size_t pos_stride;
    void *corr;
    size_t corr_stride;
    size_t ncw;
    Shards sh{};                  // sh.rows != 0: shard rows, parity inline (data + row length)
    // plane-sliced path: the syndrome kernel stores flag_gen into *flag_word when it flags a
    // codeword, and the error path skips its screen when the word holds another value (and no
    // erasures are given): nothing was flagged by this call
    uint32_t *flag_word = nullptr;
    uint32_t flag_gen = 0;
};

struct EncodeArgs {
    const void *data;
    size_t data_stride;
    unsigned len;
    void *parity;
    size_t parity_stride;
    size_t ncw;
    Shards sh{};                  // sh.rows != 0: shard rows, parity inline (data + row length)
};

// Row k's data and parity pointers and data length (plain batches: the strided arrays; shard
// batches: the row, its parity right after its data).
template <typename T, typename P, class A>
__host__ __device__ __forceinline__ void row_ptrs(const A &a, size_t k, P *&data, T *&parity, unsigned &len) {
    if (!a.sh.rows) {
        len = a.len;
        data = static_cast<P *>(a.data) + k * a.data_stride;
        parity = static_cast<T *>(a.parity) + k * a.parity_stride;
        return;
    }
    const size_t off = shard_row(a.sh, k, a.data_stride, a.len, len);
    data = static_cast<P *>(a.data) + off;
    parity = const_cast<T *>(reinterpret_cast<const T *>(data)) + len;
}

// Generic per-codeword kernels (ezrs_generic.hip): every codec, every length.
hipError_t launch_encode_generic(const DevCodec &c, const EncodeArgs &a, hipStream_t s);
hipError_t launch_decode_generic(const DevCodec &c, const DecodeArgs &a, hipStream_t s);
// Syndrome workspace layouts the error path reads.  Rows: [ncw][32] bytes (bit-sliced kernels).
// Tiled (plane-sliced kernels): codeword k's syndrome j at (k / 256) * kSynTile + 256 j + k % 256,
// so the syndrome kernel stores four codewords' syndrome j as one dword and the error path's loads
// of one syndrome across a wavefront's codewords fall in one or two cache lines.
constexpr size_t kSynTile = 256 * 32;
enum class SynLayout { Rows, Tiled };
// Error path behind the sliced syndrome kernels: decodes the codewords whose result holds the
// sentinel, starting from the syndromes in syn_ws.
hipError_t launch_decode_flagged(const DevCodec &c, const DecodeArgs &a, const uint8_t *syn_ws,
                                 SynLayout layout, hipStream_t s);

// Bit-sliced GF(2^8) kernels (ezrs_bitslice.hip) for the codecs of gen/ezrs_bs_tables.inc.
int bitslice_codec_id(const DevCodec &d);   // -1 if the codec has no bit-sliced path
// Encode needs a workspace of bs_encode_ws_bytes(ncw) device bytes.
size_t bs_encode_ws_bytes(size_t ncw);
hipError_t launch_bs_encode(int id, const DevCodec &d, const EncodeArgs &a, void *ws, hipStream_t s);
hipError_t launch_bs_syndromes(int id, const DevCodec &d, const DecodeArgs &a, uint8_t *syn_ws,
                               hipStream_t s);

// Plane-sliced GF(2^8) kernels (ezrs_ps.hip) for the codecs of gen/ezrs_ps_tables.inc: row pitch
// <= 256 bytes; decode needs the parity inside the row.
int planeslice_codec_id(const DevCodec &d);   // -1 if the codec has no plane-sliced path
size_t ps_ws_bytes(size_t ncw);
bool ps_can_encode(const DevCodec &d, const EncodeArgs &a);
bool ps_can_decode(const DevCodec &d, const DecodeArgs &a);
hipError_t launch_ps_encode(int id, const DevCodec &d, const EncodeArgs &a, void *ws, hipStream_t s);
hipError_t launch_ps_syndromes(int id, const DevCodec &d, const DecodeArgs &a, uint8_t *syn_ws,
                               hipStream_t s);

// GF(2^16) kernels (ezrs_wide.hip) for the codecs of gen/ezrs_wide_tables.inc: remainder networks
// + syndrome/parity finish + wavefront-per-codeword error path.  Decode needs inline parity.
int wide_codec_id(const DevCodec &d);        // -1 if the codec has no wide fast path
size_t wide_ws_bytes(int id, size_t ncw);
// blob: syndrome leader slots [32] | log beta [32] | log Q [NR][NR] (host copy; the Q part is
// also uploaded to the device)
bool wide_build_consts(int id, const CodecMath &m, std::vector<uint16_t> &blob);
size_t wide_cols_count(unsigned nroots);   // u16 entries of the device column tables (blob + 64)
bool wide_can_encode(const DevCodec &d, const EncodeArgs &a);
bool wide_can_decode(const DevCodec &d, const DecodeArgs &a);
hipError_t launch_wide_encode(int id, const DevCodec &d, const EncodeArgs &a, const uint16_t *blob_host,
                              const uint16_t *cols_dev, void *ws, hipStream_t s);
hipError_t launch_wide_decode(int id, const DevCodec &d, const DecodeArgs &a, const uint16_t *blob_host,
                              const uint16_t *cols_dev, void *ws, hipStream_t s);

} // namespace ezrs
