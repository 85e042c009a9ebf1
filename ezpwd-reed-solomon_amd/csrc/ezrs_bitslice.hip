// ezrs_bitslice.hip -- bit-sliced GF(2^8) RS encode / syndrome kernels for MI355X (gfx950).
//
// Why bit-slicing: RS(255,223) encode+decode is ~15 k GF(2^8) multiply-accumulates per codeword.
// One LDS log/antilog lookup per MAC caps a table kernel near 5 % of the 8 TB/s HBM roofline.
// Here a 32-bit VGPR holds one bit of 32 symbol slots, so a constant GF multiply is an XOR
// network; each network is split into nibble groups (all 15 XOR combinations of an input nibble
// are formed once) and every output bit costs one v_bitop3_b32 (3-input XOR) per input byte.
//
// Work decomposition (one 128-thread workgroup = 2 waves = one 512-codeword tile):
//   * lane l owns codewords tile0 + l + 64c, c = 0..7; its 32 register slots are (c, segment s),
//     s = position mod 4, at bit 8s + c.  Segment interleaving keeps every step's input a natural
//     little-endian dword of 4 consecutive symbols of one codeword (no byte shuffles).
//   * wave r ("role") owns syndromes [S0[r], S0[r]+NS[r]): 16 syndromes x 8 bits = 128 state VGPRs.
//   * the tile streams through LDS in chunks of 64 positions ([512 rows][17 dwords], odd row
//     pitch: conflict-free column reads); each role bit-transposes half the chunk in place (3-stage
//     delta swap, 48 ops per 8 dwords) so the transposition is not duplicated across the roles.
//   * per chunk and role: state *= d^16, then 16 Horner y-steps (d = g^4) -- all constants are
//     straight-line XOR networks generated from the codec (gen/ezrs_bs_tables.inc).
//   * the 4 segment partials are folded in-register (tree: x g, << 8; x g^2, << 16), leaving the
//     syndromes of the lane's 8 codewords in byte lane 3.
//
// Decode (k_bs_syndromes): codewords whose 32 syndromes are zero (and carry no erasures) get
// result 0 -- exactly what decode_symbols returns (rs_base:1416-1434); all others get a sentinel
// and their syndromes are written to the workspace for the error-path kernel
// (ezrs_generic.hip: decode_from_syndromes), which runs the reference's BM/Chien/Forney.
// Encode (k_bs_encode): syndromes of the data word -> parity via the GF(2) map Q (generated),
// written straight to the caller's parity rows.
#include "ezrs_internal.hpp"
#include "gen/ezrs_bs_tables.inc"

namespace ezrs {
namespace bs {

constexpr int kTile = 512;        // codewords per workgroup
constexpr int kPitch = 17;        // LDS row pitch in dwords (64 data bytes + 4 pad)
constexpr int kThreads = 128;

// In-place 8x8 bit transpose of (register index) x (bit position mod 8): afterwards D[b] bit 8s+c
// holds what D[c] bit 8s+b held.  3 delta-swap stages, 4 ops per register pair.
__device__ __forceinline__ void transpose8(uint32_t (&D)[8]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int sh = 1 << k;
        const uint32_t M = k == 0 ? 0x55555555u : k == 1 ? 0x33333333u : 0x0F0F0F0Fu;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if (c & sh) continue;
            const uint32_t x = D[c], y = D[c | sh];
            D[c] = (x & M) | ((y << sh) & ~M);
            D[c | sh] = ((x >> sh) & M) | (y & ~M);
        }
    }
}

// Stage chunk k (positions [64k, 64k+64) of the zero-front-padded word) of the tile into LDS.
// Row rho = codeword cw0 + rho; symbol index u = position - pad; u < 0 reads as zero.
__device__ __forceinline__ void load_chunk(uint32_t *tile, const uint8_t *base, size_t stride,
                                           size_t cw0, size_t ncw, int k, int pad) {
#pragma unroll 4
    for (int j = 0; j < kTile * 4 / kThreads; ++j) {
        const int pi = threadIdx.x + kThreads * j;
        const int row = pi >> 2, q = pi & 3;
        const size_t cw = cw0 + row;
        const long u0 = 64L * k - pad + 16 * q;
        uint32_t v[4] = {0u, 0u, 0u, 0u};
        if (cw < ncw && u0 + 16 > 0) {
            const uint8_t *p = base + cw * stride;
            if ((long)(cw * stride) + u0 >= 0) {
                __builtin_memcpy(v, p + u0, 16);
            } else {
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (u0 + e >= 0) v[e >> 2] |= (uint32_t)p[u0 + e] << (8 * (e & 3));
            }
            if (u0 < 0) {
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const long lo = u0 + 4 * w;           // symbol index of byte 0 of dword w
                    if (lo + 4 <= 0) v[w] = 0;
                    else if (lo < 0) v[w] &= 0xFFFFFFFFu << (8 * (-lo));
                }
            }
        }
        uint32_t *d = tile + row * kPitch + 4 * q;
        d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
    }
}

// In-place bit transposition of y-steps [8*role, 8*role+8) of the chunk: the dwords of the lane's
// 8 codewords become 8 bit-planes (plane b stored where codeword b's dword was).
__device__ __forceinline__ void transpose_half(uint32_t *tile, int role, int lane) {
#pragma unroll 1
    for (int yy = 0; yy < 8; ++yy) {
        const int y = 8 * role + yy;
        uint32_t D[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) D[c] = tile[(lane + 64 * c) * kPitch + y];
        transpose8(D);
#pragma unroll
        for (int b = 0; b < 8; ++b) tile[(lane + 64 * b) * kPitch + y] = D[b];
    }
}

// Run the Horner chunks of one word (decode: codeword, encode: data) through the tile.  Each role
// runs its own copy of the loop (R is a template parameter): with a per-chunk role branch the
// compiler hoists the common LDS plane loads of all 16 y-steps above the branch and spills.
template <class C, int R>
__device__ __forceinline__ void syndromes_tile(uint32_t (&S)[16][8], uint32_t *tile,
                                               const uint8_t *base, size_t stride, size_t cw0,
                                               size_t ncw, int nchunks, int pad) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) S[i][q] = 0;
    for (int k = 0; k < nchunks; ++k) {
        load_chunk(tile, base, stride, cw0, ncw, k, pad);
        __syncthreads();
        transpose_half(tile, R, lane);
        __syncthreads();
        C::template horner_chunk<R>(S, tile, lane, k == 0);
        __syncthreads();
    }
    C::template fold<R>(S);
}

// Byte lane 3 of 8 planes -> per-codeword bytes: after transpose8, R[c] >> 24 is the symbol of
// codeword c.
__device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (a >> 24) | ((b >> 16) & 0xFF00u) | ((c >> 8) & 0xFF0000u) | (d & 0xFF000000u);
}

constexpr int32_t kSentinel = INT32_MIN;

template <class C, int R>
__device__ __forceinline__ uint32_t nonzero_mask(const uint32_t (&S)[16][8]) {
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) nz |= S[i][q];
    return nz >> 24;                             // bit c: codeword c has a nonzero syndrome
}

// Write the role's syndromes of the flagged codewords (bits of fl) to their workspace slots.
template <class C, int R>
__device__ __forceinline__ void write_syndromes(uint32_t (&S)[16][8], uint32_t fl, size_t cw,
                                                uint8_t *syn_ws) {
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i) transpose8(S[i]);   // S[i][c] >> 24: codeword c's S_i
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (!(fl >> c & 1)) continue;
        uint8_t *dst = syn_ws + (cw + 64 * c) * 32 + C::S0[R];
#pragma unroll
        for (int i = 0; i < C::NS[R]; i += 4) {
            if (i + 4 <= C::NS[R]) {
                const uint32_t w = pack4(S[i][c], S[i + 1][c], S[i + 2][c], S[i + 3][c]);
                __builtin_memcpy(dst + i, &w, 4);
            } else {
#pragma unroll
                for (int e = i; e < C::NS[R]; ++e) dst[e] = (uint8_t)(S[e][c] >> 24);
            }
        }
    }
}

template <class C, int R>
__device__ __forceinline__ void syndromes_body(uint32_t *tile, uint32_t (*flags)[64],
                                               const uint8_t *data, size_t stride, unsigned nsym,
                                               size_t ncw, const uint32_t *neras, int32_t *result,
                                               uint8_t *syn_ws) {
    const int lane = threadIdx.x & 63;
    const size_t cw0 = (size_t)blockIdx.x * kTile;
    const int nchunks = (int)((nsym + 63) / 64);
    const int pad = nchunks * 64 - (int)nsym;
    uint32_t S[16][8];
    syndromes_tile<C, R>(S, tile, data, stride, cw0, ncw, nchunks, pad);
    flags[R][lane] = nonzero_mask<C, R>(S);
    __syncthreads();
    uint32_t fl = flags[0][lane] | flags[1][lane];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const size_t cw = cw0 + lane + 64 * c;
        if (cw >= ncw) { fl &= ~(1u << c); continue; }
        if (neras && neras[cw]) fl |= 1u << c;      // erasures: the error path validates them
        if (R == 0) result[cw] = (fl >> c & 1) ? kSentinel : 0;
    }
    if (fl) write_syndromes<C, R>(S, fl, cw0 + lane, syn_ws);
}

template <class C>
__global__ void __launch_bounds__(kThreads, 2)
    k_bs_syndromes(const uint8_t *data, size_t stride, unsigned nsym, size_t ncw,
                   const uint32_t *neras, int32_t *result, uint8_t *syn_ws) {
    __shared__ uint32_t tile[kTile * kPitch];
    __shared__ uint32_t flags[2][64];
    if (threadIdx.x < 64)
        syndromes_body<C, 0>(tile, flags, data, stride, nsym, ncw, neras, result, syn_ws);
    else
        syndromes_body<C, 1>(tile, flags, data, stride, nsym, ncw, neras, result, syn_ws);
}

template <class C, int R>
__device__ __forceinline__ void publish(const uint32_t (&S)[16][8], uint32_t *qin, int lane) {
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i) {
        qin[lane * 65 + 2 * (C::S0[R] + i)] = pack4(S[i][0], S[i][1], S[i][2], S[i][3]);
        qin[lane * 65 + 2 * (C::S0[R] + i) + 1] = pack4(S[i][4], S[i][5], S[i][6], S[i][7]);
    }
}

template <class C, int R>
__device__ __forceinline__ void parity_store(uint32_t (&S)[16][8], const uint32_t *qin, int lane,
                                             uint8_t *parity, size_t pstride, size_t cw,
                                             size_t ncw) {
    C::template parity_map<R>(S, qin, lane);
#pragma unroll
    for (int j = 0; j < C::NS[R]; ++j) transpose8(S[j]);  // S[j][c] >> 24: parity j of codeword c
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (cw + 64 * c >= ncw) continue;
        uint8_t *dst = parity + (cw + 64 * c) * pstride + C::S0[R];
#pragma unroll
        for (int j = 0; j < C::NS[R]; j += 4) {
            if (j + 4 <= C::NS[R]) {
                const uint32_t w = pack4(S[j][c], S[j + 1][c], S[j + 2][c], S[j + 3][c]);
                __builtin_memcpy(dst + j, &w, 4);
            } else {
#pragma unroll
                for (int e = j; e < C::NS[R]; ++e) dst[e] = (uint8_t)(S[e][c] >> 24);
            }
        }
    }
}

template <class C, int R>
__device__ __forceinline__ void encode_body(uint32_t *tile, const uint8_t *data, size_t stride,
                                            unsigned len, uint8_t *parity, size_t pstride,
                                            size_t ncw) {
    const int lane = threadIdx.x & 63;
    const size_t cw0 = (size_t)blockIdx.x * kTile;
    const int nchunks = (int)((len + 63) / 64);
    const int pad = nchunks * 64 - (int)len;
    uint32_t S[16][8];
    syndromes_tile<C, R>(S, tile, data, stride, cw0, ncw, nchunks, pad);
    // Both roles publish their syndromes (byte lane 3, 4 bit-planes per dword) for Q.
    uint32_t *qin = tile;                           // [64 lanes][65 dwords]
    publish<C, R>(S, qin, lane);
    __syncthreads();
    parity_store<C, R>(S, qin, lane, parity, pstride, cw0 + lane, ncw);
}

template <class C>
__global__ void __launch_bounds__(kThreads, 2)
    k_bs_encode(const uint8_t *data, size_t stride, unsigned len, uint8_t *parity,
                size_t pstride, size_t ncw) {
    __shared__ uint32_t tile[kTile * kPitch];
    if (threadIdx.x < 64) encode_body<C, 0>(tile, data, stride, len, parity, pstride, ncw);
    else encode_body<C, 1>(tile, data, stride, len, parity, pstride, ncw);
}

} // namespace bs

// ------------------------------------------------------------------------------------------------
namespace {

template <class C> bool matches(const DevCodec &d) {
    return d.mm == 8 && d.nroots == C::NR && d.fcr == C::FCR && d.prim == C::PRIM &&
           (d.dual != 0) == C::DUAL && d.poly == C::POLY;
}

} // namespace

int bitslice_codec_id(const DevCodec &d) {
    int id = 0, found = -1;
#define EZRS_BS_MATCH(C) \
    if (found < 0 && matches<bs::C>(d)) found = id; \
    ++id;
    EZRS_BS_CODEC_LIST(EZRS_BS_MATCH)
#undef EZRS_BS_MATCH
    return found;
}

hipError_t launch_bs_encode(int id, const EncodeArgs &a, hipStream_t s) {
    const unsigned grid = (unsigned)((a.ncw + bs::kTile - 1) / bs::kTile);
    int k = 0;
#define EZRS_BS_ENC(C)                                                                            \
    if (k++ == id) {                                                                              \
        hipLaunchKernelGGL(bs::k_bs_encode<bs::C>, dim3(grid), dim3(bs::kThreads), 0, s,          \
                           static_cast<const uint8_t *>(a.data), a.data_stride, a.len,            \
                           static_cast<uint8_t *>(a.parity), a.parity_stride, a.ncw);             \
        return hipGetLastError();                                                                 \
    }
    EZRS_BS_CODEC_LIST(EZRS_BS_ENC)
#undef EZRS_BS_ENC
    return hipErrorInvalidValue;
}

hipError_t launch_bs_syndromes(int id, const DevCodec &d, const DecodeArgs &a, uint8_t *syn_ws,
                               hipStream_t s) {
    const unsigned grid = (unsigned)((a.ncw + bs::kTile - 1) / bs::kTile);
    int k = 0;
#define EZRS_BS_SYN(C)                                                                            \
    if (k++ == id) {                                                                              \
        hipLaunchKernelGGL(bs::k_bs_syndromes<bs::C>, dim3(grid), dim3(bs::kThreads), 0, s,       \
                           static_cast<const uint8_t *>(a.data), a.data_stride,                   \
                           a.len + d.nroots, a.ncw, a.neras, a.result, syn_ws);                   \
        return hipGetLastError();                                                                 \
    }
    EZRS_BS_CODEC_LIST(EZRS_BS_SYN)
#undef EZRS_BS_SYN
    return hipErrorInvalidValue;
}

} // namespace ezrs
