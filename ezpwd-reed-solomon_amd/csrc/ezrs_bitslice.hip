// ezrs_bitslice.hip -- bit-sliced GF(2^8) RS encode / syndrome kernels for MI355X (gfx950).
//
// Why bit-slicing: RS(255,223) encode+decode is ~15 k GF(2^8) multiply-accumulates per codeword.
// One LDS log/antilog lookup per MAC caps a table kernel near 5 % of the 8 TB/s HBM roofline.
// Here a 32-bit VGPR holds one bit of 32 symbol slots, so a constant GF multiply is an XOR
// network; each network is split into nibble groups (all 15 XOR combinations of an input nibble
// are formed once) and every output bit costs one v_bitop3_b32 (3-input XOR) per input byte.
//
// Work decomposition (one 128-thread workgroup = 2 waves = one 512-codeword tile):
//   * lane l owns the 8 codewords at tile rows 32*(l>>2) + (l&3) + 4c, c = 0..7; its 32 register
//     slots are (c, segment s), s = position mod 4, at bit 8s + c.  Segment interleaving keeps
//     every step's input a natural little-endian dword of 4 consecutive symbols of one codeword.
//   * wave r ("role") owns syndromes [S0[r], S0[r]+NS[r]): 16 syndromes x 8 bits = 128 state VGPRs.
//   * the tile streams through LDS in chunks of 32 positions: 16 blocks of 32 rows x 32 bytes,
//     block pitch 1028 B (one pad dword: a column read by 32 lanes hits 32 distinct banks).  Chunks
//     arrive by LDS-DMA (global_load_lds_dwordx4, per-lane unaligned row addresses) into two
//     buffers, so chunk k+1 streams in while chunk k is computed.
//   * per chunk and role: state *= d^8, then 8 Horner y-steps (d = g^4); each y-step reads the 8
//     raw dwords of its slots from LDS (the next step's are in flight meanwhile) and bit-transposes
//     them in registers (3-stage delta swap, 48 ops) -- straight-line XOR networks generated from
//     the codec (gen/ezrs_bs_tables.inc).
//   * the 4 segment partials are folded in-register (x g, << 8; x g^2, << 16), leaving the
//     syndromes of the lane's 8 codewords in byte lane 3.
//
// Decode (k_bs_syndromes): codewords whose syndromes are all zero (and carry no erasures) get
// result 0 -- exactly what decode_symbols returns (rs_base:1416-1434); all others get a sentinel
// and their syndromes go to the workspace for the error-path kernel (ezrs_generic.hip:
// k_decode_flagged), which runs the reference's BM/Chien/Forney on them.
// Encode (k_bs_encode): syndromes of the data word -> parity via the GF(2) map Q (generated),
// staged through LDS and stored as whole parity rows.
#include "ezrs_internal.hpp"
#include "gen/ezrs_bs_tables.inc"

namespace ezrs {
namespace bs {

constexpr int kTile = 512;                 // codewords per workgroup
constexpr int kThreads = 128;
constexpr int kChunk = 32;                 // positions per LDS chunk
constexpr int kBlockDw = 257;              // 32 rows x 8 dwords + 1 pad dword
constexpr int kBufDw = 16 * kBlockDw;      // one chunk buffer (16 blocks)
// Two chunk buffers; encode later reuses the space for the syndrome exchange (64 x 65 dwords) and
// the parity image (512 rows x 32 bytes).
constexpr int kLdsDw = 2 * kBufDw > 64 * 65 + kTile * 8 ? 2 * kBufDw : 64 * 65 + kTile * 8;
constexpr int32_t kSentinel = INT32_MIN;

typedef __attribute__((address_space(3))) void lds_void;

// LDS dword index of (lane, slot c, dword y of the chunk) is lane_base + 32 c + y.
__device__ __forceinline__ int lane_base(int lane) { return (lane >> 2) * kBlockDw + (lane & 3) * 8; }
__device__ __forceinline__ int tile_row(int lane, int c) { return 32 * (lane >> 2) + (lane & 3) + 4 * c; }

struct Word {
    const uint8_t *base;   // row 0 of the batch
    size_t stride;         // bytes between rows
    size_t cw0, ncw;       // first row of the tile, rows in the batch
    int pad;               // leading zero positions (position = symbol index + pad)
};

// Issue this wave's 8 LDS-DMA pieces of chunk k: block b = 8*wave + i; lane j fetches row 32b + j/2,
// bytes [32k - pad + 16 (j&1), +16) of it.  Rows past the batch re-read the last row (discarded);
// pieces that would start before the batch are clamped (rebuilt by fixup_chunk0).
__device__ __forceinline__ void issue_chunk(uint32_t *buf, const Word &w, int k) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        const int b = 8 * wave + i;
        size_t cw = w.cw0 + 32 * b + (lane >> 1);
        if (cw >= w.ncw) cw = w.ncw - 1;
        long off = (long)(cw * w.stride) + (long)kChunk * k - w.pad + 16 * (lane & 1);
        if (off < 0) off = 0;
        __builtin_amdgcn_global_load_lds(static_cast<const void *>(w.base + off),
                                         (lds_void *)(buf + b * kBlockDw), 16, 0, 0);
    }
}

// Chunk 0 holds the `pad` leading zero positions: zero them, and rebuild the rows whose DMA piece
// was clamped at the start of the batch.
__device__ __forceinline__ void fixup_chunk0(uint32_t *buf, const Word &w) {
    for (int row = threadIdx.x; row < kTile; row += kThreads) {
        uint32_t *r = buf + (row >> 5) * kBlockDw + (row & 31) * 8;
        const size_t cw = w.cw0 + row;
        if (cw < w.ncw && (long)(cw * w.stride) < w.pad) {
            const uint8_t *p = w.base + cw * w.stride;
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                uint32_t v = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int u = 4 * d + e - w.pad;
                    if (u >= 0) v |= (uint32_t)p[u] << (8 * e);
                }
                r[d] = v;
            }
        } else {
#pragma unroll
            for (int d = 0; d < 8; ++d) {
                const int lo = 4 * d - w.pad;              // symbol index of byte 0 of dword d
                if (lo + 4 <= 0) r[d] = 0;
                else if (lo < 0) r[d] &= 0xFFFFFFFFu << (8 * (-lo));
            }
        }
    }
}

// Syndromes (in byte lane 3 after the fold) of the tile's words.  Each role runs its own copy of
// the loop (R is a template parameter): with a per-chunk role branch the compiler hoists the
// common LDS plane loads of all y-steps above the branch and spills.
template <class C, int R>
__device__ __forceinline__ void syndromes_tile(uint32_t (&S)[16][8], uint32_t *lds,
                                               const Word &w, int nchunks) {
    const int lb = lane_base(threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) S[i][q] = 0;
#ifndef EZRS_BS_ABLATE_DMA
    issue_chunk(lds, w, 0);
#endif
    for (int k = 0; k < nchunks; ++k) {
        uint32_t *buf = lds + (k & 1) * kBufDw;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (k == 0 && w.pad) {
            fixup_chunk0(buf, w);
            __syncthreads();
        }
#ifndef EZRS_BS_ABLATE_DMA   // timing-only builds (tools/micro/bs_ablate): drop the HBM stream
        if (k + 1 < nchunks) issue_chunk(lds + ((k + 1) & 1) * kBufDw, w, k + 1);
#endif
#ifndef EZRS_BS_ABLATE_COMPUTE  // timing-only builds: drop the XOR networks
        C::template horner_chunk<R>(S, buf, lb, k == 0);
#else
        S[0][0] ^= buf[lb];
#endif
    }
    __syncthreads();
    C::template fold<R>(S);
}

// Byte lane 3 of four registers -> one dword (register a in byte 0).
__device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (a >> 24) | ((b >> 16) & 0xFF00u) | ((c >> 8) & 0xFF0000u) | (d & 0xFF000000u);
}

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
__device__ __forceinline__ void write_syndromes(uint32_t (&S)[16][8], uint32_t fl, size_t cw0,
                                                int lane, uint8_t *syn_ws) {
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i) transpose8(S[i]);   // S[i][c] >> 24: codeword c's S_i
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (!(fl >> c & 1)) continue;
        uint8_t *dst = syn_ws + (cw0 + tile_row(lane, c)) * 32 + C::S0[R];
#pragma unroll
        for (int i = 0; i < C::NS[R]; i += 4) {
            if (i + 4 <= C::NS[R]) {
                const uint32_t v = pack4(S[i][c], S[i + 1][c], S[i + 2][c], S[i + 3][c]);
                __builtin_memcpy(dst + i, &v, 4);
            } else {
#pragma unroll
                for (int e = i; e < C::NS[R]; ++e) dst[e] = (uint8_t)(S[e][c] >> 24);
            }
        }
    }
}

template <class C, int R>
__device__ __forceinline__ void syndromes_body(uint32_t *lds, uint32_t (*flags)[64],
                                               const Word &w, int nchunks,
                                               const uint32_t *neras, int32_t *result,
                                               uint8_t *syn_ws) {
    const int lane = threadIdx.x & 63;
    uint32_t S[16][8];
    syndromes_tile<C, R>(S, lds, w, nchunks);
    flags[R][lane] = nonzero_mask<C, R>(S);
    __syncthreads();
    uint32_t fl = flags[0][lane] | flags[1][lane];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const size_t cw = w.cw0 + tile_row(lane, c);
        if (cw >= w.ncw) { fl &= ~(1u << c); continue; }
        if (neras && neras[cw]) fl |= 1u << c;      // erasures: the error path validates them
        if (R == 0) result[cw] = (fl >> c & 1) ? kSentinel : 0;
    }
    if (fl) write_syndromes<C, R>(S, fl, w.cw0, lane, syn_ws);
}

template <class C>
__global__ void __launch_bounds__(kThreads, 2)
    k_bs_syndromes(const uint8_t *data, size_t stride, unsigned nsym, size_t ncw,
                   const uint32_t *neras, int32_t *result, uint8_t *syn_ws) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDw];
    __shared__ uint32_t flags[2][64];
    const int nchunks = (int)((nsym + kChunk - 1) / kChunk);
    const Word w{data, stride, (size_t)blockIdx.x * kTile, ncw, nchunks * kChunk - (int)nsym};
    if (threadIdx.x < 64) syndromes_body<C, 0>(lds, flags, w, nchunks, neras, result, syn_ws);
    else syndromes_body<C, 1>(lds, flags, w, nchunks, neras, result, syn_ws);
}

template <class C, int R>
__device__ __forceinline__ void publish(const uint32_t (&S)[16][8], uint32_t *qin, int lane) {
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i) {
        qin[lane * 65 + 2 * (C::S0[R] + i)] = pack4(S[i][0], S[i][1], S[i][2], S[i][3]);
        qin[lane * 65 + 2 * (C::S0[R] + i) + 1] = pack4(S[i][4], S[i][5], S[i][6], S[i][7]);
    }
}

// Q map, then this role's parity bytes of the lane's 8 codewords into the LDS parity image
// [512 rows][NR bytes, padded to a dword multiple].
template <class C, int R>
__device__ __forceinline__ void parity_stage(uint32_t (&S)[16][8], const uint32_t *qin, int lane,
                                             uint8_t *pimg, int ppitch) {
    C::template parity_map<R>(S, qin, lane);
#pragma unroll
    for (int j = 0; j < C::NS[R]; ++j) transpose8(S[j]);  // S[j][c] >> 24: parity j of codeword c
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        uint8_t *dst = pimg + tile_row(lane, c) * ppitch + C::S0[R];
#pragma unroll
        for (int j = 0; j < C::NS[R]; j += 4) {
            if (j + 4 <= C::NS[R] && ((C::S0[R] + j) & 3) == 0) {
                *reinterpret_cast<uint32_t *>(dst + j) =
                    pack4(S[j][c], S[j + 1][c], S[j + 2][c], S[j + 3][c]);
            } else {
#pragma unroll
                for (int e = j; e < j + 4 && e < C::NS[R]; ++e) dst[e] = (uint8_t)(S[e][c] >> 24);
            }
        }
    }
}

template <class C, int R>
__device__ __forceinline__ void encode_body(uint32_t *lds, const Word &w, int nchunks,
                                            uint8_t *parity, size_t pstride) {
    const int lane = threadIdx.x & 63;
    uint32_t S[16][8];
    syndromes_tile<C, R>(S, lds, w, nchunks);
    // Both roles publish their syndromes (byte lane 3, 4 bit-planes per dword) for Q.
    uint32_t *qin = lds;                            // [64 lanes][65 dwords]
    publish<C, R>(S, qin, lane);
    __syncthreads();
    constexpr int ppitch = (C::NR + 3) & ~3;
    uint8_t *pimg = reinterpret_cast<uint8_t *>(lds + 64 * 65);
    parity_stage<C, R>(S, qin, lane, pimg, ppitch);
    __syncthreads();
    // Whole parity rows out: 16-byte pieces, consecutive threads on consecutive pieces of a row.
    constexpr int per_row = (C::NR + 15) / 16;
    for (int pi = threadIdx.x; pi < kTile * per_row; pi += kThreads) {
        const int row = pi / per_row, h = pi % per_row;
        const size_t cw = w.cw0 + row;
        if (cw >= w.ncw) continue;
        const int n = C::NR - 16 * h < 16 ? C::NR - 16 * h : 16;
        uint8_t *dst = parity + cw * pstride + 16 * h;
        const uint8_t *src = pimg + row * ppitch + 16 * h;
        if (n == 16) {
            uint32_t v[4];
            __builtin_memcpy(v, src, 16);
            __builtin_memcpy(dst, v, 16);
        } else {
            for (int e = 0; e < n; ++e) dst[e] = src[e];
        }
    }
}

template <class C>
__global__ void __launch_bounds__(kThreads, 2)
    k_bs_encode(const uint8_t *data, size_t stride, unsigned len, uint8_t *parity,
                size_t pstride, size_t ncw) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDw];
    const int nchunks = (int)((len + kChunk - 1) / kChunk);
    const Word w{data, stride, (size_t)blockIdx.x * kTile, ncw, nchunks * kChunk - (int)len};
    if (threadIdx.x < 64) encode_body<C, 0>(lds, w, nchunks, parity, pstride);
    else encode_body<C, 1>(lds, w, nchunks, parity, pstride);
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
