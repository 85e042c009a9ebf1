// ezrs_bitslice.hip -- bit-sliced GF(2^8) RS encode / syndrome kernels for MI355X (gfx950).
//
// Why bit-slicing: RS(255,223) encode+decode is ~15 k GF(2^8) multiply-accumulates per codeword.
// One LDS log/antilog lookup per MAC caps a table kernel near 5 % of the 8 TB/s HBM roofline.
// Here a 32-bit VGPR holds one bit of 32 symbol slots, so a constant GF multiply is an XOR
// network; each network is split into nibble groups (all 15 XOR combinations of an input nibble
// are formed once) and every output bit costs one v_bitop3_b32 (3-input XOR) per input byte.
//
// Work decomposition (one 256-thread workgroup = 4 waves = one 512-codeword tile):
//   * lane l owns the 8 consecutive codewords at tile rows 8l + c, c = 0..7; its 32 register
//     slots are (c, segment s), s = position mod 4, at bit 8s + c.  Segment interleaving keeps
//     every step's input a natural little-endian dword of 4 consecutive symbols of one codeword.
//   * wave r ("role") owns syndromes [S0[r], S0[r]+NS[r]): 8 syndromes x 8 bits = 64 state VGPRs,
//     so two workgroups (8 waves) share a CU.
//   * the tile streams through LDS in chunks of 128 positions: lane l's 8 rows x 128 bytes form
//     block l (pitch 1028 B; the pad dword makes a column read by 32 lanes hit 32 distinct banks).
//     A block is exactly one LDS-DMA instruction (global_load_lds_dwordx4, 64 lanes x 16 B at
//     per-lane unaligned row addresses): 128 contiguous bytes per row and request is what lets
//     the row-strided stream run near HBM speed (tools/micro/dma_patterns.hip).  The other
//     workgroup on the CU computes while this one waits for its chunk.
//   * each chunk is bit-transposed once, in place (role r: y-steps 8r..8r+7; 48 ops per 8 dwords),
//     then every role runs 2 Horner blocks of 16 y-steps in d = g^4 (state *= d^16, then straight-
//     line XOR networks over the bit-planes, generated from the codec: gen/ezrs_bs_tables.inc).
//   * the 4 segment partials are folded in-register (x g, << 8; x g^2, << 16), leaving the
//     syndromes of the lane's 8 codewords in byte lane 3.
//
// Decode (k_bs_syndromes): codewords whose syndromes are all zero (and carry no erasures) get
// result 0 -- exactly what decode_symbols returns (rs_base:1416-1434); all others get a sentinel
// and their syndromes go to the workspace for the error-path kernel (ezrs_generic.hip:
// k_decode_flagged), which runs the reference's BM/Chien/Forney on them.
// Encode: k_bs_encode_syn computes the syndromes of the data words into a workspace of bit-planes
// of 32-codeword groups; k_bs_parity maps them to parity with the GF(2) map Q (generated) on full
// 32-slot registers and stores each codeword's parity bytes.
#include "ezrs_internal.hpp"
#include "gen/ezrs_bs_tables.inc"

namespace ezrs {
namespace bs {

constexpr int kTile = 512;                 // codewords per workgroup
constexpr int kThreads = 256;
constexpr int kRoles = 4;
constexpr int kChunk = 128;                // positions per LDS chunk
constexpr int kBlockDw = 257;              // 8 rows x 32 dwords + 1 pad dword
constexpr int kBufDw = 64 * kBlockDw;      // one chunk (64 blocks); encode later reuses it for
                                           // the syndrome exchange (64 x 65 dwords) and the
                                           // parity image (512 rows x 32 bytes)
static_assert(kBufDw >= 64 * 65 + kTile * 8, "encode staging does not fit");
constexpr int32_t kSentinel = INT32_MIN;

typedef __attribute__((address_space(3))) void lds_void;

// LDS dword index of (lane, slot c, dword y of the chunk) is lane_base + 32 c + y.
__device__ __forceinline__ int lane_base(int lane) { return lane * kBlockDw; }
__device__ __forceinline__ int tile_row(int lane, int c) { return 8 * lane + c; }

struct Word {
    const uint8_t *base;   // row 0 of the batch
    size_t stride;         // bytes between rows
    size_t cw0, ncw;       // first row of the tile, rows in the batch
    int pad;               // leading zero positions (position = symbol index + pad)
};

// Issue this wave's 16 LDS-DMA pieces of chunk k: block b = 16*wave + i; lane j fetches row
// 8b + j/8, bytes [128k - pad + 16 (j&7), +16) of it.  Rows past the batch re-read the last row
// (discarded); pieces that would start before the batch are clamped (rebuilt by fixup_chunk0).
__device__ __forceinline__ void issue_chunk(uint32_t *buf, const Word &w, int k) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int b = 16 * wave + i;
        size_t cw = w.cw0 + 8 * b + (lane >> 3);
        if (cw >= w.ncw) cw = w.ncw - 1;
        long off = (long)(cw * w.stride) + (long)kChunk * k - w.pad + 16 * (lane & 7);
        if (off < 0) off = 0;
        __builtin_amdgcn_global_load_lds(static_cast<const void *>(w.base + off),
                                         (lds_void *)(buf + b * kBlockDw), 16, 0, 0);
    }
}

// Chunk 0 holds the `pad` leading zero positions: zero them, and rebuild the rows whose DMA piece
// was clamped at the start of the batch.
__device__ __forceinline__ void fixup_chunk0(uint32_t *buf, const Word &w) {
    for (int row = threadIdx.x; row < kTile; row += kThreads) {
        uint32_t *r = buf + (row >> 3) * kBlockDw + (row & 7) * 32;
        const size_t cw = w.cw0 + row;
        const int nd = (w.pad + 3) >> 2;                  // dwords touched by the pad
        if (cw < w.ncw && (long)(cw * w.stride) < w.pad) {
            const uint8_t *p = w.base + cw * w.stride;
            for (int d = 0; d < 32; ++d) {
                uint32_t v = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int u = 4 * d + e - w.pad;
                    if (u >= 0) v |= (uint32_t)p[u] << (8 * e);
                }
                r[d] = v;
            }
        } else {
            for (int d = 0; d < nd; ++d) {
                const int lo = 4 * d - w.pad;              // symbol index of byte 0 of dword d
                if (lo + 4 <= 0) r[d] = 0;
                else r[d] &= 0xFFFFFFFFu << (8 * (-lo));
            }
        }
    }
}

// In-place bit transposition of this role's 8 y-steps of the chunk: raw dwords (one per row)
// become bit-planes (plane b of slot (c, s) = bit b of row c's symbol 4y + s).
template <int R>
__device__ __forceinline__ void transpose_chunk(uint32_t *buf, int lb) {
#pragma unroll 2
    for (int t = 0; t < 8; ++t) {
        uint32_t *p = buf + lb + 8 * R + t;
        uint32_t D[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) D[c] = p[32 * c];
        transpose8(D);
#pragma unroll
        for (int b = 0; b < 8; ++b) p[32 * b] = D[b];
    }
}

// Syndromes (in byte lane 3 after the fold) of the tile's words.  Each role runs its own copy of
// the loop (R is a template parameter): with a per-chunk role branch the compiler hoists the
// common LDS plane loads of all y-steps above the branch and spills.
template <class C, int R>
__device__ __forceinline__ void syndromes_tile(uint32_t (&S)[16][8], uint32_t *buf,
                                               const Word &w, int nchunks) {
    const int lb = lane_base(threadIdx.x & 63);
    // Leading halves of 8 y-steps (32 positions) that hold only pad: Horner over zeros from a
    // zero state is a no-op, so they are not computed (a shortened word, or encode's 223 symbols
    // in 2 x 128 positions, skip them).
    const int skip = w.pad >> 5;
    bool started = false;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) S[i][q] = 0;
    for (int k = 0; k < nchunks; ++k) {
#ifndef EZRS_BS_ABLATE_DMA   // timing-only builds (tools/micro/bs_ablate): drop the HBM stream
        issue_chunk(buf, w, k);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        __syncthreads();
        if (k == 0 && w.pad) {
            fixup_chunk0(buf, w);
            __syncthreads();
        }
#ifndef EZRS_BS_ABLATE_TRANSPOSE  // timing-only builds: drop the bit transposition
        transpose_chunk<R>(buf, lb);
#endif
        __syncthreads();
#ifndef EZRS_BS_ABLATE_COMPUTE  // timing-only builds: drop the XOR networks
#pragma unroll 1   // one copy of each role's network: the 4 roles' code must share the I-cache
        for (int blk = 0; blk < 2; ++blk) {
            const int h0 = 4 * k + 2 * blk;          // global index of the block's first half
            if (h0 + 1 < skip) continue;
            if (started) C::template block_mul<R>(S);
            const uint32_t *p = buf + lb + 16 * blk;
            if (h0 >= skip) C::template horner_half<R, 0>(S, p);
            C::template horner_half<R, 1>(S, p + 8);
            started = true;
        }
#else
        S[0][0] ^= buf[lb];
#endif
        __syncthreads();   // the next chunk overwrites the buffer
    }
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
    uint32_t fl = flags[0][lane] | flags[1][lane] | flags[2][lane] | flags[3][lane];
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
    __shared__ __attribute__((aligned(16))) uint32_t lds[kBufDw];
    __shared__ uint32_t flags[kRoles][64];
    const int nchunks = (int)((nsym + kChunk - 1) / kChunk);
    const Word w{data, stride, (size_t)blockIdx.x * kTile, ncw, nchunks * kChunk - (int)nsym};
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: syndromes_body<C, 0>(lds, flags, w, nchunks, neras, result, syn_ws); break;
    case 1: syndromes_body<C, 1>(lds, flags, w, nchunks, neras, result, syn_ws); break;
    case 2: syndromes_body<C, 2>(lds, flags, w, nchunks, neras, result, syn_ws); break;
    default: syndromes_body<C, 3>(lds, flags, w, nchunks, neras, result, syn_ws); break;
    }
}

// Encode, stage 1 (k_bs_encode_syn): syndromes of the data words, written to the workspace as
// bit-planes of 32-codeword groups: dword ((G/64) * 8NR + 8i + q) * 64 + G%64 holds bit q of
// S_i for codewords 32G .. 32G+31 (bit s <-> codeword 32G + s).  Lane l's byte lane 3 holds
// codewords 8l .. 8l+7, i.e. byte l&3 of group l>>2's planes: gathered through LDS.
template <class C, int R>
__device__ __forceinline__ void encode_syn_body(uint32_t *lds, const Word &w, int nchunks,
                                                uint32_t *ws) {
    const int lane = threadIdx.x & 63;
    uint32_t S[16][8];
    syndromes_tile<C, R>(S, lds, w, nchunks);
    constexpr int NPL = 8 * C::NR;
    uint8_t *stage = reinterpret_cast<uint8_t *>(lds);     // [NPL planes][16 groups] dwords
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            stage[(((C::S0[R] + i) * 8 + q) * 16 + (lane >> 2)) * 4 + (lane & 3)] =
                (uint8_t)(S[i][q] >> 24);
    __syncthreads();
    const size_t tile = w.cw0 / kTile;
    uint32_t *dst = ws + (tile >> 2) * NPL * 64 + (tile & 3) * 16;
    for (int idx = threadIdx.x; idx < NPL * 16; idx += kThreads)
        dst[(idx >> 4) * 64 + (idx & 15)] = lds[idx];
}

template <class C>
__global__ void __launch_bounds__(kThreads, 2)
    k_bs_encode_syn(const uint8_t *data, size_t stride, unsigned len, size_t ncw, uint32_t *ws) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kBufDw];
    const int nchunks = (int)((len + kChunk - 1) / kChunk);
    const Word w{data, stride, (size_t)blockIdx.x * kTile, ncw, nchunks * kChunk - (int)len};
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: encode_syn_body<C, 0>(lds, w, nchunks, ws); break;
    case 1: encode_syn_body<C, 1>(lds, w, nchunks, ws); break;
    case 2: encode_syn_body<C, 2>(lds, w, nchunks, ws); break;
    default: encode_syn_body<C, 3>(lds, w, nchunks, ws); break;
    }
}

// Bytes s of a[0..3] -> one dword (a[0] in byte 0).
__device__ __forceinline__ uint32_t gather4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                            int s) {
    const uint32_t sel = (uint32_t)s | ((uint32_t)(s + 4) << 8) | 0x0c0c0000u;  // 0x0c: zero byte
    const uint32_t x01 = __builtin_amdgcn_perm(a1, a0, sel), x23 = __builtin_amdgcn_perm(a3, a2, sel);
    return __builtin_amdgcn_perm(x23, x01, 0x05040100u);
}

template <class C, int P>
__device__ __forceinline__ void parity_pass(const uint32_t *ws, size_t G, uint8_t *parity,
                                            size_t pstride, size_t ncw) {
    constexpr int NPL = 8 * C::NR;
    constexpr int NJ = C::NR - 8 * P < 8 ? C::NR - 8 * P : 8;
    uint32_t O[8][8];
    C::template q_pass<P>(O, ws + (G >> 6) * NPL * 64 + (G & 63), 64);
#pragma unroll
    for (int j = 0; j < NJ; ++j) transpose8(O[j]);   // O[j][c] byte s: symbol 8P+j of cw 32G+8s+c
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const size_t k = 32 * G + 8 * s + c;
            if (k >= ncw) continue;
            uint8_t *dst = parity + k * pstride + 8 * P;
            if (NJ == 8) {
                const uint32_t v[2] = {gather4(O[0][c], O[1][c], O[2][c], O[3][c], s),
                                       gather4(O[4][c], O[5][c], O[6][c], O[7][c], s)};
                __builtin_memcpy(dst, v, 8);
            } else if (NJ == 4) {
                const uint32_t v = gather4(O[0][c], O[1][c], O[2][c], O[3][c], s);
                __builtin_memcpy(dst, &v, 4);
            } else {
#pragma unroll
                for (int j = 0; j < NJ; ++j) dst[j] = (uint8_t)(O[j][c] >> (8 * s));
            }
        }
    }
}

// Encode, stage 2: parity = Q(syndromes) over full 32-codeword registers, one pass of 8 parity
// symbols per workgroup row (blockIdx.y), 64 groups per wave.
template <class C>
__global__ void __launch_bounds__(256)
    k_bs_parity(const uint32_t *ws, uint8_t *parity, size_t pstride, size_t ncw) {
    const size_t G = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + (threadIdx.x & 63);
    if (32 * G >= ncw) return;
    switch (blockIdx.y) {
    case 0: parity_pass<C, 0>(ws, G, parity, pstride, ncw); break;
    case 1: if constexpr (C::NPASS > 1) parity_pass<C, 1>(ws, G, parity, pstride, ncw); break;
    case 2: if constexpr (C::NPASS > 2) parity_pass<C, 2>(ws, G, parity, pstride, ncw); break;
    default: if constexpr (C::NPASS > 3) parity_pass<C, 3>(ws, G, parity, pstride, ncw); break;
    }
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

size_t bs_encode_ws_bytes(size_t ncw) { return (ncw + 2047) / 2048 * 2048 * 32; }

hipError_t launch_bs_encode(int id, const EncodeArgs &a, void *ws, hipStream_t s) {
    const unsigned grid = (unsigned)((a.ncw + bs::kTile - 1) / bs::kTile);
    const unsigned pgrid = (unsigned)((a.ncw + 8191) / 8192);   // 256 groups of 32 per block
    uint32_t *w = static_cast<uint32_t *>(ws);
    int k = 0;
#define EZRS_BS_ENC(C)                                                                            \
    if (k++ == id) {                                                                              \
        hipLaunchKernelGGL(bs::k_bs_encode_syn<bs::C>, dim3(grid), dim3(bs::kThreads), 0, s,      \
                           static_cast<const uint8_t *>(a.data), a.data_stride, a.len, a.ncw, w); \
        hipLaunchKernelGGL(bs::k_bs_parity<bs::C>, dim3(pgrid, bs::C::NPASS), dim3(256), 0, s,    \
                           w, static_cast<uint8_t *>(a.parity), a.parity_stride, a.ncw);          \
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
