// ezrs_bitslice.hip -- bit-sliced GF(2^8) RS encode / syndrome kernels for MI355X (gfx950).
//
// Why bit-slicing: RS(255,223) encode+decode is ~15 k GF(2^8) multiply-accumulates per codeword.
// One LDS log/antilog lookup per MAC caps a table kernel near 5 % of the 8 TB/s HBM roofline.
// Here a 32-bit VGPR holds one bit of 32 symbol slots, so a constant GF multiply is an XOR
// network; each network is split into nibble groups (all 15 XOR combinations of an input nibble
// are formed once) and every output bit costs one v_bitop3_b32 (3-input XOR) per input byte.
//
// Work decomposition (one 256-thread workgroup = 4 waves = one 256-codeword tile; 4 workgroups
// share a CU, so the others compute while one waits for its chunk or sits in a barrier):
//   * lane l owns the 4 consecutive codewords at tile rows 4l + c, c = 0..3; its 32 register
//     slots are (c, segment sigma), sigma = position mod 8: slot bit 8s + k holds codeword k & 3,
//     segment 4 (k >> 2) + s.  Every y-step's input is two natural little-endian dwords (8
//     consecutive symbols) of each of the lane's 4 codewords.
//   * wave r ("role") owns syndromes [S0[r], S0[r]+NS[r]): 8 syndromes x 8 bits = 64 state VGPRs.
//   * the tile streams through LDS in chunks of 128 positions: region m (one LDS-DMA instruction,
//     global_load_lds_dwordx4, 64 lanes x 16 B at per-lane row addresses; pitch 1028 B) holds the
//     128-byte row pieces of lanes m and m + 32.  128 contiguous bytes per row and request is what
//     lets the row-strided stream run fast (tools/micro/dma_patterns.hip: 128-B pieces 4.5 TB/s
//     latency-bound, 64-B pieces 2.6); a ds_read_b32 half-wave (lanes 0-31 or 32-63) touches each
//     region once, at bank (m + y) mod 32: conflict-free.
//   * each chunk is bit-transposed once, in place (role r: y-steps 4r..4r+3; 48 ops per 8 dwords),
//     then every role runs one Horner block of 16 y-steps in d = g^8 (state *= d^16, then
//     straight-line XOR networks over the bit-planes, generated from the codec:
//     gen/ezrs_bs_tables.inc).
//   * the 8 segment partials are folded in-register (x g^4, << 4; x g, << 8; x g^2, << 16),
//     leaving the syndromes of the lane's 4 codewords at bits 28..31.
//
// Decode (k_bs_syndromes): codewords whose syndromes are all zero (and carry no erasures) get
// result 0 -- exactly what decode_symbols returns (rs_base:1416-1434); all others get a sentinel
// and their syndromes go to the workspace for the error-path kernel (ezrs_errors.hip:
// k_decode_errors), which runs the reference's BM/Chien/Forney on them.
// Encode: k_bs_encode_syn computes the syndromes of the data words into a workspace of bit-planes
// of 32-codeword groups; k_bs_parity maps them to parity with the GF(2) map Q (generated) on full
// 32-slot registers and stores each codeword's parity bytes.
#include "ezrs_internal.hpp"
#include "gen/ezrs_bs_tables.inc"

namespace ezrs {
namespace bs {

constexpr int kTile = 256;                 // codewords per workgroup
constexpr int kThreads = 256;
constexpr int kRoles = 4;
constexpr int kChunk = 128;                // positions per LDS chunk (= one 16-y-step block)
constexpr int kRegionDw = 257;             // one LDS-DMA region: 8 rows x 32 dwords + 1 pad dword
constexpr int kBufDw = 32 * kRegionDw;     // one chunk of the tile
static_assert(kBufDw >= 8 * 32 * (kTile / 32), "encode staging does not fit");
constexpr int32_t kSentinel = INT32_MIN;

typedef __attribute__((address_space(3))) void lds_void;

// Region m holds rows i = 2c + e (c = 0..3, e = 0..1) = row c of lane m + 32 e, 32 dwords each.
// Lane l's row c dword t is at lane_base(l) + 64 c + t; after the in-place transposition the
// dwords 2y, 2y+1 of its 4 rows hold bit-planes b = (row b & 3, dword 2y + (b >> 2)) of y-step y.
__device__ __forceinline__ int lane_base(int lane) { return (lane & 31) * kRegionDw + 32 * (lane >> 5); }
__device__ __forceinline__ int tile_row(int lane, int c) { return 4 * lane + c; }

template <int I, int N, class F> __device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

struct Word {
    const uint8_t *base;   // row 0 of the batch
    size_t stride;         // bytes between rows
    size_t cw0, ncw;       // first row of the tile, rows in the batch
    int pad;               // leading zero positions (position = symbol index + pad)
};

// Issue this wave's 8 LDS-DMA pieces of chunk k: region m = 8 wave + i; lane j fetches bytes
// [128k - pad + 16 (j&7), +16) of region row j >> 3 = 2c + e, i.e. tile row 4 (m + 32 e) + c.
// Rows past the batch re-read the last row (discarded); pieces that would start before the batch
// are clamped (rebuilt by fixup_chunk0).
__device__ __forceinline__ void issue_chunk(uint32_t *buf, const Word &w, int k) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int ri = lane >> 3;                       // region row 2c + e
    const int rsub = 128 * (ri & 1) + (ri >> 1);    // tile row - 4 m
    const long col = (long)kChunk * k - w.pad + 16 * (lane & 7);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = 8 * wave + i;
        size_t cw = w.cw0 + 4 * m + rsub;
        if (cw >= w.ncw) cw = w.ncw - 1;
        long off = (long)(cw * w.stride) + col;
        if (off < 0) off = 0;
        __builtin_amdgcn_global_load_lds(static_cast<const void *>(w.base + off),
                                         (lds_void *)(buf + m * kRegionDw), 16, 0, 0);
    }
}

// Chunk 0 holds the `pad` leading zero positions: zero them, and rebuild the rows whose DMA piece
// was clamped at the start of the batch.
__device__ __forceinline__ void fixup_chunk0(uint32_t *buf, const Word &w) {
    for (int row = threadIdx.x; row < kTile; row += kThreads) {
        uint32_t *r = buf + lane_base(row >> 2) + 64 * (row & 3);
        const size_t cw = w.cw0 + row;
        const int nd = (w.pad + 3) >> 2;                  // dwords touched by the pad
        if (cw < w.ncw && (long)(cw * w.stride) < w.pad) {
            const uint8_t *p = w.base + cw * w.stride;
            for (int d = 0; d < kChunk / 4; ++d) {
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

// In-place bit transposition of this role's 4 y-steps of the chunk: the 8 raw dwords of a y-step
// (D[k] = dword 2y + (k >> 2) of row k & 3) become its 8 bit-planes, plane b where D[b] was.
template <int R>
__device__ __forceinline__ void transpose_chunk(uint32_t *buf, int lb) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t *p = buf + lb + 2 * (4 * R + t);
        uint32_t D[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) D[k] = p[64 * (k & 3) + (k >> 2)];
        transpose8(D);
#pragma unroll
        for (int k = 0; k < 8; ++k) p[64 * (k & 3) + (k >> 2)] = D[k];
    }
}

// Syndromes (at bits 28..31 after the fold) of the tile's words.  Each role runs its own copy of
// the loop (R is a template parameter): with a per-chunk role branch the compiler hoists the
// common LDS plane loads of all y-steps above the branch and spills.
template <class C, int R>
__device__ __forceinline__ void syndromes_tile(uint32_t (&S)[16][8], uint32_t *buf,
                                               const Word &w, int nchunks) {
    const int lb = lane_base(threadIdx.x & 63);
    // Leading pad positions are zeroed data: Horner over zeros from a zero state is a no-op.  Whole
    // pad chunks (a heavily shortened word) are not evaluated.
    const int skip = w.pad / kChunk;
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
        if (k >= skip) {
            if (k > skip) static_for<0, C::NS[R]>([&](auto i) { C::template mul<R, i>(S[i]); });
            C::template horner_block<R>(S, buf + lb);
        }
#else
        S[0][0] ^= buf[lb];
#endif
        __syncthreads();   // the next chunk overwrites the buffer
    }
    static_for<0, C::NS[R]>([&](auto i) { C::template fold<R, i>(S[i]); });
}

template <class C, int R>
__device__ __forceinline__ uint32_t nonzero_mask(const uint32_t (&S)[16][8]) {
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) nz |= S[i][q];
    return nz >> 28;                             // bit c: codeword c has a nonzero syndrome
}

// Write the role's syndromes of the flagged codewords (bits of fl) to their workspace slots, one
// syndrome at a time (after transpose8, S[i][4+c] >> 24 is codeword c's S_i).
template <class C, int R>
__device__ __forceinline__ void write_syndromes(uint32_t (&S)[16][8], uint32_t fl, size_t cw0,
                                                int lane, uint8_t *syn_ws) {
    uint8_t *dst = syn_ws + (cw0 + tile_row(lane, 0)) * 32 + C::S0[R];
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i) {
        transpose8(S[i]);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (fl >> c & 1) dst[32 * c + i] = (uint8_t)(S[i][4 + c] >> 24);
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
    int32_t res[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const size_t cw = w.cw0 + tile_row(lane, c);
        if (cw >= w.ncw) fl &= ~(1u << c);
        else if (neras && neras[cw]) fl |= 1u << c;  // erasures: the error path validates them
        res[c] = (fl >> c & 1) ? kSentinel : 0;
    }
    if (R == 0) {
        const size_t cw = w.cw0 + tile_row(lane, 0);
        if (cw + 3 < w.ncw) {
            __builtin_memcpy(result + cw, res, 16);
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (cw + c < w.ncw) result[cw + c] = res[c];
        }
    }
    if (fl) write_syndromes<C, R>(S, fl, w.cw0, lane, syn_ws);
}

template <class C>
__global__ void __launch_bounds__(kThreads, 4)
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
// S_i for codewords 32G .. 32G+31 (bit s <-> codeword 32G + s).  Lane l's bits 28..31 hold
// codewords 4l .. 4l+3, i.e. nibble l&7 of group l>>3's planes: pairs of lanes form a byte (DPP),
// gathered through LDS.
template <class C, int R>
__device__ __forceinline__ void encode_syn_body(uint32_t *lds, const Word &w, int nchunks,
                                                uint32_t *ws) {
    const int lane = threadIdx.x & 63;
    uint32_t S[16][8];
    syndromes_tile<C, R>(S, lds, w, nchunks);
    constexpr int NPL = 8 * C::NR;
    constexpr int NG = kTile / 32;                         // groups per tile
    uint8_t *stage = reinterpret_cast<uint8_t *>(lds);     // [NPL planes][NG groups] dwords
#pragma unroll
    for (int i = 0; i < C::NS[R]; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t nib = S[i][q] >> 28;
            // lane l+1's nibble (row_shr:1 within each row of 16 lanes: l odd reads l-1 ... so
            // even lanes pull their odd neighbour with row_shl:1)
            const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nib, 0x101, 0xF, 0xF, false);
            if (!(lane & 1))
                stage[(((C::S0[R] + i) * 8 + q) * NG + (lane >> 3)) * 4 + ((lane >> 1) & 3)] =
                    (uint8_t)(nib | (hi << 4));
        }
    __syncthreads();
    const size_t tile = w.cw0 / kTile;                     // groups 8 tile .. 8 tile + 7
    uint32_t *dst = ws + (tile >> 3) * NPL * 64 + (tile & 7) * NG;
    for (int idx = threadIdx.x; idx < NPL * NG; idx += kThreads)
        dst[(idx / NG) * 64 + (idx % NG)] = lds[idx];
}

template <class C>
__global__ void __launch_bounds__(kThreads, 4)
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

// Encode, stage 2: parity = Q(syndromes) over full 32-codeword registers.  One 256-thread block
// covers 64 groups (2048 codewords).  The block first copies its 64 groups' workspace planes
// (8 NR x 64 dwords) into LDS with coalesced 16-byte loads -- all in flight at once, instead of 32
// dependent rounds of global loads per wave -- then wave P computes parity symbols 8P..8P+7 of
// every group from LDS, and, in the same LDS, stages them as [codeword][NR] bytes so that each
// codeword's parity leaves as one contiguous run.
constexpr int kParGroups = 64;                      // groups of 32 codewords per parity block
constexpr int kParCw = 32 * kParGroups;

template <class C, int P>
__device__ __forceinline__ void parity_compute(uint32_t (&O)[8][8], const uint32_t *in) {
    constexpr int NJ = C::NR - 8 * P < 8 ? C::NR - 8 * P : 8;
    C::template q_pass<P>(O, in, 64);
#pragma unroll
    for (int j = 0; j < NJ; ++j) transpose8(O[j]);   // O[j][c] byte s: symbol 8P+j of cw 32G+8s+c
}

template <class C, int P>
__device__ __forceinline__ void parity_stage(const uint32_t (&O)[8][8], uint8_t *stage, int g) {
    constexpr int NJ = C::NR - 8 * P < 8 ? C::NR - 8 * P : 8;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            uint8_t *dst = stage + g * (32 * C::NR + 16) + (8 * s + c) * C::NR + 8 * P;
            if (NJ == 8) {
                reinterpret_cast<uint32_t *>(dst)[0] = gather4(O[0][c], O[1][c], O[2][c], O[3][c], s);
                reinterpret_cast<uint32_t *>(dst)[1] = gather4(O[4][c], O[5][c], O[6][c], O[7][c], s);
            } else if (NJ == 4) {
                reinterpret_cast<uint32_t *>(dst)[0] = gather4(O[0][c], O[1][c], O[2][c], O[3][c], s);
            } else {
#pragma unroll
                for (int j = 0; j < NJ; ++j) dst[j] = (uint8_t)(O[j][c] >> (8 * s));
            }
        }
}

template <class C>
__global__ void __launch_bounds__(256)
    k_bs_parity(const uint32_t *ws, uint8_t *parity, size_t pstride, size_t ncw) {
    constexpr int kDw = 8 * C::NR * kParGroups;          // input planes, dwords
    // staged parity: group g's 32 rows in a region of 32 NR + 16 bytes (the pad spreads the
    // groups' stores over the LDS banks); the region reuses the input buffer
    constexpr int kRegion = 32 * C::NR + 16;
    constexpr int kLdsDw = kDw > kParGroups * kRegion / 4 ? kDw : kParGroups * kRegion / 4;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsDw];
    const uint4 *src = reinterpret_cast<const uint4 *>(ws + (size_t)blockIdx.x * kDw);
    for (int i = threadIdx.x; i < kDw / 4; i += 256) reinterpret_cast<uint4 *>(lds)[i] = src[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t O[8][8];
    switch (wave) {
    case 0: parity_compute<C, 0>(O, lds + lane); break;
    case 1: if constexpr (C::NPASS > 1) parity_compute<C, 1>(O, lds + lane); break;
    case 2: if constexpr (C::NPASS > 2) parity_compute<C, 2>(O, lds + lane); break;
    default: if constexpr (C::NPASS > 3) parity_compute<C, 3>(O, lds + lane); break;
    }
    __syncthreads();                                      // the inputs are consumed
    uint8_t *stage = reinterpret_cast<uint8_t *>(lds);
    switch (wave) {
    case 0: parity_stage<C, 0>(O, stage, lane); break;
    case 1: if constexpr (C::NPASS > 1) parity_stage<C, 1>(O, stage, lane); break;
    case 2: if constexpr (C::NPASS > 2) parity_stage<C, 2>(O, stage, lane); break;
    default: if constexpr (C::NPASS > 3) parity_stage<C, 3>(O, stage, lane); break;
    }
    __syncthreads();
    // one codeword's NR parity bytes per lane and round: consecutive lanes -> consecutive rows
    const size_t cw0 = (size_t)blockIdx.x * kParCw;
    for (int r = threadIdx.x; r < kParCw; r += 256) {
        const size_t k = cw0 + r;
        if (k >= ncw) break;
        uint8_t *dst = parity + k * pstride;
        const uint8_t *src8 = stage + (r >> 5) * kRegion + (r & 31) * C::NR;
        if constexpr (C::NR % 16 == 0) {
#pragma unroll
            for (int o = 0; o < C::NR; o += 16) {
                uint4 v = *reinterpret_cast<const uint4 *>(src8 + o);
                __builtin_memcpy(dst + o, &v, 16);
            }
        } else if constexpr (C::NR % 4 == 0) {
#pragma unroll
            for (int o = 0; o < C::NR; o += 4) {
                uint32_t v = *reinterpret_cast<const uint32_t *>(src8 + o);
                __builtin_memcpy(dst + o, &v, 4);
            }
        } else {
            for (int o = 0; o < C::NR; ++o) dst[o] = src8[o];
        }
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

hipError_t launch_bs_encode(int id, const DevCodec &, const EncodeArgs &a, void *ws, hipStream_t s) {
    const unsigned grid = (unsigned)((a.ncw + bs::kTile - 1) / bs::kTile);
    const unsigned pgrid = (unsigned)((a.ncw + bs::kParCw - 1) / bs::kParCw);
    uint32_t *w = static_cast<uint32_t *>(ws);
    int k = 0;
#define EZRS_BS_ENC(C)                                                                            \
    if (k++ == id) {                                                                              \
        hipLaunchKernelGGL(bs::k_bs_encode_syn<bs::C>, dim3(grid), dim3(bs::kThreads), 0, s,      \
                           static_cast<const uint8_t *>(a.data), a.data_stride, a.len, a.ncw, w); \
        hipLaunchKernelGGL(bs::k_bs_parity<bs::C>, dim3(pgrid), dim3(256), 0, s,                  \
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
