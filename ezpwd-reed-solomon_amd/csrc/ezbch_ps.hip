// ezbch_ps.hip -- plane-sliced BCH remainders on MI355X (gfx950): the encode of BCH codecs whose
// ECC is a whole number of bytes of at most 64 bits (C5: BCH(1023,983,4), 40 bits); the same tile
// loop (ezbch_ps_tile.hpp) starts the fused decode in ezbch.hip.
//
// The remainder of a row: ECC = d(x) x^E mod g(x), data bits MSB first, ECC left-justified
// big-endian (c++/ezpwd/bch:196-205; Djelic encode_bch).  The derivation is in
// codegen/gen_bch_ps.py: with bit b of the byte q places from the row's end the coefficient of
// x^(8q + b), every bit plane of a row has the same weights w(q) = x^(8q) mod g, so a 32-bit word
// holding one byte position of four rows is XORed whole into an E-word state; a three-level fold
// inside each byte combines the planes (sum_b x^b U_b).  XOR networks only, no tables: the LFSR
// kernel (k_bch_encode, ezbch.hip) spends a dependent 256-entry table read per data byte.
//
// A workgroup of kTW wavefronts per 256-row tile (four rows per lane, byte k of a word = row
// 4l + k), two tile images per workgroup: the tile's rows arrive by 1 KiB LDS-DMA instructions as
// they lie in memory, the next tile's while this one is computed.  Wave w runs the networks of
// frame pieces [NP w / kTW, NP (w+1) / kTW), folds its partial state (the fold is linear) and the
// partial ECC bytes are XORed through LDS; each wave then finishes one of its lanes' four rows
// (encode: stores its ECC).
// Rows are read as aligned dwords and aligned with v_alignbyte (an odd pitch -- C5's 127 -- puts
// the four rows of the 64 lanes in distinct banks), then transposed 4 x 4 bytes into position
// words.  The frame is right-aligned on the last byte read (encode: the data, decode: data + ECC).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ezbch_ps_tile.hpp"

namespace ezrs {
namespace bps {

template <class C>
__global__ void __launch_bounds__(64 * kTW) k_bch_ps(BpsArgs a) {
    constexpr int TW = tile_waves<C>();
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const rsrc_t orsrc = make_rsrc(a.ecc, a.espan);
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = lane_id();
    // rows 4l + k, k = w (TW = 4) or 2w, 2w + 1; rows past ncw: offsets past the buffer's range
    tile_loop<C, false, (4 / TW) * EccStore<C::EB>::N>(a, lds, [&](uint32_t tile, uint8_t *, const uint32_t (&out)[C::EB]) {
#pragma unroll
        for (int j = 0; j < 4 / TW; ++j) {
            const uint32_t k = (4 / TW) * w + j;
            uint32_t wd[2];
            row_bytes<C::EB>(out, k, wd);
            EccStore<C::EB>::run(orsrc, (tile * kRows + 4u * l + k) * (uint32_t)a.estride, wd);
        }
    });
}

template <class C> constexpr bool bps_match(int m, int t) { return C::M == m && C::T == t; }

} // namespace bps

// Codec id of the plane-sliced path (EZBCH_PS_CODEC_LIST order), -1 if none.
int bps_codec_id(int m, int t, int ecc_bits) {
    int id = 0, found = -1;
#define EZBCH_PS_MATCH(N, M, T) \
    if (found < 0 && M == m && T == t && bps::BPS_##N::E == ecc_bits) found = id; \
    ++id;
    EZBCH_PS_CODEC_LIST(EZBCH_PS_MATCH)
#undef EZBCH_PS_MATCH
    return found;
}

int bps_frame(int id) {
    int k = 0, f = -1;
#define EZBCH_PS_F(N, M, T) if (k++ == id) f = bps::BPS_##N::F;
    EZBCH_PS_CODEC_LIST(EZBCH_PS_F)
#undef EZBCH_PS_F
    return f;
}

hipError_t launch_bps(int id, const BpsArgs &a, int ncu, hipStream_t s) {
    const unsigned cap = 2u * (unsigned)(ncu > 0 ? ncu : 256);             // 2 workgroups per CU (LDS)
    const unsigned grid = a.ntiles < cap ? a.ntiles : cap;
    if (!grid) return hipSuccess;
    int k = 0;
#define EZBCH_PS_LAUNCH(N, M, T)                                                                    \
    if (k++ == id) {                                                                                \
        hipLaunchKernelGGL((bps::k_bch_ps<bps::BPS_##N>), dim3(grid), dim3(64 * bps::tile_waves<bps::BPS_##N>()), 0, s, a); \
    }
    EZBCH_PS_CODEC_LIST(EZBCH_PS_LAUNCH)
#undef EZBCH_PS_LAUNCH
    return hipGetLastError();
}

} // namespace ezrs
