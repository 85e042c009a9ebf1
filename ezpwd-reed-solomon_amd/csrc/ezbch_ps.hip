// ezbch_ps.hip -- plane-sliced BCH remainders on MI355X (gfx950): the encode of BCH codecs whose
// ECC is a whole number of bytes of at most 64 bits (C5: BCH(1023,983,4), 40 bits), and the
// remainder difference their decode starts from.
//
// The remainder of a row: ECC = d(x) x^E mod g(x), data bits MSB first, ECC left-justified
// big-endian (c++/ezpwd/bch:196-205; Djelic encode_bch).  The derivation is in
// codegen/gen_bch_ps.py: with bit b of the byte q places from the row's end the coefficient of
// x^(8q + b), every bit plane of a row has the same weights w(q) = x^(8q) mod g, so a 32-bit word
// holding one byte position of four rows is XORed whole into an E-word state; a three-level fold
// inside each byte combines the planes (sum_b x^b U_b).  XOR networks only, no tables: the LFSR
// kernel (k_bch_encode, ezbch.hip) spends a dependent 256-entry table read per data byte.
//
// One wavefront per 256-row tile (four rows per lane, byte k of a word = row 4l + k), each with
// its own LDS image: the tile's rows arrive by 1 KiB LDS-DMA instructions as they lie in memory,
// the next tile's as soon as this one's main loop has read its image; no barrier, no exchange.
// Rows are read as aligned dwords and aligned with v_alignbyte (an odd pitch -- C5's 127 -- puts
// the four rows of the 64 lanes in distinct banks), then transposed 4 x 4 bytes into position words.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gen/ezbch_ps_tables.inc"
#include "ezbch_ps.hpp"

namespace ezrs {
namespace bps {

constexpr int kRows = 256;                    // rows per tile (per wavefront)
constexpr int kGuard = 128;                   // LDS bytes before the image: frame positions before a
                                              // row's first byte read there (then masked)
constexpr int kImage = 32768;                 // 32 DMA instructions of 1 KiB: 256 rows of <= 128 B
constexpr int kSlot = kGuard + kImage + 64;   // LDS per wavefront (4 per CU)
constexpr uint32_t kOob = 0xF0000000u;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef int rsrc_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lane_id() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Buffer descriptor of [base, base + span): out-of-range bytes read as zero.
__device__ __forceinline__ rsrc_t make_rsrc(const uint8_t *base, uint32_t span) {
    const uint64_t p = (uint64_t)(uintptr_t)base;
    rsrc_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(p >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)span);
    r.w = 0x00020000;
    return r;
}

__device__ __forceinline__ uint32_t lds_addr(const uint8_t *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
}

// 4x4 byte transpose: out[t] byte k = in[k] byte t.
__device__ __forceinline__ void transpose4x4(const uint32_t (&a)[4], uint32_t *out) {
    const uint32_t t01 = __builtin_amdgcn_perm(a[1], a[0], 0x05010400u);
    const uint32_t t23 = __builtin_amdgcn_perm(a[3], a[2], 0x05010400u);
    const uint32_t u01 = __builtin_amdgcn_perm(a[1], a[0], 0x07030602u);
    const uint32_t u23 = __builtin_amdgcn_perm(a[3], a[2], 0x07030602u);
    out[0] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
    out[1] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
    out[2] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);
    out[3] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);
}

// Bytes s of a0..a3 -> one dword (a0 in byte 0).
__device__ __forceinline__ uint32_t gather4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int s) {
    const uint32_t sel = (uint32_t)s | ((uint32_t)(s + 4) << 8) | 0x0c0c0000u;   // 0x0c: zero byte
    const uint32_t x01 = __builtin_amdgcn_perm(a1, a0, sel), x23 = __builtin_amdgcn_perm(a3, a2, sel);
    return __builtin_amdgcn_perm(x23, x01, 0x05040100u);
}

// The tile's bytes [toff, toff + bytes) into the image, 1 KiB per instruction.
__device__ __forceinline__ void issue_tile(uint32_t img, rsrc_t rsrc, uint32_t toff, uint32_t bytes) {
    const uint32_t n = (bytes + 1023) >> 10, lo16 = 16u * lane_id();
    for (uint32_t i = 0; i < n; ++i)
        asm volatile("s_mov_b32 m0, %0\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %1, %2, 0 offen lds"
                     :: "s"(img + i * 1024u), "v"(toff + i * 1024u + lo16), "s"(rsrc) : "memory", "m0");
}

// Raw dwords of rows 4l + k at one 16-position piece (aligned afterwards with v_alignbyte)
struct Raw {
    u32x2 e[4][2];
    uint32_t d4[4];
};
template <int OFF>
__device__ __forceinline__ void issue_at(Raw &r, const uint32_t (&at4)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        asm volatile("ds_read2_b32 %0, %3 offset0:%4 offset1:%5\n\t"
                     "ds_read2_b32 %1, %3 offset0:%6 offset1:%7\n\t"
                     "ds_read_b32 %2, %3 offset:%8"
                     : "=&v"(r.e[k][0]), "=&v"(r.e[k][1]), "=&v"(r.d4[k])
                     : "v"(at4[k]), "n"(OFF / 4), "n"(OFF / 4 + 1), "n"(OFF / 4 + 2), "n"(OFF / 4 + 3), "n"(OFF + 16)
                     : "memory");
}
__device__ __forceinline__ void wait_raw(Raw &r) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(r.e[0][0]), "+v"(r.e[0][1]), "+v"(r.d4[0]), "+v"(r.e[1][0]), "+v"(r.e[1][1]), "+v"(r.d4[1]),
                   "+v"(r.e[2][0]), "+v"(r.e[2][1]), "+v"(r.d4[2]), "+v"(r.e[3][0]), "+v"(r.e[3][1]), "+v"(r.d4[3])
                 :: "memory");
}

// Frame block B (positions 8B .. 8B+7) of the four rows into the state: positions before a row's
// first byte (fb, wave-uniform) and -- encode -- the ECC positions contribute nothing.
template <class C, bool DEC, int B>
__device__ __forceinline__ void block(uint32_t (&U)[C::E], uint32_t (&X)[8], int fb) {
    constexpr int pa = 8 * B;
    if constexpr (!DEC && pa + 8 > C::F - C::EB) {
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (pa + t >= C::F - C::EB) X[t] = 0;
    }
    if (pa < fb) {                                           // wave-uniform
        const int d = fb - pa;
#pragma unroll
        for (int t = 0; t < 8; ++t) X[t] = t < d ? 0u : X[t];
    }
    C::template block<B, B == 0>(U, X);
}

// Piece I (blocks 2I, 2I+1): wait for its reads, issue the next piece's, run its networks.
template <class C, bool DEC, int I>
__device__ __forceinline__ void piece(uint32_t (&U)[C::E], Raw &cur, const uint32_t (&at)[4],
                                      const uint32_t (&at4)[4], int fb) {
    constexpr int NP = C::NB / 2;
    if constexpr (I < NP) {
        wait_raw(cur);
        Raw nxt;
        if constexpr (I + 1 < NP) issue_at<16 * (I + 1)>(nxt, at4);
        __builtin_amdgcn_sched_barrier(0);
        u32x4 R[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t d[5] = {cur.e[k][0].x, cur.e[k][0].y, cur.e[k][1].x, cur.e[k][1].y, cur.d4[k]};
#pragma unroll
            for (int j = 0; j < 4; ++j) R[k][j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], at[k]);
        }
        uint32_t X[8];
        {
            const uint32_t c0[4] = {R[0].x, R[1].x, R[2].x, R[3].x};
            const uint32_t c1[4] = {R[0].y, R[1].y, R[2].y, R[3].y};
            transpose4x4(c0, X);
            transpose4x4(c1, X + 4);
        }
        block<C, DEC, 2 * I>(U, X, fb);
        __builtin_amdgcn_sched_barrier(0);
        {
            const uint32_t c2[4] = {R[0].z, R[1].z, R[2].z, R[3].z};
            const uint32_t c3[4] = {R[0].w, R[1].w, R[2].w, R[3].w};
            transpose4x4(c2, X);
            transpose4x4(c3, X + 4);
        }
        block<C, DEC, 2 * I + 1>(U, X, fb);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (I + 1 < NP) piece<C, DEC, I + 1>(U, nxt, at, at4, fb);
    }
}

template <class C, bool DEC>
__global__ void __launch_bounds__(64) k_bch_ps(BpsArgs a) {
    static_assert(C::NB % 2 == 0 && C::F <= 128, "frame: whole 16-position pieces, rows <= 128 B");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSlot];
    const rsrc_t rsrc = make_rsrc(a.base, a.span);
    const uint32_t img = __builtin_amdgcn_readfirstlane(lds_addr(lds)) + kGuard;
    const uint32_t tb = kRows * a.stride;                    // a tile's bytes
    uint32_t tile = blockIdx.x;
    if (tile < a.ntiles) issue_tile(img, rsrc, tile * tb, tb);
    for (; tile < a.ntiles; tile += gridDim.x) {
        const uint32_t toff = tile * tb;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the tile landed (and the stores went)
        if (toff + tb >= a.span) {
            // a 16-byte DMA piece that crosses the span's end comes back all-zero: re-read the last
            // 64 bytes one by one (out-of-range bytes read as zero)
            const uint32_t off = a.span - 64u + lane_id();
            uint32_t v;
            asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(v) : "v"(off), "s"(rsrc) : "memory");
            if (off >= toff && off < a.span)
                asm volatile("ds_write_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(img + (off - toff)), "v"(v) : "memory");
        }
        int fb = a.fb;
        asm volatile("" : "+s"(fb));
        // byte address of frame position 0 of rows 4l + k (the rows' first bytes at position fb)
        uint32_t at[4], at4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            at[k] = img + (4u * lane_id() + k) * a.stride - (uint32_t)fb;
            at4[k] = at[k] & ~3u;
        }
        uint32_t U[C::E];
        {
            Raw cur;
            issue_at<0>(cur, at4);
            asm volatile("s_setprio 1");
            piece<C, DEC, 0>(U, cur, at, at4, fb);
            asm volatile("s_setprio 0");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the image is read: the next tile may land
        const uint32_t nt = tile + gridDim.x;
        if (nt < a.ntiles) issue_tile(img, rsrc, nt * tb, tb);
        C::fold(U);
        // ECC byte e of row 4l + k in byte k of out[e]: bits E-1-8e .. E-8-8e of the remainder, MSB first
        uint32_t out[C::EB];
#pragma unroll
        for (int e = 0; e < C::EB; ++e) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) v |= (U[C::E - 1 - 8 * e - j] & 0x01010101u) << (7 - j);
            out[e] = v;
        }
        const size_t k0 = (size_t)tile * kRows + 4u * lane_id();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k0 + k >= a.ncw) break;
            uint32_t w[2] = {0u, 0u};
#pragma unroll
            for (int e = 0; e < C::EB; e += 4) {
                const uint32_t b0 = out[e], b1 = e + 1 < C::EB ? out[e + 1 < C::EB ? e + 1 : e] : 0u,
                               b2 = e + 2 < C::EB ? out[e + 2 < C::EB ? e + 2 : e] : 0u,
                               b3 = e + 3 < C::EB ? out[e + 3 < C::EB ? e + 3 : e] : 0u;
                w[e / 4] = gather4(b0, b1, b2, b3, k);
            }
            if constexpr (!DEC) {
                __builtin_memcpy(a.ecc + (k0 + k) * a.estride, w, C::EB);
            } else {
                // the difference left-justified, byte 0 at the top (ezbch.hip data_remainder ^ ECC)
                const uint64_t r = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
                a.rem[k0 + k] = r;
                a.result[k0 + k] = r ? kBpsFlag : 0;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // no DMA may land after the exit
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

hipError_t launch_bps(int id, bool dec, const BpsArgs &a, int ncu, hipStream_t s) {
    const unsigned cap = 4u * (unsigned)(ncu > 0 ? ncu : 256);             // 4 wavefronts per CU (LDS)
    const unsigned grid = a.ntiles < cap ? a.ntiles : cap;
    if (!grid) return hipSuccess;
    int k = 0;
#define EZBCH_PS_LAUNCH(N, M, T)                                                                    \
    if (k++ == id) {                                                                                \
        if (dec) hipLaunchKernelGGL((bps::k_bch_ps<bps::BPS_##N, true>), dim3(grid), dim3(64), 0, s, a);  \
        else hipLaunchKernelGGL((bps::k_bch_ps<bps::BPS_##N, false>), dim3(grid), dim3(64), 0, s, a);     \
    }
    EZBCH_PS_CODEC_LIST(EZBCH_PS_LAUNCH)
#undef EZBCH_PS_LAUNCH
    return hipGetLastError();
}

} // namespace ezrs
