// ezbch_ps_tile.hpp -- the tile machinery of the plane-sliced BCH remainder kernels (see
// ezbch_ps.hip): images, networks, fold and the persistent tile loop, shared by the encode kernel
// (ezbch_ps.hip) and the fused decode kernel (ezbch.hip), which hand the loop what to do with each
// tile's remainders.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gen/ezbch_ps_tables.inc"
#include "ezbch_ps.hpp"

namespace ezrs {
namespace bps {

constexpr int kRows = 256;                    // rows per tile
constexpr int kTW = 4;                        // wavefronts per tile (per workgroup), at most; two
                                              // (r06i): decode 1.44 vs 0.90 ms at 8 M, encode equal
constexpr int kGuard = 128;                   // LDS bytes before an image: frame positions before a
                                              // row's first byte read there (then masked)
constexpr int kImage = 32768;                 // 32 DMA instructions of 1 KiB: 256 rows of <= 128 B
constexpr int kImgSlot = kGuard + kImage + 64;
constexpr int kXch = 8 * 256;                 // per wave: <= 8 ECC-byte words of 64 lanes
constexpr int kLds = 2 * kImgSlot + kTW * kXch;  // per workgroup: 2 per CU

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
// first byte (fb, wave-uniform) contribute nothing.
template <class C, bool DEC, int B, bool FIRST>
__device__ __forceinline__ void block(uint32_t (&U)[C::E], uint32_t (&X)[8], int fb) {
    constexpr int pa = 8 * B;
    if (pa < fb) {                                           // wave-uniform
        const int d = fb - pa;
#pragma unroll
        for (int t = 0; t < 8; ++t) X[t] = t < d ? 0u : X[t];
    }
    C::template block<B, FIRST, DEC ? 0 : C::EB>(U, X);
}

// Piece I (blocks 2I, 2I+1) of pieces [I0, IE): wait for its reads, issue the next piece's, run its
// networks.
template <class C, bool DEC, int I, int I0, int IE>
__device__ __forceinline__ void piece(uint32_t (&U)[C::E], Raw &cur, const uint32_t (&at)[4],
                                      const uint32_t (&at4)[4], int fb) {
    if constexpr (I < IE) {
        wait_raw(cur);
        Raw nxt;
        if constexpr (I + 1 < IE) issue_at<16 * (I + 1)>(nxt, at4);
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
        block<C, DEC, 2 * I, I == I0>(U, X, fb);
        __builtin_amdgcn_sched_barrier(0);
        {
            const uint32_t c2[4] = {R[0].z, R[1].z, R[2].z, R[3].z};
            const uint32_t c3[4] = {R[0].w, R[1].w, R[2].w, R[3].w};
            transpose4x4(c2, X);
            transpose4x4(c3, X + 4);
        }
        block<C, DEC, 2 * I + 1, false>(U, X, fb);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (I + 1 < IE) piece<C, DEC, I + 1, I0, IE>(U, nxt, at, at4, fb);
    }
}

// Wavefronts per tile of a codec: kTW, or one per 16-position piece of a shorter frame
template <class C> constexpr int tile_waves() { return C::NB / 2 < kTW ? C::NB / 2 : kTW; }

// Wave W's share of a tile: pieces [NP W / TW, NP (W+1) / TW) of the image at img.
template <class C, bool DEC, int W>
__device__ __forceinline__ void part_tile(uint32_t (&U)[C::E], uint32_t img, uint32_t stride, int fb) {
    constexpr int TW = tile_waves<C>(), NP = C::NB / 2, I0 = W * NP / TW, IE = (W + 1) * NP / TW;
    // byte address of frame position 0 of rows 4l + k (the rows' first bytes at position fb)
    uint32_t at[4], at4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        at[k] = img + (4u * lane_id() + k) * stride - (uint32_t)fb;
        at4[k] = at[k] & ~3u;
    }
    Raw cur;
    issue_at<16 * I0>(cur, at4);
    asm volatile("s_setprio 1");                     // without: encode 0.404 vs 0.398 ms at 8 M (r06i)
    piece<C, DEC, I0, I0, IE>(U, cur, at, at4, fb);
    asm volatile("s_setprio 0");
}

// Stores of one row's ECC bytes w (byte 0 first) at byte offset off: dwords, then a short, then a
// byte; an offset past the buffer's range stores nothing.
template <int EB> struct EccStore {
    static constexpr int N = EB / 4 + ((EB & 3) >= 2) + (EB & 1);   // instructions per row
    static __device__ __forceinline__ void run(rsrc_t r, uint32_t off, const uint32_t (&w)[2]) {
#pragma unroll
        for (int o = 0; o + 4 <= EB; o += 4)
            asm volatile("buffer_store_dword %0, %1, %2, 0 offen offset:%3" :: "v"(w[o / 4]), "v"(off), "s"(r), "n"(o) : "memory");
        constexpr int o2 = EB / 4 * 4;
        if constexpr ((EB & 3) >= 2)
            asm volatile("buffer_store_short %0, %1, %2, 0 offen offset:%3" :: "v"(w[o2 / 4]), "v"(off), "s"(r), "n"(o2) : "memory");
        constexpr int o1 = EB & ~1;
        if constexpr (EB & 1)
            asm volatile("buffer_store_byte %0, %1, %2, 0 offen offset:%3"
                         :: "v"(w[o1 / 4] >> (8 * (o1 & 3))), "v"(off), "s"(r), "n"(o1) : "memory");
    }
};

// The persistent loop over a launch's tiles.  Per tile, once the waves' partial ECC bytes are
// summed, fin(tile, image, out) runs in every wave (all threads of the workgroup): out[e] byte k is
// byte e of the ECC (encode) or of the remainder XOR the received ECC (decode) of row
// tile * 256 + 4l + k, and image[j] (LDS) is byte tile * 256 * stride + j of the batch.  NV: the
// vector-memory instructions fin issues per tile, left in flight by the next tile's wait, or -1
// when their number varies (the wait then takes them all).  NSLOT: 2 -- the next tile's rows land
// in the other image while this one is computed; 1 -- one image (X = its offset in lds), the next
// tile's DMA issued once fin is done with it (three workgroups per CU cover each other's waits).
template <class C, bool DEC, int NV, int NSLOT = 2, class Fin>
__device__ __forceinline__ void tile_loop(const BpsArgs &a, uint8_t *lds, Fin &&fin) {
    static_assert(NSLOT == 1 || NSLOT == 2, "one or two images");
    constexpr uint32_t kX = NSLOT * kImgSlot;             // exchange words after the images
    constexpr int TW = tile_waves<C>();
    static_assert(C::NB % (2 * TW) == 0 && (TW == 2 || TW == 4) && C::F <= 128 && C::EB <= 8,
                  "frame: whole 16-position pieces per wave");
    const rsrc_t rsrc = make_rsrc(a.base, a.span);
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = lane_id();
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    const uint32_t tb = kRows * a.stride;                    // a tile's bytes
    const uint32_t ndma = (tb + 1023) >> 10;
    auto issue = [&](uint32_t tile, uint32_t slot) {       // this wave's share of a tile's DMA
        const uint32_t img = lds0 + slot * kImgSlot + kGuard, toff = tile * tb + 16u * l;
        for (uint32_t i = w; i < ndma; i += TW)
            asm volatile("s_mov_b32 m0, %0\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %1, %2, 0 offen lds"
                         :: "s"(__builtin_amdgcn_readfirstlane(img + i * 1024u)), "v"(toff + i * 1024u), "s"(rsrc)
                         : "memory", "m0");
    };
    uint32_t tile = blockIdx.x;
    if (tile < a.ntiles) issue(tile, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t it = 0; tile < a.ntiles; ++it, tile += gridDim.x) {
        const uint32_t slot = NSLOT == 2 ? (it & 1) : 0u, img = lds0 + slot * kImgSlot + kGuard;
        // this wave's share of the tile's DMA (issued an iteration ago) has landed; the last tile's
        // fin may leave its stores in flight
        if constexpr (NV >= 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NV) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t toff = tile * tb;
        if (w == 0 && toff + tb >= a.span) {
            // a 16-byte DMA piece that crosses the span's end comes back all-zero: re-read the last
            // 64 bytes one by one (out-of-range bytes read as zero)
            const uint32_t off = a.span - 64u + l;
            uint32_t v;
            asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(v) : "v"(off), "s"(rsrc) : "memory");
            if (off >= toff && off < a.span)
                asm volatile("ds_write_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(img + (off - toff)), "v"(v) : "memory");
        }
        // all shares of the image are in, and every wave is done with the other image and the
        // exchange words
        asm volatile("s_barrier" ::: "memory");
        const uint32_t nt = tile + gridDim.x;
        if (NSLOT == 2 && nt < a.ntiles) issue(nt, slot ^ 1);
        int fb = a.fb;
        asm volatile("" : "+s"(fb));
        uint32_t U[C::E];
        if constexpr (TW == 4) {
            if (w == 0) part_tile<C, DEC, 0>(U, img, a.stride, fb);
            else if (w == 1) part_tile<C, DEC, 1>(U, img, a.stride, fb);
            else if (w == 2) part_tile<C, DEC, 2>(U, img, a.stride, fb);
            else part_tile<C, DEC, 3>(U, img, a.stride, fb);
        } else {
            if (w == 0) part_tile<C, DEC, 0>(U, img, a.stride, fb);
            else part_tile<C, DEC, 1>(U, img, a.stride, fb);
        }
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
        // the other waves' partial bytes
        uint32_t *xw = (uint32_t *)(lds + kX);
#pragma unroll
        for (int e = 0; e < C::EB; ++e) xw[w * (kXch / 4) + e * 64 + l] = out[e];
        __syncthreads();
#pragma unroll
        for (int o = 1; o < TW; ++o) {
            const uint32_t p = (w + o) % TW;
#pragma unroll
            for (int e = 0; e < C::EB; ++e) out[e] ^= xw[p * (kXch / 4) + e * 64 + l];
        }
        fin(tile, lds + slot * kImgSlot + kGuard, out);
        if constexpr (NSLOT == 1) {
            if (nt < a.ntiles) {
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // fin is done with the image
                issue(nt, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // no DMA may land after the exit
}

// The ECC bytes of row 4l + k (byte e of out[] -> byte e of the pair, byte 0 first)
template <int EB>
__device__ __forceinline__ void row_bytes(const uint32_t (&out)[EB], uint32_t k, uint32_t (&wd)[2]) {
    uint32_t b[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = e < EB ? out[e < EB ? e : 0] : 0u;
    wd[0] = gather4(b[0], b[1], b[2], b[3], (int)k);
    wd[1] = gather4(b[4], b[5], b[6], b[7], (int)k);
}

} // namespace bps
} // namespace ezrs
