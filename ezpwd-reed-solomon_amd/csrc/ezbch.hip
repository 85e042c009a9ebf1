// ezbch.hip -- batched binary BCH on MI355X (gfx950) and its C ABI (include/ezbch.h).
//
// Semantics: the Djelic / Linux lib/bch.c codec that the reference wraps as ezpwd::bch_base,
// ezpwd::bch<N,T> and ezpwd::BCH<N,K,T> (c++/ezpwd/bch:48-463) together with ezpwd::correct_bch
// (c++/ezpwd/bch_base:168-199), applied independently to every codeword of a batch:
//   encode : ECC = d(x) x^ecc_bits mod g(x), data bits MSB first, ECC left-justified big-endian in
//            ecc_bytes bytes, zero-initialised (bch:196-205)
//   decode : decode_bch's result (count / -EBADMSG / -EINVAL) and, as correct_bch, the reported
//            bits flipped in data and ECC; locations e address data[e/8] bit e%8 (ECC beyond
//            8*len), reported in ascending order (the reference's order is unpinned).
//
// Kernels: one lane per codeword, 256-codeword workgroups.
//   k_bch_encode    byte-at-a-time LFSR over the data with a left-justified remainder of NW 64-bit
//                   words (NW = 1, 2, 4: ecc_bits <= 64, 128, 256) and a 256-entry step table in LDS;
//                   each row is read as aligned dwords (v_alignbyte).
//   k_bch_decode<T> the same remainder XOR the received ECC; zero -> result 0.  Otherwise, in the
//                   same lane: syndromes S_1..S_2t from the set bits of the difference, binary
//                   Berlekamp-Massey (odd steps; static register arrays), and the locator's roots:
//                   degree 1 directly, degrees 2..4 as an affine GF(2)-linear equation
//                   A4 y^4 + A2 y^2 + A1 y = delta solved by elimination over the m basis bits,
//                   degree > 4 by a Chien search over the codeword's bit positions.
//   k_bch_decode_big t <= 64, ecc_bits <= 1024 with run-time t (per-lane arrays).
//   k_bch_*_wave     every larger init_bch-valid codec: one wavefront per codeword (see below).
// There is no CPU path.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/ezbch.h"
#include "ezbch_ps_tile.hpp"
#include "ezrs_internal.hpp"

using ezrs::BpsArgs;
using ezrs::bps_codec_id;
using ezrs::bps_frame;
using ezrs::launch_bps;

namespace {

constexpr int kBigT = 64;                    // runtime-t decode (k_bch_decode_big<NW>)
constexpr int kMaxNW = 16;                   // 64-bit words of the widest remainder
constexpr int kMaxM = 15;
constexpr int kThreads = 256;
constexpr int kEBADMSG = 74, kEINVAL = 22;   // Linux errno values, negated as decode_bch returns them

struct DevBch {
    int m, n, t, ecc_bits, ecc_bytes;
    int lds_tabs;             // exp/log tables staged in LDS (m <= 12)
    int nw;                   // 64-bit words of the remainder (1 .. 16; the wave path: 64 nwl)
    int nwl;                  // wave path (t > 64 or ecc_bits > 1024): remainder words per lane, else 0
    uint64_t emask[kMaxNW];   // the ecc_bits significant bits of a left-justified remainder
    const uint64_t *step;     // [256][nw] byte-step remainder table
    const uint16_t *ex;       // [2n] alpha^i
    const uint16_t *lg;       // [n+1] log_alpha (lg[0] unused)
    const uint64_t *syn_tab;  // ecc_bits <= 64, t <= 4: [8][256] the odd syndromes S1, S3, S5, S7
                              // (16 bits each) of remainder byte b (from the top) holding value v
    int bps;                  // plane-sliced remainder kernels (ezbch_ps.hip): codec id, or -1
    int ncu;                  // compute units of the device
};

struct BchArgs {
    const uint8_t *data;      // rows read by both kernels
    uint8_t *wdata;           // the same rows, written by decode (corrections); null for encode
    size_t dstride;
    unsigned len;
    uint8_t *ecc;
    size_t estride;
    int32_t *result;
    uint32_t *errloc;
    size_t lstride;
    size_t ncw;
    int staged;               // the block's data rows are copied to LDS with coalesced loads
    int lds_fix;              // decode, staged rows with their ECC inline: corrections go to the LDS
                              // image and only the 16-byte pieces holding them are written back
    int ecc_only;             // decode_bch's "ecc = recv XOR calc" form: no data, nothing corrected
    const uint32_t *syn;      // decode_bch's syndrome form: S_1..S_2t per codeword (ecc_only set)
    size_t sstride;
};

constexpr size_t kLdsLimit = 65536;

// LDS layout: [0, 2048 nw) byte-step table | exp/log tables (decode, m <= 12) | staged rows
__host__ __device__ inline size_t tabs_offset(const DevBch &b) { return (size_t)2048 * b.nw; }
__host__ __device__ inline size_t rows_offset(const DevBch &b, bool tabs) {
    return tabs_offset(b) + (tabs && b.lds_tabs ? (((size_t)3 * b.n + 1) * 2 + 15) / 16 * 16 : 0);
}

// staged rows: kThreads rows at the batch pitch from a dword-aligned start (+ 3 + 3 slack; C5's
// 256 rows of 127 bytes then fit four blocks per CU)
__host__ __device__ inline size_t rows_bytes(const BchArgs &a) { return (size_t)kThreads * a.dstride + 8; }

size_t lds_bytes(const DevBch &b, bool tabs, const BchArgs &a) {
    return rows_offset(b, tabs) + (a.staged ? rows_bytes(a) : 0);
}

// Rows are staged when the batch has a row pitch the block's span can hold within 64 KiB of LDS.
int want_staging(const DevBch &b, bool tabs, const BchArgs &a) {
    return a.ncw > 1 && a.len > 0 && a.dstride >= a.len &&
           rows_offset(b, tabs) + rows_bytes(a) <= kLdsLimit;
}

// ECC bytes inline after each row's data, rows packed back to back (the rows form at pitch len +
// ecc_bytes): the staged image holds them too, and a written-back piece holds no byte outside the
// rows (a gap between rows is never rewritten)
int ecc_inline(const DevBch &b, const BchArgs &a) {
    return a.ecc == a.data + a.len && a.estride == a.dstride && a.dstride == a.len + (size_t)b.ecc_bytes;
}

// ---- device ------------------------------------------------------------------------------------
struct GF {
    const uint16_t *ex, *lg;
    int n;
    __device__ uint32_t mul(uint32_t a, uint32_t b) const { return (a && b) ? ex[lg[a] + lg[b]] : 0u; }
    __device__ uint32_t div(uint32_t a, uint32_t b) const { return a ? ex[lg[a] + n - lg[b]] : 0u; }
    __device__ uint32_t inv(uint32_t a) const { return ex[n - lg[a]]; }
    __device__ uint32_t sq(uint32_t a) const { return a ? ex[2 * lg[a]] : 0u; }
    __device__ uint32_t sqrt(uint32_t a) const {
        if (!a) return 0u;
        const uint32_t l = lg[a];
        return ex[(l & 1) ? (l + n) >> 1 : l >> 1];
    }
};

// The bytes p[0..len) in order, read as the aligned dwords that hold them.
template <class F>
__device__ __forceinline__ void for_each_byte(const uint8_t *p, unsigned len, F &&f) {
    if (!len) return;
    const unsigned a = (unsigned)((uintptr_t)p & 3u);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p - a);
    const unsigned nd = (a + len + 3) >> 2;
    uint32_t lo = q[0];
    unsigned i = 0, j = 1;
    for (; i + 4 <= len; i += 4, ++j) {
        const uint32_t hi = j < nd ? q[j] : 0u;
        const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, a);
        f(w & 0xffu);
        f((w >> 8) & 0xffu);
        f((w >> 16) & 0xffu);
        f(w >> 24);
        lo = hi;
    }
    if (i < len) {
        uint32_t w = __builtin_amdgcn_alignbyte(j < nd ? q[j] : 0u, lo, a);
        for (; i < len; ++i, w >>= 8) f(w & 0xffu);
    }
}

// A left-justified multiword remainder: w[0] holds the most significant 64 bits.
template <int NW> struct Rem {
    uint64_t w[NW];
};

template <int NW>
__device__ __forceinline__ Rem<NW> data_remainder(const uint64_t *step, const uint8_t *p,
                                                  unsigned len) {
    Rem<NW> r;
#pragma unroll
    for (int i = 0; i < NW; ++i) r.w[i] = 0;
    for_each_byte(p, len, [&](uint32_t byte) {
        const uint64_t *s = step + NW * ((uint32_t)(r.w[0] >> 56) ^ byte);
#pragma unroll
        for (int i = 0; i < NW; ++i)
            r.w[i] = ((r.w[i] << 8) | (i + 1 < NW ? r.w[i + 1 < NW ? i + 1 : i] >> 56 : 0)) ^ s[i];
    });
    return r;
}

__device__ __forceinline__ void stage_tables(const DevBch &b, uint8_t *smem, bool tabs) {
    uint64_t *step = reinterpret_cast<uint64_t *>(smem);
    for (int i = threadIdx.x; i < 256 * b.nw; i += kThreads) step[i] = b.step[i];
    if (tabs && b.lds_tabs) {
        uint16_t *ex = reinterpret_cast<uint16_t *>(smem + tabs_offset(b)), *lg = ex + 2 * b.n;
        for (int i = threadIdx.x; i < 2 * b.n; i += kThreads) ex[i] = b.ex[i];
        for (int i = threadIdx.x; i <= b.n; i += kThreads) lg[i] = b.lg[i];
    }
    __syncthreads();
}

// This lane's data row: staged -- the block's rows are one contiguous span of global memory, copied
// into LDS with coalesced dword loads (a lane-per-row read of 127-byte rows touches a new cache line
// per lane and load) -- or read in place.
__device__ __forceinline__ const uint8_t *block_rows(uint8_t *smem, const DevBch &b, bool tabs,
                                                     const BchArgs &a) {
    const size_t k0 = (size_t)blockIdx.x * kThreads;
    if (!a.staged) return a.data + (k0 + threadIdx.x) * a.dstride;
    const size_t nrows = a.ncw - k0 < (size_t)kThreads ? a.ncw - k0 : (size_t)kThreads;
    const uint8_t *base = a.data + k0 * a.dstride;
    const size_t span = (nrows - 1) * a.dstride + a.len + (a.lds_fix ? (size_t)b.ecc_bytes : 0);
    const unsigned off = (unsigned)((uintptr_t)base & 3u);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(base - off);
    uint8_t *rows = smem + rows_offset(b, tabs);
    uint32_t *dst = reinterpret_cast<uint32_t *>(rows);
    const unsigned nd = (unsigned)((off + span + 3) >> 2);
    for (unsigned i = threadIdx.x; i < nd; i += kThreads) dst[i] = src[i];
    __syncthreads();
    return rows + off + threadIdx.x * a.dstride;
}

// Flip bit el of this lane's staged row (data, then its inline ECC).
__device__ __forceinline__ void fix_bit_lds(uint8_t *rows, const uint8_t *row, uint32_t el) {
    const uint32_t o = (uint32_t)(row - rows) + (el >> 3);
    atomicXor(reinterpret_cast<uint32_t *>(rows + (o & ~3u)), (1u << (el & 7)) << (8 * (o & 3)));
}

// Once every lane of the wave has flipped its bits in the image: each lane writes back the 16-byte
// pieces (on the global 16-byte grid) that hold its corrected bits, from the image -- a piece wholly
// inside the bytes of the wave's 64 rows as one store (a piece shared by two rows of the wave may
// be written by both lanes, with the same bytes), a piece reaching past them byte by byte over the
// wave's own bytes only (the neighbouring waves and blocks write the rest).
template <int T>
__device__ __forceinline__ void write_pieces(const uint8_t *rows, const uint8_t *row, const uint32_t (&loc)[T], int cnt,
                                             const DevBch &b, const BchArgs &a) {
    const size_t k0 = (size_t)blockIdx.x * kThreads;
    const size_t nrows = a.ncw - k0 < (size_t)kThreads ? a.ncw - k0 : (size_t)kThreads;
    const unsigned w = threadIdx.x >> 6;
    const size_t wend = 64u * w + 64u < nrows ? 64u * w + 64u : nrows;     // the wave's rows [64 w, wend)
    uint8_t *base = a.wdata + k0 * a.dstride;
    const unsigned off = (unsigned)((uintptr_t)base & 3u);
    uint8_t *g = base - off;                                                // image byte 0
    const int lo = (int)(off + 64u * w * a.dstride),
              hi = (int)(off + (wend - 1) * a.dstride + a.len + (size_t)b.ecc_bytes);
    const uint32_t gmis = (uint32_t)((uintptr_t)g & 15u);                  // image offset -> piece grid
    int last = -1000;
#pragma unroll
    for (int i = 0; i < T; ++i) {
        if (i >= cnt) break;
        const uint32_t o = (uint32_t)(row - rows) + (loc[i] >> 3);
        const int p0 = (int)((o + gmis) & ~15u) - (int)gmis;              // image offset of the piece
        if (p0 == last) continue;
        last = p0;
        if (p0 >= lo && p0 + 16 <= hi) {
            const uint32_t *s4 = reinterpret_cast<const uint32_t *>(rows + p0);   // dword aligned
            *reinterpret_cast<uint4 *>(g + p0) = make_uint4(s4[0], s4[1], s4[2], s4[3]);
        } else {
            for (int q = p0 < lo ? lo : p0; q < p0 + 16 && q < hi; ++q) g[q] = rows[q];
        }
    }
}

template <int NW>
__global__ void __launch_bounds__(kThreads) k_bch_encode(DevBch b, BchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    stage_tables(b, smem, false);
    const uint8_t *row = block_rows(smem, b, false, a);
    const size_t k = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= a.ncw) return;
    const Rem<NW> r = data_remainder<NW>(reinterpret_cast<const uint64_t *>(smem), row, a.len);
    uint8_t *e = a.ecc + k * a.estride;
    // ecc_bytes = ceil(m t / 8) may pass the NW words when ecc_bits < m t: those bytes are zero
    for (int i = 0; i < b.ecc_bytes; ++i)
        e[i] = (i >> 3) < NW ? (uint8_t)(r.w[(i >> 3) < NW ? i >> 3 : 0] >> (56 - 8 * (i & 7))) : (uint8_t)0;
}

// y -> A4 y^4 + A2 y^2 + A1 y is GF(2)-linear.  With the images of the polynomial-basis vectors
// 1 << i (= alpha^i) in echelon form: returns the kernel dimension, or -1 if A(y) = delta has no
// solution; y0 = a particular solution, k1, k2 = the first two kernel basis vectors.
// MM: m known at compile time (the plane-sliced decode's codec), or 0
template <int MM = 0>
__device__ int solve_affine(const GF &f, int m, uint32_t A4, uint32_t A2, uint32_t A1,
                            uint32_t delta, uint32_t &y0, uint32_t &k1, uint32_t &k2) {
    constexpr int kM = MM ? MM : kMaxM;
    if constexpr (MM != 0) m = MM;
    const int l4 = A4 ? (int)f.lg[A4] : -1, l2 = A2 ? (int)f.lg[A2] : -1, l1 = A1 ? (int)f.lg[A1] : -1;
    uint32_t v[kM], c[kM];
    int pb[kM];
    int dim = 0;
    uint32_t q1 = 0, q2 = 0;                // k1, k2: selects, not a store indexed by dim (scratch)
#pragma unroll
    for (int i = 0; i < kM; ++i) {
        v[i] = 0;
        c[i] = 0;
        pb[i] = -1;
        if (i < m) {
            uint32_t w = 0;
            if (l4 >= 0) w ^= f.ex[l4 + 4 * i];
            if (l2 >= 0) w ^= f.ex[l2 + 2 * i];
            if (l1 >= 0) w ^= f.ex[l1 + i];
            uint32_t cc = 1u << i;
#pragma unroll
            for (int k = 0; k < i; ++k)
                if (pb[k] >= 0 && ((w >> pb[k]) & 1u)) {
                    w ^= v[k];
                    cc ^= c[k];
                }
            v[i] = w;
            c[i] = cc;
            pb[i] = w ? 31 - __clz(w) : -1;
            q1 = (!w && dim == 0) ? cc : q1;
            q2 = (!w && dim == 1) ? cc : q2;
            dim += !w;
        }
    }
    uint32_t y = 0, rem = delta;
#pragma unroll
    for (int k = 0; k < kM; ++k)
        if (pb[k] >= 0 && ((rem >> pb[k]) & 1u)) {
            rem ^= v[k];
            y ^= c[k];
        }
    y0 = y;
    k1 = q1;
    k2 = q2;
    return rem ? -1 : dim;
}

// Roots X of sigma(X) = X^L + a X^(L-1) + b X^(L-2) + c X^(L-3) + d for L = 2..4 (sigma(0) != 0);
// returns L if there are L distinct roots, else 0.
template <int MM = 0>
__device__ int small_roots(const GF &f, int m, int L, uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                           uint32_t (&X)[4]) {
    uint32_t A4, A2, A1, delta, s = 0;
    int want;                               // kernel dimension of L distinct roots
    if (L == 2) {                           // y = X:         y^2 + a y = b
        A4 = 0; A2 = 1; A1 = a; delta = b; want = 1;
    } else if (L == 3) {                    // y = X + a:     y^4 + (a^2 + b) y^2 + (ab + c) y = 0, y != 0
        A4 = 1; A2 = f.sq(a) ^ b; A1 = f.mul(a, b) ^ c; delta = 0; want = 2; s = a;
    } else if (a == 0) {                    // y = X:         y^4 + b y^2 + c y = d
        A4 = 1; A2 = b; A1 = c; delta = d; want = 2;
    } else {                                // X = s + 1/y, s^2 = c/a:  y^4 + (as + b)/e y^2 + a/e y = 1/e
        s = f.sqrt(f.div(c, a));
        const uint32_t s2 = f.sq(s);
        const uint32_t e = f.sq(s2) ^ f.mul(a, f.mul(s2, s)) ^ f.mul(b, s2) ^ f.mul(c, s) ^ d;
        if (!e) return 0;                   // X = s is a double root
        const uint32_t ie = f.inv(e);
        A4 = 1; A2 = f.mul(f.mul(a, s) ^ b, ie); A1 = f.mul(a, ie); delta = ie; want = 2;
    }
    uint32_t y0, k1, k2;
    if (solve_affine<MM>(f, m, A4, A2, A1, delta, y0, k1, k2) != want) return 0;
    // L = 2: y0, y0 + k1; L = 3 (y0 = 0): the three nonzero kernel elements + s; L = 4: the four
    // solutions y, X = 1/y + s (a != 0) or y.  Selects, every X[i] written: a store per case
    // would be merged into one indexed by L, in scratch memory.
    const bool l3 = L == 3, inv = L == 4 && a;
    const uint32_t y[4] = {l3 ? k1 : y0, l3 ? k2 : y0 ^ k1, l3 ? k1 ^ k2 : y0 ^ k2, y0 ^ k1 ^ k2};
#pragma unroll
    for (int i = 0; i < 4; ++i) X[i] = inv ? f.inv(y[i] ? y[i] : 1u) ^ s : (l3 ? y[i] ^ s : y[i]);
    return L;
}

// Chien search over the codeword's bit positions p < nbits: X = alpha^p is a root of
// sigma(X) = sum_j C_j X^(L-j).  Returns the number of roots (their p in P[0..min(cnt,T)).
template <int T>
__device__ int chien(const GF &f, const uint32_t (&C)[2 * T + 2], int L, uint32_t nbits,
                     uint32_t (&P)[T]) {
    int lt[T + 1];
#pragma unroll
    for (int j = 0; j <= T; ++j) lt[j] = (j <= L && C[j]) ? (int)f.lg[C[j]] : -1;
    int cnt = 0;
    for (uint32_t p = 0; p < nbits; ++p) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j <= T; ++j)
            if (lt[j] >= 0) {
                v ^= f.ex[lt[j]];
                lt[j] += L - j;
                if (lt[j] >= f.n) lt[j] -= f.n;
            }
        if (!v) {
#pragma unroll
            for (int i = 0; i < T; ++i)
                if (i == cnt) P[i] = p;
            ++cnt;
        }
    }
    return cnt;
}

template <int J, int W>
__device__ __forceinline__ uint32_t coef(const uint32_t (&C)[W]) {
    if constexpr (J < W) return C[J];
    else return 0u;
}

// decode_bch on the masked ECC difference r (left-justified): the count and the ascending error
// locations, or -EBADMSG.
template <int T, int NW, int MM = 0>
__device__ int locate(const DevBch &b, const GF &f, Rem<NW> r, uint32_t nbits,
                      uint32_t (&loc)[T], const uint32_t *sin = nullptr) {
    uint64_t any = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) any |= r.w[i];
    if (!any && !sin) return 0;             // only unused ECC bits differ
    const uint32_t n = (uint32_t)b.n;
    uint32_t S[2 * T + 1];
#pragma unroll
    for (int j = 0; j <= 2 * T; ++j) S[j] = (sin && j > 0) ? sin[j - 1] : 0u;
    if (sin) {                              // a caller's syndrome outside GF(2^m) indexes no table
        uint32_t bad = 0;
#pragma unroll
        for (int j = 1; j <= 2 * T; ++j) bad |= S[j] > n;
        if (bad) return -EINVAL;
    }
    bool tab = false;
    if constexpr (NW == 1 && T <= 4) {
        if (b.syn_tab && !sin) {            // the odd syndromes are GF(2)-linear in the remainder's
            tab = true;                     // bits: one table entry per remainder byte
            uint64_t acc = 0;
            for (int bb = 0; bb < b.ecc_bytes; ++bb)
                acc ^= b.syn_tab[bb * 256 + (uint32_t)((r.w[0] >> (56 - 8 * bb)) & 255u)];
#pragma unroll
            for (int j = 1; j < 2 * T; j += 2) S[j] = (uint32_t)(acc >> (8 * (j - 1))) & 0xFFFFu;
        }
    }
#pragma unroll
    for (int wi = 0; wi < NW && !sin && !tab; ++wi) {
        uint64_t x = r.w[wi];
        while (x) {                         // S_j = r(alpha^j), j odd
            const int lz = __clzll(x);
            x &= ~(0x8000000000000000ull >> lz);
            const uint32_t p = (uint32_t)(b.ecc_bits - 1 - (64 * wi + lz));
            uint32_t p2 = 2 * p;
            if (p2 >= n) p2 -= n;
            uint32_t e = p;
#pragma unroll
            for (int j = 1; j < 2 * T; j += 2) {
                S[j] ^= f.ex[e];
                e += p2;
                if (e >= n) e -= n;
            }
        }
    }
    if (!sin) {
#pragma unroll
        for (int j = 1; j <= T; ++j) S[2 * j] = f.sq(S[j]);
    }

    // Berlekamp-Massey; for a binary code the even-step discrepancies vanish.  B holds x^m B.
    constexpr int W = 2 * T + 2;
    uint32_t C[W], B[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        C[j] = j == 0;
        B[j] = j == 1;
    }
    int L = 0;
    // Log domain: the syndromes' logs once (an even one is twice the log of its half), the
    // discrepancy's quotient by its log, and only the coefficients that can be nonzero: before odd
    // step rr, deg C <= rr - 1 and deg B <= rr (B = x at rr = 1; C + q B, x^2 C, x^2 B keep it),
    // so the update touches C[1..rr].
    constexpr uint32_t kNoLog = 0xFFFFu;
    uint32_t lS[2 * T + 1];
#pragma unroll
    for (int j = 1; j <= 2 * T; ++j) {
        if (j % 2 || sin) {                 // a caller's even syndromes are taken as given
            lS[j] = S[j] ? (uint32_t)f.lg[S[j]] : kNoLog;
        } else {
            const uint32_t h = lS[j / 2];
            lS[j] = h == kNoLog ? kNoLog : (2 * h >= n ? 2 * h - n : 2 * h);
        }
    }
    uint32_t lbd = 0;                       // log of the last nonzero discrepancy (bd = 1)
#pragma unroll
    for (int rr = 1; rr < 2 * T; rr += 2) {
        uint32_t d = S[rr];
#pragma unroll
        for (int i = 1; i < rr; ++i)
            if (C[i] && lS[rr - i] != kNoLog) d ^= f.ex[f.lg[C[i]] + lS[rr - i]];
        if (d) {
            const bool grow = 2 * L <= rr - 1;
            const uint32_t ld = f.lg[d];
            const uint32_t lq = ld >= lbd ? ld - lbd : ld + n - lbd;    // log (d / bd)
            uint32_t old[W];
#pragma unroll
            for (int j = 0; j < W; ++j) old[j] = C[j];
#pragma unroll
            for (int j = 1; j <= rr && j < W; ++j)
                if (B[j]) C[j] ^= f.ex[lq + f.lg[B[j]]];
            if (grow) {
                L = rr - L;
                lbd = ld;
            }
#pragma unroll
            for (int j = W - 1; j >= 0; --j) B[j] = j >= 2 ? (grow ? old[j - 2] : B[j - 2]) : 0u;
        } else {
#pragma unroll
            for (int j = W - 1; j >= 0; --j) B[j] = j >= 2 ? B[j - 2] : 0u;
        }
    }
    if (L > T) return -kEBADMSG;
    if (L == 0) return 0;
    uint32_t lead = 0;
#pragma unroll
    for (int j = 0; j <= T; ++j)
        if (j == L) lead = C[j];
    if (!lead) return -kEBADMSG;            // the length exceeds the locator's true degree

    uint32_t P[T];                          // root exponents: X = alpha^P
    int nr = 0;
    if (L == 1) {
        P[0] = f.lg[C[1]];
        nr = 1;
    } else if (L <= 4) {
        uint32_t X[4];
        nr = small_roots<MM>(f, b.m, L, C[1], C[2], coef<3>(C), coef<4>(C), X);
#pragma unroll
        for (int i = 0; i < T && i < 4; ++i)
            if (i < nr) P[i] = f.lg[X[i]];
    } else {
        if constexpr (T > 4) nr = chien<T>(f, C, L, nbits, P);
    }
    if (nr != L) return -kEBADMSG;

    uint32_t el[T];
    bool ok = true;
#pragma unroll
    for (int i = 0; i < T; ++i) {
        el[i] = 0xFFFFFFFFu;
        if (i < L) {
            if (P[i] >= nbits) {
                ok = false;
            } else {
                const uint32_t e = nbits - 1 - P[i];
                el[i] = (e & ~7u) | (7u - (e & 7u));
            }
        }
    }
    if (!ok) return -kEBADMSG;
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j + 1 < T - i; ++j) {
            const uint32_t x = el[j], y = el[j + 1];
            el[j] = x < y ? x : y;
            el[j + 1] = x < y ? y : x;
        }
#pragma unroll
    for (int i = 0; i < T; ++i) loc[i] = el[i];
    return L;
}

// One codeword of k_bch_decode<T, NW>; with `fix` (lds_fix) its corrections go to the staged image
// (row: this lane's row in it) instead of the rows in global memory, and loc[0 .. cnt_out) are
// left for write_pieces.
template <int T, int NW>
__device__ __forceinline__ void decode_one(const DevBch &b, const BchArgs &a, uint8_t *smem, const uint8_t *row,
                                           size_t k, uint8_t *rows, bool fix, uint32_t (&loc)[T], int &cnt_out) {
    if (8ull * a.len > (unsigned long long)(b.n - b.ecc_bits)) {   // decode_bch's length check
        a.result[k] = -kEINVAL;
        return;
    }
    if (a.syn) {                                        // syndrome form: locations only
        const uint16_t *sx = reinterpret_cast<const uint16_t *>(smem + tabs_offset(b));
        const GF f{b.lds_tabs ? sx : b.ex, b.lds_tabs ? sx + 2 * b.n : b.lg, b.n};
        Rem<NW> z;
#pragma unroll
        for (int i = 0; i < NW; ++i) z.w[i] = 0;
        uint32_t loc[T];
        const int cnt = locate<T, NW>(b, f, z, 8u * a.len + (uint32_t)b.ecc_bits, loc, a.syn + k * a.sstride);
        a.result[k] = cnt;
        if (a.errloc)
            for (int i = 0; i < cnt; ++i) a.errloc[k * a.lstride + i] = loc[i];
        return;
    }
    uint8_t *d = a.ecc_only ? nullptr : a.wdata + k * a.dstride, *e = a.ecc + k * a.estride;
    const uint8_t *er = fix ? row + a.len : e;           // the received ECC (staged when inline)
    Rem<NW> r;
    if (a.ecc_only) {
#pragma unroll
        for (int i = 0; i < NW; ++i) r.w[i] = 0;
    } else {
        r = data_remainder<NW>(reinterpret_cast<const uint64_t *>(smem), row, a.len);
    }
    for (int i = 0; i < b.ecc_bytes && (i >> 3) < NW; ++i)    // bytes past NW words: unused bits
        r.w[i >> 3] ^= (uint64_t)er[i] << (56 - 8 * (i & 7));
    uint64_t any = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) any |= r.w[i];
    if (!any) {
        a.result[k] = 0;
        return;
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) r.w[i] &= b.emask[i];
    const uint16_t *sx = reinterpret_cast<const uint16_t *>(smem + tabs_offset(b));
    const GF f{b.lds_tabs ? sx : b.ex, b.lds_tabs ? sx + 2 * b.n : b.lg, b.n};
    const int cnt = locate<T, NW>(b, f, r, 8u * a.len + (uint32_t)b.ecc_bits, loc);
    a.result[k] = cnt;
    if (fix && cnt > 0) cnt_out = cnt;
#pragma unroll
    for (int i = 0; i < T; ++i) {
        if (i < cnt) {
            const uint32_t el = loc[i];
            if (a.errloc) a.errloc[k * a.lstride + i] = el;
            if (a.ecc_only) continue;
            if (fix) fix_bit_lds(rows, row, el);
            else if (el < 8u * a.len) d[el >> 3] ^= (uint8_t)(1u << (el & 7));
            else e[(el >> 3) - a.len] ^= (uint8_t)(1u << (el & 7));
        }
    }
}

template <int T, int NW>
__global__ void __launch_bounds__(kThreads) k_bch_decode(DevBch b, BchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    stage_tables(b, smem, true);
    const uint8_t *row = a.ecc_only ? nullptr : block_rows(smem, b, true, a);
    const size_t k = (size_t)blockIdx.x * kThreads + threadIdx.x;
    uint8_t *rows = smem + rows_offset(b, true);
    uint32_t loc[T];
    int cnt = 0;
    if (k < a.ncw) decode_one<T, NW>(b, a, smem, row, k, rows, a.lds_fix != 0, loc, cnt);
    if (!a.lds_fix) return;                             // (uniform over the block)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    write_pieces<T>(rows, row, loc, cnt, b, a);
}

// ---- plane-sliced codecs, ECC inline (C5): the fused decode ------------------------------------
// The encode's tile loop (ezbch_ps_tile.hpp) leaves each row's remainder XOR its received ECC in
// registers; a nonzero one is located (locate<T, 1>, the GF tables staged in LDS), its bits are
// flipped in the tile's LDS image, and after a workgroup barrier each row writes back the 16-byte
// pieces of the global grid that hold its flips -- a piece reaching outside the tile's bytes only
// over the tile's own, byte by byte.  One pass over the rows: read once, corrected pieces written.
// One tile image per workgroup and three workgroups per CU: the per-row locate is a chain of
// dependent table reads, and a third wave per SIMD hides more of it than a second image hides of
// the DMA (8 M: 0.644 vs 0.780 ms with two images and two workgroups per CU, r06r)
constexpr int kDecSlots = 1;
constexpr int kDecLds = kDecSlots * ezrs::bps::kImgSlot + ezrs::bps::kTW * ezrs::bps::kXch;
constexpr int kDecPerCu = 3;                   // workgroups per CU (LDS)

template <class C>
__global__ void __launch_bounds__(64 * ezrs::bps::kTW, kDecPerCu) k_bch_ps_decode(DevBch b, BchArgs a, BpsArgs p) {
    namespace bp = ezrs::bps;
    constexpr int TW = bp::tile_waves<C>(), T = C::T, NR = 4 / TW;
    constexpr uint32_t n = (1u << C::M) - 1;
    static_assert(T <= 4, "odd syndromes S1 .. S7 from the nibble tables");
    constexpr uint32_t kTabs = ((3 * n + 1) * 2 + 15) / 16 * 16, kNib = 2 * C::EB * 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDecLds + kTabs + 8 * kNib];
    uint16_t *ex = reinterpret_cast<uint16_t *>(lds + kDecLds), *lg = ex + 2 * n;
    // syndrome tables by nibble of the remainder (from the top): the byte tables are linear in the
    // byte, so nibble q's entry for v is the byte table's for v << 4 (q even) or v
    uint64_t *nib = reinterpret_cast<uint64_t *>(lds + kDecLds + kTabs);
    for (uint32_t i = threadIdx.x; i < 2 * n; i += blockDim.x) ex[i] = b.ex[i];
    for (uint32_t i = threadIdx.x; i <= n; i += blockDim.x) lg[i] = b.lg[i];
    for (uint32_t i = threadIdx.x; i < kNib; i += blockDim.x) {
        const uint32_t q = i >> 4, v = i & 15u;
        nib[i] = b.syn_tab[(q >> 1) * 256 + ((q & 1) ? v : v << 4)];
    }
    __syncthreads();
    const GF f{ex, lg, (int)n};
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = bp::lane_id();
    const uint32_t nbits = 8u * a.len + (uint32_t)b.ecc_bits, tb = bp::kRows * p.stride;
    // rows 4l + k, k = w (TW = 4) or 2w, 2w + 1
    bp::tile_loop<C, true, -1, kDecSlots>(p, lds, [&](uint32_t tile, uint8_t *image, const uint32_t (&out)[C::EB]) {
        uint32_t loc[NR][T];
        int cnt[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const uint32_t k = NR * w + j, r = 4u * l + k;
            const size_t row = (size_t)tile * bp::kRows + r;
            cnt[j] = 0;
            if (row >= a.ncw) continue;
            uint32_t wd[2];
            bp::row_bytes<C::EB>(out, k, wd);
            Rem<1> rm;
            rm.w[0] = (((uint64_t)__builtin_bswap32(wd[0]) << 32) | __builtin_bswap32(wd[1])) & b.emask[0];
            int c = 0;
            if (rm.w[0]) {
                uint64_t acc = 0;
#pragma unroll
                for (uint32_t q = 0; q < 2 * C::EB; ++q) acc ^= nib[q * 16 + (uint32_t)((rm.w[0] >> (60 - 4 * q)) & 15u)];
                uint32_t S[2 * T];                          // S_1 .. S_2T; S_2j = S_j^2
#pragma unroll
                for (int jj = 1; jj < 2 * T; jj += 2) S[jj - 1] = (uint32_t)(acc >> (8 * (jj - 1))) & 0xFFFFu;
#pragma unroll
                for (int jj = 1; jj <= T; ++jj) S[2 * jj - 1] = f.sq(S[jj - 1]);
                c = locate<T, 1, C::M>(b, f, rm, nbits, loc[j], S);
            }
            a.result[row] = c;
            if (c <= 0) continue;
            cnt[j] = c;
#pragma unroll
            for (int i = 0; i < T; ++i) {
                if (i >= c) break;
                if (a.errloc) a.errloc[row * a.lstride + i] = loc[j][i];
                const uint32_t o = r * p.stride + (loc[j][i] >> 3);
                atomicXor(reinterpret_cast<uint32_t *>(image + (o & ~3u)), (1u << (loc[j][i] & 7)) << (8 * (o & 3)));
            }
        }
        __syncthreads();                                    // every row's flips are in the image
        const uint32_t toff = tile * tb, hi = p.span - toff < tb ? p.span - toff : tb;
        uint8_t *g = a.wdata + toff;                        // image byte 0
        const uint32_t gmis = (uint32_t)((uintptr_t)g & 15u);
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const uint32_t r = 4u * l + NR * w + j;
            int last = -1000;
#pragma unroll
            for (int i = 0; i < T; ++i) {
                if (i >= cnt[j]) break;
                const uint32_t o = r * p.stride + (loc[j][i] >> 3);
                const int p0 = (int)((o + gmis) & ~15u) - (int)gmis;   // image offset of the piece
                if (p0 == last) continue;
                last = p0;
                if (p0 >= 0 && p0 + 16 <= (int)hi) {
                    uint4 v;
                    __builtin_memcpy(&v, image + p0, 16);
                    *reinterpret_cast<uint4 *>(g + p0) = v;
                } else {
                    for (int q = p0 < 0 ? 0 : p0; q < p0 + 16 && q < (int)hi; ++q) g[q] = image[q];
                }
            }
        }
    });
}

// ---- t > 16 or ecc_bits > 256: the same decode with run-time t ------------------------------
// The working polynomials are per-lane arrays indexed at run time (scratch memory): slower than
// the register-resident k_bch_decode<T, NW>, for the codecs it does not instantiate.

// Chien search over p < nbits, run-time degree L (as chien<T>)
__device__ int chien_big(const GF &f, const uint32_t *C, int L, uint32_t nbits, uint32_t *P, int T) {
    int lt[kBigT + 1];
    for (int j = 0; j <= L; ++j) lt[j] = C[j] ? (int)f.lg[C[j]] : -1;
    int cnt = 0;
    for (uint32_t p = 0; p < nbits; ++p) {
        uint32_t v = 0;
        for (int j = 0; j <= L; ++j)
            if (lt[j] >= 0) {
                v ^= f.ex[lt[j]];
                lt[j] += L - j;
                if (lt[j] >= f.n) lt[j] -= f.n;
            }
        if (!v) {
            if (cnt < T) P[cnt] = p;
            ++cnt;
        }
    }
    return cnt;
}

// locate<T, NW> with run-time t <= kBigT
template <int NW>
__device__ int locate_big(const DevBch &b, const GF &f, Rem<NW> r, uint32_t nbits, uint32_t *loc,
                          const uint32_t *sin = nullptr) {
    uint64_t any = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) any |= r.w[i];
    if (!any && !sin) return 0;
    const int T = b.t;
    const uint32_t n = (uint32_t)b.n;
    uint32_t S[2 * kBigT + 1];
    for (int j = 0; j <= 2 * T; ++j) S[j] = (sin && j > 0) ? sin[j - 1] : 0u;
    if (sin) {                              // a caller's syndrome outside GF(2^m) indexes no table
        uint32_t bad = 0;
        for (int j = 1; j <= 2 * T; ++j) bad |= S[j] > n;
        if (bad) return -EINVAL;
    }
#pragma unroll
    for (int wi = 0; wi < NW && !sin; ++wi) {
        uint64_t x = r.w[wi];
        while (x) {                         // S_j = r(alpha^j), j odd
            const int lz = __clzll(x);
            x &= ~(0x8000000000000000ull >> lz);
            const uint32_t p = (uint32_t)(b.ecc_bits - 1 - (64 * wi + lz));
            uint32_t p2 = 2 * p;
            if (p2 >= n) p2 -= n;
            uint32_t e = p;
            for (int j = 1; j < 2 * T; j += 2) {
                S[j] ^= f.ex[e];
                e += p2;
                if (e >= n) e -= n;
            }
        }
    }
    if (!sin)
        for (int j = 1; j <= T; ++j) S[2 * j] = f.sq(S[j]);
    // Berlekamp-Massey as in locate<T, NW>
    const int W = 2 * T + 2;
    uint32_t C[2 * kBigT + 2], B[2 * kBigT + 2], old[2 * kBigT + 2];
    for (int j = 0; j < W; ++j) {
        C[j] = j == 0;
        B[j] = j == 1;
    }
    int L = 0;
    uint32_t bd = 1;
    for (int rr = 1; rr < 2 * T; rr += 2) {
        uint32_t d = S[rr];
        for (int i = 1; i < rr; ++i) d ^= f.mul(C[i], S[rr - i]);
        if (d) {
            const bool grow = 2 * L <= rr - 1;
            const uint32_t q = f.div(d, bd);
            for (int j = 0; j < W; ++j) {
                old[j] = C[j];
                C[j] ^= f.mul(q, B[j]);
            }
            if (grow) {
                L = rr - L;
                bd = d;
            }
            for (int j = W - 1; j >= 0; --j) B[j] = j >= 2 ? (grow ? old[j - 2] : B[j - 2]) : 0u;
        } else {
            for (int j = W - 1; j >= 0; --j) B[j] = j >= 2 ? B[j - 2] : 0u;
        }
    }
    if (L > T) return -kEBADMSG;
    if (L == 0) return 0;
    if (!C[L]) return -kEBADMSG;
    uint32_t P[kBigT];
    int nr;
    if (L == 1) {
        P[0] = f.lg[C[1]];
        nr = 1;
    } else if (L <= 4) {
        uint32_t X[4];
        nr = small_roots(f, b.m, L, C[1], C[2], C[3], L >= 4 ? C[4] : 0u, X);
        for (int i = 0; i < nr && i < 4; ++i) P[i] = f.lg[X[i]];
    } else {
        nr = chien_big(f, C, L, nbits, P, T);
    }
    if (nr != L) return -kEBADMSG;
    for (int i = 0; i < L; ++i) {
        if (P[i] >= nbits) return -kEBADMSG;
        const uint32_t e = nbits - 1 - P[i];
        const uint32_t el = (e & ~7u) | (7u - (e & 7u));
        int j = i;                          // insertion into the ascending list
        while (j > 0 && loc[j - 1] > el) {
            loc[j] = loc[j - 1];
            --j;
        }
        loc[j] = el;
    }
    return L;
}

template <int NW>
__global__ void __launch_bounds__(kThreads) k_bch_decode_big(DevBch b, BchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    stage_tables(b, smem, true);
    const uint8_t *row = a.ecc_only ? nullptr : block_rows(smem, b, true, a);
    const size_t k = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= a.ncw) return;
    if (8ull * a.len > (unsigned long long)(b.n - b.ecc_bits)) {   // decode_bch's length check
        a.result[k] = -kEINVAL;
        return;
    }
    if (a.syn) {                                        // syndrome form: locations only
        const uint16_t *sx = reinterpret_cast<const uint16_t *>(smem + tabs_offset(b));
        const GF f{b.lds_tabs ? sx : b.ex, b.lds_tabs ? sx + 2 * b.n : b.lg, b.n};
        Rem<NW> z;
#pragma unroll
        for (int i = 0; i < NW; ++i) z.w[i] = 0;
        uint32_t loc[kBigT];
        const int cnt = locate_big<NW>(b, f, z, 8u * a.len + (uint32_t)b.ecc_bits, loc, a.syn + k * a.sstride);
        a.result[k] = cnt;
        if (a.errloc)
            for (int i = 0; i < cnt; ++i) a.errloc[k * a.lstride + i] = loc[i];
        return;
    }
    uint8_t *d = a.ecc_only ? nullptr : a.wdata + k * a.dstride, *e = a.ecc + k * a.estride;
    Rem<NW> r;
    if (a.ecc_only) {
#pragma unroll
        for (int i = 0; i < NW; ++i) r.w[i] = 0;
    } else {
        r = data_remainder<NW>(reinterpret_cast<const uint64_t *>(smem), row, a.len);
    }
    for (int i = 0; i < b.ecc_bytes && (i >> 3) < NW; ++i)    // bytes past NW words: unused bits
        r.w[i >> 3] ^= (uint64_t)e[i] << (56 - 8 * (i & 7));
    uint64_t any = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) any |= r.w[i];
    if (!any) {
        a.result[k] = 0;
        return;
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) r.w[i] &= b.emask[i];
    const uint16_t *sx = reinterpret_cast<const uint16_t *>(smem + tabs_offset(b));
    const GF f{b.lds_tabs ? sx : b.ex, b.lds_tabs ? sx + 2 * b.n : b.lg, b.n};
    uint32_t loc[kBigT];
    const int cnt = locate_big<NW>(b, f, r, 8u * a.len + (uint32_t)b.ecc_bits, loc);
    a.result[k] = cnt;
    for (int i = 0; i < cnt; ++i) {
        const uint32_t el = loc[i];
        if (a.errloc) a.errloc[k * a.lstride + i] = el;
        if (a.ecc_only) continue;
        if (el < 8u * a.len) d[el >> 3] ^= (uint8_t)(1u << (el & 7));
        else e[(el >> 3) - a.len] ^= (uint8_t)(1u << (el & 7));
    }
}

// ---- t > 64 or ecc_bits > 1024: one wavefront per codeword -------------------------------------
// Every init_bch-valid codec (m <= 15: ecc_bits < 32768) runs here.  The remainder is spread over
// the wave, lane l holding 64-bit words l*NWL .. l*NWL+NWL-1 of the left-justified remainder; one
// data byte shifts the whole wave's remainder by 8 bits (the carry from lane l+1 by a lane shuffle)
// and XORs row fb of the byte-step table [256][64 NWL] (global memory, one coalesced row per byte).
// Decode: syndromes lane-parallel over the odd indices (from the set bits of the remainder), even
// ones by one log-table lookup (S_(2^k o) = S_o^(2^k)); binary Berlekamp-Massey with the locator
// and B in LDS (discrepancy as a wave XOR reduction, updates lane-parallel); roots in closed form
// for degree <= 4 (as the lane path), else a lane-parallel Chien search over the bit positions;
// locations rank-sorted ascending.  The per-codeword chains (a byte step, a BM step) are serial,
// so this path is for correctness over the whole parameter range, not the C5 rate.
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v, int d) {
    const uint32_t lo = __shfl_down((uint32_t)v, d, 64), hi = __shfl_down((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d, 64);
    return v;
}
// x mod (2^m - 1) for x < 2^30
__device__ __forceinline__ uint32_t mod_n(uint32_t x, int m, uint32_t n) {
    x = (x & n) + (x >> m);
    x = (x & n) + (x >> m);
    return x >= n ? x - n : x;
}

// Remainder of the data bytes p[0..len): w[j] = word lane*NWL + j.
template <int NWL>
__device__ void wave_remainder(const DevBch &b, const uint8_t *p, unsigned len, uint64_t (&w)[NWL]) {
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int j = 0; j < NWL; ++j) w[j] = 0;
    const size_t nw = (size_t)64 * NWL;
    for (unsigned c0 = 0; c0 < len; c0 += 64) {
        const uint32_t mine = c0 + lane < len ? p[c0 + lane] : 0u;
        const unsigned cnt = len - c0 < 64u ? len - c0 : 64u;
        for (unsigned i = 0; i < cnt; ++i) {
            const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)i);
            const uint32_t fb = ((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(w[0] >> 56), 0) ^ v) & 0xffu;
            const uint64_t nxt = lane == 63 ? 0ull : shfl_down64(w[0], 1);
            const uint64_t *row = b.step + fb * nw + (size_t)lane * NWL;
#pragma unroll
            for (int j = 0; j < NWL; ++j) {
                const uint64_t lo = j + 1 < NWL ? w[j + 1 < NWL ? j + 1 : j] : nxt;
                w[j] = ((w[j] << 8) | (lo >> 56)) ^ row[j];
            }
        }
    }
}

template <int NWL>
__global__ void __launch_bounds__(64) k_bch_encode_wave(DevBch b, BchArgs a) {
    const size_t k = blockIdx.x;
    const int lane = (int)threadIdx.x;
    uint64_t w[NWL];
    wave_remainder<NWL>(b, a.data + k * a.dstride, a.len, w);
    uint8_t *e = a.ecc + k * a.estride;
#pragma unroll
    for (int j = 0; j < NWL; ++j) {
        const int wi = lane * NWL + j;
        for (int bb = 0; bb < 8; ++bb) {
            const int i = 8 * wi + bb;
            if (i < b.ecc_bytes) e[i] = (uint8_t)(w[j] >> (56 - 8 * bb));
        }
    }
}

// Per-wave LDS of the decode: S[0..2t] u16 | C[W] u16 | B[W] u16 | lgC[W] i32 | P[t] u32 | E[t] u32 | cnt
__host__ __device__ inline size_t wave_w(int t) { return ((size_t)2 * t + 2 + 63) / 64 * 64; }
__host__ __device__ inline size_t wave_lds_bytes(int t) {
    return ((size_t)2 * t + 2) * 2 + wave_w(t) * (2 + 2 + 4) + (size_t)t * 8 + 16;
}

template <int NWL>
__global__ void __launch_bounds__(64) k_bch_decode_wave(DevBch b, BchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int T = b.t, lane = (int)threadIdx.x, m = b.m;
    const uint32_t n = (uint32_t)b.n;
    const size_t W = wave_w(T);
    uint16_t *S = reinterpret_cast<uint16_t *>(smem);
    uint16_t *C = S + 2 * T + 2, *B = C + W;
    int32_t *lgC = reinterpret_cast<int32_t *>(B + W);
    uint32_t *P = reinterpret_cast<uint32_t *>(lgC + W), *E = P + T;
    const GF f{b.ex, b.lg, b.n};
    const size_t k = blockIdx.x;
    if (8ull * a.len > (unsigned long long)(b.n - b.ecc_bits)) {   // decode_bch's length check
        if (lane == 0) a.result[k] = -kEINVAL;
        return;
    }
    const uint32_t nbits = 8u * a.len + (uint32_t)b.ecc_bits;
    uint8_t *d = a.ecc_only ? nullptr : a.wdata + k * a.dstride, *e = a.ecc + k * a.estride;
    // syndromes S_1 .. S_2t
    if (a.syn) {
        const uint32_t *sin = a.syn + k * a.sstride;
        uint32_t bad = 0;
        for (int j = 1 + lane; j <= 2 * T; j += 64) {
            const uint32_t v = sin[j - 1];
            bad |= v > n;
            S[j] = (uint16_t)v;
        }
        if (__ballot(bad != 0)) {
            if (lane == 0) a.result[k] = -kEINVAL;
            return;
        }
    } else {
        uint64_t w[NWL];
        if (a.ecc_only) {
#pragma unroll
            for (int j = 0; j < NWL; ++j) w[j] = 0;
        } else {
            wave_remainder<NWL>(b, a.data + k * a.dstride, a.len, w);
        }
        uint64_t any = 0;
#pragma unroll
        for (int j = 0; j < NWL; ++j) {
            const int wi = lane * NWL + j;
            for (int bb = 0; bb < 8; ++bb) {               // XOR the received ECC (big-endian words)
                const int i = 8 * wi + bb;
                if (i < b.ecc_bytes) w[j] ^= (uint64_t)e[i] << (56 - 8 * bb);
            }
            const int hi = b.ecc_bits - 64 * wi;           // significant bits of word wi
            w[j] &= hi >= 64 ? ~0ull : hi <= 0 ? 0ull : ~0ull << (64 - hi);
            any |= w[j];
        }
        if (!__ballot(any != 0)) {
            if (lane == 0) a.result[k] = 0;
            return;
        }
        // odd S_j from the set bits (powers p) of the remainder, lane-parallel over j
        for (int j0 = 1; j0 < 2 * T; j0 += 128) {
            const int j = j0 + 2 * lane;
            uint32_t acc = 0;
#pragma unroll
            for (int jj = 0; jj < NWL; ++jj)
                for (int ls = 0; ls < 64; ++ls) {
                    uint64_t x = readlane64(w[jj], ls);
                    const int wi = ls * NWL + jj;
                    while (x) {
                        const int lz = __clzll(x);
                        x &= ~(0x8000000000000000ull >> lz);
                        const uint32_t pw = (uint32_t)(b.ecc_bits - 1 - (64 * wi + lz));
                        if (j < 2 * T) acc ^= f.ex[mod_n((uint32_t)j * pw, m, n)];
                    }
                }
            if (j < 2 * T) S[j] = (uint16_t)acc;
        }
        __syncthreads();
        // even S_(2^k o) = S_o^(2^k): one lookup each
        for (int j = 2 + 2 * lane; j <= 2 * T; j += 128) {
            int o = j, sh = 0;
            while (!(o & 1)) { o >>= 1; ++sh; }
            const uint32_t so = S[o];
            S[j] = so ? (uint16_t)f.ex[mod_n((uint32_t)f.lg[so] << sh, m, n)] : (uint16_t)0;
        }
    }
    __syncthreads();
    // Berlekamp-Massey (as locate_big): C = 1, B = x
    for (size_t j = lane; j < W; j += 64) {
        C[j] = j == 0;
        B[j] = j == 1;
    }
    __syncthreads();
    int L = 0;
    uint32_t bd = 1;
    for (int rr = 1; rr < 2 * T; rr += 2) {
        uint32_t part = 0;
        const int top = L < rr - 1 ? L : rr - 1;
        for (int i = 1 + lane; i <= top; i += 64) part ^= f.mul(C[i], S[rr - i]);
        const uint32_t dd = S[rr] ^ wave_xor(part);
        const int ch = (int)(W / 64);
        if (dd) {
            const bool grow = 2 * L <= rr - 1;
            const uint32_t q = f.div(dd, bd);
            for (int c = ch - 1; c >= 0; --c) {            // top-down: [j-2] still holds the old values
                const int j = 64 * c + lane;
                const uint32_t cj = C[j], bj = B[j], c2 = j >= 2 ? C[j - 2] : 0u, b2 = j >= 2 ? B[j - 2] : 0u;
                __syncthreads();
                C[j] = (uint16_t)(cj ^ f.mul(q, bj));
                B[j] = (uint16_t)(j >= 2 ? (grow ? c2 : b2) : 0u);
                __syncthreads();
            }
            if (grow) {
                L = rr - L;
                bd = dd;
            }
        } else {
            for (int c = ch - 1; c >= 0; --c) {
                const int j = 64 * c + lane;
                const uint32_t b2 = j >= 2 ? B[j - 2] : 0u;
                __syncthreads();
                B[j] = (uint16_t)b2;
                __syncthreads();
            }
        }
    }
    int res;
    if (L > T || (L > 0 && !C[L])) {
        res = -kEBADMSG;
    } else if (L == 0) {
        res = 0;
    } else {
        int nr;
        if (L <= 4) {
            if (L == 1) {
                if (lane == 0) P[0] = f.lg[C[1]];
                nr = 1;
            } else {
                uint32_t X[4];
                nr = small_roots(f, m, L, C[1], C[2], C[3], L >= 4 ? C[4] : 0u, X);
                if (lane == 0)
                    for (int i = 0; i < nr && i < 4; ++i) P[i] = f.lg[X[i]];
            }
        } else {
            for (size_t j = lane; j <= (size_t)L; j += 64) lgC[j] = C[j] ? (int32_t)f.lg[C[j]] : -1;
            __syncthreads();
            nr = 0;
            for (uint32_t p0 = 0; p0 < nbits && nr < L; p0 += 64) {
                const uint32_t pp = p0 + lane;
                uint32_t v = 0;
                for (int j = 0; j <= L; ++j) {
                    const int lc = lgC[j];
                    if (lc >= 0) v ^= f.ex[mod_n((uint32_t)lc + mod_n((uint32_t)(L - j) * pp, m, n), m, n)];
                }
                const uint64_t hit = __ballot(pp < nbits && v == 0);
                if (hit) {
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(hit >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)hit, 0u));
                    if ((hit >> lane) & 1 && nr + (int)below < T) P[nr + below] = pp;
                    nr += __popcll(hit);
                }
            }
        }
        __syncthreads();
        res = L;
        if (nr != L) res = -kEBADMSG;
        else {
            uint32_t bad = 0;
            for (int i = lane; i < L; i += 64) bad |= P[i] >= nbits;
            if (__ballot(bad != 0)) res = -kEBADMSG;
        }
        if (res > 0) {
            // error bit e = nbits-1-P, reported as (e & ~7) | (7 - e & 7); rank-sort ascending
            for (int i = lane; i < L; i += 64) {
                const uint32_t ei = nbits - 1 - P[i], el = (ei & ~7u) | (7u - (ei & 7u));
                int rank = 0;
                for (int q2 = 0; q2 < L; ++q2) {
                    const uint32_t eq = nbits - 1 - P[q2], lq = (eq & ~7u) | (7u - (eq & 7u));
                    rank += lq < el;
                }
                E[rank] = el;
            }
            __syncthreads();
            if (a.errloc)
                for (int i = lane; i < L; i += 64) a.errloc[k * a.lstride + i] = E[i];
            if (!a.ecc_only && !a.syn && lane == 0)
                for (int i = 0; i < L; ++i) {                  // serial: two errors may share a byte
                    const uint32_t el = E[i];
                    if (el < 8u * a.len) d[el >> 3] ^= (uint8_t)(1u << (el & 7));
                    else e[(el >> 3) - a.len] ^= (uint8_t)(1u << (el & 7));
                }
        }
    }
    if (lane == 0) a.result[k] = res;
}

// The wavefront-per-codeword kernels take one workgroup per codeword: batches go in chunks of at
// most kWaveChunk codewords, so the grid stays far below the 2^32-thread launch limit.
constexpr size_t kWaveChunk = (size_t)1 << 24;

BchArgs wave_chunk(const BchArgs &a, size_t k0) {
    BchArgs c = a;
    c.ncw = a.ncw - k0 < kWaveChunk ? a.ncw - k0 : kWaveChunk;
    if (c.data) c.data += k0 * a.dstride;
    if (c.wdata) c.wdata += k0 * a.dstride;
    if (c.ecc) c.ecc += k0 * a.estride;
    if (c.result) c.result += k0;
    if (c.errloc) c.errloc += k0 * a.lstride;
    if (c.syn) c.syn += k0 * a.sstride;
    return c;
}

// Launches of the plane-sliced kernels over a batch: 256-row tiles, every byte offset of a launch
// below 0xE0000000 (32-bit buffer offsets).
template <class F>
hipError_t bps_chunks(const BchArgs &a, F &&launch) {
    const size_t pitch = a.dstride > a.estride ? a.dstride : a.estride;
    size_t per = (size_t)0xE0000000u / (pitch ? pitch : 1) / 256 * 256;
    if (per > ((size_t)1 << 28)) per = (size_t)1 << 28;       // 8-byte remainders: 32-bit offsets
    if (per == 0) per = 256;
    for (size_t k0 = 0; k0 < a.ncw; k0 += per) {
        const size_t n = a.ncw - k0 < per ? a.ncw - k0 : per;
        const hipError_t e = launch(k0, n);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// The plane-sliced path takes rows of its frame (encode: data <= F bytes, decode: data + ECC) at a
// pitch of at most 128 bytes; decode also needs the ECC right after the data (the row is one
// polynomial).
bool bps_ok(const DevBch &b, const BchArgs &a, bool dec) {
    if (b.bps < 0 || a.ecc_only || a.syn || a.len == 0 || a.dstride > 128 || a.ncw == 0) return false;
    if (8ull * a.len > (unsigned long long)(b.n - b.ecc_bits)) return false;
    if ((int)(a.len + (dec ? b.ecc_bytes : 0)) > bps_frame(b.bps)) return false;
    if (dec && !(a.ecc == a.data + a.len && a.estride == a.dstride)) return false;
    if (!dec && (a.estride < b.ecc_bytes || a.estride > 4096)) return false;
    return a.dstride >= a.len;
}

hipError_t launch_encode(const DevBch &b, BchArgs a, hipStream_t s) {
    if (bps_ok(b, a, false)) {
        return bps_chunks(a, [&](size_t k0, size_t n) {
            const BpsArgs p{a.data + k0 * a.dstride, (uint32_t)((n - 1) * a.dstride + a.len), (uint32_t)a.dstride,
                            (uint32_t)n, (uint32_t)((n + 255) / 256), bps_frame(b.bps) - (int)a.len,
                            a.ecc + k0 * a.estride, a.estride,
                            (uint32_t)((n - 1) * a.estride + b.ecc_bytes)};
            return launch_bps(b.bps, p, b.ncu, s);
        });
    }
    if (b.nwl) {
        for (size_t k0 = 0; k0 < a.ncw; k0 += kWaveChunk) {      // one workgroup per codeword
            const BchArgs c = wave_chunk(a, k0);
            const unsigned g = (unsigned)c.ncw;
            if (b.nwl == 1) hipLaunchKernelGGL(k_bch_encode_wave<1>, dim3(g), dim3(64), 0, s, b, c);
            else if (b.nwl == 2) hipLaunchKernelGGL(k_bch_encode_wave<2>, dim3(g), dim3(64), 0, s, b, c);
            else if (b.nwl == 4) hipLaunchKernelGGL(k_bch_encode_wave<4>, dim3(g), dim3(64), 0, s, b, c);
            else hipLaunchKernelGGL(k_bch_encode_wave<8>, dim3(g), dim3(64), 0, s, b, c);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const unsigned grid = (unsigned)((a.ncw + kThreads - 1) / kThreads);
    a.staged = want_staging(b, false, a);
    const size_t sh = lds_bytes(b, false, a);
    if (b.nw == 1) hipLaunchKernelGGL(k_bch_encode<1>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else if (b.nw == 2) hipLaunchKernelGGL(k_bch_encode<2>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else if (b.nw == 4) hipLaunchKernelGGL(k_bch_encode<4>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else if (b.nw == 8) hipLaunchKernelGGL(k_bch_encode<8>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else hipLaunchKernelGGL(k_bch_encode<16>, dim3(grid), dim3(kThreads), sh, s, b, a);
    return hipGetLastError();
}

hipError_t launch_bps_decode(const DevBch &b, const BchArgs &a, const BpsArgs &p, hipStream_t s) {
    const unsigned cap = (unsigned)kDecPerCu * (unsigned)(b.ncu > 0 ? b.ncu : 256);
    const unsigned grid = p.ntiles < cap ? p.ntiles : cap;
    if (!grid) return hipSuccess;
    int k = 0;
#define EZBCH_PS_DECODE(N, M, T)                                                                     \
    if (k++ == b.bps)                                                                                \
        hipLaunchKernelGGL((k_bch_ps_decode<ezrs::bps::BPS_##N>), dim3(grid),                       \
                           dim3(64 * ezrs::bps::tile_waves<ezrs::bps::BPS_##N>()), 0, s, b, a, p);
    EZBCH_PS_CODEC_LIST(EZBCH_PS_DECODE)
#undef EZBCH_PS_DECODE
    return hipGetLastError();
}

hipError_t launch_decode(const DevBch &b, BchArgs a, hipStream_t s) {
    if (bps_ok(b, a, true) && ecc_inline(b, a)) {            // packed rows, ECC inline: fused decode
        return bps_chunks(a, [&](size_t k0, size_t n) {
            BchArgs c = a;
            c.ncw = n;
            c.data += k0 * a.dstride;
            c.wdata += k0 * a.dstride;
            c.ecc += k0 * a.estride;
            c.result += k0;
            if (c.errloc) c.errloc += k0 * a.lstride;
            const BpsArgs p{c.data, (uint32_t)((n - 1) * a.dstride + a.len + b.ecc_bytes), (uint32_t)a.dstride,
                            (uint32_t)n, (uint32_t)((n + 255) / 256), bps_frame(b.bps) - (int)(a.len + b.ecc_bytes),
                            nullptr, 0, 0};
            return launch_bps_decode(b, c, p, s);
        });
    }
    if (b.nwl) {
        const size_t sh = wave_lds_bytes(b.t);
        for (size_t k0 = 0; k0 < a.ncw; k0 += kWaveChunk) {      // one workgroup per codeword
            const BchArgs c = wave_chunk(a, k0);
            const unsigned g = (unsigned)c.ncw;
            if (b.nwl == 1) hipLaunchKernelGGL(k_bch_decode_wave<1>, dim3(g), dim3(64), sh, s, b, c);
            else if (b.nwl == 2) hipLaunchKernelGGL(k_bch_decode_wave<2>, dim3(g), dim3(64), sh, s, b, c);
            else if (b.nwl == 4) hipLaunchKernelGGL(k_bch_decode_wave<4>, dim3(g), dim3(64), sh, s, b, c);
            else hipLaunchKernelGGL(k_bch_decode_wave<8>, dim3(g), dim3(64), sh, s, b, c);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const unsigned grid = (unsigned)((a.ncw + kThreads - 1) / kThreads);
    a.lds_fix = !a.ecc_only && !a.syn && ecc_inline(b, a) && b.t <= 16 && b.nw <= 4;  // k_bch_decode<T, NW>
    a.staged = a.ecc_only ? 0 : want_staging(b, true, a);
    if (!a.staged) a.lds_fix = 0;
    const size_t sh = lds_bytes(b, true, a);
    // (T, NW) instantiations: NW = 1 for ecc_bits <= 64 (t <= 12 since m >= 5), NW = 2 for
    // ecc_bits <= 128 (m t > 64: t >= 5), NW = 4 for ecc_bits <= 256 (t >= 9)
#define EZBCH_CASE(T, NW)                                                                     \
    if (b.t == T && b.nw == NW) {                                                             \
        hipLaunchKernelGGL((k_bch_decode<T, NW>), dim3(grid), dim3(kThreads), sh, s, b, a);   \
        return hipGetLastError();                                                             \
    }
    EZBCH_CASE(1, 1) EZBCH_CASE(2, 1) EZBCH_CASE(3, 1) EZBCH_CASE(4, 1) EZBCH_CASE(5, 1)
    EZBCH_CASE(6, 1) EZBCH_CASE(7, 1) EZBCH_CASE(8, 1) EZBCH_CASE(9, 1) EZBCH_CASE(10, 1)
    EZBCH_CASE(11, 1) EZBCH_CASE(12, 1)
    EZBCH_CASE(5, 2) EZBCH_CASE(6, 2) EZBCH_CASE(7, 2) EZBCH_CASE(8, 2) EZBCH_CASE(9, 2)
    EZBCH_CASE(10, 2) EZBCH_CASE(11, 2) EZBCH_CASE(12, 2) EZBCH_CASE(13, 2) EZBCH_CASE(14, 2)
    EZBCH_CASE(15, 2) EZBCH_CASE(16, 2)
    EZBCH_CASE(9, 4) EZBCH_CASE(10, 4) EZBCH_CASE(11, 4) EZBCH_CASE(12, 4) EZBCH_CASE(13, 4)
    EZBCH_CASE(14, 4) EZBCH_CASE(15, 4) EZBCH_CASE(16, 4)
#undef EZBCH_CASE
    // everything else init_bch accepts up to t = 64, ecc_bits = 1024
    if (b.nw == 1) hipLaunchKernelGGL(k_bch_decode_big<1>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else if (b.nw == 2) hipLaunchKernelGGL(k_bch_decode_big<2>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else if (b.nw == 4) hipLaunchKernelGGL(k_bch_decode_big<4>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else if (b.nw == 8) hipLaunchKernelGGL(k_bch_decode_big<8>, dim3(grid), dim3(kThreads), sh, s, b, a);
    else hipLaunchKernelGGL(k_bch_decode_big<16>, dim3(grid), dim3(kThreads), sh, s, b, a);
    return hipGetLastError();
}

// ---- host --------------------------------------------------------------------------------------
thread_local std::string g_err;

int hip_fail(hipError_t e, const char *what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return -ENODEV;
    return -EIO;
}

#define HIP_TRY(expr)                                          \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) return hip_fail(e_, #expr);      \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// init_bch's default primitive polynomials, m = 5..15
const unsigned kDefaultPoly[11] = {0x25, 0x43, 0x83, 0x11d, 0x211, 0x409,
                                   0x805, 0x1053, 0x201b, 0x402b, 0x8003};

// Field tables and generator of init_bch(m, t, poly) (bch_base:49-69); false where init_bch fails.
struct HostBch {
    unsigned m = 0, n = 0, t = 0, poly = 0, ecc_bits = 0, ecc_bytes = 0;
    std::vector<uint16_t> ex, lg;
    std::vector<uint8_t> g;   // generator coefficients, x^0 first

    bool build(unsigned m_, unsigned t_, unsigned poly_) {
        if (m_ < 5 || m_ > 15) return false;
        m = m_;
        n = (1u << m) - 1;
        t = t_;
        if (t < 1 || m * t >= n) return false;
        poly = poly_ ? poly_ : kDefaultPoly[m - 5];
        if ((poly >> m) != 1) return false;
        ex.assign(2 * n, 0);
        lg.assign(n + 1, 0);
        std::vector<char> seen(n + 1, 0);
        for (unsigned i = 0, x = 1; i < n; ++i) {
            if (seen[x]) return false;                  // not primitive
            seen[x] = 1;
            ex[i] = ex[i + n] = (uint16_t)x;
            lg[x] = (uint16_t)i;
            x <<= 1;
            if (x >> m) x ^= poly;
        }
        std::vector<char> root(n, 0);                   // cyclotomic cosets of 1, 3, .., 2t-1
        for (unsigned i = 0; i < t; ++i)
            for (unsigned k = 0, j = 2 * i + 1; k < m; ++k, j = (2 * j) % n) root[j] = 1;
        std::vector<unsigned> gc(1, 1);
        auto mul = [&](unsigned a, unsigned b) -> unsigned { return (a && b) ? ex[lg[a] + lg[b]] : 0u; };
        for (unsigned j = 0; j < n; ++j) {
            if (!root[j]) continue;
            const unsigned r = ex[j];
            gc.push_back(0);
            for (size_t k = gc.size() - 1; k > 0; --k) gc[k] = gc[k - 1] ^ mul(gc[k], r);
            gc[0] = mul(gc[0], r);
        }
        g.resize(gc.size());
        for (size_t k = 0; k < gc.size(); ++k) {
            if (gc[k] > 1) return false;
            g[k] = (uint8_t)gc[k];
        }
        ecc_bits = (unsigned)g.size() - 1;
        ecc_bytes = (m * t + 7) / 8;
        return true;
    }

    // the lane path: t <= 64 and ecc_bits <= 1024; the wave path above
    bool wave() const { return t > (unsigned)kBigT || ecc_bits > 64u * kMaxNW; }
    unsigned nwl() const {
        const unsigned w = (ecc_bits + 63) / 64;             // 64-bit words
        return !wave() ? 0 : w <= 64 ? 1 : w <= 128 ? 2 : w <= 256 ? 4 : 8;
    }
    unsigned words() const {
        if (wave()) return 64 * nwl();
        return ecc_bits <= 64 ? 1 : ecc_bits <= 128 ? 2 : ecc_bits <= 256 ? 4 : ecc_bits <= 512 ? 8 : 16;
    }
    // step[v] = (v x^(E+8 nw 64-8) mod g) left-justified over nw words (w[0] most significant):
    // the remainder update for one data byte; laid out [v][word]
    std::vector<uint64_t> step_table() const {
        const unsigned E = ecc_bits, nw = words(), W = 64 * nw;
        std::vector<uint64_t> gl(nw, 0), tab(256 * nw);
        for (unsigned i = 0; i < E; ++i)
            if (g[i]) {
                const unsigned bit = W - E + i;                  // from the LSB of the whole
                gl[nw - 1 - bit / 64] |= 1ull << (bit % 64);
            }
        for (unsigned v = 0; v < 256; ++v) {
            std::vector<uint64_t> c(nw, 0);
            c[0] = (uint64_t)v << 56;
            for (int k = 0; k < 8; ++k) {
                const bool top = c[0] >> 63;
                for (unsigned i = 0; i < nw; ++i)
                    c[i] = (c[i] << 1) | (i + 1 < nw ? c[i + 1] >> 63 : 0);
                if (top)
                    for (unsigned i = 0; i < nw; ++i) c[i] ^= gl[i];
            }
            for (unsigned i = 0; i < nw; ++i) tab[v * nw + i] = c[i];
        }
        return tab;
    }
};

} // namespace

struct ezbch_codec {
    int device = 0;
    HostBch h;
    DevBch dev{};
    uint64_t *d_step = nullptr;
    uint16_t *d_tabs = nullptr;
    uint64_t *d_syn = nullptr;    // DevBch::syn_tab
    std::mutex mu;                // guards the host-pipeline buffers
    void *d_stage = nullptr;
    size_t stage_bytes = 0;
    void *h_stage = nullptr;      // pinned host staging (gathers, compact ECC)
    size_t hstage_bytes = 0;
    hipStream_t stream = nullptr;
};

namespace {

int create_impl(ezbch_codec **out, unsigned m, unsigned t, unsigned poly, int device, long want_k) {
    if (!out) return -EINVAL;
    *out = nullptr;
    HostBch h;
    if (!h.build(m, t, poly)) {
        g_err = "init_bch: invalid parameters (need 5 <= m <= 15, t >= 1, m*t < 2^m-1, a primitive "
                "polynomial of degree m)";
        return -EINVAL;
    }
    if (want_k >= 0 && (long)(h.n - h.ecc_bits) != want_k) {
        g_err = "BCH<N,K,T>: K does not match the codec init_bch builds (N - ecc_bits)";
        return -EINVAL;
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0 || device < 0 || device >= ndev) {
        g_err = "no usable HIP device";
        return -ENODEV;
    }
    ezbch_codec *c = new (std::nothrow) ezbch_codec;
    if (!c) return -ENOMEM;
    c->device = device;
    c->h = std::move(h);
    DeviceGuard dg(device);
    const std::vector<uint64_t> tab = c->h.step_table();
    const size_t nt = c->h.ex.size() + c->h.lg.size();
    if ((e = hipMalloc(&c->d_step, tab.size() * 8)) != hipSuccess ||
        (e = hipMalloc(&c->d_tabs, nt * sizeof(uint16_t))) != hipSuccess ||
        (e = hipMemcpy(c->d_step, tab.data(), tab.size() * 8, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c->d_tabs, c->h.ex.data(), c->h.ex.size() * 2, hipMemcpyHostToDevice)) !=
            hipSuccess ||
        (e = hipMemcpy(c->d_tabs + c->h.ex.size(), c->h.lg.data(), c->h.lg.size() * 2,
                       hipMemcpyHostToDevice)) != hipSuccess) {
        ezbch_destroy(c);
        return hip_fail(e, "BCH tables");
    }
    DevBch &d = c->dev;
    d.m = (int)m;
    d.n = (int)c->h.n;
    d.t = (int)t;
    d.ecc_bits = (int)c->h.ecc_bits;
    d.ecc_bytes = (int)c->h.ecc_bytes;
    d.lds_tabs = m <= 12;
    d.nw = (int)c->h.words();
    d.nwl = (int)c->h.nwl();
    for (int i = 0; i < kMaxNW && !d.nwl; ++i) {
        const int hi = (int)c->h.ecc_bits - 64 * i;             // significant bits in word i
        d.emask[i] = hi >= 64 ? ~0ull : hi <= 0 ? 0ull : ~0ull << (64 - hi);
    }
    d.step = c->d_step;
    d.ex = c->d_tabs;
    d.lg = c->d_tabs + c->h.ex.size();
    if (!d.nwl && d.nw == 1 && t <= 4) {    // syndrome byte tables (locate<T, 1>)
        std::vector<uint64_t> st(8 * 256, 0);
        const unsigned n = c->h.n, eb = c->h.ecc_bits;
        for (unsigned bb = 0; bb < 8; ++bb)
            for (unsigned v = 0; v < 256; ++v)
                for (unsigned i = 0; i < 8; ++i) {
                    if (!(v >> i & 1)) continue;
                    const unsigned lz = 63 - (56 - 8 * bb + i);      // the bit's leading-zero index
                    if (lz >= eb) continue;                           // masked (unused ECC bits)
                    const unsigned p = eb - 1 - lz;                   // S_j += alpha^(j p)
                    for (unsigned j = 1; j < 2 * t; j += 2)
                        st[bb * 256 + v] ^= (uint64_t)c->h.ex[(uint64_t)j * p % n] << (8 * (j - 1));
                }
        if ((e = hipMalloc(&c->d_syn, st.size() * 8)) != hipSuccess ||
            (e = hipMemcpy(c->d_syn, st.data(), st.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) {
            ezbch_destroy(c);
            return hip_fail(e, "BCH syndrome tables");
        }
        d.syn_tab = c->d_syn;
    }
    d.bps = !d.nwl && c->h.ecc_bits % 8 == 0 && c->h.poly == kDefaultPoly[m - 5]
                ? bps_codec_id((int)m, (int)t, (int)c->h.ecc_bits) : -1;
    if (hipDeviceGetAttribute(&d.ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) d.ncu = 256;
    *out = c;
    return 0;
}

int check_args(const ezbch_codec *c, const uint8_t *data, size_t dstride, unsigned len,
               const uint8_t *ecc, size_t estride, size_t ncw) {
    if (!data || !ecc) return -EINVAL;
    if (ncw > 1 && (estride < c->h.ecc_bytes || dstride < len)) return -EINVAL;
    return 0;
}

// Row form: the ECC follows the data in each row.
int check_rows(const ezbch_codec *c, const uint8_t *rows, size_t stride, unsigned len, size_t ncw) {
    if (!rows) return -EINVAL;
    if (ncw > 1 && stride < (size_t)len + c->h.ecc_bytes) return -EINVAL;
    return 0;
}

int ensure_hstage(ezbch_codec *c, size_t bytes) {
    if (c->hstage_bytes >= bytes) return 0;
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->hstage_bytes = 0;
    HIP_TRY(hipHostMalloc(&c->h_stage, bytes, hipHostMallocDefault));
    c->hstage_bytes = bytes;
    return 0;
}

int ensure_stage(ezbch_codec *c, size_t bytes) {
    if (!c->stream) HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (c->stage_bytes >= bytes) return 0;
    if (c->d_stage) (void)hipFree(c->d_stage);
    c->d_stage = nullptr;
    c->stage_bytes = 0;
    HIP_TRY(hipMalloc(&c->d_stage, bytes));
    c->stage_bytes = bytes;
    return 0;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

} // namespace

extern "C" {

const char *ezbch_last_error(void) { return g_err.c_str(); }

int ezbch_create(ezbch_codec **out, unsigned m, unsigned t, unsigned prim_poly, int device) {
    return create_impl(out, m, t, prim_poly, device, -1);
}

int ezbch_create_nkt(ezbch_codec **out, unsigned n, unsigned k, unsigned t, int device) {
    unsigned m = 0;
    while (m < 16 && ((1u << m) - 1) < n) ++m;
    if (((1u << m) - 1) != n) {
        if (out) *out = nullptr;
        g_err = "BCH<N,K,T>: N must be 2^m - 1";
        return -EINVAL;
    }
    return create_impl(out, m, t, 0, device, (long)k);
}

int ezbch_destroy(ezbch_codec *c) {
    if (!c) return 0;
    DeviceGuard g(c->device);
    if (c->d_step) (void)hipFree(c->d_step);
    if (c->d_tabs) (void)hipFree(c->d_tabs);
    if (c->d_syn) (void)hipFree(c->d_syn);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int ezbch_get_info(const ezbch_codec *c, ezbch_info *info) {
    if (!c || !info) return -EINVAL;
    info->m = c->h.m;
    info->n = c->h.n;
    info->t = c->h.t;
    info->ecc_bits = c->h.ecc_bits;
    info->ecc_bytes = c->h.ecc_bytes;
    info->prim_poly = c->h.poly;
    info->device = c->device;
    return 0;
}

int ezbch_encode(const ezbch_codec *c, const uint8_t *data, size_t data_stride, unsigned len,
                 uint8_t *ecc, size_t ecc_stride, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_args(c, data, data_stride, len, ecc, ecc_stride, ncw)) return r;
    DeviceGuard g(c->device);
    BchArgs a{data, nullptr, data_stride, len, ecc, ecc_stride, nullptr, nullptr, 0, ncw, 0};
    hipError_t e = launch_encode(c->dev, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(e, "BCH encode launch");
}

int ezbch_encode_rows(const ezbch_codec *c, uint8_t *rows, size_t stride, unsigned len,
                      size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_rows(c, rows, stride, len, ncw)) return r;
    return ezbch_encode(c, rows, stride, len, rows + len, stride, ncw, stream);
}

int ezbch_decode(const ezbch_codec *c, uint8_t *data, size_t data_stride, unsigned len,
                 uint8_t *ecc, size_t ecc_stride, int32_t *result, uint32_t *errloc,
                 size_t errloc_stride, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!result) return -EINVAL;
    if (!ecc) {   // ECC inside the row
        if (int r = check_rows(c, data, data_stride, len, ncw)) return r;
        ecc = data + len;
        ecc_stride = data_stride;
    }
    if (int r = check_args(c, data, data_stride, len, ecc, ecc_stride, ncw)) return r;
    if (errloc && ncw > 1 && errloc_stride < c->h.t) return -EINVAL;
    DeviceGuard g(c->device);
    BchArgs a{data, data, data_stride, len, ecc, ecc_stride, result, errloc, errloc_stride, ncw, 0, 0};
    hipError_t e = launch_decode(c->dev, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(e, "BCH decode launch");
}

int ezbch_decode_ecc(const ezbch_codec *c, const uint8_t *ecc, size_t ecc_stride, unsigned len,
                     int32_t *result, uint32_t *errloc, size_t errloc_stride, size_t ncw,
                     void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!result || !ecc) return -EINVAL;
    if (ncw > 1 && ecc_stride < c->h.ecc_bytes) return -EINVAL;
    if (errloc && ncw > 1 && errloc_stride < c->h.t) return -EINVAL;
    DeviceGuard g(c->device);
    BchArgs a{nullptr, nullptr, 0, len, const_cast<uint8_t *>(ecc), ecc_stride, result, errloc,
              errloc_stride, ncw, 0, 0, 1};
    hipError_t e = launch_decode(c->dev, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(e, "BCH decode launch");
}

int ezbch_decode_syn(const ezbch_codec *c, const uint32_t *syn, size_t syn_stride, unsigned len,
                     int32_t *result, uint32_t *errloc, size_t errloc_stride, size_t ncw,
                     void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!result || !syn) return -EINVAL;
    if (ncw > 1 && syn_stride < 2 * (size_t)c->h.t) return -EINVAL;
    if (errloc && ncw > 1 && errloc_stride < c->h.t) return -EINVAL;
    DeviceGuard g(c->device);
    BchArgs a{nullptr, nullptr, 0, len, nullptr, 0, result, errloc, errloc_stride, ncw, 0, 0, 1,
              syn, syn_stride};
    hipError_t e = launch_decode(c->dev, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(e, "BCH decode launch");
}

namespace {

// Host encode: rows' data bytes go to the device (one linear copy of the span when the pitch is at
// most twice the row, else a CPU gather into pinned staging), the kernel writes a compact
// [n][ecc_bytes] block, only that block comes back and a CPU scatter places each row's ECC.  The
// caller's data bytes are never written.
int bch_encode_host_core(ezbch_codec *c, const uint8_t *data, size_t data_stride, unsigned len,
                         uint8_t *ecc, size_t ecc_stride, size_t ncw, size_t chunk) {
    const size_t eb = c->h.ecc_bytes;
    // a single row is staged at pitch len whatever its stride (a stride below len, 0 included, is
    // legal for one codeword and must not size the staging)
    const bool span = ncw == 1 || data_stride <= 2 * (size_t)len + eb;
    const size_t drow = ncw == 1 ? len : span ? data_stride : len;
    const bool ecc_direct = ecc_stride == eb || ncw == 1;
    if (!chunk) chunk = ((size_t)64 << 20) / (drow ? drow : 1) + 1;
    if (chunk > ncw) chunk = ncw;
    const size_t b_in = align_up(chunk * drow + 16), b_ecc = align_up(chunk * eb);
    if (int r = ensure_stage(c, b_in + b_ecc)) return r;
    if (int r = ensure_hstage(c, (span ? 0 : align_up(chunk * len)) + (ecc_direct ? 0 : b_ecc) + 256))
        return r;
    uint8_t *st = static_cast<uint8_t *>(c->d_stage), *dec = st + b_in;
    uint8_t *hs = static_cast<uint8_t *>(c->h_stage);
    uint8_t *hin = hs, *hecc = hs + (span ? 0 : align_up(chunk * len));
    for (size_t k0 = 0; k0 < ncw; k0 += chunk) {
        const size_t n = ncw - k0 < chunk ? ncw - k0 : chunk;
        const uint8_t *hd = data + k0 * data_stride;
        if (span) {
            HIP_TRY(hipMemcpyAsync(st, hd, (n - 1) * data_stride + len, hipMemcpyHostToDevice, c->stream));
        } else {
            for (size_t r = 0; r < n; ++r) std::memcpy(hin + r * len, hd + r * data_stride, len);
            HIP_TRY(hipMemcpyAsync(st, hin, n * len, hipMemcpyHostToDevice, c->stream));
        }
        BchArgs a{st, nullptr, drow, len, dec, eb, nullptr, nullptr, 0, n, 0};
        HIP_TRY(launch_encode(c->dev, a, c->stream));
        HIP_TRY(hipMemcpyAsync(ecc_direct ? ecc + k0 * eb : hecc, dec, n * eb, hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (!ecc_direct)
            for (size_t r = 0; r < n; ++r) std::memcpy(ecc + (k0 + r) * ecc_stride, hecc + r * eb, eb);
    }
    return 0;
}

} // namespace

int ezbch_encode_host(ezbch_codec *c, const uint8_t *data, size_t data_stride, unsigned len,
                      uint8_t *ecc, size_t ecc_stride, size_t ncw, size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_args(c, data, data_stride, len, ecc, ecc_stride, ncw)) return r;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return bch_encode_host_core(c, data, data_stride, len, ecc, ecc_stride, ncw, chunk);
}

int ezbch_encode_rows_host(ezbch_codec *c, uint8_t *rows, size_t stride, unsigned len, size_t ncw,
                           size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_rows(c, rows, stride, len, ncw)) return r;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return bch_encode_host_core(c, rows, stride, len, rows + len, stride, ncw, chunk);
}

int ezbch_decode_syn_host(ezbch_codec *c, const uint32_t *syn, size_t syn_stride, unsigned len,
                          int32_t *result, uint32_t *errloc, size_t errloc_stride, size_t ncw) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!result || !syn) return -EINVAL;
    const size_t S = 2 * (size_t)c->h.t, T = c->h.t;
    if (ncw > 1 && syn_stride < S) return -EINVAL;
    if (errloc && ncw > 1 && errloc_stride < T) return -EINVAL;
    if (ncw == 1) syn_stride = S, errloc_stride = T;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const size_t b_syn = align_up(ncw * S * 4), b_res = align_up(ncw * 4);
    if (int r = ensure_stage(c, b_syn + b_res + ncw * T * 4)) return r;
    uint8_t *st = static_cast<uint8_t *>(c->d_stage);
    uint32_t *dsyn = reinterpret_cast<uint32_t *>(st);
    int32_t *dres = reinterpret_cast<int32_t *>(st + b_syn);
    uint32_t *dloc = reinterpret_cast<uint32_t *>(st + b_syn + b_res);
    HIP_TRY(hipMemcpy2DAsync(dsyn, S * 4, syn, syn_stride * 4, S * 4, ncw, hipMemcpyHostToDevice, c->stream));
    if (int r = ezbch_decode_syn(c, dsyn, S, len, dres, errloc ? dloc : nullptr, T, ncw, c->stream)) return r;
    HIP_TRY(hipMemcpyAsync(result, dres, ncw * 4, hipMemcpyDeviceToHost, c->stream));
    if (errloc)
        HIP_TRY(hipMemcpy2DAsync(errloc, errloc_stride * 4, dloc, T * 4, T * 4, ncw, hipMemcpyDeviceToHost,
                                 c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int ezbch_decode_host(ezbch_codec *c, uint8_t *data, size_t data_stride, unsigned len,
                      uint8_t *ecc, size_t ecc_stride, int32_t *result, uint32_t *errloc,
                      size_t errloc_stride, size_t ncw, size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!result) return -EINVAL;
    if (!ecc) {
        if (int r = check_rows(c, data, data_stride, len, ncw)) return r;
        ecc = data + len;
        ecc_stride = data_stride;
    }
    if (int r = check_args(c, data, data_stride, len, ecc, ecc_stride, ncw)) return r;
    if (errloc && ncw > 1 && errloc_stride < c->h.t) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const size_t eb = c->h.ecc_bytes, row = (size_t)len + eb, T = c->h.t;
    if (!chunk) chunk = ((size_t)64 << 20) / row + 1;
    if (chunk > ncw) chunk = ncw;
    const size_t b_rows = align_up(chunk * row), b_res = align_up(chunk * 4);
    if (int r = ensure_stage(c, b_rows + b_res + align_up(errloc ? chunk * T * 4 : 0))) return r;
    uint8_t *st = static_cast<uint8_t *>(c->d_stage);
    int32_t *dres = reinterpret_cast<int32_t *>(st + b_rows);
    uint32_t *dloc = reinterpret_cast<uint32_t *>(st + b_rows + b_res);
    for (size_t k0 = 0; k0 < ncw; k0 += chunk) {
        const size_t n = ncw - k0 < chunk ? ncw - k0 : chunk;
        if (len)
            HIP_TRY(ezrs::copy2d(st, row, data + k0 * data_stride, data_stride, len, n,
                                     hipMemcpyHostToDevice, c->stream));
        HIP_TRY(ezrs::copy2d(st + len, row, ecc + k0 * ecc_stride, ecc_stride, eb, n,
                                 hipMemcpyHostToDevice, c->stream));
        if (errloc)   // copy-in/copy-out: entries the decode does not write keep their value
            HIP_TRY(ezrs::copy2d(dloc, T * 4, errloc + k0 * errloc_stride, errloc_stride * 4,
                                     T * 4, n, hipMemcpyHostToDevice, c->stream));
        BchArgs a{st, st, row, len, st + len, row, dres, errloc ? dloc : nullptr, T, n, 0};
        HIP_TRY(launch_decode(c->dev, a, c->stream));
        if (len)
            HIP_TRY(ezrs::copy2d(data + k0 * data_stride, data_stride, st, row, len, n,
                                     hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(ezrs::copy2d(ecc + k0 * ecc_stride, ecc_stride, st + len, row, eb, n,
                                 hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(result + k0, dres, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (errloc)
            HIP_TRY(ezrs::copy2d(errloc + k0 * errloc_stride, errloc_stride * 4, dloc, T * 4,
                                     T * 4, n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return 0;
}

} // extern "C"
