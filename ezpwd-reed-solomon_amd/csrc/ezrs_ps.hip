// ezrs_ps.hip -- plane-sliced GF(2^8) RS syndrome kernels for MI355X (gfx950).
//
// Computes the syndromes S_i = r(alpha^((fcr+i)*prim)) of c++/ezpwd/rs_base:1390-1414 for batches
// of 255-symbol codewords.  Decode: a codeword whose syndromes are all zero (and that carries no
// erasures) gets result 0, exactly decode_symbols' early return (rs_base:1416-1434); every other
// codeword gets a sentinel and its syndromes go to the workspace for the error path
// (ezrs_generic.hip: k_decode_flagged).  Encode: the syndromes of the data symbols go to a
// workspace and k_ps_parity maps them to parity (parity = V^-1 S).
//
// Arithmetic (codegen/gen_ps.py has the derivation): a 32-bit word holds one position of four
// codewords, bit 8k + b = bit-plane b of codeword k.  Each bit is a GF(2) stream, so only one root
// per cyclotomic coset ("leader") is evaluated -- V_{b,2e} = V_{b,e}^2 -- and the per-plane values
// are folded into syndromes (S = sum_b alpha^b V_b) once per tile.  For RS(255,223) the main loop
// keeps 16 leaders x 8 bits = 128 state words per codeword slot set, half the state (and half the
// XORs per input symbol) of a per-symbol bit-slicing of the 32 syndromes.
//
// Work decomposition (one 512-thread workgroup per CU, persistent over tiles):
//   * tile = 256 consecutive codewords; lane l of every wave owns codewords 4l..4l+3 of the tile.
//   * the tile's rows are one contiguous span (row pitch <= 256 B): it is copied to LDS by linear
//     1-KiB LDS-DMA instructions through a buffer resource (out-of-range bytes read as zero), double
//     buffered: the next tile lands while this one is computed.  (Row-gather DMA shapes measured
//     4.1-5.3 TB/s, whole-tile linear loads 6.2-6.7 TB/s: tools/micro/ps_stream2.hip.)
//   * wave (g, q), g = wave / 4, q = wave % 4: leader group g (8 leaders, 64 state words) over
//     position slice q (64 positions decode, 56 encode).  Each lane reads its 4 rows' bytes with
//     aligned ds_read_b32 + v_alignbyte (gfx950 LDS does not serve unaligned reads), transposes
//     4x4 bytes with v_perm, and runs the generated XOR networks.
//   * slice q's partials are multiplied by alpha^(-q S e) and summed across the 4 slices through
//     LDS (two pairwise exchange rounds in the consumed tile buffer); each wave then owns the
//     totals of two leaders and runs their expansion + plane fold (generated epilogue).
//   * global stores of a tile are issued after the next tile's top barrier, so the vmcnt wait of
//     that barrier only covers memory operations issued a whole tile earlier.
#include "ezrs_internal.hpp"
#include "gen/ezrs_ps_tables.inc"

namespace ezrs {
namespace ps {

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kTile = 256;                          // codewords per tile
constexpr int kGuard = 256;                         // bytes before each tile image (pad reads)
constexpr int kTileMax = 65536;                     // tile bytes: 256 rows x pitch <= 256 B
constexpr int kBufBytes = kGuard + kTileMax + 64;
constexpr int32_t kSentinel = INT32_MIN;
constexpr int kN = 255;

typedef __attribute__((address_space(3))) void lds_void;

// Timing-only builds (tools/micro/ps_stamps.hip): per-phase s_memtime stamps of the first
// workgroups.  Never defined in the library.
#ifdef EZRS_PS_STAMPS
__device__ unsigned long long g_ps_stamps[8][8][16][8];    // [wg][wave][tile][phase]
#define PS_STAMP(ph) do { if (blockIdx.x < 8 && it < 16 && lane == 0) \
    g_ps_stamps[blockIdx.x][wave][it][ph] = __builtin_amdgcn_s_memtime(); } while (0)
__device__ unsigned long long g_py_stamps[16][2][8][8];  // [wg][wave][tile][phase]
__device__ unsigned long long g_pg_stamps[16][8][16][8];  // [wg][wave][tile][phase]
#define PG_STAMP(ph) do { __builtin_amdgcn_sched_barrier(0); if (blockIdx.x < 16 && it < 16 && lane == 0) \
    g_pg_stamps[blockIdx.x][stamp_wave][it][ph] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#define PY_STAMP(ph) do { __builtin_amdgcn_sched_barrier(0); if (blockIdx.x < 16 && it < 8 && lane == 0) \
    g_py_stamps[blockIdx.x][Q][it][ph] = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define PS_STAMP(ph) do { } while (0)
#define PY_STAMP(ph) do { } while (0)
#define PG_STAMP(ph) do { } while (0)
#endif

struct PsArgs {
    const uint8_t *base;        // row 0 of the batch
    uint32_t span;              // bytes readable from base
    uint32_t stride;            // row pitch in bytes (<= 256)
    uint32_t ncw;               // codewords
    uint32_t ntiles;
    int lo;                     // full-frame position of the rows' first byte (the pad)
    int hi;                     // one past the last evaluated position (255 decode, 255-NR encode)
    const uint32_t *neras;      // decode: erasure counts (nullable)
    int32_t *result;            // decode
    uint8_t *ws;                // decode: [ncw][32] flagged syndromes; encode: [NR][ws_pitch]
    size_t ws_pitch;            // encode: codewords per syndrome row (a multiple of 2048)
    int ablate;                 // timing experiments only (tools/micro): bit 0 no main loop, 1 no
                                // exchange, 2 no epilogue, 3 no DMA, 4 no result stores; 0 in the
                                // library
};

template <int I, int N, class F> __device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// In-place 8x8 bit transpose of (register index) x (bit position mod 8).
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

// Issue this wave's share of the tile's linear LDS-DMA (1 KiB per instruction).
__device__ __forceinline__ void issue_tile(uint8_t *buf, const PsArgs &a, __amdgpu_buffer_rsrc_t rsrc,
                                           uint32_t tile, int wave, int lane) {
    const uint32_t tb = a.stride * kTile;                 // tile bytes
    const uint32_t ninstr = (tb + 1023) >> 10;
    const uint32_t t0 = tile * tb;
    for (uint32_t i = wave; i < ninstr; i += kWaves)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void *)(buf + kGuard + i * 1024), 16,
                                                 t0 + i * 1024 + 16 * lane, 0, 0, 0);
}

// The 8 position words of positions p0..p0+7 for the lane's 4 rows: X[t] byte k = row k symbol.
__device__ __forceinline__ void load_block(const uint8_t *buf, const int (&rb)[4], const uint32_t (&sh)[4],
                                           int p0, uint32_t (&X)[8]) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int o = rb[k] + p0;                         // rb: row start - lo, relative to buf
        const uint32_t *d = reinterpret_cast<const uint32_t *>(buf + (o & ~3));
        const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
        lo[k] = __builtin_amdgcn_alignbyte(d1, d0, sh[k]);
        hi[k] = __builtin_amdgcn_alignbyte(d2, d1, sh[k]);
    }
    transpose4x4(lo, X);
    transpose4x4(hi, X + 4);
}

// Main loop of one wave: group G over slice positions [q S, q S + S) (S = 8 NB).
template <class C, int G, int NB>
__device__ __forceinline__ void main_slice(uint32_t (&V)[C::NLG][8], const uint8_t *buf,
                                           const int (&rb)[4], const uint32_t (&sh)[4], int s0,
                                           int lo, int hi) {
    static_for<0, NB>([&](auto B) {
        const int p0 = s0 + 8 * B;                        // full-frame position of word X[0]
        if (p0 + 8 > lo && p0 < hi) {                     // wave-uniform
            uint32_t X[8];
            load_block(buf, rb, sh, p0, X);
            if (p0 < lo || p0 + 8 > hi) {
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (p0 + t < lo || p0 + t >= hi) X[t] = 0;
            }
            C::template block<G, decltype(B)::value>(V, X);
        }
    });
}

// Reduction of the slice partials: wave (g, q) ends with the totals of leader slots
// 2 idx, 2 idx + 1 of group g, idx = 2 (q & 1) + (q >> 1)  (gen_ps.py assigns leaders to match).
template <class C, int q>
__device__ __forceinline__ void reduce(uint32_t (&V)[C::NLG][8], uint32_t (&T)[2][8], uint8_t *buf,
                                       int wave, int lane) {
    uint4 *r1 = reinterpret_cast<uint4 *>(buf);          // 8 waves x 8 x 1 KiB
    // round 1: partner q ^ 1; keep slots [4 (q & 1), +4), send the other 4 (32 words)
    constexpr int keep1 = 4 * (q & 1), send1 = 4 - keep1;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ss = send1 + s;
            uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
            // select the slot at run time (wave-uniform) without dynamic register indexing
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if (c == ss) { w0 = V[c][4 * h]; w1 = V[c][4 * h + 1]; w2 = V[c][4 * h + 2]; w3 = V[c][4 * h + 3]; }
            r1[(wave * 8 + 2 * s + h) * 64 + lane] = make_uint4(w0, w1, w2, w3);
        }
    __syncthreads();
    const int partner1 = wave ^ 1;
    uint32_t K[4][8];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint4 v = r1[(partner1 * 8 + 2 * s + h) * 64 + lane];
            uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if (c == keep1 + s) { m0 = V[c][4 * h]; m1 = V[c][4 * h + 1]; m2 = V[c][4 * h + 2]; m3 = V[c][4 * h + 3]; }
            K[s][4 * h] = m0 ^ v.x; K[s][4 * h + 1] = m1 ^ v.y;
            K[s][4 * h + 2] = m2 ^ v.z; K[s][4 * h + 3] = m3 ^ v.w;
        }
    __syncthreads();                                      // r1 is read; round 2 reuses it
    // round 2: partner q ^ 2; keep K slots [2 (q >> 1), +2), send the other 2 (16 words)
    constexpr int keep2 = 2 * (q >> 1), send2 = 2 - keep2;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c == send2 + s) { w0 = K[c][4 * h]; w1 = K[c][4 * h + 1]; w2 = K[c][4 * h + 2]; w3 = K[c][4 * h + 3]; }
            r1[(wave * 4 + 2 * s + h) * 64 + lane] = make_uint4(w0, w1, w2, w3);
        }
    __syncthreads();
    const int partner2 = wave ^ 2;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint4 v = r1[(partner2 * 4 + 2 * s + h) * 64 + lane];
            uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (c == keep2 + s) { m0 = K[c][4 * h]; m1 = K[c][4 * h + 1]; m2 = K[c][4 * h + 2]; m3 = K[c][4 * h + 3]; }
            T[s][4 * h] = m0 ^ v.x; T[s][4 * h + 1] = m1 ^ v.y;
            T[s][4 * h + 2] = m2 ^ v.z; T[s][4 * h + 3] = m3 ^ v.w;
        }
}

// Deferred global stores of one tile (issued after the next tile's top barrier).
template <class C> struct Pending {
    uint32_t D[C::NQ][4];       // syndrome bytes of the lane's 4 codewords, per quad slot
    uint32_t flags;             // decode: bit k = codeword 4 lane + k is flagged
    int32_t res[4];
    size_t cw0;                 // first codeword of the lane
    bool live;
};

template <class C, bool ENC, int G, int I>
__device__ __forceinline__ void flush(const Pending<C> &pd, const PsArgs &a, int lane) {
    if (!pd.live) return;
    if constexpr (ENC) {
        // workspace [NR][ws_pitch]: syndrome-major, one byte per codeword (coalesced dwords)
        uint8_t *dst = a.ws + pd.cw0;
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int si = C::SYN[G][I][qd][j];
                if (si >= 0) *reinterpret_cast<uint32_t *>(dst + si * a.ws_pitch) = pd.D[qd][j];
            }
    } else {
        if (G == 0 && I == 0) {   // one wave writes the results
            if (pd.cw0 + 3 < a.ncw) {
                *reinterpret_cast<int4 *>(a.result + pd.cw0) =
                    make_int4(pd.res[0], pd.res[1], pd.res[2], pd.res[3]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (pd.cw0 + k < a.ncw) a.result[pd.cw0 + k] = pd.res[k];
            }
        }
        if (pd.flags) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!(pd.flags >> k & 1)) continue;
                uint8_t *dst = a.ws + (pd.cw0 + k) * 32;
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int si = C::SYN[G][I][qd][j];
                        if (si >= 0) dst[si] = (uint8_t)(pd.D[qd][j] >> (8 * k));
                    }
            }
        }
    }
    (void)lane;
}

template <class C, bool ENC, int G, int I>
__device__ __forceinline__ void wave_body(const PsArgs &a, uint8_t *lds, uint32_t (*flags)[64],
                                          int wave, int lane) {
    constexpr int S = ENC ? C::S_ENC : C::S_DEC;
    constexpr int NB = S / 8;
    constexpr int q = 2 * (I & 1) + (I >> 1);              // slice (inverse of I = 2 (q&1) + (q>>1))
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.base, (short)0, (int)a.span, 0x00020000);
    // the lane's row starts relative to the tile image, shifted so that position p' of row k is
    // at byte rb[k] + p' of the buffer
    int rb[4];
    uint32_t sh[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rb[k] = kGuard + (4 * lane + k) * (int)a.stride - a.lo;
        sh[k] = (uint32_t)rb[k] & 3u;
    }
    Pending<C> pd;
    pd.live = false;
    uint8_t *buf = lds;
    uint32_t tile = blockIdx.x;
    if (tile < a.ntiles) issue_tile(buf, a, rsrc, tile, wave, lane);
    for (int it = 0; tile < a.ntiles; tile += gridDim.x, ++it) {
        (void)it;
        PS_STAMP(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                                   // the tile has landed
        PS_STAMP(1);
        flush<C, ENC, G, I>(pd, a, lane);
        if (tile == a.ntiles - 1) {
            // A buffer load whose dword crosses the end of the range reads zero there: re-read the
            // span's last bytes (the last row's tail) directly.
            if (wave == 0) {
                const uint32_t t0 = tile * a.stride * kTile;
                const uint32_t tail = a.span - t0 < 64u ? a.span - t0 : 64u;
                if ((uint32_t)lane < tail) {
                    const uint32_t off = a.span - tail + lane;
                    buf[kGuard + (off - t0)] = a.base[off];
                }
            }
            __syncthreads();
        }
        const size_t cw0 = (size_t)tile * kTile + 4 * lane;
        uint32_t ne = 0;
        if (!ENC && a.neras) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (cw0 + k < a.ncw && a.neras[cw0 + k]) ne |= 1u << k;
        }
        uint32_t V[C::NLG][8];
#pragma unroll
        for (int s = 0; s < C::NLG; ++s)
#pragma unroll
            for (int t = 0; t < 8; ++t) V[s][t] = 0;
        main_slice<C, G, NB>(V, buf, rb, sh, q * S, a.lo, a.hi);
        if constexpr (q != 0) C::template fixup<G, S>(V, q);
        PS_STAMP(2);
        __syncthreads();                                   // every wave is done with the image
        PS_STAMP(3);
        uint32_t T[2][8];
        reduce<C, q>(V, T, buf, wave, lane);
        __syncthreads();                                   // the exchange area is read
        // the next tile lands while this one's syndromes are folded (and the other workgroup on
        // this CU computes)
        if (tile + gridDim.x < a.ntiles) issue_tile(buf, a, rsrc, tile + gridDim.x, wave, lane);
        PS_STAMP(4);
        uint32_t Qd[C::NQ][8];
        C::template epilogue<G, I>(T, Qd);
        // quads -> bytes: after transpose8, Qd[qd][j] byte k = syndrome j of the quad, codeword k
        uint32_t nz = 0;
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            uint32_t vm = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (C::SYN[G][I][qd][j] >= 0) vm |= 0x01010101u << j;
#pragma unroll
            for (int t = 0; t < 8; ++t) nz |= Qd[qd][t] & vm;
            transpose8(Qd[qd]);
#pragma unroll
            for (int j = 0; j < 4; ++j) pd.D[qd][j] = Qd[qd][j];
        }
        pd.cw0 = cw0;
        pd.live = true;
        PS_STAMP(5);
        if constexpr (!ENC) {
            uint32_t fl = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (nz >> (8 * k) & 0xFF) fl |= 1u << k;
            flags[wave][lane] = fl;
            __syncthreads();
            fl = ne;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) fl |= flags[w][lane];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (cw0 + k >= a.ncw) fl &= ~(1u << k);
                pd.res[k] = (fl >> k & 1) ? kSentinel : 0;
            }
            pd.flags = fl;
        }
    }
    flush<C, ENC, G, I>(pd, a, lane);
}

// Two workgroups per CU (16 waves, <= 128 VGPRs): while one waits for its tile or sits in a
// barrier, the other computes.
template <class C, bool ENC>
__global__ void __launch_bounds__(kThreads, 4) k_ps_syndromes(PsArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kBufBytes];
    __shared__ uint32_t flags[kWaves][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // wave (g, q): g = wave >> 2, q = wave & 3; epilogue index idx = 2 (q & 1) + (q >> 1)
    switch (wave) {
    case 0: wave_body<C, ENC, 0, 0>(a, lds, flags, wave, lane); break;
    case 1: wave_body<C, ENC, 0, 2>(a, lds, flags, wave, lane); break;
    case 2: wave_body<C, ENC, 0, 1>(a, lds, flags, wave, lane); break;
    case 3: wave_body<C, ENC, 0, 3>(a, lds, flags, wave, lane); break;
    case 4: wave_body<C, ENC, 1, 0>(a, lds, flags, wave, lane); break;
    case 5: wave_body<C, ENC, 1, 2>(a, lds, flags, wave, lane); break;
    case 6: wave_body<C, ENC, 1, 1>(a, lds, flags, wave, lane); break;
    default: wave_body<C, ENC, 1, 3>(a, lds, flags, wave, lane); break;
    }
}

// ---- helpers of the gather-layout kernels ------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(const uint8_t *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
}

typedef int pw_rsrc_t __attribute__((ext_vector_type(4)));

// Buffer descriptor of [base, base + span): raw (stride 0), out-of-range bytes read as zero.
__device__ __forceinline__ pw_rsrc_t pw_rsrc(const uint8_t *base, uint32_t span) {
    const uint64_t p = (uint64_t)(uintptr_t)base;
    pw_rsrc_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(p >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)span);
    r.w = 0x00020000;
    return r;
}

// ---- pair-wave syndromes ---------------------------------------------------------------------
// Two waves (one workgroup, 4 per CU) own a tile of 256 codewords (lane l: rows l + 64k, byte k
// of its words) and
// stream it through ONE 32 KiB LDS window of 128 positions x 256 rows.  Full 128-byte row chunks
// per DMA instruction (8 lanes per row, 8 rows per instruction) keep the gather at line
// granularity (narrow per-row pieces -- a per-wave design with 32-position windows -- measured
// 1.5-1.8 TB/s for the fetch alone: tools/micro/pw_dma.hip).  Wave q
// evaluates ALL leaders over the 16-position pieces p = q, q+2, q+4, q+6 of every window (an even
// split for any codec length) with the blocks of those positions (no fixups), then the waves swap
// the partials of the leaders the other owns and each folds its own leaders' syndromes (generated
// PY_ epilogues).
//
// LDS layout: instruction (k, m) (k = byte in word, m = lane block) covers the 8 consecutive rows
// 64k + l, l = 8m..8m+7, at (8k + m) KiB; lane j of it loads row 64k + l, l = 8m + j/8, 16-byte
// piece p = (j & 7) ^ f(l), f(l) = (l >> 1) & 7, so piece p of row 64k + l sits at
//   (8k + l/8) KiB + 128 (l & 7) + 16 (p ^ f(l)):
// the XOR swizzle makes every 16-lane group of a ds_read_b128 hit 16 distinct bank quads.
// Encode leaves the syndromes in tile-lane order (workspace column tile*256 + 4l + k holds
// codeword tile*256 + 64k + l); k_ps_parity<C, true> undoes it.
constexpr int kPyWin = 128;                                 // positions per window
constexpr int kPyWinBytes = kTile * kPyWin;                 // 32 KiB

template <class C, bool ENC, int Q>
__device__ __forceinline__ void py_body(const PsArgs &a, uint8_t *buf, uint32_t (*flags)[64], int lane) {
    constexpr int NL = C::NL, NLW = C::NLW;
    constexpr int HI = ENC ? kN - C::NR : kN;                   // one past the last position
    constexpr int W_HI = (HI - 1) / kPyWin;
    const int w_lo = a.lo / kPyWin;
    const pw_rsrc_t rsrc = pw_rsrc(a.base, a.span);
    const uint32_t lbuf = __builtin_amdgcn_readfirstlane(lds_addr(buf));
    // Per-lane DMA and LDS-read offsets are recomputed where they are used, from a laundered lane
    // id (an empty volatile asm the compiler cannot hoist), so that they do not occupy registers
    // across the 128-word state.
    auto fresh_lane = [&]() { uint32_t l = (uint32_t)lane; asm volatile("" : "+v"(l)); return l; };
    // DMA role: this wave issues instructions k = 2Q, 2Q+1, m = 0..7; lane j -> row 64k + 8m + j/8,
    // piece (j & 7) ^ f(8m + j/8), and (8m + j/8) >> 1 & 7 only depends on m & 1
    auto doff = [&](uint32_t l, int kk, int mp) {
        const uint32_t dslot = l >> 3;
        const uint32_t p = (l & 7) ^ ((4 * mp + (dslot >> 1)) & 7);
        return (64 * (2 * Q + kk) + dslot) * a.stride + 16 * p;
    };
    const uint32_t m_step = 8u * a.stride;                      // rows 64k + l, l += 8
    // read role: piece p = 2 pp + Q of row 64k + lane at rd(pp) + 8 KiB k
    auto rd = [&](uint32_t l, int pp) {
        return 1024 * (l >> 3) + 128 * (l & 7) + 16 * ((2 * pp + Q) ^ ((l >> 1) & 7));
    };
    const uint32_t tile_bytes = a.stride * kTile;

    // (LDS-DMA and the window's LDS reads are inline asm, as in the per-wave kernel: the compiler
    // would otherwise wait for every outstanding vector memory operation in front of each LDS read)
    auto issue = [&](uint32_t toff, int w) {
        const uint32_t base = toff + (uint32_t)(kPyWin * w - a.lo);
        const uint32_t l = fresh_lane();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const uint32_t d0 = base + doff(l, kk, 0), d1 = base + doff(l, kk, 1);
#pragma unroll
            for (int m = 0; m < 8; ++m)
                asm volatile("s_mov_b32 m0, %0\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dwordx4 %1, %2, 0 offen lds"
                             :: "s"(lbuf + (8 * (2 * Q + kk) + m) * 1024), "v"((m & 1 ? d1 : d0) + m * m_step),
                                "s"(rsrc) : "memory", "m0");
        }
    };
    // Fix-ups of this wave's pieces (the reader patches what it reads, after the window landed):
    // pieces straddling the span's start/end come back all-zero; positions before lo hold the
    // previous row's bytes.
    auto fix = [&](uint32_t toff, int w) {
#pragma unroll 1
        for (int i = 0; i < 16; ++i) {
            const int k = i >> 2, pp = i & 3;
            const int64_t r0 = (int64_t)toff + (int64_t)(64 * k + lane) * a.stride;
            const int64_t o = r0 + kPyWin * w + 16 * (2 * pp + Q) - a.lo;
            const bool straddle = (o < 0 && o > -16) || (o < (int64_t)a.span && o + 16 > (int64_t)a.span);
            if (!straddle && o >= r0) continue;
            const uint32_t dst = lbuf + rd(lane, pp) + 8192 * k;
#pragma unroll 1
            for (int j = 0; j < 16; ++j) {
                const int64_t g = o + j;
                uint32_t v = 0;
                if (g >= r0 && !straddle) continue;                // the DMA'd byte stands
                if (g >= r0 && g < (int64_t)a.span)                // (asm: see pw_fix)
                    asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)"
                                 : "=&v"(v) : "v"(a.base + g) : "memory");
                asm volatile("ds_write_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(dst + j), "v"(v) : "memory");
            }
        }
    };

    // deferred stores of the previous tile (issued once the next tile's first window landed):
    // encode its syndromes, decode its results (flagged codewords' syndromes go out at once)
    uint32_t pend[ENC ? C::NQW : 1][4];
    size_t pend_cw0 = 0, pend_col = 0;
    uint32_t pend_fl = 0;
    bool pending = false;
    auto flush = [&]() {
        if (!pending) return;
        if constexpr (ENC) {
            uint8_t *dst = a.ws + pend_col;
#pragma unroll
            for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int si = C::SYN[Q][qd][jj];
                    if (si >= 0) *reinterpret_cast<uint32_t *>(dst + (size_t)si * a.ws_pitch) = pend[qd][jj];
                }
        } else {
            if (Q == 0) {
                int32_t res[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) res[k] = (pend_fl >> k & 1) ? kSentinel : 0;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (pend_cw0 + 64 * k < a.ncw) a.result[pend_cw0 + 64 * k] = res[k];
            }
        }
        pending = false;
    };

    uint32_t tile = blockIdx.x;
    if (tile < a.ntiles) issue(tile * tile_bytes, w_lo);
    for (int it = 0; tile < a.ntiles; tile += gridDim.x, ++it) {
        (void)it;
        PY_STAMP(0);
        const uint32_t toff = tile * tile_bytes;
        uint32_t V[NL][8];
#pragma unroll
        for (int s = 0; s < NL; ++s)
#pragma unroll
            for (int t = 0; t < 8; ++t) V[s][t] = 0;
        static_for<0, W_HI + 1>([&](auto Wc) {
            constexpr int W = decltype(Wc)::value;
            if (W < w_lo) return;                                // wave-uniform
            if (W > w_lo) issue(toff, W);                        // the window buffer is free
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();                                     // window W landed (both waves)
            PY_STAMP(1 + 2 * W);
            if (W == w_lo) flush();
            if (__builtin_expect(kPyWin * W - a.lo < 0 ||
                                 (int64_t)toff + tile_bytes + kPyWin * W - a.lo + kPyWin > (int64_t)a.span, 0))
                fix(toff, W);
            static_for<0, 4>([&](auto Pc) {
                constexpr int pp = decltype(Pc)::value;
                constexpr int p16 = kPyWin * W + 16 * (2 * pp + Q); // first position of the piece
                if constexpr (p16 < HI) {
                    uint4 R[4];
                    asm volatile("ds_read_b128 %0, %4\n\t"
                                 "ds_read_b128 %1, %4 offset:8192\n\t"
                                 "ds_read_b128 %2, %4 offset:16384\n\t"
                                 "ds_read_b128 %3, %4 offset:24576\n\t"
                                 "s_waitcnt lgkmcnt(0)"
                                 : "=&v"(R[0]), "=&v"(R[1]), "=&v"(R[2]), "=&v"(R[3])
                                 : "v"(lbuf + rd(fresh_lane(), pp)) : "memory");
                    uint32_t X[16];
                    {
                        const uint32_t c0[4] = {R[0].x, R[1].x, R[2].x, R[3].x};
                        const uint32_t c1[4] = {R[0].y, R[1].y, R[2].y, R[3].y};
                        const uint32_t c2[4] = {R[0].z, R[1].z, R[2].z, R[3].z};
                        const uint32_t c3[4] = {R[0].w, R[1].w, R[2].w, R[3].w};
                        transpose4x4(c0, X);
                        transpose4x4(c1, X + 4);
                        transpose4x4(c2, X + 8);
                        transpose4x4(c3, X + 12);
                    }
                    static_for<0, 2>([&](auto Bc) {
                        constexpr int p0 = p16 + 8 * decltype(Bc)::value;
                        if constexpr (p0 < HI) {
                            uint32_t Y[8];
#pragma unroll
                            for (int t = 0; t < 8; ++t) Y[t] = p0 + t < HI ? X[p0 - p16 + t] : 0u;
                            C::template block<p0 / 8>(V, Y);
                        }
                    });
                }
            });
            __syncthreads();                                     // both waves are done with the window
            PY_STAMP(2 + 2 * W);
        });
        // swap partials through the (free) window buffer: wave Q sends the leaders the other owns
        {
            uint4 *x = reinterpret_cast<uint4 *>(buf);
#pragma unroll
            for (int i = 0; i < NLW; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int s = C::OWN[Q ^ 1][i];
                    x[((Q * NLW + i) * 2 + h) * 64 + lane] =
                        make_uint4(V[s][4 * h], V[s][4 * h + 1], V[s][4 * h + 2], V[s][4 * h + 3]);
                }
        }
        __syncthreads();
        uint32_t T[NLW][8];
        {
            const uint4 *x = reinterpret_cast<const uint4 *>(buf);
#pragma unroll
            for (int i = 0; i < NLW; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int s = C::OWN[Q][i];
                    const uint4 v = x[(((Q ^ 1) * NLW + i) * 2 + h) * 64 + lane];
                    T[i][4 * h] = V[s][4 * h] ^ v.x;
                    T[i][4 * h + 1] = V[s][4 * h + 1] ^ v.y;
                    T[i][4 * h + 2] = V[s][4 * h + 2] ^ v.z;
                    T[i][4 * h + 3] = V[s][4 * h + 3] ^ v.w;
                }
        }
        __syncthreads();                                         // the exchange area is read
        PY_STAMP(5);
        if (tile + gridDim.x < a.ntiles) issue(toff + gridDim.x * tile_bytes, w_lo);
        const size_t cw0 = (size_t)tile * kTile + lane;          // byte k <-> codeword cw0 + 64k
        uint32_t nz = 0;
        uint32_t D[C::NQW][4];
        C::template epilogue<Q>(T, [&](auto Qc, uint32_t (&Qw)[8]) {
            constexpr int qd = decltype(Qc)::value;
            if constexpr (!ENC) {
                uint32_t vm = 0;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if (C::SYN[Q][qd][jj] >= 0) vm |= 0x01010101u << jj;
#pragma unroll
                for (int t = 0; t < 8; ++t) nz |= Qw[t] & vm;
            }
            transpose8(Qw);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) D[qd][jj] = Qw[jj];
        });
        if constexpr (ENC) {
#pragma unroll
            for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) pend[qd][jj] = D[qd][jj];
        }
        pend_cw0 = cw0;
        pend_col = (size_t)tile * kTile + 4 * lane;
        pending = true;
        PY_STAMP(6);
        if constexpr (!ENC) {
            uint32_t fl = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (nz >> (8 * k) & 0xFF) fl |= 1u << k;
            // OR with the other wave's flags (asm: the compiler would wait for the DMA in flight)
            const uint32_t fa = lds_addr(reinterpret_cast<uint8_t *>(&flags[Q][lane]));
            const uint32_t fb = lds_addr(reinterpret_cast<uint8_t *>(&flags[Q ^ 1][lane]));
            asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(fa), "v"(fl) : "memory");
            __syncthreads();
            uint32_t fo;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(fo) : "v"(fb) : "memory");
            fl |= fo;
            if (a.neras) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (cw0 + 64 * k < a.ncw && a.neras[cw0 + 64 * k]) fl |= 1u << k;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (cw0 + 64 * k >= a.ncw) fl &= ~(1u << k);
            pend_fl = fl;
            if (fl) {                                            // flagged: syndromes for the error path
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!(fl >> k & 1)) continue;
                    uint8_t *dst = a.ws + (cw0 + 64 * k) * 32;
#pragma unroll
                    for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            const int si = C::SYN[Q][qd][jj];
                            if (si >= 0) dst[si] = (uint8_t)(D[qd][jj] >> (8 * k));
                        }
                }
            }
        }
    }
    flush();
}

template <class C, bool ENC>
__global__ void __attribute__((amdgpu_flat_work_group_size(128, 128), amdgpu_waves_per_eu(2)))
k_py_syndromes(PsArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[kPyWinBytes];
    __shared__ uint32_t flags[2][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wave == 0) py_body<C, ENC, 0>(a, buf, flags, lane);
    else py_body<C, ENC, 1>(a, buf, flags, lane);
}

// ---- group syndromes (default) -----------------------------------------------------------------
// NW = 4 waves (one workgroup, 2 per CU) share a whole tile of 256 codewords (lane l: rows
// l + 64k, byte k of its words) held in LDS in the swizzled gather layout of the pair kernel: two
// 32 KiB halves (positions 0..127, 128..255), each 128-byte row chunk fetched by 8 lanes of one
// LDS-DMA instruction.  Fetching both halves of every row together keeps each cache line read
// once (windows fetched a half at a time re-read the lines the halves share from HBM once the
// L2 no longer holds them: 3.5-4.4 TB/s vs 6.2-6.7 TB/s, tools/micro/py_dma.hip).  Wave q
// evaluates ALL leaders over the 16-position pieces g = q, q + 4, q + 8, q + 12 with the PW blocks
// of those positions (no fixups); two rounds of pairwise exchange through the consumed tile
// buffer (recursive halving by owner bits: PG4_*::SEND / KEEP) leave each wave the totals of the
// leaders it owns, whose syndromes it folds.  The next tile is fetched while the epilogues run
// (and the other workgroup on the CU computes).
constexpr int kPgTileBytes = 2 * kPyWinBytes;               // 64 KiB

template <class C, bool ENC, int Q>
__device__ __forceinline__ void pg_body(const PsArgs &a, uint8_t *buf, uint32_t (*flags)[64], int lane) {
    constexpr int NW = C::NW, NL = C::NL, NLW = C::NLW;
    constexpr int stamp_wave = Q;
    (void)stamp_wave;
    constexpr int NPW = 16 / NW;                                // pieces per wave
    constexpr int IPW = 32 / NW;                                // DMA instructions per wave per half
    constexpr int HI = ENC ? kN - C::NR : kN;                   // one past the last position
    const int w_lo = a.lo / kPyWin;                             // first half holding positions >= lo
    const pw_rsrc_t rsrc = pw_rsrc(a.base, a.span);
    const uint32_t lbuf = __builtin_amdgcn_readfirstlane(lds_addr(buf));
    auto fresh_lane = [&]() { uint32_t l = (uint32_t)lane; asm volatile("" : "+v"(l)); return l; };
    // DMA: instruction i = 8k + m of a half covers rows 64k + 8m .. +7; lane j -> row 64k + 8m + j/8,
    // piece (j & 7) ^ f(8m + j/8), f(l) = (l >> 1) & 7 (only depends on m & 1 and j/8)
    auto doff = [&](uint32_t l, int k, int mp) {
        const uint32_t dslot = l >> 3;
        const uint32_t p = (l & 7) ^ ((4 * mp + (dslot >> 1)) & 7);
        return (64 * k + dslot) * a.stride + 16 * p;
    };
    const uint32_t m_step = 8u * a.stride;
    auto rd = [&](uint32_t l, int p) {                          // piece p of row 64k + l: + 8 KiB k
        return 1024 * (l >> 3) + 128 * (l & 7) + 16 * (p ^ ((l >> 1) & 7));
    };
    const uint32_t tile_bytes = a.stride * kTile;

    auto issue = [&](uint32_t toff) {
        if (a.ablate & 8) return;
        const uint32_t l = fresh_lane();
        for (int w = w_lo; w < 2; ++w) {                        // wave-uniform
            const uint32_t base = toff + (uint32_t)(kPyWin * w - a.lo);
#pragma unroll
            for (int ii = 0; ii < IPW; ii += 2) {
                const int i = Q * IPW + ii, k = i >> 3, m0 = i & 7;   // m0 even: (m0, m0 + 1)
                const uint32_t d0 = base + doff(l, k, 0) + m0 * m_step, d1 = base + doff(l, k, 1) + (m0 + 1) * m_step;
                asm volatile("s_mov_b32 m0, %0\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dwordx4 %1, %2, 0 offen lds"
                             :: "s"(lbuf + w * kPyWinBytes + i * 1024), "v"(d0), "s"(rsrc) : "memory", "m0");
                asm volatile("s_mov_b32 m0, %0\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dwordx4 %1, %2, 0 offen lds"
                             :: "s"(lbuf + w * kPyWinBytes + (i + 1) * 1024), "v"(d1), "s"(rsrc) : "memory", "m0");
            }
        }
    };
    // fix-ups of this wave's pieces (see pw_fix): straddling the span's ends, or before lo
    auto fix = [&](uint32_t toff) {
#pragma unroll 1
        for (int i = 0; i < 4 * NPW; ++i) {
            const int k = i & 3, g = Q + NW * (i >> 2), w = g >> 3, p = g & 7;
            if (w < w_lo) continue;
            const int64_t r0 = (int64_t)toff + (int64_t)(64 * k + lane) * a.stride;
            const int64_t o = r0 + kPyWin * w + 16 * p - a.lo;
            const bool straddle = (o < 0 && o > -16) || (o < (int64_t)a.span && o + 16 > (int64_t)a.span);
            if (!straddle && o >= r0) continue;
            const uint32_t dst = lbuf + w * kPyWinBytes + rd(lane, p) + 8192 * k;
#pragma unroll 1
            for (int j = 0; j < 16; ++j) {
                const int64_t gg = o + j;
                uint32_t v = 0;
                if (gg >= r0 && !straddle) continue;
                if (gg >= r0 && gg < (int64_t)a.span)
                    asm volatile("global_load_ubyte %0, %1, off\n\ts_waitcnt vmcnt(0)"
                                 : "=&v"(v) : "v"(a.base + gg) : "memory");
                asm volatile("ds_write_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(dst + j), "v"(v) : "memory");
            }
        }
    };

    uint32_t pend[ENC ? C::NQW : 1][4];
    size_t pend_cw0 = 0, pend_col = 0;
    uint32_t pend_fl = 0;
    bool pending = false;
    auto flush = [&]() {
        if (!pending || (a.ablate & 16)) return;
        if constexpr (ENC) {
            uint8_t *dst = a.ws + pend_col;
#pragma unroll
            for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int si = C::SYN[Q][qd][jj];
                    if (si >= 0) *reinterpret_cast<uint32_t *>(dst + (size_t)si * a.ws_pitch) = pend[qd][jj];
                }
        } else if (Q == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (pend_cw0 + 64 * k < a.ncw) a.result[pend_cw0 + 64 * k] = (pend_fl >> k & 1) ? kSentinel : 0;
        }
        pending = false;
    };

    uint32_t tile = blockIdx.x;
    if (tile < a.ntiles) issue(tile * tile_bytes);
    for (int it = 0; tile < a.ntiles; tile += gridDim.x, ++it) {
        (void)it;
        PG_STAMP(0);
        const uint32_t toff = tile * tile_bytes;
        uint32_t V[NL][8];
#pragma unroll
        for (int s = 0; s < NL; ++s)
#pragma unroll
            for (int t = 0; t < 8; ++t) V[s][t] = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PG_STAMP(1);
        __syncthreads();                                         // the tile landed (all waves)
        PG_STAMP(2);
        flush();
        if (__builtin_expect(a.lo > 0 || (int64_t)toff + tile_bytes + kPyWin > (int64_t)a.span, 0)) fix(toff);
        if (!(a.ablate & 1)) static_for<0, NPW>([&](auto Jc) {
            constexpr int g = Q + NW * decltype(Jc)::value, w = g >> 3, p = g & 7;
            constexpr int p16 = kPyWin * w + 16 * p;             // first position of the piece
            if constexpr (p16 < HI) {
                if (w < w_lo) return;                            // wave-uniform (shortened codes)
                uint4 R[4];
                asm volatile("ds_read_b128 %0, %4\n\t"
                             "ds_read_b128 %1, %4 offset:8192\n\t"
                             "ds_read_b128 %2, %4 offset:16384\n\t"
                             "ds_read_b128 %3, %4 offset:24576\n\t"
                             "s_waitcnt lgkmcnt(0)"
                             : "=&v"(R[0]), "=&v"(R[1]), "=&v"(R[2]), "=&v"(R[3])
                             : "v"(lbuf + w * kPyWinBytes + rd(fresh_lane(), p)) : "memory");
                uint32_t X[16];
                {
                    const uint32_t c0[4] = {R[0].x, R[1].x, R[2].x, R[3].x};
                    const uint32_t c1[4] = {R[0].y, R[1].y, R[2].y, R[3].y};
                    const uint32_t c2[4] = {R[0].z, R[1].z, R[2].z, R[3].z};
                    const uint32_t c3[4] = {R[0].w, R[1].w, R[2].w, R[3].w};
                    transpose4x4(c0, X);
                    transpose4x4(c1, X + 4);
                    transpose4x4(c2, X + 8);
                    transpose4x4(c3, X + 12);
                }
                static_for<0, 2>([&](auto Bc) {
                    constexpr int p0 = p16 + 8 * decltype(Bc)::value;
                    if constexpr (p0 < HI) {
                        uint32_t Y[8];
#pragma unroll
                        for (int t = 0; t < 8; ++t) Y[t] = p0 + t < HI ? X[p0 - p16 + t] : 0u;
                        C::template block<p0 / 8>(V, Y);
                    }
                });
            }
        });
        PG_STAMP(3);
        __syncthreads();                                         // every wave is done with the tile
        PG_STAMP(4);
        // recursive-halving exchange through the tile buffer
        if (!(a.ablate & 2)) static_for<0, C::ROUNDS>([&](auto Rc) {
            constexpr int r = decltype(Rc)::value, P = Q ^ (1 << r), NS = C::NSEND[r];
            uint4 *x = reinterpret_cast<uint4 *>(buf);
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                const int s = C::SEND[Q][r][i];
                if (s < 0) continue;
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    x[((Q * NS + i) * 2 + h) * 64 + lane] =
                        make_uint4(V[s][4 * h], V[s][4 * h + 1], V[s][4 * h + 2], V[s][4 * h + 3]);
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                const int s = C::KEEP[Q][r][i];
                if (s < 0) continue;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint4 v = x[((P * NS + i) * 2 + h) * 64 + lane];
                    V[s][4 * h] ^= v.x;
                    V[s][4 * h + 1] ^= v.y;
                    V[s][4 * h + 2] ^= v.z;
                    V[s][4 * h + 3] ^= v.w;
                }
            }
            __syncthreads();                                     // read before reuse / the next DMA
        });
        PG_STAMP(5);
        if (tile + gridDim.x < a.ntiles) issue(toff + gridDim.x * tile_bytes);
        uint32_t T[NLW][8];
#pragma unroll
        for (int i = 0; i < NLW; ++i)
#pragma unroll
            for (int t = 0; t < 8; ++t) T[i][t] = C::OWN[Q][i] >= 0 ? V[C::OWN[Q][i] < 0 ? 0 : C::OWN[Q][i]][t] : 0u;
        const size_t cw0 = (size_t)tile * kTile + lane;          // byte k <-> codeword cw0 + 64k
        uint32_t nz = 0;
        uint32_t D[C::NQW][4];
#pragma unroll
        for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) D[qd][jj] = T[0][jj + qd];
        if (!(a.ablate & 4)) C::template epilogue<Q>(T, [&](auto Qc, uint32_t (&Qw)[8]) {
            constexpr int qd = decltype(Qc)::value;
            if constexpr (!ENC) {
                uint32_t vm = 0;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if (C::SYN[Q][qd][jj] >= 0) vm |= 0x01010101u << jj;
#pragma unroll
                for (int t = 0; t < 8; ++t) nz |= Qw[t] & vm;
            }
            transpose8(Qw);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) D[qd][jj] = Qw[jj];
        });
        pend_cw0 = cw0;
        pend_col = (size_t)tile * kTile + 4 * lane;
        pending = true;
        PG_STAMP(6);
        if constexpr (ENC) {
#pragma unroll
            for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) pend[qd][jj] = D[qd][jj];
        } else {
            uint32_t fl = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (nz >> (8 * k) & 0xFF) fl |= 1u << k;
            // OR over the waves (asm: the compiler would wait for the DMA in flight)
            const uint32_t fa = lds_addr(reinterpret_cast<uint8_t *>(&flags[Q][lane]));
            asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(fa), "v"(fl) : "memory");
            __syncthreads();
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                if (q == Q) continue;
                const uint32_t fb = lds_addr(reinterpret_cast<uint8_t *>(&flags[q][lane]));
                uint32_t fo;
                asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(fo) : "v"(fb) : "memory");
                fl |= fo;
            }
            if (a.neras) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (cw0 + 64 * k < a.ncw && a.neras[cw0 + 64 * k]) fl |= 1u << k;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (cw0 + 64 * k >= a.ncw) fl &= ~(1u << k);
            pend_fl = fl;
            if (fl) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (!(fl >> k & 1)) continue;
                    uint8_t *dst = a.ws + (cw0 + 64 * k) * 32;
#pragma unroll
                    for (int qd = 0; qd < C::NQW; ++qd)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) {
                            const int si = C::SYN[Q][qd][jj];
                            if (si >= 0) dst[si] = (uint8_t)(D[qd][jj] >> (8 * k));
                        }
                }
            }
        }
    }
    flush();
}

template <class C, bool ENC>
__global__ void __attribute__((amdgpu_flat_work_group_size(256, 256), amdgpu_waves_per_eu(2)))
k_pg_syndromes(PsArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[kPgTileBytes];
    __shared__ uint32_t flags[4][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    switch (wave) {
    case 0: pg_body<C, ENC, 0>(a, buf, flags, lane); break;
    case 1: pg_body<C, ENC, 1>(a, buf, flags, lane); break;
    case 2: pg_body<C, ENC, 2>(a, buf, flags, lane); break;
    default: pg_body<C, ENC, 3>(a, buf, flags, lane); break;
    }
}

// ---- encode, stage 2: parity = V^-1 S on 32-codeword bit-sliced registers -------------------
// Syndromes (encode workspace) -> parity rows.
// One 256-thread block covers 64 groups of 32 codewords (2048).  Phase 1: wave w transposes
// syndromes w, w+4, ... of every group (lane = group; the workspace row of syndrome i holds one
// byte per codeword, so a lane's 32 bytes are contiguous and a wave's loads are too) into bit
// planes in LDS (plane 8 i + q, group G at dword (8 i + q) * 64 + G; slot 8 k + m <-> codeword
// 32 G + 4 m + k).  Phase 2: wave P computes parity symbols 8P..8P+7 (generated q_pass),
// transposes them back to bytes and stages each codeword's parity row in LDS (per-group regions
// padded by 8 bytes: conflict-free 8-byte stores); then the rows are stored.
constexpr int kParGroups = 64;
constexpr int kParCw = 32 * kParGroups;

// Bytes s of a[0..3] -> one dword (a[0] in byte 0).
__device__ __forceinline__ uint32_t gather4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int s) {
    const uint32_t sel = (uint32_t)s | ((uint32_t)(s + 4) << 8) | 0x0c0c0000u;   // 0x0c: zero byte
    const uint32_t x01 = __builtin_amdgcn_perm(a1, a0, sel), x23 = __builtin_amdgcn_perm(a3, a2, sel);
    return __builtin_amdgcn_perm(x23, x01, 0x05040100u);
}

template <class C, bool PERM>
__global__ void __launch_bounds__(256) k_ps_parity(const uint8_t *ws, size_t ws_pitch, uint8_t *parity,
                                                   size_t pstride, size_t ncw) {
    constexpr int NR = C::NR;
    constexpr int kRegion = 32 * NR + 8;                       // bytes per group in the stage
    constexpr int kPlanes = 8 * NR * kParGroups;               // dwords
    constexpr int kStage = kParGroups * kRegion / 4;           // dwords
    constexpr int kLds = kPlanes > kStage ? kPlanes : kStage;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t g0 = (size_t)blockIdx.x * kParGroups;
    const uint8_t *src = ws + (g0 + lane) * 32;                // ws rows are padded to 2048 cw
    for (int i = wave; i < NR; i += 4) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(src + i * ws_pitch);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(src + i * ws_pitch + 16);
        uint32_t D[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        transpose8(D);                                         // D[q] bit 8k + m: cw 4m + k
#pragma unroll
        for (int qq = 0; qq < 8; ++qq) lds[(8 * i + qq) * 64 + lane] = D[qq];
    }
    __syncthreads();
    uint32_t O[8][8];
    switch (wave) {
    case 0: C::template q_pass<0>(O, lds + lane, 64); break;
    case 1: if constexpr (C::NPASS > 1) C::template q_pass<1>(O, lds + lane, 64); break;
    case 2: if constexpr (C::NPASS > 2) C::template q_pass<2>(O, lds + lane, 64); break;
    default: if constexpr (C::NPASS > 3) C::template q_pass<3>(O, lds + lane, 64); break;
    }
    __syncthreads();                                           // planes consumed
    uint8_t *stage = reinterpret_cast<uint8_t *>(lds);
    if (wave < C::NPASS) {
        const int nj = NR - 8 * wave < 8 ? NR - 8 * wave : 8;
#pragma unroll
        for (int jl = 0; jl < 8; ++jl)
            if (jl < nj) transpose8(O[jl]);                    // O[jl][m] byte k: symbol of cw 4m+k
        uint8_t *reg = stage + lane * kRegion + 8 * wave;
#pragma unroll
        for (int m = 0; m < 8; ++m)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint8_t *row = reg + (4 * m + k) * NR;
                const uint32_t lo = gather4(O[0][m], O[1][m], O[2][m], O[3][m], k);
                if (nj == 8) {
                    const uint32_t hi = gather4(O[4][m], O[5][m], O[6][m], O[7][m], k);
                    *reinterpret_cast<uint2 *>(row) = make_uint2(lo, hi);
                } else if (nj == 4) {
                    *reinterpret_cast<uint32_t *>(row) = lo;
                } else {
                    for (int jl = 0; jl < nj; ++jl) row[jl] = (uint8_t)(O[jl][m] >> (8 * k));
                }
            }
    }
    __syncthreads();
    const size_t cwb = g0 * 32;
    for (int r = threadIdx.x; r < kParCw; r += 256) {
        // workspace column -> codeword (PERM: tile-lane order of the pair kernel, 4l + j <-> 64j + l)
        const size_t x = cwb + r;
        const size_t k = PERM ? ((x & ~(size_t)255) | ((x & 3) << 6) | ((x >> 2) & 63)) : x;
        if (k >= ncw) continue;
        uint8_t *dst = parity + k * pstride;
        const uint8_t *s8 = stage + (r >> 5) * kRegion + (r & 31) * NR;
        if constexpr (NR % 8 == 0) {
#pragma unroll
            for (int o = 0; o < NR; o += 8) {
                uint2 v = *reinterpret_cast<const uint2 *>(s8 + o);
                __builtin_memcpy(dst + o, &v, 8);
            }
        } else if constexpr (NR % 4 == 0) {
#pragma unroll
            for (int o = 0; o < NR; o += 4) {
                uint32_t v = *reinterpret_cast<const uint32_t *>(s8 + o);
                __builtin_memcpy(dst + o, &v, 4);
            }
        } else {
            for (int o = 0; o < NR; ++o) dst[o] = s8[o];
        }
    }
}


// 8-wave form of k_ps_parity: wave P computes parity symbols 4P..4P+3 (q_pass4), halving each
// wave's share of the map and doubling the waves that hide the phases' latencies.
template <class C, bool PERM>
__global__ void __launch_bounds__(512) k_ps_parity8(const uint8_t *ws, size_t ws_pitch, uint8_t *parity,
                                                    size_t pstride, size_t ncw) {
    constexpr int NR = C::NR;
    constexpr int kRegion = 32 * NR + 8;                       // bytes per group in the stage
    constexpr int kPlanes = 8 * NR * kParGroups;               // dwords
    constexpr int kStage = kParGroups * kRegion / 4;           // dwords
    constexpr int kLds = kPlanes > kStage ? kPlanes : kStage;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t g0 = (size_t)blockIdx.x * kParGroups;
    const uint8_t *src = ws + (g0 + lane) * 32;                // ws rows are padded to 2048 cw
    for (int i = wave; i < NR; i += 8) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(src + i * ws_pitch);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(src + i * ws_pitch + 16);
        uint32_t D[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        transpose8(D);                                         // D[q] bit 8k + m: cw 4m + k
#pragma unroll
        for (int qq = 0; qq < 8; ++qq) lds[(8 * i + qq) * 64 + lane] = D[qq];
    }
    __syncthreads();
    uint32_t O[4][8];
    switch (wave) {
    case 0: C::template q_pass4<0>(O, lds + lane, 64); break;
    case 1: if constexpr (C::NPASS4 > 1) C::template q_pass4<1>(O, lds + lane, 64); break;
    case 2: if constexpr (C::NPASS4 > 2) C::template q_pass4<2>(O, lds + lane, 64); break;
    case 3: if constexpr (C::NPASS4 > 3) C::template q_pass4<3>(O, lds + lane, 64); break;
    case 4: if constexpr (C::NPASS4 > 4) C::template q_pass4<4>(O, lds + lane, 64); break;
    case 5: if constexpr (C::NPASS4 > 5) C::template q_pass4<5>(O, lds + lane, 64); break;
    case 6: if constexpr (C::NPASS4 > 6) C::template q_pass4<6>(O, lds + lane, 64); break;
    default: if constexpr (C::NPASS4 > 7) C::template q_pass4<7>(O, lds + lane, 64); break;
    }
    __syncthreads();                                           // planes consumed
    uint8_t *stage = reinterpret_cast<uint8_t *>(lds);
    if (wave < C::NPASS4) {
        const int nj = NR - 4 * wave < 4 ? NR - 4 * wave : 4;
#pragma unroll
        for (int jl = 0; jl < 4; ++jl)
            if (jl < nj) transpose8(O[jl]);                    // O[jl][m] byte k: symbol of cw 4m+k
        uint8_t *reg = stage + lane * kRegion + 4 * wave;
#pragma unroll
        for (int m = 0; m < 8; ++m)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint8_t *row = reg + (4 * m + k) * NR;
                if (nj == 4) {
                    *reinterpret_cast<uint32_t *>(row) = gather4(O[0][m], O[1][m], O[2][m], O[3][m], k);
                } else {
                    for (int jl = 0; jl < nj; ++jl) row[jl] = (uint8_t)(O[jl][m] >> (8 * k));
                }
            }
    }
    __syncthreads();
    const size_t cwb = g0 * 32;
    for (int r = threadIdx.x; r < kParCw; r += 512) {
        const size_t x = cwb + r;
        const size_t k = PERM ? ((x & ~(size_t)255) | ((x & 3) << 6) | ((x >> 2) & 63)) : x;
        if (k >= ncw) continue;
        uint8_t *dst = parity + k * pstride;
        const uint8_t *s8 = stage + (r >> 5) * kRegion + (r & 31) * NR;
        if constexpr (NR % 8 == 0) {
#pragma unroll
            for (int o = 0; o < NR; o += 8) {
                uint2 v = *reinterpret_cast<const uint2 *>(s8 + o);
                __builtin_memcpy(dst + o, &v, 8);
            }
        } else if constexpr (NR % 4 == 0) {
#pragma unroll
            for (int o = 0; o < NR; o += 4) {
                uint32_t v = *reinterpret_cast<const uint32_t *>(s8 + o);
                __builtin_memcpy(dst + o, &v, 4);
            }
        } else {
            for (int o = 0; o < NR; ++o) dst[o] = s8[o];
        }
    }
}

} // namespace ps

// ------------------------------------------------------------------------------------------------
namespace {

template <class C> bool ps_matches(const DevCodec &d) {
    return d.mm == 8 && d.nroots == C::NR && d.fcr == C::FCR && d.prim == C::PRIM && !d.dual &&
           d.poly == C::POLY;
}

// Syndrome kernel: 0 = pair (default), 3 = 4-wave group, 2 = 8-wave slices; EZRS_PS_VARIANT =
// pair | group4 | slices selects one for comparison runs.
int ps_variant() {
    static const int v = [] {
        const char *e = getenv("EZRS_PS_VARIANT");
        if (e && std::string(e) == "slices") return 2;
        if (e && std::string(e) == "group4") return 3;
        return 0;
    }();
    return v;
}

// Workgroups per launch (persistent over tiles): 2 per CU for the 8-wave slices and the 4-wave
// group kernels (64 KiB LDS each), 4 per CU for the pair kernel (32 KiB each).
unsigned syn_grid(const DevCodec &d, uint32_t ntiles, int var) {
    const uint32_t per_cu = var == 0 ? 4u : 2u;
    const uint32_t nwg = per_cu * (uint32_t)(d.ncu > 0 ? d.ncu : 256);
    return ntiles < nwg ? ntiles : nwg;
}

template <class C, bool ENC>
void launch_syn(int var, unsigned grid, const ps::PsArgs &p, hipStream_t s) {
    if (var == 0)
        hipLaunchKernelGGL((ps::k_py_syndromes<typename C::PY, ENC>), dim3(grid), dim3(128), 0, s, p);
    else if (var == 3)
        hipLaunchKernelGGL((ps::k_pg_syndromes<typename C::PG4, ENC>), dim3(grid), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((ps::k_ps_syndromes<typename C::PS, ENC>), dim3(grid), dim3(ps::kThreads), 0, s, p);
}

#define EZRS_PS_TRIPLE(C)                                                                         \
    struct T_##C {                                                                                \
        using PS = ps::PS_##C;                                                                    \
        using PY = ps::PY_##C;                                                                    \
        using PG4 = ps::PG4_##C;                                                                  \
    };
EZRS_PS_CODEC_LIST(EZRS_PS_TRIPLE)
#undef EZRS_PS_TRIPLE

} // namespace

int planeslice_codec_id(const DevCodec &d) {
    int id = 0, found = -1;
#define EZRS_PS_MATCH(C) \
    if (found < 0 && ps_matches<ps::PS_##C>(d)) found = id; \
    ++id;
    EZRS_PS_CODEC_LIST(EZRS_PS_MATCH)
#undef EZRS_PS_MATCH
    return found;
}

// Encode workspace: [NR][ws_pitch] bytes, ws_pitch = ncw rounded up to 2048 (the parity kernel's
// block); >= 32 bytes per codeword as decode needs.
static size_t ps_pitch(size_t ncw) { return (ncw + 2047) / 2048 * 2048; }
size_t ps_ws_bytes(size_t ncw) { return ps_pitch(ncw) * 32; }

// Largest batch one launch takes: the tile span must stay below 4 GiB (32-bit buffer offsets).
static size_t ps_max_rows(size_t stride) { return ((size_t)0xF0000000u / stride) / 2048 * 2048; }

bool ps_can_encode(const DevCodec &, const EncodeArgs &a) {
    return a.data_stride >= 1 && a.data_stride <= 256;
}

bool ps_can_decode(const DevCodec &d, const DecodeArgs &a) {
    const bool inline_par = a.parity == static_cast<char *>(a.data) + a.len && a.parity_stride == a.data_stride;
    return inline_par && a.data_stride <= 256 && a.data_stride >= a.len + d.nroots;
}

hipError_t launch_ps_encode(int id, const DevCodec &d, const EncodeArgs &a, void *ws, hipStream_t s) {
    const size_t maxr = ps_max_rows(a.data_stride);
    const int var = ps_variant();
    for (size_t k0 = 0; k0 < a.ncw; k0 += maxr) {
        const size_t n = a.ncw - k0 < maxr ? a.ncw - k0 : maxr;
        ps::PsArgs p{};
        p.base = static_cast<const uint8_t *>(a.data) + k0 * a.data_stride;
        p.span = (uint32_t)((n - 1) * a.data_stride + a.len);
        p.stride = (uint32_t)a.data_stride;
        p.ncw = (uint32_t)n;
        p.ntiles = (uint32_t)((n + ps::kTile - 1) / ps::kTile);
        p.lo = (int)(d.load - a.len);              // leading zero positions of a shortened code
        p.hi = (int)d.load;                        // data positions only
        p.ws = static_cast<uint8_t *>(ws);
        p.ws_pitch = ps_pitch(n);
        uint8_t *par = static_cast<uint8_t *>(a.parity) + k0 * a.parity_stride;
        const unsigned grid = syn_grid(d, p.ntiles, var);
        const unsigned pgrid = (unsigned)((n + ps::kParCw - 1) / ps::kParCw);
        int k = 0;
        // syndromes of the data positions, then parity = V^-1 S (the pair and group kernels leave
        // the workspace in tile-lane column order: PERM)
#define EZRS_PS_ENC(C)                                                                            \
        if (k++ == id) {                                                                          \
            launch_syn<T_##C, true>(var, grid, p, s);                                             \
            if (var == 2)                                                                         \
                hipLaunchKernelGGL((ps::k_ps_parity8<ps::PS_##C, false>), dim3(pgrid), dim3(512), 0, s, \
                                   static_cast<const uint8_t *>(ws), p.ws_pitch, par, a.parity_stride, n); \
            else                                                                                  \
                hipLaunchKernelGGL((ps::k_ps_parity8<ps::PS_##C, true>), dim3(pgrid), dim3(512), 0, s, \
                                   static_cast<const uint8_t *>(ws), p.ws_pitch, par, a.parity_stride, n); \
        }
        EZRS_PS_CODEC_LIST(EZRS_PS_ENC)
#undef EZRS_PS_ENC
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_ps_syndromes(int id, const DevCodec &d, const DecodeArgs &a, uint8_t *syn_ws,
                               hipStream_t s) {
    const size_t maxr = ps_max_rows(a.data_stride);
    const int var = ps_variant();
    for (size_t k0 = 0; k0 < a.ncw; k0 += maxr) {
        const size_t n = a.ncw - k0 < maxr ? a.ncw - k0 : maxr;
        ps::PsArgs p{};
        p.base = static_cast<const uint8_t *>(a.data) + k0 * a.data_stride;
        p.span = (uint32_t)((n - 1) * a.data_stride + a.len + d.nroots);
        p.stride = (uint32_t)a.data_stride;
        p.ncw = (uint32_t)n;
        p.ntiles = (uint32_t)((n + ps::kTile - 1) / ps::kTile);
        p.lo = (int)(d.load - a.len);
        p.hi = ps::kN;
        p.neras = a.neras ? a.neras + k0 : nullptr;
        p.result = a.result + k0;
        p.ws = syn_ws + k0 * 32;
        const unsigned grid = syn_grid(d, p.ntiles, var);
        int k = 0;
#define EZRS_PS_SYN(C)                                                                            \
        if (k++ == id) launch_syn<T_##C, false>(var, grid, p, s);
        EZRS_PS_CODEC_LIST(EZRS_PS_SYN)
#undef EZRS_PS_SYN
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace ezrs
