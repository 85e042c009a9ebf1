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
#else
#define PS_STAMP(ph) do { } while (0)
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

// ---- encode, stage 2: parity = V^-1 S on 32-codeword bit-sliced registers -------------------
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

template <class C>
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
        const size_t k = cwb + r;
        if (k >= ncw) break;
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

int ps_grid(const DevCodec &d, uint32_t ntiles) {
    const uint32_t nwg = 2u * (uint32_t)(d.ncu > 0 ? d.ncu : 256);   // 2 workgroups per CU
    return (int)(ntiles < nwg ? ntiles : nwg);
}

} // namespace

int planeslice_codec_id(const DevCodec &d) {
    int id = 0, found = -1;
#define EZRS_PS_MATCH(C) \
    if (found < 0 && ps_matches<ps::C>(d)) found = id; \
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
        const unsigned grid = (unsigned)ps_grid(d, p.ntiles);
        const unsigned pgrid = (unsigned)((n + ps::kParCw - 1) / ps::kParCw);
        int k = 0;
#define EZRS_PS_ENC(C)                                                                            \
        if (k++ == id) {                                                                          \
            hipLaunchKernelGGL((ps::k_ps_syndromes<ps::C, true>), dim3(grid), dim3(ps::kThreads), \
                               0, s, p);                                                         \
            hipLaunchKernelGGL(ps::k_ps_parity<ps::C>, dim3(pgrid), dim3(256), 0, s,              \
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
        const unsigned grid = (unsigned)ps_grid(d, p.ntiles);
        int k = 0;
#define EZRS_PS_SYN(C)                                                                            \
        if (k++ == id)                                                                            \
            hipLaunchKernelGGL((ps::k_ps_syndromes<ps::C, false>), dim3(grid), dim3(ps::kThreads),\
                               0, s, p);
        EZRS_PS_CODEC_LIST(EZRS_PS_SYN)
#undef EZRS_PS_SYN
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace ezrs
