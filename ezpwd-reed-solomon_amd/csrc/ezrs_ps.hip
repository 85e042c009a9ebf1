// ezrs_ps.hip -- plane-sliced GF(2^8) RS kernels for MI355X (gfx950): syndromes (decode) and
// parity (encode) of batches of 255-symbol codewords.
//
// Decode computes the syndromes S_i = r(alpha^((fcr+i)*prim)) of c++/ezpwd/rs_base:1390-1414.  A
// codeword whose syndromes are all zero (and that carries no erasures) gets result 0, exactly
// decode_symbols' early return (rs_base:1416-1434); every other codeword gets a sentinel and its
// syndromes go to the workspace for the error path (ezrs_errors.hip: k_decode_errors).  Encode
// computes the parity of encode_symbols (rs_base:1296-1332) directly from the data symbols.
//
// Arithmetic (codegen/gen_ps.py has the derivation): a 32-bit word holds one position of four
// codewords, bit 8k + b = bit-plane b of codeword k.  Each bit is a GF(2) stream.  Only one root per
// cyclotomic coset ("leader") is evaluated -- V_{b,2e} = V_{b,e}^2 -- and the per-plane values are
// expanded and folded into syndromes (S = sum_b alpha^b V_b) once per tile: 16 leaders x 8 bits
// for RS(255,223).  Encode evaluates the syndromes of the data positions; k_ps_parity8 maps them to
// parity (parity = V^-1 S, bit-sliced over 32 codewords per lane).
//
// Tile kernel k_pt_lin: one 512-thread workgroup (8 waves) per 256-codeword tile, two workgroups per
// CU (80 KiB of LDS each, <= 128 VGPRs: 4 waves per SIMD), persistent over tiles.
//   * The tile's rows are one contiguous span of HBM; 1 KiB LDS-DMA instructions copy it to LDS as it
//     lies (every line fetched once), the next tile's while this tile's epilogue runs.  Lane l owns
//     rows 4l .. 4l+3 (byte k of its words = row 4l + k); with an odd pitch the row starts fall in 32
//     distinct banks, so the row reads (4-byte aligned, then v_alignbyte) are conflict-free.
//   * Waves split the leaders into GN groups and the 16-position pieces into QN = 8 / GN quarters;
//     every quarter runs quarter 0's networks and then multiplies its partials by alpha^(-16 q e).
//   * A recursive-halving exchange through the consumed image leaves every wave the totals of the
//     leaders its generated epilogue folds: 4 syndromes (one quad) per wave.
//   * Shard batches (SH): per-row offsets and pads come from a per-tile row table; the bytes before a
//     shortened row's own pad (the previous row's, in the linear image) are masked off.
//   * All LDS traffic, LDS-DMA and global stores are inline asm with counted s_waitcnt: the
//     compiler would otherwise wait for every DMA in flight at each LDS access or barrier.
//   * Measured and dropped: a row-pitched, swizzled image gathered by unaligned per-lane LDS-DMA
//     (conflict-free aligned ds_read_b128, no v_alignbyte) -- encode 0.177 / decode 0.139 ms per
//     1 M-codeword call against 0.143 / 0.109 for the linear image; the parity pass fused into this
//     kernel every 8 tiles (workgroups reach it in lockstep, nothing overlaps it: 0.143 vs 0.144 ms);
//     a persistent parity kernel (one workgroup per CU, planes and row stage in separate LDS, the
//     next chunk's workspace loads in flight during the map): 0.149 vs 0.144 ms.
//
#include "ezrs_internal.hpp"

#include <atomic>
#include "gen/ezrs_ps_tables.inc"
#ifdef EZRS_PS_ONLY_223
// timing-experiment builds only (tools/build_variant.sh): the plane-sliced path for RS(255,223)
// alone (every other codec takes the generic kernels), so a variant compiles in about a minute
#undef EZRS_PS_CODEC_LIST
#define EZRS_PS_CODEC_LIST(X) X(RS_255_223)
#endif

namespace ezrs {
namespace ps {

constexpr int kTile = 256;                          // codewords per tile
constexpr int32_t kSentinel = INT32_MIN;
constexpr int kN = 255;

typedef __attribute__((address_space(3))) void lds_void;

#ifdef EZRS_PS_STAMPS
// tools/micro/pt_stamps.hip: phase stamps of the linear tile kernel, [wg][wave][tile][phase]
__device__ unsigned long long g_pt_stamps[16][8][8][8];
#define PT_STAMP(ph) do { __builtin_amdgcn_sched_barrier(0); if (blockIdx.x < 16 && pt_it < 8 && \
    __lane_id() == 0) g_pt_stamps[blockIdx.x][pt_w][pt_it][ph] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
// tools/micro/pq_stamps.hip: the same for the 4-wave kernel, [wg][wave][tile][phase]
__device__ unsigned long long g_pq_stamps[512][4][9][8];
__device__ unsigned long long g_pq_rt[512][4];             // wave 0: realtime + memtime at start / end
__device__ unsigned g_pq_hw[512][2];                       // wave 0: HW_ID, XCC_ID
#define PQ_STAMP(ph) do { __builtin_amdgcn_sched_barrier(0); if (blockIdx.x < 512 && pq_it < 9 && \
    __lane_id() == 0) g_pq_stamps[blockIdx.x][W][pq_it][ph] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#define PQ_RT(i) do { __builtin_amdgcn_sched_barrier(0); if (blockIdx.x < 512 && W == 0 && __lane_id() == 0) { \
    g_pq_rt[blockIdx.x][2 * (i)] = __builtin_amdgcn_s_memrealtime(); \
    g_pq_rt[blockIdx.x][2 * (i) + 1] = __builtin_amdgcn_s_memtime(); \
    if ((i) == 0) { g_pq_hw[blockIdx.x][0] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)); \
                    g_pq_hw[blockIdx.x][1] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11)); } } \
    __builtin_amdgcn_sched_barrier(0); } while (0)
// tools/micro/par_stamps.hip: the parity kernel's phases, [block][wave][phase]
__device__ unsigned long long g_par_stamps[64][8][8];
__device__ unsigned long long g_par_rt[4096][2];           // s_memrealtime (100 MHz) at wave 0's start / end
__device__ unsigned g_par_hw[4096];                        // HW_ID of wave 0
#define PAR_STAMP(ph) do { __builtin_amdgcn_sched_barrier(0); if (__lane_id() == 0) { \
    if (blockIdx.x < 64) g_par_stamps[blockIdx.x][wave][ph] = __builtin_amdgcn_s_memtime(); \
    if (wave == 0 && (ph == 0 || ph == 7) && blockIdx.x < 4096) { \
        g_par_rt[blockIdx.x][ph == 7] = __builtin_amdgcn_s_memrealtime(); \
        if (ph == 0) g_par_hw[blockIdx.x] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)); } } \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define PT_STAMP(ph) do { } while (0)
#define PQ_STAMP(ph) do { } while (0)
#define PQ_RT(i) do { } while (0)
#define PAR_STAMP(ph) do { } while (0)
#endif

struct PsArgs {
    const uint8_t *base;        // row 0 of the batch
    uint32_t span;              // bytes readable from base
    uint32_t stride;            // row pitch in bytes (<= 256)
    uint32_t ncw;               // codewords
    uint32_t ntiles;
    int lo;                     // full-frame position of the rows' first byte (the pad)
    int32_t *result;            // decode
    uint8_t *ws;                // decode: tiled syndromes (kSynTile); encode: [NR][ws_pitch]
    size_t ws_pitch;            // encode: codewords per syndrome row (a multiple of 2048); decode:
                                // the launch's first codeword mod 256 (its place in the tiled layout)
    uint32_t srows;             // shard batches (Shards): codewords per shard, 0 = a plain batch
    int stail_lo;               // full-frame position of a shard's last row's first byte
    uint32_t spitch;            // shard pitch in bytes
    int ablate;                 // timing experiments only (tools/pt_ablate.py, EZRS_PT_ABLATE): bit 0
                                // no main loop, 1 no exchange, 2 no fold, 3 no DMA, 5 nothing flagged
    uint32_t *flag;             // decode: gen stored here when a codeword is flagged (DecodeArgs)
    uint32_t gen;
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

// ---- LDS and buffer-resource helpers ----------------------------------------------------------
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

// Bytes s of a[0..3] -> one dword (a[0] in byte 0).
__device__ __forceinline__ uint32_t gather4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int s) {
    const uint32_t sel = (uint32_t)s | ((uint32_t)(s + 4) << 8) | 0x0c0c0000u;   // 0x0c: zero byte
    const uint32_t x01 = __builtin_amdgcn_perm(a1, a0, sel), x23 = __builtin_amdgcn_perm(a3, a2, sel);
    return __builtin_amdgcn_perm(x23, x01, 0x05040100u);
}

// ---- tile kernel (default) ---------------------------------------------------------------------
namespace pt {

constexpr int kThreads = 512;
constexpr int kLds = 81920;                   // 80 KiB: two workgroups per CU
constexpr int kGuard = 256;                   // bytes before the image: row 0's pad positions
constexpr int kImage = 65536;                 // the tile image (256 rows x pitch <= 256 B)
constexpr int kFlags = kGuard + kImage;       // decode flags [8][64] after the image
constexpr int kTab = kFlags + 2048;           // shard batches: per-row image offset and pad [256]
constexpr uint32_t kOob = 0xF0000000u;        // a buffer offset past every span (ps_max_rows)
static_assert(kTab + 1024 <= kLds, "tile kernel LDS");
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// The lane id, recomputed (v_mbcnt) wherever it is used: values derived from it are then not
// hoisted out of the tile loop, where they would pin registers across the state.
__device__ __forceinline__ uint32_t fresh(uint32_t = 0) {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

template <int N> __device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ void store_dword(pw_rsrc_t r, uint32_t off, uint32_t v) {
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen" :: "v"(v), "v"(off), "s"(r) : "memory");
}
__device__ __forceinline__ void store_byte(pw_rsrc_t r, uint32_t off, uint32_t v) {
    asm volatile("buffer_store_byte %0, %1, %2, 0 offen" :: "v"(v), "v"(off), "s"(r) : "memory");
}

// Recursive-halving exchange, sub-rounds S.. (see gen_ps.py PtRole): send the XS items to the
// area, then add the partner's XV items.  lx = this lane's byte in wave 0's slot 0.
template <class C, int W, int S, int J = 0>
__device__ __forceinline__ void xsend(uint32_t (&V)[C::NI][8], uint32_t lx) {
    if constexpr (J < C::XCAP) {
        constexpr int it = C::XS[W][S][J];
        if constexpr (it >= 0) {
            const u32x4 w0 = {V[it][0], V[it][1], V[it][2], V[it][3]};
            const u32x4 w1 = {V[it][4], V[it][5], V[it][6], V[it][7]};
            asm volatile("ds_write_b128 %0, %1 offset:%3\n\t"
                         "ds_write_b128 %0, %2 offset:%4"
                         :: "v"(lx + W * C::XCAP * 2048u), "v"(w0), "v"(w1), "n"(J * 2048),
                            "n"(J * 2048 + 1024) : "memory");
        }
        xsend<C, W, S, J + 1>(V, lx);
    }
}
// Add the partner PW's items of sub-round S (XV) into V, the reads two items ahead of the XORs:
// LDS latency is paid once per sub-round, not once per item.
template <class C, int W, int S>
constexpr int xnext(int j) {
    ++j;
    while (j < C::XCAP && C::XV[W][S][j] < 0) ++j;
    return j;
}
template <class C, int PW, int J>
__device__ __forceinline__ void xread(u32x4 (&b)[2], uint32_t lx) {
    asm volatile("ds_read_b128 %0, %2 offset:%3\n\t"
                 "ds_read_b128 %1, %2 offset:%4"
                 : "=&v"(b[0]), "=&v"(b[1]) : "v"(lx + PW * C::XCAP * 2048u), "n"(J * 2048), "n"(J * 2048 + 1024)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void xwait(u32x4 (&b)[2]) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(b[0]), "+v"(b[1]) : "n"(N) : "memory");
}
// cur = item J and nx = item xnext(J) are in flight
template <class C, int W, int S, int PW, int J>
__device__ __forceinline__ void xrecv_run(uint32_t (&V)[C::NI][8], uint32_t lx, u32x4 (&cur)[2], u32x4 (&nx)[2]) {
    if constexpr (J < C::XCAP) {
        constexpr int J1 = xnext<C, W, S>(J), J2 = xnext<C, W, S>(J1);
        u32x4 nn[2];
        if constexpr (J2 < C::XCAP) {
            xread<C, PW, J2>(nn, lx);
            xwait<4>(cur);
        } else if constexpr (J1 < C::XCAP) {
            xwait<2>(cur);
        } else {
            xwait<0>(cur);
        }
        constexpr int it = C::XV[W][S][J];
        V[it][0] ^= cur[0].x; V[it][1] ^= cur[0].y; V[it][2] ^= cur[0].z; V[it][3] ^= cur[0].w;
        V[it][4] ^= cur[1].x; V[it][5] ^= cur[1].y; V[it][6] ^= cur[1].z; V[it][7] ^= cur[1].w;
        xrecv_run<C, W, S, PW, J1>(V, lx, nx, nn);
    }
}
template <class C, int W, int S, int PW>
__device__ __forceinline__ void xrecv_pipe(uint32_t (&V)[C::NI][8], uint32_t lx) {
    constexpr int J0 = xnext<C, W, S>(-1), J1 = xnext<C, W, S>(J0);
    u32x4 a[2], b[2];
    if constexpr (J0 < C::XCAP) xread<C, PW, J0>(a, lx);
    if constexpr (J1 < C::XCAP) xread<C, PW, J1>(b, lx);
    xrecv_run<C, W, S, PW, J0>(V, lx, a, b);
}
template <class C, int W, int S>
__device__ __forceinline__ void xrecv(uint32_t (&V)[C::NI][8], uint32_t lx) {
    xrecv_pipe<C, W, S, W ^ (C::GN << C::XR[S])>(V, lx);
}
template <class C, int W, int S>
__device__ __forceinline__ void exchange(uint32_t (&V)[C::NI][8], uint32_t lx) {
    if constexpr (S < C::NSUB) {
        xsend<C, W, S>(V, lx);
        wait_lgkm();
        barrier();
        xrecv<C, W, S>(V, lx);
        barrier();                                           // read before the area is reused
        exchange<C, W, S + 1>(V, lx);
    }
}

// The tile's rows are one contiguous span; 64 line-aligned 1 KiB DMA instructions copy it to LDS as
// it lies (fetch-efficient: every 128-byte line is read once, by one instruction).  Lane l owns rows
// 4l .. 4l+3 (byte k of its words = row 4l + k): with an odd pitch P the rows' starts 4lP fall in
// 32 distinct LDS banks, so the row reads (ds_read2_b32, 4-byte aligned, then v_alignbyte by the
// row's byte phase (kP - lo) mod 4) are conflict-free (an even pitch is correct, with conflicts).
// One tile buffer per workgroup; the other workgroup on the CU computes while this one's next tile
// lands.  The exchange uses the whole 80 KiB once the image is consumed.

// Shard batches: byte offset (from the span base) and pad (full-frame position of the first byte)
// of codeword k.  Row j of shard q sits at q * spitch + j * stride; a shard's last row is shortened.
__device__ __forceinline__ uint32_t row_at(const PsArgs &a, uint32_t k, int &lo) {
    const uint32_t q = k / a.srows, j = k - q * a.srows;
    lo = j + 1 == a.srows ? a.stail_lo : a.lo;
    return q * a.spitch + j * a.stride;
}

// A shard tile's DMA start moved down to the 16-byte grid (its image then begins up to 15 bytes
// early; the row table's offsets are taken from the same start): the 1 KiB LDS-DMA pieces of a
// tile that starts mid-row are otherwise misaligned 16-byte loads, each split in the memory
// pipeline (r05r: 1 MiB shards decode 114.7 us against 80.2 us for a plain batch of as many
// codewords).  Kept as is when the widened span would pass the image.
__device__ __forceinline__ uint32_t sh_align(uint32_t off, uint32_t &bytes) {
    const uint32_t mis = off & 15u;
    if (bytes + mis > (uint32_t)kImage) return off;
    bytes += mis;
    return off - mis;
}

__device__ __forceinline__ void issue_tile_lin(uint32_t lbuf, pw_rsrc_t rsrc, uint32_t toff, uint32_t tile_bytes,
                                               int w, int ablate) {
    if (ablate & 8) return;
    const uint32_t ninstr = (tile_bytes + 1023) >> 10;
    const uint32_t lo16 = 16u * fresh();
    for (uint32_t i = w; i < ninstr; i += 8)
        asm volatile("s_mov_b32 m0, %0\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %1, %2, 0 offen lds"
                     :: "s"(lbuf + kGuard + i * 1024u), "v"(toff + i * 1024u + lo16), "s"(rsrc) : "memory", "m0");
}

// Positions pa .. pa+7 (words X) with the network of quarter 0's block B0; positions before lo
// (the zero pad of a shortened code: the image holds the previous row's bytes there) and at or
// past HI contribute nothing.  pa, lo wave-uniform.
// F: the wave's first block (sets the state: never skipped, its masked positions are zeros).
// LO0: full-length rows (lo == 0, the common case): no run-time masks, so no branches -- the
// branches around every block cost a register shuffle each.
template <class C, int G, int HI, int B0, int PA, bool F, bool LO0>
__device__ __forceinline__ void block8_rt(uint32_t (&V)[C::NI][8], uint32_t (&X)[8], int lo) {
    constexpr int dhi = HI - PA;
    if constexpr (dhi <= 0 && !F) return;
    if constexpr (dhi < 8) {
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (t >= dhi) X[t] = 0;
    }
    if constexpr (!LO0) {
        const int dlo = lo - PA;                             // wave-uniform
        if (!F && dlo >= 8) return;
#pragma unroll
        for (int t = 0; t < 8; ++t) X[t] = t < dlo ? 0u : X[t];
    }
    C::template block<G, B0, F>(V, X);
}

// Rows 4l + k, positions pa .. pa+15 (k = 0..3): R[k] = 16 bytes of row k.
__device__ __forceinline__ void read_rows_lin(u32x4 (&R)[4], uint32_t lbuf, uint32_t stride, int pa, int lo,
                                              const uint32_t (&ph)[4]) {
    const uint32_t base = lbuf + kGuard + 4u * fresh() * stride + (uint32_t)(pa - lo);
    u32x2 e[4][2];
    uint32_t d4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t at = (base + k * stride) & ~3u;
        asm volatile("ds_read2_b32 %0, %3 offset1:1\n\t"
                     "ds_read2_b32 %1, %3 offset0:2 offset1:3\n\t"
                     "ds_read_b32 %2, %3 offset:16"
                     : "=&v"(e[k][0]), "=&v"(e[k][1]), "=&v"(d4[k]) : "v"(at) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(e[0][0]), "+v"(e[0][1]), "+v"(d4[0]), "+v"(e[1][0]), "+v"(e[1][1]), "+v"(d4[1]),
                   "+v"(e[2][0]), "+v"(e[2][1]), "+v"(d4[2]), "+v"(e[3][0]), "+v"(e[3][1]), "+v"(d4[3])
                 :: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t d[5] = {e[k][0].x, e[k][0].y, e[k][1].x, e[k][1].y, d4[k]};
#pragma unroll
        for (int j = 0; j < 4; ++j) R[k][j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], ph[k]);
    }
}

// Shard batches: rows 4l + k from their row-table entries e (image offset of position 0 | pad << 24,
// written at the tile's start); in the pieces below the shortened rows' pad (pa < tail_lo, only in
// tiles that hold a shortened row) the bytes before each row's own pad -- the previous row's, in
// the linear image -- are masked off.
__device__ __forceinline__ void read_rows_shard(u32x4 (&R)[4], uint32_t lbuf, int pa, int tail_lo, const u32x4 &e) {
    u32x2 d2[4][2];
    uint32_t d4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t at = (lbuf + (e[k] & 0xFFFFFFu) + (uint32_t)pa) & ~3u;
        asm volatile("ds_read2_b32 %0, %3 offset1:1\n\t"
                     "ds_read2_b32 %1, %3 offset0:2 offset1:3\n\t"
                     "ds_read_b32 %2, %3 offset:16"
                     : "=&v"(d2[k][0]), "=&v"(d2[k][1]), "=&v"(d4[k]) : "v"(at) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(d2[0][0]), "+v"(d2[0][1]), "+v"(d4[0]), "+v"(d2[1][0]), "+v"(d2[1][1]), "+v"(d4[1]),
                   "+v"(d2[2][0]), "+v"(d2[2][1]), "+v"(d4[2]), "+v"(d2[3][0]), "+v"(d2[3][1]), "+v"(d4[3])
                 :: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t d[5] = {d2[k][0].x, d2[k][0].y, d2[k][1].x, d2[k][1].y, d4[k]};
        const uint32_t sh = lbuf + (e[k] & 0xFFFFFFu) + (uint32_t)pa;      // byte phase in bits 0..1
#pragma unroll
        for (int j = 0; j < 4; ++j) R[k][j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
    }
    if (pa < tail_lo) {                                      // wave-uniform
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int z8 = 8 * ((int)(e[k] >> 24) - pa);     // pad bits at the piece's start
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = min(max(z8 - 32 * j, 0), 32);
                R[k][j] &= (uint32_t)(0xFFFFFFFFull << c);
            }
        }
    }
}

// Quarter Q's pieces, each with its own networks (block index = its absolute 8-position block).
template <class C, int G, int Q, int HI, bool SH, bool LO0>
__device__ __forceinline__ void lin_pass(uint32_t (&V)[C::NI][8], uint32_t lbuf, uint32_t stride, int lo,
                                         const uint32_t (&ph)[4], int tail_lo) {
    constexpr int BQ = Q;
    constexpr int NP = C::NP0[G] + C::NP1[G];
    static_assert(16 * (C::PIECE[G][0] + Q) < HI, "the wave's first block sets its state");
    u32x4 e = {0, 0, 0, 0};
    if constexpr (SH)
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(e) : "v"(lbuf + kTab + 16u * fresh()) : "memory");
    static_for<0, NP>([&](auto Ic) {
        constexpr int I = decltype(Ic)::value;
        constexpr int p0 = C::PIECE[G][I];
        if constexpr (16 * p0 < HI) {
            constexpr int pa = 16 * (p0 + Q);
            if constexpr (pa < HI) {
                u32x4 R[4];
                if constexpr (SH) read_rows_shard(R, lbuf, pa, tail_lo, e);
                else read_rows_lin(R, lbuf, stride, pa, lo, ph);
                uint32_t X[8];
                {
                    const uint32_t c0[4] = {R[0].x, R[1].x, R[2].x, R[3].x};
                    const uint32_t c1[4] = {R[0].y, R[1].y, R[2].y, R[3].y};
                    transpose4x4(c0, X);
                    transpose4x4(c1, X + 4);
                }
                block8_rt<C, G, HI, 2 * (p0 + BQ), pa, I == 0, LO0>(V, X, lo);
                {
                    const uint32_t c2[4] = {R[0].z, R[1].z, R[2].z, R[3].z};
                    const uint32_t c3[4] = {R[0].w, R[1].w, R[2].w, R[3].w};
                    transpose4x4(c2, X);
                    transpose4x4(c3, X + 4);
                }
                block8_rt<C, G, HI, 2 * (p0 + BQ) + 1, pa + 8, false, LO0>(V, X, lo);
            }
        }
    });
}

// Fix-up, exchange (through the consumed image), next tile's DMA, fold and stores of wave W.
template <class C, bool ENC, int W>
__device__ __forceinline__ void wave_tail_lin(uint32_t (&V)[C::NI][8], const PsArgs &a, uint32_t lbuf,
                                              uint32_t tile, uint32_t noff, uint32_t nbytes,
                                              pw_rsrc_t rsrc, pw_rsrc_t rout, pw_rsrc_t rws, int pt_it = 0) {
    const int pt_w = W;
    (void)pt_it; (void)pt_w;
    constexpr int G = W % C::GN, Q = W / C::GN;
    if (!(a.ablate & 2)) {
        exchange<C, W, 0>(V, lbuf + 16u * fresh());         // slot (W XCAP + j) at 2 KiB each
    }
    PT_STAMP(4);
    if (noff != kOob) issue_tile_lin(lbuf, rsrc, noff, nbytes, W, a.ablate);
    uint32_t T[C::NOWN][8];
#pragma unroll
    for (int i = 0; i < C::NOWN; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) T[i][t] = C::OWN[W][i] >= 0 ? V[C::OWN[W][i] < 0 ? 0 : C::OWN[W][i]][t] : 0u;
    uint32_t Qs[8] = {0, 0, 0, 0, 0, 0, 0, 0}, nz = 0;
    constexpr uint32_t vm = (C::SYN[W][0][0] >= 0 ? 0x01010101u : 0u) | (C::SYN[W][0][1] >= 0 ? 0x02020202u : 0u) |
                            (C::SYN[W][0][2] >= 0 ? 0x04040404u : 0u) | (C::SYN[W][0][3] >= 0 ? 0x08080808u : 0u);
    if (!(a.ablate & 4))
        C::template epilogue<W>(T, [&](auto, uint32_t (&Qw)[8]) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                nz |= Qw[t] & vm;
                Qs[t] = Qw[t];
            }
        }, [](auto) {});
    PT_STAMP(5);
    const uint32_t cw0 = tile * kTile + 4u * fresh();        // byte k <-> codeword cw0 + k
    if constexpr (ENC) {
        transpose8(Qs);                                      // Qs[jj] byte k: syndrome jj, codeword k
        // syndrome-major workspace in codeword order: the dword at column cw0 holds cw0 .. cw0+3
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
            if (C::SYN[W][0][jj] >= 0) store_dword(rws, (uint32_t)(C::SYN[W][0][jj] * a.ws_pitch) + cw0, Qs[jj]);
    } else {
        uint32_t fl = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (nz >> (8 * k) & 0xFF) fl |= 1u << k;
        const uint32_t fa = lbuf + kFlags + 256u * W + 4u * fresh();
        asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(fa), "v"(fl) : "memory");
        barrier();
        {
            uint32_t f[8];
            const uint32_t fb = lbuf + kFlags + 4u * fresh();
            asm volatile("ds_read_b32 %0, %8\n\t"
                         "ds_read_b32 %1, %8 offset:256\n\t"
                         "ds_read_b32 %2, %8 offset:512\n\t"
                         "ds_read_b32 %3, %8 offset:768\n\t"
                         "ds_read_b32 %4, %8 offset:1024\n\t"
                         "ds_read_b32 %5, %8 offset:1280\n\t"
                         "ds_read_b32 %6, %8 offset:1536\n\t"
                         "ds_read_b32 %7, %8 offset:1792\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]),
                           "=&v"(f[5]), "=&v"(f[6]), "=&v"(f[7]) : "v"(fb) : "memory");
            fl = f[0] | f[1] | f[2] | f[3] | f[4] | f[5] | f[6] | f[7];
            if (a.ablate & 32) fl = 0;                       // timing runs: keep the error path idle
        }
        if constexpr (W == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                store_dword(rout, (cw0 + k) * 4u, (fl >> k & 1) ? (uint32_t)kSentinel : 0u);
            if (fl != 0 && a.flag) *a.flag = a.gen;          // this call flagged a codeword
        }
        if (__ballot(fl != 0) != 0) {                        // flagged codewords: their syndromes
            transpose8(Qs);                                  // Qs[jj] byte k: syndrome jj, codeword k
            // tiled layout (ezrs_internal.hpp kSynTile): syndrome j of the 256 codewords of a tile in
            // one 256-byte row, so a lane's four codewords are one dword (unflagged ones included)
            if (a.ws_pitch == 0) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if (C::SYN[W][0][jj] >= 0)
                        store_dword(rws, tile * (uint32_t)kSynTile + 256u * C::SYN[W][0][jj] + 4u * fresh(),
                                    Qs[jj]);
            } else {                                         // a launch not starting a tile (shards)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t g = (uint32_t)a.ws_pitch + cw0 + k;
                    const uint32_t row = (fl >> k & 1) ? (g >> 8) * (uint32_t)kSynTile + (g & 255u) : kOob;
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        if (C::SYN[W][0][jj] >= 0) store_byte(rws, row + 256u * C::SYN[W][0][jj], Qs[jj] >> (8 * k));
                }
            }
        }
    }
    PT_STAMP(6);
}

template <class C, bool ENC, int W, bool SH, bool LO0>
__device__ __forceinline__ void pt_run_lin(const PsArgs &a, uint8_t *lds) {
    constexpr int G = W % C::GN, Q = W / C::GN;
    const int w = W;
    constexpr int HI = ENC ? kN - (int)C::NR : kN;
    const pw_rsrc_t rsrc = pw_rsrc(a.base, a.span);
    const uint32_t lbuf = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    const pw_rsrc_t rout = pw_rsrc(reinterpret_cast<const uint8_t *>(a.result), ENC ? 0u : a.ncw * 4u);
    const pw_rsrc_t rws = pw_rsrc(a.ws, ENC ? (uint32_t)(C::NR * a.ws_pitch)
                                            : (uint32_t)((a.ws_pitch + a.ncw + 255) / 256 * kSynTile));
    constexpr bool shards = SH;
    // byte range of tile t: plain batches t * 256 rows of pitch stride; shard batches from its first
    // row's start to the next tile's (the span's end for the last tile)
    auto tile_range = [&](uint32_t t, uint32_t &bytes) -> uint32_t {
        if (!shards) {
            bytes = a.stride * kTile;
            return t * bytes;
        }
        int lo;
        const uint32_t t0 = t * kTile, off = row_at(a, t0, lo);
        bytes = (t0 + kTile < a.ncw ? row_at(a, t0 + kTile, lo) : a.span) - off;
        return sh_align(off, bytes);
    };
    uint32_t tile = blockIdx.x;
    uint32_t tbytes, toff = tile < a.ntiles ? tile_range(tile, tbytes) : 0u;
    if (tile < a.ntiles) issue_tile_lin(lbuf, rsrc, toff, tbytes, w, a.ablate);
    int pt_it = 0, pt_w = w;
    (void)pt_it; (void)pt_w;
    for (; tile < a.ntiles; tile += gridDim.x, ++pt_it) {
        // run-time values re-read each tile: nothing derived from them is hoisted out of the loop
        int lo = a.lo;
        asm volatile("" : "+s"(lo));
        uint32_t ph[4];                                      // byte phase of row k's start
#pragma unroll
        for (int k = 0; k < 4; ++k) ph[k] = (lbuf + kGuard + k * a.stride - (uint32_t)lo) & 3u;
        uint32_t nbytes = 0;
        const uint32_t noff = tile + gridDim.x < a.ntiles ? tile_range(tile + gridDim.x, nbytes) : kOob;
        uint32_t V[C::NI][8];                                // set by the wave's first block
        PT_STAMP(0);
        wait_vm<0>();                                        // the tile landed (and the stores went)
        if constexpr (SH) {                                  // row table: wave w writes rows 32w ..
            const uint32_t j = fresh();
            if (j < 32u) {
                const uint32_t r = 32u * (uint32_t)w + j, k = tile * kTile + r;
                uint32_t e = kGuard;
                if (k < a.ncw) {
                    int rlo;
                    const uint32_t at = row_at(a, k, rlo);
                    e = (kGuard + at - toff - (uint32_t)rlo) | ((uint32_t)rlo << 24);
                }
                asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(lbuf + kTab + 4u * r), "v"(e) : "memory");
            }
        }
        barrier();
        PT_STAMP(1);
        if (toff + tbytes >= a.span) {                       // last tile: the span's final bytes
            // a 16-byte DMA piece that crosses the span's end comes back all-zero: re-read the last
            // 64 bytes one by one (out-of-range bytes read as zero)
            if (w == 0) {
                const uint32_t off = a.span - 64u + fresh();
                uint32_t v;
                asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                             : "=&v"(v) : "v"(off), "s"(rsrc) : "memory");
                if (off >= toff && off < a.span)
                    asm volatile("ds_write_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                                 :: "v"(lbuf + kGuard + (off - toff)), "v"(v) : "memory");
            }
            barrier();
        }
        // every main loop over the other workgroup's tails (r04k C2 on k_pt_lin 1115 vs 1091 GB/s)
        asm volatile("s_setprio 1");
        int tlo = lo;                                        // shard batches: pad of the tile's rows
        if constexpr (SH) {
            const uint32_t t0 = tile * kTile, kt = (t0 / a.srows) * a.srows + a.srows - 1;
            if (kt < t0 + kTile && kt < a.ncw) tlo = a.stail_lo;
        }
        lin_pass<C, G, Q, HI, SH, LO0>(V, lbuf, a.stride, lo, ph, tlo);
        asm volatile("s_setprio 0");
        PT_STAMP(2);
        barrier();                                           // the image is consumed
        PT_STAMP(3);
        wave_tail_lin<C, ENC, W>(V, a, lbuf, tile, noff, nbytes, rsrc, rout, rws, pt_it);
        toff = noff;
        tbytes = nbytes;
    }
    wait_vm<0>();                                            // no DMA may land after the exit
}

template <class C, bool ENC, bool SH, bool LO0>
__global__ void __attribute__((amdgpu_flat_work_group_size(kThreads, kThreads), amdgpu_waves_per_eu(4)))
k_pt_lin(PsArgs a) {
    static_assert(C::NQ == 1, "one quad (4 syndromes) per wave");
    static_assert(C::GN <= 2 && C::GN * C::QN == 8, "8 waves: at most two leader groups");
    static_assert(8 * C::XCAP * 2048 <= kLds, "exchange area");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (w) {                                             // each wave's pieces and tail, compiled
    case 0: pt_run_lin<C, ENC, 0, SH, LO0>(a, lds); break;
    case 1: pt_run_lin<C, ENC, 1, SH, LO0>(a, lds); break;
    case 2: pt_run_lin<C, ENC, 2, SH, LO0>(a, lds); break;
    case 3: pt_run_lin<C, ENC, 3, SH, LO0>(a, lds); break;
    case 4: pt_run_lin<C, ENC, 4, SH, LO0>(a, lds); break;
    case 5: pt_run_lin<C, ENC, 5, SH, LO0>(a, lds); break;
    case 6: pt_run_lin<C, ENC, 6, SH, LO0>(a, lds); break;
    default: pt_run_lin<C, ENC, 7, SH, LO0>(a, lds); break;
    }
}

} // namespace pt

// ---- 4-wave tile kernel k_pq_lin (PQ_<codec>, codegen gen_pq) -----------------------------------
// One 256-thread workgroup (4 waves) per 256-codeword tile, two workgroups per CU (80 KiB LDS
// each), up to 256 VGPRs (2 waves per SIMD).  Wave W evaluates EVERY coset leader (NI x 8 state
// words) over its own contiguous run of 8-position blocks with each block's own network: the
// tile's rows are read and their Four-Russians combinations formed once (the 8-wave kernel reads
// every position twice, once per leader group, and fixes up three quarters by alpha^(-16 q e)).
// The next piece's LDS reads are in flight while the current piece's networks run.  Then a
// two-round recursive-halving exchange through the consumed image leaves each wave the totals of
// the leaders whose two quads of syndromes it folds.  Image, DMA, flags and stores as k_pt_lin.
namespace pq {

using pt::kGuard;
using pt::kImage;
using pt::kOob;
using pt::u32x2;
using pt::u32x4;
constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kLds = 81920;                   // 80 KiB: two workgroups per CU
constexpr int kFlags = kGuard + kImage;       // decode flags [4][64] after the image
constexpr int kTab = kFlags + 1024;           // shard batches: per-row image offset and pad [256]
static_assert(kTab + 1024 <= kLds, "pq tile kernel LDS");

// Raw dwords of rows 4l + k at one 16-position piece (4-byte aligned reads, aligned afterwards).
struct Raw {
    u32x2 e[4][2];
    uint32_t d4[4];
};

// the piece at byte offset OFF (a multiple of 8) from the rows' dword-aligned position-0 addresses
// at4[k]: the offset rides in the instructions' immediates
template <int OFF>
__device__ __forceinline__ void issue_at(Raw &r, const uint32_t (&at4)[4]) {
    static_assert(OFF % 4 == 0 && OFF / 4 + 4 < 256, "ds_read2 dword offsets");
#pragma unroll
    for (int k = 0; k < 4; ++k)
        asm volatile("ds_read2_b32 %0, %3 offset0:%4 offset1:%5\n\t"
                     "ds_read2_b32 %1, %3 offset0:%6 offset1:%7\n\t"
                     "ds_read_b32 %2, %3 offset:%8"
                     : "=&v"(r.e[k][0]), "=&v"(r.e[k][1]), "=&v"(r.d4[k])
                     : "v"(at4[k]), "n"(OFF / 4), "n"(OFF / 4 + 1), "n"(OFF / 4 + 2), "n"(OFF / 4 + 3), "n"(OFF + 16)
                     : "memory");
}
// a final single-block piece: bytes OFF .. OFF+11 only (the dwords block B+1 would need are not
// read, so no dead in-flight register is left for the allocator to move)
template <int OFF>
__device__ __forceinline__ void issue_half(Raw &r, const uint32_t (&at4)[4]) {
    static_assert(OFF % 4 == 0 && OFF / 4 + 2 < 256, "ds_read2 dword offsets");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        asm volatile("ds_read2_b32 %0, %2 offset0:%3 offset1:%4\n\t"
                     "ds_read_b32 %1, %2 offset:%5"
                     : "=&v"(r.e[k][0]), "=&v"(r.e[k][1].x) : "v"(at4[k]), "n"(OFF / 4), "n"(OFF / 4 + 1), "n"(OFF + 8)
                     : "memory");
    }                                                        // e[k][1].y and d4[k] stay unset
}
template <int OFF, bool HALF>
__device__ __forceinline__ void issue_piece(Raw &r, const uint32_t (&at4)[4]) {
    if constexpr (HALF) issue_half<OFF>(r, at4);
    else issue_at<OFF>(r, at4);
}
__device__ __forceinline__ void wait_raw(Raw &r) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(r.e[0][0]), "+v"(r.e[0][1]), "+v"(r.d4[0]), "+v"(r.e[1][0]), "+v"(r.e[1][1]), "+v"(r.d4[1]),
                   "+v"(r.e[2][0]), "+v"(r.e[2][1]), "+v"(r.d4[2]), "+v"(r.e[3][0]), "+v"(r.e[3][1]), "+v"(r.d4[3])
                 :: "memory");
}
// byte address of row 4l + k at position 0 (plain batches: packed rows of pitch `stride`, the
// first byte at position lo; shard batches: the row-table entry e[k] = image offset of position 0 |
// pad << 24)
template <bool SH>
__device__ __forceinline__ void row_addrs(uint32_t (&at)[4], uint32_t lbuf, uint32_t stride, int lo, const u32x4 &e) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if constexpr (SH) at[k] = lbuf + (e[k] & 0xFFFFFFu);
        else at[k] = lbuf + kGuard + (4u * pt::fresh() + k) * stride - (uint32_t)lo;
    }
}
// aligned 16 bytes of each row; shard batches: bytes before a shortened row's own pad masked off
template <bool SH>
__device__ __forceinline__ void align_rows(u32x4 (&R)[4], const Raw &r, const uint32_t (&at)[4], int pa,
                                          int tail_lo, uint32_t pads) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t d[5] = {r.e[k][0].x, r.e[k][0].y, r.e[k][1].x, r.e[k][1].y, r.d4[k]};
#pragma unroll
        for (int j = 0; j < 4; ++j) R[k][j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], at[k]);
    }
    if constexpr (SH) {
        // bytes before a shortened row's own first byte (the previous row's, in the linear image):
        // every shard's last row has the same pad tail_lo, so the byte masks are wave-uniform and a
        // row only selects them (rows with the batch's pad lo are masked by block8 when lo > 0)
        if (pa < tail_lo) {                                  // wave-uniform
            uint32_t mt[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = min(max(8 * (tail_lo - pa) - 32 * j, 0), 32);
                mt[j] = __builtin_amdgcn_readfirstlane((uint32_t)(0xFFFFFFFFull << c));
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t keep = ((pads >> (8 * k)) & 0xFFu) == (uint32_t)tail_lo ? 0u : 0xFFFFFFFFu;
#pragma unroll
                for (int j = 0; j < 4; ++j) R[k][j] &= keep | mt[j];
            }
        }
    }
}

// block B (positions 8B .. 8B+7, words X) into every leader (F: the wave's first block sets the
// state); positions at/after HI contribute nothing, nor -- unless LO0 (full-length rows, the common
// case, compiled without the run-time masks and their branches) -- positions before lo
template <class C, int HI, int B, bool F, bool LO0>
__device__ __forceinline__ void block8(uint32_t (&V)[C::NI][8], uint32_t (&X)[8], int lo) {
    constexpr int pa = 8 * B;
    if constexpr (pa >= HI) return;
    if constexpr (HI - pa < 8) {
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (t >= HI - pa) X[t] = 0;
    }
    if constexpr (!LO0) {
        const int dlo = lo - pa;                             // wave-uniform
#pragma unroll
        for (int t = 0; t < 8; ++t) X[t] = t < dlo ? 0u : X[t];
    }
    C::template block<B, F>(V, X);
}

// Piece I of wave W (blocks B and B+1 from the run's start, 16 positions): wait for its reads,
// issue the next piece's, run its networks.
template <class C, bool ENC, int W, bool SH, bool LO0, int I>
__device__ __forceinline__ void piece(uint32_t (&V)[C::NI][8], Raw &cur, const uint32_t (&at)[4],
                                      const uint32_t (&at4)[4], int lo, int tail_lo, uint32_t pads) {
    constexpr int E = ENC ? 1 : 0;
    constexpr int HI = ENC ? kN - (int)C::NR : kN;
    // blocks at or past HI (encode: the parity positions) are neither read nor run
    constexpr int b0 = C::B0[E][W], b1 = C::B0[E][W + 1] < (HI + 7) / 8 ? C::B0[E][W + 1] : (HI + 7) / 8;
    constexpr int B = b0 + 2 * I;
    if constexpr (B < b1) {
        wait_raw(cur);
        Raw nxt;
        if constexpr (B + 2 < b1) issue_piece<8 * (B + 2), (B + 3 >= b1)>(nxt, at4);
        __builtin_amdgcn_sched_barrier(0);
        u32x4 R[4];
        align_rows<SH>(R, cur, at, 8 * B, tail_lo, pads);
        uint32_t X[8];
        {
            const uint32_t c0[4] = {R[0].x, R[1].x, R[2].x, R[3].x};
            const uint32_t c1[4] = {R[0].y, R[1].y, R[2].y, R[3].y};
            transpose4x4(c0, X);
            transpose4x4(c1, X + 4);
        }
        block8<C, HI, B, I == 0, LO0>(V, X, lo);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (B + 1 < b1) {
            const uint32_t c2[4] = {R[0].z, R[1].z, R[2].z, R[3].z};
            const uint32_t c3[4] = {R[0].w, R[1].w, R[2].w, R[3].w};
            transpose4x4(c2, X);
            transpose4x4(c3, X + 4);
            block8<C, HI, B + 1, false, LO0>(V, X, lo);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (B + 2 < b1) piece<C, ENC, W, SH, LO0, I + 1>(V, nxt, at, at4, lo, tail_lo, pads);
    }
}

template <class C, bool ENC, int W, bool SH, bool LO0>
__device__ __forceinline__ void pq_pass(uint32_t (&V)[C::NI][8], uint32_t lbuf, uint32_t stride, int lo,
                                        int tail_lo) {
    constexpr int E = ENC ? 1 : 0;
    constexpr int b0 = C::B0[E][W];
    u32x4 e = {0, 0, 0, 0};
    if constexpr (SH)
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(e) : "v"(lbuf + kTab + 16u * pt::fresh()) : "memory");
    Raw cur;
    uint32_t at[4], at4[4];
    row_addrs<SH>(at, lbuf, stride, lo, e);
#pragma unroll
    for (int k = 0; k < 4; ++k) at4[k] = at[k] & ~3u;        // byte phase at[k] & 3 for v_alignbyte
    // shard batches: the four rows' pads, one byte each (the row table entry is dead after this)
    const uint32_t pads = SH ? (e[0] >> 24) | (e[1] >> 24) << 8 | (e[2] >> 24) << 16 | (e[3] >> 24) << 24 : 0u;
    constexpr int HI = ENC ? kN - (int)C::NR : kN;
    constexpr int b1 = C::B0[E][W + 1] < (HI + 7) / 8 ? C::B0[E][W + 1] : (HI + 7) / 8;
    issue_piece<8 * b0, (b0 + 1 >= b1)>(cur, at4);
    piece<C, ENC, W, SH, LO0, 0>(V, cur, at, at4, lo, tail_lo, pads);
}

// Recursive-halving exchange (partner W ^ (1 << XR[s])), slots of XCAP items x 2 KiB per wave.
template <class C, int W, int S, int J = 0>
__device__ __forceinline__ void xsend(uint32_t (&V)[C::NI][8], uint32_t lx) {
    if constexpr (J < C::XCAP) {
        constexpr int it = C::XS[W][S][J];
        if constexpr (it >= 0) {
            const u32x4 w0 = {V[it][0], V[it][1], V[it][2], V[it][3]};
            const u32x4 w1 = {V[it][4], V[it][5], V[it][6], V[it][7]};
            asm volatile("ds_write_b128 %0, %1 offset:%3\n\t"
                         "ds_write_b128 %0, %2 offset:%4"
                         :: "v"(lx + W * C::XCAP * 2048u), "v"(w0), "v"(w1), "n"(J * 2048),
                            "n"(J * 2048 + 1024) : "memory");
        }
        xsend<C, W, S, J + 1>(V, lx);
    }
}
template <class C, int W, int S>
__device__ __forceinline__ void xrecv(uint32_t (&V)[C::NI][8], uint32_t lx) {
    pt::xrecv_pipe<C, W, S, W ^ (1 << C::XR[S])>(V, lx);
}
template <class C, int W, int S>
__device__ __forceinline__ void exchange(uint32_t (&V)[C::NI][8], uint32_t lx) {
    if constexpr (S < C::NSUB) {
        xsend<C, W, S>(V, lx);
        pt::wait_lgkm();
        pt::barrier();
        xrecv<C, W, S>(V, lx);
        pt::barrier();                                       // read before the area is reused
        exchange<C, W, S + 1>(V, lx);
    }
}

// The tile's DMA, wave w taking every fourth 1 KiB instruction
__device__ __forceinline__ void issue_tile(uint32_t lbuf, pw_rsrc_t rsrc, uint32_t toff, uint32_t tile_bytes, int w) {
#ifdef EZRS_PQ_ABL_NODMA
    return;                                                  // timing-only builds (pq_stamps)
#endif
    const uint32_t ninstr = (tile_bytes + 1023) >> 10;
    const uint32_t lo16 = 16u * pt::fresh();
    for (uint32_t i = (uint32_t)w; i < ninstr; i += kWaves)
        asm volatile("s_mov_b32 m0, %0\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %1, %2, 0 offen lds"
                     :: "s"(lbuf + kGuard + i * 1024u), "v"(toff + i * 1024u + lo16), "s"(rsrc) : "memory", "m0");
}

// Exchange, next tile's DMA, fold and stores of wave W.
template <class C, bool ENC, int W>
__device__ __forceinline__ void wave_tail(uint32_t (&V)[C::NI][8], const PsArgs &a, uint32_t lbuf, uint32_t tile,
                                          uint32_t noff, uint32_t nbytes, pw_rsrc_t rsrc, pw_rsrc_t rout,
                                          pw_rsrc_t rws, int pq_it = 0) {
    (void)pq_it;
    exchange<C, W, 0>(V, lbuf + 16u * pt::fresh());
    PQ_STAMP(4);
    if (noff != kOob) issue_tile(lbuf, rsrc, noff, nbytes, W);
    uint32_t T[C::NOWN][8];
#pragma unroll
    for (int i = 0; i < C::NOWN; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) T[i][t] = C::OWN[W][i] >= 0 ? V[C::OWN[W][i] < 0 ? 0 : C::OWN[W][i]][t] : 0u;
    uint32_t Qs[C::NQ][8], nz = 0;
    C::template epilogue<W>(T, [&](auto qc, uint32_t (&Qw)[8]) {
        constexpr int qd = decltype(qc)::value;
        constexpr uint32_t vm = (C::SYN[W][qd][0] >= 0 ? 0x01010101u : 0u) | (C::SYN[W][qd][1] >= 0 ? 0x02020202u : 0u) |
                                (C::SYN[W][qd][2] >= 0 ? 0x04040404u : 0u) | (C::SYN[W][qd][3] >= 0 ? 0x08080808u : 0u);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            nz |= Qw[t] & vm;
            Qs[qd][t] = Qw[t];
        }
    }, [](auto) {});
    PQ_STAMP(5);
    const uint32_t cw0 = tile * kTile + 4u * pt::fresh();    // byte k <-> codeword cw0 + k
    if constexpr (ENC) {
        static_for<0, C::NQ>([&](auto qc) {
            constexpr int qd = decltype(qc)::value;
            transpose8(Qs[qd]);                              // Qs[qd][jj] byte k: syndrome jj, codeword k
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                if (C::SYN[W][qd][jj] >= 0)
                    pt::store_dword(rws, (uint32_t)(C::SYN[W][qd][jj] * a.ws_pitch) + cw0, Qs[qd][jj]);
        });
    } else {
        uint32_t fl = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (nz >> (8 * k) & 0xFF) fl |= 1u << k;
        const uint32_t fa = lbuf + kFlags + 256u * W + 4u * pt::fresh();
        asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(fa), "v"(fl) : "memory");
        pt::barrier();
        {
            uint32_t f[4];
            const uint32_t fb = lbuf + kFlags + 4u * pt::fresh();
            asm volatile("ds_read_b32 %0, %4\n\t"
                         "ds_read_b32 %1, %4 offset:256\n\t"
                         "ds_read_b32 %2, %4 offset:512\n\t"
                         "ds_read_b32 %3, %4 offset:768\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]) : "v"(fb) : "memory");
            fl = f[0] | f[1] | f[2] | f[3];
        }
        if constexpr (W == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                pt::store_dword(rout, (cw0 + k) * 4u, (fl >> k & 1) ? (uint32_t)kSentinel : 0u);
            if (fl != 0 && a.flag) *a.flag = a.gen;          // this call flagged a codeword
        }
        if (__ballot(fl != 0) != 0) {                        // flagged codewords: their syndromes
            static_for<0, C::NQ>([&](auto qc) {
                constexpr int qd = decltype(qc)::value;
                transpose8(Qs[qd]);
                if (a.ws_pitch == 0) {
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        if (C::SYN[W][qd][jj] >= 0)
                            pt::store_dword(rws, tile * (uint32_t)kSynTile + 256u * C::SYN[W][qd][jj] + 4u * pt::fresh(),
                                            Qs[qd][jj]);
                } else {                                     // a launch not starting a tile (shards)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t g = (uint32_t)a.ws_pitch + cw0 + k;
                        const uint32_t row = (fl >> k & 1) ? (g >> 8) * (uint32_t)kSynTile + (g & 255u) : kOob;
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj)
                            if (C::SYN[W][qd][jj] >= 0)
                                pt::store_byte(rws, row + 256u * C::SYN[W][qd][jj], Qs[qd][jj] >> (8 * k));
                    }
                }
            });
        }
    }
}

template <class C, bool ENC, int W, bool SH, bool LO0>
__device__ __forceinline__ void pq_run(const PsArgs &a, uint8_t *lds) {
    const pw_rsrc_t rsrc = pw_rsrc(a.base, a.span);
    const uint32_t lbuf = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    const pw_rsrc_t rout = pw_rsrc(reinterpret_cast<const uint8_t *>(a.result), ENC ? 0u : a.ncw * 4u);
    const pw_rsrc_t rws = pw_rsrc(a.ws, ENC ? (uint32_t)(C::NR * a.ws_pitch)
                                            : (uint32_t)((a.ws_pitch + a.ncw + 255) / 256 * kSynTile));
    auto tile_range = [&](uint32_t t, uint32_t &bytes) -> uint32_t {
        if (!SH) {
            bytes = a.stride * kTile;
            return t * bytes;
        }
        int lo;
        const uint32_t t0 = t * kTile, off = pt::row_at(a, t0, lo);
        bytes = (t0 + kTile < a.ncw ? pt::row_at(a, t0 + kTile, lo) : a.span) - off;
        return pt::sh_align(off, bytes);
    };
    uint32_t tile = blockIdx.x;
    PQ_RT(0);
    uint32_t tbytes, toff = tile < a.ntiles ? tile_range(tile, tbytes) : 0u;
    if (tile < a.ntiles) issue_tile(lbuf, rsrc, toff, tbytes, W);
    int pq_it = 0;
    (void)pq_it;
    for (; tile < a.ntiles; tile += gridDim.x, ++pq_it) {
        PQ_STAMP(0);
        int lo = a.lo;
        asm volatile("" : "+s"(lo));
        uint32_t nbytes = 0;
        const uint32_t noff = tile + gridDim.x < a.ntiles ? tile_range(tile + gridDim.x, nbytes) : kOob;
        uint32_t V[C::NI][8];                                // set by the wave's first block
        pt::wait_vm<0>();                                    // the tile landed (and the stores went)
        if constexpr (SH) {                                  // row table: wave W writes rows 64W ..
            const uint32_t r = 64u * (uint32_t)W + pt::fresh(), k = tile * kTile + r;
            uint32_t e = kGuard;
            if (k < a.ncw) {
                int rlo;
                const uint32_t at = pt::row_at(a, k, rlo);
                e = (kGuard + at - toff - (uint32_t)rlo) | ((uint32_t)rlo << 24);
            }
            asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(lbuf + kTab + 4u * r), "v"(e) : "memory");
        }
        pt::barrier();
        if (toff + tbytes >= a.span) {                       // last tile: the span's final bytes
            if (W == 0) {
                const uint32_t off = a.span - 64u + pt::fresh();
                uint32_t v;
                asm volatile("buffer_load_ubyte %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                             : "=&v"(v) : "v"(off), "s"(rsrc) : "memory");
                if (off >= toff && off < a.span)
                    asm volatile("ds_write_b8 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                                 :: "v"(lbuf + kGuard + (off - toff)), "v"(v) : "memory");
            }
            pt::barrier();
        }
        int tlo = lo;                                        // shard batches: pad of the tile's rows
        if constexpr (SH) {
            const uint32_t t0 = tile * kTile, kt = (t0 / a.srows) * a.srows + a.srows - 1;
            if (kt < t0 + kTile && kt < a.ncw) tlo = a.stail_lo;
        }
        PQ_STAMP(1);
        // the main loop outranks the other workgroup's waves on the SIMD (their exchange, DMA and
        // fold): r04j C2 1203 vs 1169 GB/s; r06c: tails over main loops 1503, equal priority 1430,
        // main loops over tails 1558 GB/s (profiles/r06/r06c_priority_ab.txt)
        asm volatile("s_setprio 1");
        pq_pass<C, ENC, W, SH, LO0>(V, lbuf, a.stride, lo, tlo);
        asm volatile("s_setprio 0");
        PQ_STAMP(2);
        pt::barrier();                                       // the image is consumed
        PQ_STAMP(3);
        wave_tail<C, ENC, W>(V, a, lbuf, tile, noff, nbytes, rsrc, rout, rws, pq_it);
        PQ_STAMP(6);
        toff = noff;
        tbytes = nbytes;
    }
    pt::wait_vm<0>();                                        // no DMA may land after the exit
    PQ_RT(1);
}

template <class C, bool ENC, bool SH, bool LO0>
__global__ void __attribute__((amdgpu_flat_work_group_size(kThreads, kThreads), amdgpu_waves_per_eu(2)))
k_pq_lin(PsArgs a) {
    static_assert(kWaves * C::XCAP * 2048 <= kGuard + kImage, "exchange area");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    switch (w) {
    case 0: pq_run<C, ENC, 0, SH, LO0>(a, lds); break;
    case 1: pq_run<C, ENC, 1, SH, LO0>(a, lds); break;
    case 2: pq_run<C, ENC, 2, SH, LO0>(a, lds); break;
    default: pq_run<C, ENC, 3, SH, LO0>(a, lds); break;
    }
}

} // namespace pq


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

// wave P runs pass P (parity symbols 4P .. 4P+3) with hook H
template <class C, class H>
__device__ __forceinline__ void pass_switch(int wave, uint32_t (&O)[4][8], const uint32_t *in, H &hook) {
    switch (wave) {
    case 0: C::template q_pass4<0>(O, in, 64, hook); break;
    case 1: if constexpr (C::NPASS4 > 1) C::template q_pass4<1>(O, in, 64, hook); break;
    case 2: if constexpr (C::NPASS4 > 2) C::template q_pass4<2>(O, in, 64, hook); break;
    case 3: if constexpr (C::NPASS4 > 3) C::template q_pass4<3>(O, in, 64, hook); break;
    case 4: if constexpr (C::NPASS4 > 4) C::template q_pass4<4>(O, in, 64, hook); break;
    case 5: if constexpr (C::NPASS4 > 5) C::template q_pass4<5>(O, in, 64, hook); break;
    case 6: if constexpr (C::NPASS4 > 6) C::template q_pass4<6>(O, in, 64, hook); break;
    default: if constexpr (C::NPASS4 > 7) C::template q_pass4<7>(O, in, 64, hook); break;
    }
}

// Codeword k's parity row: 8/4/1-byte copies of the staged row s8.
template <int NR>
__device__ __forceinline__ void store_parity_row(uint8_t *dst, const uint8_t *s8) {
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


// 8-wave form of k_ps_parity: wave P computes parity symbols 4P..4P+3 (q_pass4), halving each
// wave's share of the map and doubling the waves that hide the phases' latencies.
template <class C>
__global__ void __launch_bounds__(512) k_ps_parity8(const uint8_t *ws, size_t ws_pitch, uint8_t *parity,
                                                    size_t pstride, size_t ncw, Shards sh, unsigned len) {
    constexpr int NR = C::NR;
    constexpr int kRegion = 32 * NR + 8;                       // bytes per group in the stage
    constexpr int kPlanes = 8 * NR * kParGroups;               // dwords
    constexpr int kStage = kParGroups * kRegion / 4;           // dwords
    constexpr int kLds = kPlanes > kStage ? kPlanes : kStage;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t g0 = (size_t)blockIdx.x * kParGroups;
    const uint8_t *src = ws + (g0 + lane) * 32;                // ws rows are padded to 2048 cw
    PAR_STAMP(0);
    // wave w loads syndromes w + 8c (chunk c) -- every load in flight at once -- and makes chunk
    // c's planes visible when the passes reach it, so the map runs while later chunks arrive
    constexpr int NCH = (NR + 7) / 8;
    pt::u32x4 v[NCH][2];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {                            // plain loads: the compiler counts
        const int i = wave + 8 * c < NR ? wave + 8 * c : 0;   // them (past NR: a dummy row 0)
        v[c][0] = *reinterpret_cast<const pt::u32x4 *>(src + i * ws_pitch);
        v[c][1] = *reinterpret_cast<const pt::u32x4 *>(src + i * ws_pitch + 16);
        __builtin_amdgcn_sched_barrier(0);                     // issue order = chunk order
    }
    auto ready = [&](auto cc) {
        constexpr int c = decltype(cc)::value;
        const int i = wave + 8 * c;
        const pt::u32x4 a0 = v[c][0], a1 = v[c][1];
        if (i < NR) {
            uint32_t D[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
            transpose8(D);                                     // D[q] bit 8k + m: cw 4m + k
#pragma unroll
            for (int qq = 0; qq < 8; ++qq) lds[(8 * i + qq) * 64 + lane] = D[qq];
        }
        pt::wait_lgkm();                                       // raw barrier: later chunks' loads stay in flight
        pt::barrier();
    };
    ready(std::integral_constant<int, 0>{});
    PAR_STAMP(1);
    PAR_STAMP(2);
    auto hook = [&](auto ic) {                                 // before syndrome i: chunk i / 8
        constexpr int i = decltype(ic)::value;
        if constexpr (i % 8 == 0) ready(std::integral_constant<int, i / 8>{});
    };
    uint32_t O[4][8];
    pass_switch<C>(wave, O, lds + lane, hook);
    if (wave >= C::NPASS4)                                     // no pass: still takes every barrier
        static_for<1, NR>([&](auto ic) { hook(ic); });
    PAR_STAMP(3);
    __syncthreads();                                           // planes consumed
    PAR_STAMP(4);
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
    PAR_STAMP(5);
    __syncthreads();
    PAR_STAMP(6);
    const size_t cwb = g0 * 32;
    // two lanes per parity row, NR / 2 bytes each (NR % 8 == 0): a wave's store covers 32 rows
    // instead of 64 (C2 line 1549 vs 1526 GB/s; 4 or 8 lanes per row the same within noise,
    // r05y / r05z A/B); other NR: one lane per row
    if constexpr (NR % 8 == 0) {
        constexpr int LPR = 2, PB = NR / LPR;
        const int sub = threadIdx.x % LPR;
        for (int r = threadIdx.x / LPR; r < kParCw; r += 512 / LPR) {
            const size_t k = cwb + r;
            if (k >= ncw) break;
            unsigned rlen;
            uint8_t *dst = sh.rows ? parity + shard_row(sh, k, pstride, len, rlen) + rlen : parity + k * pstride;
            const uint8_t *s8 = stage + (r >> 5) * kRegion + (r & 31) * NR + PB * sub;
            if constexpr (PB == 16) {
                const uint2 lo = *reinterpret_cast<const uint2 *>(s8);      // the stage is 8-aligned
                const uint2 hi = *reinterpret_cast<const uint2 *>(s8 + 8);
                const pt::u32x4 v = {lo.x, lo.y, hi.x, hi.y};
                __builtin_memcpy(dst + PB * sub, &v, 16);
            } else if constexpr (PB % 8 == 0) {
#pragma unroll
                for (int o = 0; o < PB; o += 8) {
                    uint2 v = *reinterpret_cast<const uint2 *>(s8 + o);
                    __builtin_memcpy(dst + PB * sub + o, &v, 8);
                }
            } else {
                uint32_t v = *reinterpret_cast<const uint32_t *>(s8);
                __builtin_memcpy(dst + PB * sub, &v, 4);
            }
        }
        PAR_STAMP(7);
        return;
    }
    for (int r = threadIdx.x; r < kParCw; r += 512) {
        const size_t x = cwb + r;
        const size_t k = x;
        if (k >= ncw) continue;
        unsigned rlen;
        // shard batches: parity is the base of the rows, each row's parity after its data
        uint8_t *dst = sh.rows ? parity + shard_row(sh, k, pstride, len, rlen) + rlen : parity + k * pstride;
        store_parity_row<NR>(dst, stage + (r >> 5) * kRegion + (r & 31) * NR);
    }
    PAR_STAMP(7);
}

} // namespace ps

// ------------------------------------------------------------------------------------------------
namespace {

template <class C> bool ps_matches(const DevCodec &d) {
    return d.mm == 8 && d.nroots == C::NR && d.fcr == C::FCR && d.prim == C::PRIM && !d.dual &&
           d.poly == C::POLY;
}

// The parity stage: k_ps_parity8, one block per 2048-codeword chunk.  Measured and dropped: a
// pipelined persistent form, one block per CU over the chunks (r04n 44.2 vs 41.2 us: at two waves
// per SIMD the map loses more than the overlapped stores save); independent waves without LDS,
// each loading and transposing every syndrome itself (r06b 58 vs 38 us: four 8-byte partial
// writes per row cost more than the whole LDS-staged kernel).
template <class PS>
void launch_parity(const DevCodec &d, const uint8_t *ws, size_t ws_pitch, uint8_t *par, size_t pstride,
                   size_t n, const Shards &sh, unsigned len, unsigned nchunk, hipStream_t s) {
    (void)d;
    hipLaunchKernelGGL((ps::k_ps_parity8<PS>), dim3(nchunk), dim3(512), 0, s, ws, ws_pitch, par, pstride, n, sh, len);
}

// Workgroups per launch (persistent over tiles): 2 per CU (80 KiB LDS each).
unsigned syn_grid(const DevCodec &d, uint32_t ntiles) {
    const uint32_t nwg = 2u * (uint32_t)(d.ncu > 0 ? d.ncu : 256);
    return ntiles < nwg ? ntiles : nwg;
}


} // namespace

// Codecs with the 4-wave tile kernel (PQ_<codec>; codegen PQ_CODECS) use it for both directions
// (r04f: C2 1161 vs 1062 GB/s on k_pt_lin); the others, and variant builds with -DEZRS_NO_PQ (A/B
// timing, tools/build_variant.sh), run the 8-wave k_pt_lin.
template <class PS> struct PqFor { using type = void; };
#define EZRS_PQ_FOR(C) template <> struct PqFor<ps::PS_##C> { using type = ps::PQ_##C; };
EZRS_PQ_CODEC_LIST(EZRS_PQ_FOR)
#undef EZRS_PQ_FOR

template <class PS, class PT, bool ENC>
void launch_tile(const ps::PsArgs &p, bool shard, unsigned grid, hipStream_t s) {
    using PQ = typename PqFor<PS>::type;
#ifndef EZRS_NO_PQ
    if constexpr (!std::is_void<PQ>::value) {
        const bool lo0 = p.lo == 0;                          // full-length rows: no pad masks
        if (shard && lo0)
            hipLaunchKernelGGL((ps::pq::k_pq_lin<PQ, ENC, true, true>), dim3(grid), dim3(ps::pq::kThreads), 0, s, p);
        else if (shard)
            hipLaunchKernelGGL((ps::pq::k_pq_lin<PQ, ENC, true, false>), dim3(grid), dim3(ps::pq::kThreads), 0, s, p);
        else if (lo0)
            hipLaunchKernelGGL((ps::pq::k_pq_lin<PQ, ENC, false, true>), dim3(grid), dim3(ps::pq::kThreads), 0, s, p);
        else
            hipLaunchKernelGGL((ps::pq::k_pq_lin<PQ, ENC, false, false>), dim3(grid), dim3(ps::pq::kThreads), 0, s, p);
        return;
    }
#endif
#ifndef EZRS_PQ_ONLY                                          // (ISA inspection builds: tools/pq_isa.sh)
    const bool lo0 = p.lo == 0;                              // full-length rows: no pad masks
    if (shard && lo0)
        hipLaunchKernelGGL((ps::pt::k_pt_lin<PT, ENC, true, true>), dim3(grid), dim3(ps::pt::kThreads), 0, s, p);
    else if (shard)
        hipLaunchKernelGGL((ps::pt::k_pt_lin<PT, ENC, true, false>), dim3(grid), dim3(ps::pt::kThreads), 0, s, p);
    else if (lo0)
        hipLaunchKernelGGL((ps::pt::k_pt_lin<PT, ENC, false, true>), dim3(grid), dim3(ps::pt::kThreads), 0, s, p);
    else
        hipLaunchKernelGGL((ps::pt::k_pt_lin<PT, ENC, false, false>), dim3(grid), dim3(ps::pt::kThreads), 0, s, p);
#endif
}

int planeslice_codec_id(const DevCodec &d) {
    int id = 0, found = -1;
#define EZRS_PS_MATCH(C) \
    if (found < 0 && ps_matches<ps::PS_##C>(d)) found = id; \
    ++id;
    EZRS_PS_CODEC_LIST(EZRS_PS_MATCH)
#undef EZRS_PS_MATCH
    return found;
}

// Timing experiments only: EZRS_PT_ABLATE disables phases of the tile kernel (PsArgs::ablate).  Read
// only by variant builds compiled with -DEZRS_PT_ABLATE_ENV (tools/build_variant.sh); the release
// library never looks at the environment here, so a stray variable cannot switch correction off.
static int pt_ablate() {
#ifdef EZRS_PT_ABLATE_ENV
    const char *e = getenv("EZRS_PT_ABLATE");
    return e ? atoi(e) : 0;
#else
    return 0;
#endif
}

// Workspace: decode tiled syndromes (kSynTile); encode [NR][ws_pitch] syndromes, ws_pitch = ncw
// rounded up to 2048 (the parity kernel's block).
static size_t ps_pitch(size_t ncw) { return (ncw + 2047) / 2048 * 2048; }
size_t ps_ws_bytes(size_t ncw) { return ps_pitch(ncw) * 32; }

// Largest batch one launch takes: every buffer offset stays below 0xF0000000 (32-bit offsets;
// the tile kernel's out-of-range marker kOob is above them).
// That covers the rows' span AND the per-codeword buffers: the result array (4 B per codeword) and
// the syndrome workspace (32 B per codeword in either layout), so a short row pitch cannot wrap the
// workspace offsets.  The codec's launch_rows (ezrs_set_launch_rows, a test hook) lowers the cap
// (tests: launches split mid-batch and, for shard batches, mid-tile; the results are the same by
// construction).
static size_t ps_row_cap(const DevCodec &d) {
    const size_t hard = (size_t)0xE0000000u / 32;
    return d.launch_rows && d.launch_rows < hard ? d.launch_rows : hard;
}
static size_t ps_max_rows(const DevCodec &d, size_t stride) {
    const size_t cap = ps_row_cap(d);
    size_t m = (size_t)0xE0000000u / stride;
    if (m > cap) m = cap;
    return m >= 2048 && cap == (size_t)0xE0000000u / 32 ? m / 2048 * 2048 : m;   // a test cap: as set
}

// Shard batches: rows per launch, whole shards (byte offsets stay below 0xE0000000 as above).
static size_t ps_max_rows_shards(const DevCodec &d, const Shards &g) {
    size_t n = (size_t)0xE0000000u / g.pitch;
    const size_t byrows = ps_row_cap(d) / g.rows;
    if (byrows < n) n = byrows;
    return (n ? n : 1) * g.rows;
}
// Shard batches: a tile's rows must fit the 64 KiB image (no gaps between shards beyond a row's
// width) and every launch's span the 32-bit offsets.
static bool ps_shards_ok(const Shards &g, size_t stride) {
    return g.pitch <= (size_t)g.rows * stride && g.pitch < 0xE0000000u;
}

bool ps_can_encode(const DevCodec &, const EncodeArgs &a) {
    if (a.sh.rows) return a.data_stride <= 256 && ps_shards_ok(a.sh, a.data_stride);
    return a.data_stride >= 1 && a.data_stride <= 256;
}

bool ps_can_decode(const DevCodec &d, const DecodeArgs &a) {
    if (a.sh.rows) return a.data_stride <= 256 && ps_shards_ok(a.sh, a.data_stride);
    const bool inline_par = a.parity == static_cast<char *>(a.data) + a.len && a.parity_stride == a.data_stride;
    return inline_par && a.data_stride <= 256 && a.data_stride >= a.len + d.nroots;
}

hipError_t launch_ps_encode(int id, const DevCodec &d, const EncodeArgs &a, void *ws, hipStream_t s) {
    const size_t pitch = a.data_stride > a.parity_stride ? a.data_stride : a.parity_stride;
    const size_t maxr = a.sh.rows ? ps_max_rows_shards(d, a.sh) : ps_max_rows(d, pitch);
    for (size_t k0 = 0; k0 < a.ncw; k0 += maxr) {
        const size_t n = a.ncw - k0 < maxr ? a.ncw - k0 : maxr;
        ps::PsArgs p{};
        unsigned rlen;
        const size_t b0 = shard_row(a.sh, k0, a.data_stride, a.len, rlen);   // chunks start a shard
        const size_t last = shard_row(a.sh, n - 1, a.data_stride, a.len, rlen);
        p.base = static_cast<const uint8_t *>(a.data) + b0;
        p.span = (uint32_t)(last + rlen);
        p.stride = (uint32_t)a.data_stride;
        if (a.sh.rows) {
            p.srows = a.sh.rows;
            p.stail_lo = (int)(d.load - a.sh.tail);
            p.spitch = (uint32_t)a.sh.pitch;
        }
        p.ncw = (uint32_t)n;
        p.ntiles = (uint32_t)((n + ps::kTile - 1) / ps::kTile);
        p.lo = (int)(d.load - a.len);              // leading zero positions of a shortened code
        // shard batches: the parity kernel finds each row's parity from the rows' base
        uint8_t *par = a.sh.rows ? const_cast<uint8_t *>(p.base) : static_cast<uint8_t *>(a.parity) + k0 * a.parity_stride;
        p.ws = static_cast<uint8_t *>(ws);
        p.ws_pitch = ps_pitch(n);
        p.ablate = pt_ablate();
        const unsigned grid = syn_grid(d, p.ntiles);
        int k = 0;
#define EZRS_PS_ENC(C)                                                                            \
        if (k++ == id) {                                                                          \
            const unsigned pgrid = (unsigned)((n + ps::kParCw - 1) / ps::kParCw);                 \
            launch_tile<ps::PS_##C, ps::PT_##C, true>(p, a.sh.rows != 0, grid, s);                \
            launch_parity<ps::PS_##C>(d, static_cast<const uint8_t *>(ws), p.ws_pitch, par,     \
                                      a.parity_stride, n, a.sh, a.len, pgrid, s);                 \
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
    const size_t maxr = a.sh.rows ? ps_max_rows_shards(d, a.sh) : ps_max_rows(d, a.data_stride);
    for (size_t k0 = 0; k0 < a.ncw; k0 += maxr) {
        const size_t n = a.ncw - k0 < maxr ? a.ncw - k0 : maxr;
        ps::PsArgs p{};
        unsigned rlen;
        const size_t b0 = shard_row(a.sh, k0, a.data_stride, a.len, rlen);   // chunks start a shard
        const size_t last = shard_row(a.sh, n - 1, a.data_stride, a.len, rlen);
        p.base = static_cast<const uint8_t *>(a.data) + b0;
        p.span = (uint32_t)(last + rlen + d.nroots);
        p.stride = (uint32_t)a.data_stride;
        if (a.sh.rows) {
            p.srows = a.sh.rows;
            p.stail_lo = (int)(d.load - a.sh.tail);
            p.spitch = (uint32_t)a.sh.pitch;
        }
        p.ncw = (uint32_t)n;
        p.ntiles = (uint32_t)((n + ps::kTile - 1) / ps::kTile);
        p.lo = (int)(d.load - a.len);
        p.result = a.result + k0;
        p.ws = syn_ws + k0 / 256 * kSynTile;                  // tiled layout, global codeword index
        p.ws_pitch = k0 % 256;
        p.ablate = pt_ablate();
        p.flag = a.flag_word;
        p.gen = a.flag_gen;
        const unsigned grid = syn_grid(d, p.ntiles);
        int k = 0;
#define EZRS_PS_SYN(C)                                                                            \
        if (k++ == id) launch_tile<ps::PS_##C, ps::PT_##C, false>(p, a.sh.rows != 0, grid, s);
        EZRS_PS_CODEC_LIST(EZRS_PS_SYN)
#undef EZRS_PS_SYN
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace ezrs

