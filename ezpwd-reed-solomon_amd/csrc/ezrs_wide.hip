// ezrs_wide.hip -- GF(2^16) RS fast path (BASELINE config C4: RS(65535,65503)).
//
// Syndromes S_i = r(beta_i) (c++/ezpwd/rs_base:1390-1414) through binary minimal polynomials:
// for each cyclotomic coset ("leader" e) of the roots, R_e = r mod M_e(x) is a GF(2)-linear shift
// register over whole 16-bit symbols (XOR only; codegen/gen_wide.py has the derivation), and every
// root beta of the coset gives S = R_e(beta), 16 GF(2^16) products per syndrome.
//
//   k_wide_rem     streams 128-codeword tiles through LDS (LDS-DMA, 128-symbol windows, double
//                  buffered); wave w runs the 64-symbol networks of leaders kLPW w .. kLPW w + 3 on
//                  32-bit words that pack one position of two codewords.  Out: remainders
//                  [ncw][NLP][16] u16.
//   k_wide_finish  32 lanes per codeword evaluate the syndromes by Horner with a table-free
//                  multiply by the constant beta (mulc).  Encode: parity = Q S with
//                  Q = V^-1 diag(beta^NR) (V[i][k] = beta_i^(NR-1-k)), the unique parity whose
//                  codeword has zero syndromes -- encode_symbols' LFSR result (rs_base:1296-1332).
//                  Decode: result 0 for a codeword with zero syndromes and no erasures
//                  (rs_base:1416-1434); the others get queued for
//   k_wide_errors  one wavefront per flagged codeword: erasure locator + Berlekamp-Massey with the
//                  discrepancy as a wave reduction (rs_base:1436-1546), the roots the Chien search
//                  would find (1548-1584) by Berlekamp's trace algorithm over lane-parallel
//                  polynomials with alpha_to in LDS, sorted to the reference's order, Omega and
//                  Forney per root lane (1589-1690), the reference's partial-correction-on-failure
//                  semantics, positions in the pad-relative frame (1713-1716).
#include "ezrs_internal.hpp"
#include "gen/ezrs_wide_tables.inc"

namespace ezrs {
namespace wide {

constexpr int kRows = 128;                  // codewords per tile (64 pairs)
constexpr int kWin = 128;                   // symbols per window
constexpr int kRowBytes = 2 * kWin;         // 256 B of each row per window
constexpr int kBuf = kRows * kRowBytes;     // 32 KiB
constexpr int kLPW = 4;                     // leaders per wave
constexpr int kNBuf = 2;                    // window ring: the DMA runs kNBuf - 1 windows ahead
// (measured, C4 k_wide_rem per launch.  16-symbol networks: 2 leaders x 8 waves, 2 workgroups per
// CU 3.8 ms; 1 leader x 16 waves, 3 buffers, 1 workgroup per CU 4.7 ms; 4 leaders x 4 waves
// 3.8 ms.  32-symbol networks, 2 leaders x 8 waves: 3.27 ms.  64-symbol networks (C::CB), 4 leaders
// x 4 waves, 198 VGPRs, 2 workgroups per CU: 2.89 ms.)
constexpr int kMaxNR = 32;
constexpr int kM = 16;                      // symbol bits of every wide codec
constexpr int32_t kSentinel = INT32_MIN;

typedef int rsrc_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// Buffer descriptor of [base, base + span): raw, out-of-range bytes read as zero.
__device__ __forceinline__ rsrc_t make_rsrc(const uint8_t *base, uint32_t span) {
    const uint64_t p = (uint64_t)(uintptr_t)base;
    rsrc_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(p >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)span);
    r.w = 0x00020000;
    return r;
}

struct RemArgs {
    const uint8_t *base;        // row 0 of the batch
    size_t stride;              // row pitch, bytes
    uint32_t n;                 // symbols evaluated from each row's start
    uint32_t ncw;
    uint16_t *rem;              // [ncw][nlp][16]
    uint32_t nlp;               // leaders padded to the waves (NW * kLPW)
};

// the networks of leaders B .. B + kLPW - 1 on one 16-symbol block
template <class C, int B, int L = 0>
__device__ __forceinline__ void blocks_of(uint32_t (&S)[kLPW][16], const uint32_t (&c)[C::CB]) {
    if constexpr (L < kLPW && B + L < C::NL) {
        C::template block<B + L>(S[L], c);
        blocks_of<C, B, L + 1>(S, c);
    }
}

// LDS image of one window: row r (pair p = r >> 1) at r * 256; its 16-byte chunk c = 2b + h
// (b = 16-symbol block) at slot 2 (b ^ (p & 7)) + (h ^ q), q = (p >> 3) & 1.  Each 16-lane group
// of a ds_read_b128 holds 16 distinct p mod 16 and so reads 16 distinct bank quads.
template <class C, int W>
__device__ __forceinline__ void rem_body(const RemArgs &a, uint8_t *lds, int lane) {
    constexpr int NW = (C::NL + kLPW - 1) / kLPW;
    const size_t row0 = (size_t)blockIdx.x * kRows;
    const uint32_t rows = a.ncw - row0 < (size_t)kRows ? (uint32_t)(a.ncw - row0) : (uint32_t)kRows;
    const uint8_t *tbase = a.base + row0 * a.stride;
    const uint32_t span = (uint32_t)((rows - 1) * a.stride + 2u * a.n);
    const rsrc_t rsrc = make_rsrc(tbase, span);
    const uint32_t nwin = (a.n + kWin - 1) / kWin;
    const uint32_t z = nwin * kWin - a.n;             // leading positions of window 0 to ignore
    const uint32_t lbuf = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    const uint32_t stride = (uint32_t)a.stride;

    // DMA role: instructions i = W, W + NW, ... < 32; instruction i covers rows 4i .. 4i + 3, lane j
    // -> row 4i + j / 16, slot j % 16.
    auto issue = [&](uint32_t w, uint32_t buf) {
        uint32_t l = (uint32_t)lane;
        asm volatile("" : "+v"(l));
        const uint32_t s = l & 15, rr = l >> 4;
        const int32_t wbase = (int32_t)(2 * kWin * w) - (int32_t)(2 * z);
#pragma unroll
        for (int i = W; i < 32; i += NW) {
            const uint32_t r = 4 * i + rr, p = r >> 1, q = (p >> 3) & 1;
            const uint32_t b = (s >> 1) ^ (p & 7), h = (s & 1) ^ q;
            const uint32_t off = (uint32_t)((int32_t)(r * stride) + wbase + (int32_t)(16 * (2 * b + h)));
            asm volatile("s_mov_b32 m0, %0\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %1, %2, 0 offen lds"
                         :: "s"(lbuf + buf * kBuf + i * 1024), "v"(off), "s"(rsrc) : "memory", "m0");
        }
    };

    constexpr int IPW = 32 / NW;                       // DMA instructions per wave per window
    uint32_t S[kLPW][16];
#pragma unroll
    for (int L = 0; L < kLPW; ++L)
#pragma unroll
        for (int k = 0; k < 16; ++k) S[L][k] = 0;

    const uint32_t p = (uint32_t)lane, q = (p >> 3) & 1;
    const uint32_t rowa = lbuf + 2 * p * kRowBytes;
    for (uint32_t w = 0; w + 1 < (uint32_t)kNBuf && w < nwin; ++w) issue(w, w);
    for (uint32_t w = 0; w < nwin; ++w) {
        // window w landed (this wave's share: all but the younger windows' DMA), then every
        // wave's share (barrier); the buffer of window w - 1 is free for window w + kNBuf - 1
        if (w + kNBuf - 2 < nwin)
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(IPW * (kNBuf - 2)) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w + kNBuf - 1 < nwin) issue(w + kNBuf - 1, (w + kNBuf - 1) % kNBuf);
        const uint32_t wb = rowa + (w % kNBuf) * kBuf;
        if (w == 0 && z) {
            // positions before the row's start (the previous row's bytes, or zeros): clear them in
            // this lane's two rows (every wave writes the same zeros, each before its own reads)
            for (uint32_t t = 0; t < z; ++t) {
                const uint32_t ch = t >> 3, b = ch >> 1, h = ch & 1;
                const uint32_t o = 16 * (2 * (b ^ (p & 7)) + (h ^ q)) + 2 * (t & 7);
                asm volatile("ds_write_b16 %0, %1\n\t"
                             "ds_write_b16 %0, %1 offset:256\n\t"
                             "s_waitcnt lgkmcnt(0)" :: "v"(wb + o), "v"(0u) : "memory");
            }
            // the 16-byte piece holding a row's first symbols straddles its start: a row whose
            // piece begins before the buffer's range read it as zeros, so reload those symbols
            const uint32_t zr = z & 7, nfix = (8 - zr) & 7;
            for (uint32_t h = 0; h < 2 && nfix; ++h) {
                const uint32_t r = 2 * p + h;
                if (row0 + r >= a.ncw) break;
                for (uint32_t t = 0; t < nfix && t < a.n; ++t) {
                    const uint32_t u = z + t, ch = u >> 3, b = ch >> 1, hh = ch & 1;
                    const uint32_t o = 16 * (2 * (b ^ (p & 7)) + (hh ^ q)) + 2 * (u & 7) + 256 * h;
                    const uint32_t v = *reinterpret_cast<const uint16_t *>(tbase + r * a.stride + 2 * t);
                    asm volatile("ds_write_b16 %0, %1\n\t"
                                 "s_waitcnt lgkmcnt(0)" :: "v"(wb + o), "v"(v) : "memory");
                }
            }
        }
        // (LDS reads as inline asm with the wait per block: the compiler-scheduled form that
        // loads block b + 1 during block b measured slower, 4.09 vs 3.83 ms per C4 launch)
        static_assert(kWin % C::CB == 0 && C::CB % 16 == 0, "network blocks tile the window");
#pragma unroll
        for (int b0 = 0; b0 < kWin / 16; b0 += C::CB / 16) {
            uint32_t c[C::CB];
            static_assert(C::CB == 64, "the LDS read below covers four 16-symbol blocks");
            uint32_t xa[4], xb[4];
#pragma unroll
            for (int h2 = 0; h2 < 4; ++h2) {
                const uint32_t blk = wb + 32 * ((uint32_t)(b0 + h2) ^ (p & 7));
                xa[h2] = blk + 16 * q;
                xb[h2] = blk + 16 * (q ^ 1);
            }
            uint4 R[16];                              // [h2][A0, A1, B0, B1]: one wait for all
            asm volatile("ds_read_b128 %0, %16\n\t"
                         "ds_read_b128 %1, %17\n\t"
                         "ds_read_b128 %2, %16 offset:256\n\t"
                         "ds_read_b128 %3, %17 offset:256\n\t"
                         "ds_read_b128 %4, %18\n\t"
                         "ds_read_b128 %5, %19\n\t"
                         "ds_read_b128 %6, %18 offset:256\n\t"
                         "ds_read_b128 %7, %19 offset:256\n\t"
                         "ds_read_b128 %8, %20\n\t"
                         "ds_read_b128 %9, %21\n\t"
                         "ds_read_b128 %10, %20 offset:256\n\t"
                         "ds_read_b128 %11, %21 offset:256\n\t"
                         "ds_read_b128 %12, %22\n\t"
                         "ds_read_b128 %13, %23\n\t"
                         "ds_read_b128 %14, %22 offset:256\n\t"
                         "ds_read_b128 %15, %23 offset:256\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(R[0]), "=&v"(R[1]), "=&v"(R[2]), "=&v"(R[3]), "=&v"(R[4]), "=&v"(R[5]),
                           "=&v"(R[6]), "=&v"(R[7]), "=&v"(R[8]), "=&v"(R[9]), "=&v"(R[10]), "=&v"(R[11]),
                           "=&v"(R[12]), "=&v"(R[13]), "=&v"(R[14]), "=&v"(R[15])
                         : "v"(xa[0]), "v"(xb[0]), "v"(xa[1]), "v"(xb[1]), "v"(xa[2]), "v"(xb[2]),
                           "v"(xa[3]), "v"(xb[3])
                         : "memory");
#pragma unroll
            for (int h2 = 0; h2 < 4; ++h2) {
                const uint4 A0 = R[4 * h2], A1 = R[4 * h2 + 1], B0 = R[4 * h2 + 2], B1 = R[4 * h2 + 3];
                const uint32_t ra[8] = {A0.x, A0.y, A0.z, A0.w, A1.x, A1.y, A1.z, A1.w};
                const uint32_t rb[8] = {B0.x, B0.y, B0.z, B0.w, B1.x, B1.y, B1.z, B1.w};
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    c[16 * h2 + 2 * t] = __builtin_amdgcn_perm(rb[t], ra[t], 0x05040100u);
                    c[16 * h2 + 2 * t + 1] = __builtin_amdgcn_perm(rb[t], ra[t], 0x07060302u);
                }
            }
            blocks_of<C, kLPW * W>(S, c);
        }
    }
    // remainders of the lane's two codewords (low halves: row 2p, high halves: row 2p + 1)
#pragma unroll
    for (int L = 0; L < kLPW; ++L) {
        if (kLPW * W + L >= C::NL) break;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const size_t cw = row0 + 2 * p + h;
            if (cw >= a.ncw) continue;
            const uint32_t sel = h ? 0x07060302u : 0x05040100u;
            uint32_t d[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) d[m] = __builtin_amdgcn_perm(S[L][2 * m + 1], S[L][2 * m], sel);
            uint4 *dst = reinterpret_cast<uint4 *>(a.rem + (cw * a.nlp + kLPW * W + L) * 16);
            dst[0] = make_uint4(d[0], d[1], d[2], d[3]);
            dst[1] = make_uint4(d[4], d[5], d[6], d[7]);
        }
    }
}

// wave -> rem_body<C, W> (the leader set is a template parameter: wave-uniform networks)
template <class C, int NW, int W = 0>
__device__ __forceinline__ void static_for_waves(const RemArgs &a, uint8_t *lds, int lane, int wave) {
    if constexpr (W < NW) {
        if (wave == W) rem_body<C, W>(a, lds, lane);
        else static_for_waves<C, NW, W + 1>(a, lds, lane, wave);
    }
}

template <class C>
__global__ void __launch_bounds__(64 * ((C::NL + kLPW - 1) / kLPW)) k_wide_rem(RemArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kNBuf * kBuf];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    constexpr int NW = (C::NL + kLPW - 1) / kLPW;
    static_assert(NW <= 16 && 32 % NW == 0, "waves must split the window's 32 DMA instructions");
    static_for_waves<C, NW>(a, lds, lane, wave);
}

// ------------------------------------------------------------------------------------------------
struct FinishArgs {
    const uint16_t *rem;
    uint32_t nlp, ncw, nr;
    uint8_t leader[kMaxNR];     // syndrome i -> leader slot
    const uint16_t *cols;       // [NR][16] beta_i * 2^b, then (encode) [NR][NR][16] Q_ki * 2^b
    // encode
    uint16_t *parity;
    size_t pstride;             // elements
    // decode
    const uint32_t *neras;
    int32_t *result;
    uint16_t *syn;              // [ncw][32] polynomial form, flagged codewords only
    uint32_t *queue;            // [0] count, [1..] flagged codewords
};

constexpr int kFinGroups = 8;               // codewords per block pass (32 lanes each)
constexpr int kQRow = 2 * kMaxNR * 16 + 16; // bytes per LDS row of Q columns (padded)

// x * c for a constant c given by its columns col[b] = c * 2^b: XOR of the columns of x's set bits
// (v_bfe_i32 gives the all-ones / zero mask, v_bitop3 0x78 is y ^ (col & mask)); no table reads
__device__ __forceinline__ uint32_t mulc(uint32_t x, const uint32_t (&col)[16]) {
    uint32_t y = 0;
#pragma unroll
    for (int b = 0; b < 16; ++b)
        y = __builtin_amdgcn_bitop3_b32(y, col[b], (uint32_t)__builtin_amdgcn_sbfe((int)x, b, 1), 0x78);
    return y;
}

template <bool ENC>
__global__ void __launch_bounds__(256) k_wide_finish(FinishArgs a) {
    __shared__ uint16_t sl[kFinGroups][kMaxNR];
    __shared__ __attribute__((aligned(16))) uint8_t qc[ENC ? kMaxNR * kQRow : 16];
    __shared__ uint32_t nfl[kFinGroups], qbase;
    const unsigned lane = threadIdx.x & 31, g = threadIdx.x >> 5;
    const unsigned NR = a.nr;
    if constexpr (ENC) {                      // Q columns: row k = the 16 NR columns of parity k
        const unsigned rowb = NR * 32;
        for (unsigned t = threadIdx.x; t < NR * rowb / 16; t += 256) {
            const unsigned k = t / (rowb / 16), o = t % (rowb / 16);
            *reinterpret_cast<uint4 *>(qc + k * kQRow + 16 * o) =
                reinterpret_cast<const uint4 *>(a.cols + NR * 16 + k * NR * 16)[o];
        }
    }
    uint32_t bc[16];                          // columns of beta_lane
    if (lane < NR) {
        const uint4 *cp = reinterpret_cast<const uint4 *>(a.cols + lane * 16);
        const uint4 c0 = cp[0], c1 = cp[1];
        const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
        for (int b = 0; b < 16; ++b) bc[b] = (w[b >> 1] >> (16 * (b & 1))) & 0xFFFFu;
    }
    for (size_t base = (size_t)blockIdx.x * kFinGroups; base < a.ncw; base += (size_t)gridDim.x * kFinGroups) {
        const size_t cw = base + g;
        const bool live = cw < a.ncw;
        uint32_t S = 0;                       // S_lane = R(beta) by Horner, R = sum_k s[k] x^k
        if (live && lane < NR) {
            const uint4 *src = reinterpret_cast<const uint4 *>(a.rem + (cw * a.nlp + a.leader[lane]) * 16);
            const uint4 r0 = src[0], r1 = src[1];
            const uint32_t rw[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
            for (int k = 15; k >= 0; --k) S = mulc(S, bc) ^ ((rw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
        }
        if constexpr (ENC) {
            __syncthreads();                  // Q staged (first pass); sl free (later passes)
            sl[g][lane] = (uint16_t)S;
            __syncthreads();
            if (live && lane < NR) {
                const uint8_t *qrow = qc + lane * kQRow;
                uint32_t par = 0;
                for (unsigned i = 0; i < NR; ++i) {
                    const uint4 q0 = *reinterpret_cast<const uint4 *>(qrow + 32 * i);
                    const uint4 q1 = *reinterpret_cast<const uint4 *>(qrow + 32 * i + 16);
                    const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
                    uint32_t qcol[16];
#pragma unroll
                    for (int b = 0; b < 16; ++b) qcol[b] = (w[b >> 1] >> (16 * (b & 1))) & 0xFFFFu;
                    par ^= mulc(sl[g][i], qcol);
                }
                a.parity[cw * a.pstride + lane] = (uint16_t)par;
            }
        } else {
            // flagged codewords (nonzero syndromes or erasures) go to the error queue, one
            // atomic per block pass (a counter hit once per codeword serialises)
            const uint64_t nz = __ballot(S != 0);
            const uint32_t half = (uint32_t)(nz >> (32 * (g & 1)));
            const bool flagged = live && (half != 0 || (a.neras && a.neras[cw] != 0));
            if (flagged && lane < NR) a.syn[cw * kMaxNR + lane] = (uint16_t)S;   // zeros too
            if (lane == 0) {
                nfl[g] = flagged ? 1u : 0u;
                if (live) a.result[cw] = flagged ? kSentinel : 0;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned n = 0;
#pragma unroll
                for (int j = 0; j < kFinGroups; ++j) n += nfl[j];
                qbase = n ? atomicAdd(a.queue, n) : 0u;
            }
            __syncthreads();
            if (lane == 0 && flagged) {
                unsigned below = 0;
                for (unsigned j = 0; j < g; ++j) below += nfl[j];
                a.queue[1 + qbase + below] = (uint32_t)cw;
            }
            __syncthreads();                  // nfl / qbase reused by the next pass
        }
    }
}

// ------------------------------------------------------------------------------------------------
struct ErrArgs {
    DevCodec c;
    DecodeArgs d;
    const uint16_t *syn;
    const uint32_t *queue;
    uint16_t qsolve[16];        // y = sum_j c_j qsolve[j] solves y^2 + y = c when Tr(c) = 0
};

#ifndef EZRS_WIDE_ERR_WAVES
#define EZRS_WIDE_ERR_WAVES 16
#endif
constexpr int kErrWaves = EZRS_WIDE_ERR_WAVES;
// per-wave scratch, dwords: roots 64, omega/syndromes/lambda 3 x 32, factor pool 32 (64 u16),
// factor stack 40
constexpr int kErrScratch = 64 + 3 * 32 + 32 + 40;

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
    return v;
}

// x mod nn for x < 2 nn
__device__ __forceinline__ unsigned red1(unsigned x, unsigned nn) { return x >= nn ? x - nn : x; }
// x mod nn for any 32-bit x, nn = 2^mm - 1 (Karn's fold, rs_base:648-657): two folds leave x < nn + 2
__device__ __forceinline__ unsigned fold(unsigned x, unsigned nn, unsigned mm) {
    x = (x & nn) + (x >> mm);
    x = (x & nn) + (x >> mm);
    return red1(x, nn);
}

// ---- lane-parallel polynomials over GF(2^m): lane j holds coefficient j (degree <= 63) ----------
struct Gf {
    const uint16_t *AT;     // antilog, LDS
    const uint16_t *I;      // log, global
    unsigned nn;
};

__device__ __forceinline__ int pdeg(unsigned a) {
    const uint64_t nz = __ballot(a != 0);
    return nz ? 63 - __builtin_clzll(nz) : -1;
}
__device__ __forceinline__ unsigned plog(const Gf &g, unsigned a) { return a ? g.I[a] : g.nn; }
__device__ __forceinline__ unsigned pexp(const Gf &g, unsigned l) { return l != g.nn ? g.AT[l] : 0u; }

// a mod b: b monic of degree db >= 1 given in log form (blog), a of degree <= da
__device__ unsigned pmod(const Gf &g, unsigned a, int da, unsigned blog, int db, unsigned lane) {
    for (int t = da; t >= db; --t) {
        const unsigned c = __builtin_amdgcn_readlane(a, t);
        const unsigned bl = __shfl(blog, (int)((lane - (unsigned)(t - db)) & 63), 64);
        if (c) {
            const unsigned lc = __builtin_amdgcn_readfirstlane(g.I[c]);
            if ((int)lane >= t - db && (int)lane <= t && bl != g.nn) a ^= g.AT[red1(lc + bl, g.nn)];
        }
    }
    return a;
}

// log form of a / a[d]
__device__ __forceinline__ unsigned pmonic_log(const Gf &g, unsigned a, int d) {
    const unsigned lc = __builtin_amdgcn_readfirstlane(g.I[__builtin_amdgcn_readlane(a, d)]);
    const unsigned al = plog(g, a);
    return al != g.nn ? red1(al + g.nn - lc, g.nn) : g.nn;
}

// monic gcd(a, b) (polynomial form), its degree in dg; a != 0
__device__ unsigned pgcd(const Gf &g, unsigned a, unsigned b, int &dg, unsigned lane) {
    int da = pdeg(a), db = pdeg(b);
    if (db < 0) {                                    // gcd(a, 0) = a / a[da]
        dg = da;
        return pexp(g, pmonic_log(g, a, da));
    }
    while (db >= 0) {
        const unsigned bl = pmonic_log(g, b, db);
        const unsigned r = db > 0 ? pmod(g, a, da, bl, db, lane) : 0u;
        a = pexp(g, bl);
        da = db;
        b = r;
        db = pdeg(r);
    }
    dg = da;
    return a;
}

// f / gm for gm | f, gm monic of degree dg in log form
__device__ unsigned pdiv(const Gf &g, unsigned f, int df, unsigned gl, int dg, unsigned lane) {
    unsigned q = 0;
    for (int t = df; t >= dg; --t) {
        const unsigned c = __builtin_amdgcn_readlane(f, t);
        const unsigned bl = __shfl(gl, (int)((lane - (unsigned)(t - dg)) & 63), 64);
        if (c) {
            const unsigned lc = __builtin_amdgcn_readfirstlane(g.I[c]);
            if ((int)lane == t - dg) q = c;
            if ((int)lane >= t - dg && (int)lane <= t && bl != g.nn) f ^= g.AT[red1(lc + bl, g.nn)];
        }
    }
    return q;
}

__global__ void __launch_bounds__(64 * kErrWaves) k_wide_errors(ErrArgs ea) {
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    const DevCodec &c = ea.c;
    const DecodeArgs &a = ea.d;
    const unsigned NN = c.nn, A0 = c.nn, NR = c.nroots, FCR = c.fcr, PRM = c.prim, MM = c.mm;
    const uint32_t nq = ea.queue[0];
    if ((size_t)blockIdx.x * kErrWaves >= nq) return;      // uniform over the workgroup
    uint16_t *AT = smem;                          // alpha^e, e < NN
    for (unsigned i = threadIdx.x; i < NN; i += blockDim.x) AT[i] = c.alpha_to[i];
    const int wave = threadIdx.x >> 6;
    const unsigned lane = threadIdx.x & 63;
    // per-wave scratch: roots (u32 x 64), omega, syndromes, lambda (index form, u16 x 64 each),
    // the root finder's factor pool (u16 x 64) and stack (u32 x 40)
    uint32_t *roots = reinterpret_cast<uint32_t *>(smem + ((NN + 7) & ~7u)) + wave * kErrScratch;
    uint16_t *omg = reinterpret_cast<uint16_t *>(roots + 64);
    uint16_t *slg = omg + 64;
    uint16_t *llg = slg + 64;
    uint16_t *pool = llg + 64;
    uint32_t *stk = reinterpret_cast<uint32_t *>(pool + 64);
    __syncthreads();
    const uint16_t *I = c.index_of;
    const Gf g{AT, I, NN};
    const unsigned len = a.len, pad = c.load - len;

    for (uint32_t qi = blockIdx.x * kErrWaves + wave; qi < nq; qi += gridDim.x * kErrWaves) {
        const size_t k = ea.queue[1 + qi];
        uint16_t *data = static_cast<uint16_t *>(a.data) + k * a.data_stride;
        uint16_t *parity = static_cast<uint16_t *>(a.parity) + k * a.parity_stride;
        const uint32_t *eras = a.eras ? a.eras + k * a.eras_stride : nullptr;
        const unsigned no_eras = a.neras ? a.neras[k] : 0;
        uint32_t *pos = a.positions ? a.positions + k * a.pos_stride : nullptr;
        uint16_t *corr = a.corr ? static_cast<uint16_t *>(a.corr) + k * a.corr_stride : nullptr;
        int count;
        // argument checks of decode_symbols (rs_base:1375-1387)
        bool bad = no_eras > NR;
        if (!bad && lane < no_eras) bad = eras[lane] >= len + NR;
        if (__ballot(bad)) { if (lane == 0) a.result[k] = -1; continue; }
        const unsigned sp = lane < NR ? ea.syn[k * kMaxNR + lane] : 0u;
        if (!__ballot(sp != 0)) { if (lane == 0) a.result[k] = 0; continue; }   // 1416-1434
        const unsigned sl = sp ? I[sp] : A0;                 // syn[lane], index form
        slg[lane] = (uint16_t)sl;

        // erasure locator (1436-1450): lane j holds lambda[j] (polynomial form)
        unsigned lam = lane == 0 ? 1u : 0u;
        if (no_eras > 0) {
            const unsigned u0 = fold(PRM * (NN - 1 - (eras[0] + pad)), NN, MM);
            if (lane == 1) lam = AT[u0];
            for (unsigned i = 1; i < no_eras; ++i) {
                const unsigned u = fold(PRM * (NN - 1 - (eras[i] + pad)), NN, MM);
                const unsigned prev = __shfl_up(lam, 1, 64);
                const unsigned tmp = lane >= 1 && lane <= i + 1 && prev ? I[prev] : A0;
                if (tmp != A0) lam ^= AT[red1(u + tmp, NN)];
            }
        }
        unsigned b = lam ? I[lam] : A0;                      // b[lane], index form
        unsigned li = b;                                     // lambda[lane], index form
        // Berlekamp-Massey (1501-1546); lanes > NR hold lambda = 0, b = A0.  A step with a zero
        // discrepancy leaves lambda (and so li) as it is: the log-table read is redone only after
        // lambda changes.
        unsigned r = no_eras, el = no_eras;
        while (++r <= NR) {
            const unsigned si = lane < r ? slg[r - 1 - lane] : A0;
            const unsigned term = (li != A0 && si != A0) ? AT[red1(li + si, NN)] : 0u;
            const unsigned dsum = wave_xor(term);
            const unsigned discr = dsum ? I[dsum] : A0;
            const unsigned bprev = __shfl_up(b, 1, 64);
            const unsigned bsh = lane == 0 ? A0 : bprev;
            if (discr == A0) {
                b = lane <= NR ? bsh : A0;
            } else {
                const unsigned t = lane == 0 ? lam : lam ^ (bsh != A0 ? AT[red1(discr + bsh, NN)] : 0u);
                if (2 * el <= r + no_eras - 1) {
                    el = r + no_eras - el;
                    b = lane <= NR ? (lam == 0 ? A0 : red1(li + NN - discr, NN)) : A0;
                } else {
                    b = lane <= NR ? bsh : A0;
                }
                lam = lane <= NR ? t : 0u;
                li = lam ? I[lam] : A0;
            }
        }
        // lambda to index form, its degree (1549-1553)
        const unsigned llog = li;
        const uint64_t nzl = __ballot(lam != 0 && lane <= NR);
        const unsigned deg = 63 - __builtin_clzll(nzl);
        llg[lane] = (uint16_t)llog;
        if (deg == 0) {                                      // 1577-1595 (no root can match)
            if (lane == 0) a.result[k] = -1;
            continue;
        }
        // Roots of lambda -- the set the Chien search finds (1555-1584) -- by Berlekamp's trace
        // algorithm.  lambda has deg distinct roots in GF(2^m) iff x^(2^m) = x mod lambda
        // (x^(2^m) - x is the product of all x - a); otherwise the reference's search finds fewer
        // than deg roots and gives up.  P_k = x^(2^k) mod L (L = lambda made monic) by repeated
        // squaring; a factor F of L splits as gcd(F, Tr(beta x) mod F), Tr(y) = sum_k y^(2^k),
        // beta = alpha^b for b = 0..m-1 (a basis: two distinct roots differ in some
        // Tr(alpha^b .)).  Factors wait on a stack in LDS; a linear factor x + r gives the root
        // r = alpha^i, i in [1, NN] as the reference numbers positions.
        const unsigned Ll = pmonic_log(g, lam, (int)deg);
        const unsigned x1 = deg >= 2 ? (lane == 1 ? 1u : 0u) : (lane == 0 ? pexp(g, Ll) : 0u);
        // squaring is GF(2)-linear: (sum_j p_j x^j)^2 = sum_j p_j^2 Q_j with Q_j = x^(2j) mod L, so
        // each squaring is deg independent products per lane once the Q_j are known (x^i mod L
        // for i <= 2 deg - 2, one multiply-by-x step each)
        unsigned Ql[kMaxNR];                                 // log form of Q_j
        {
            unsigned X = lane == 0 ? 1u : 0u;
#pragma unroll
            for (int i = 0; i <= 2 * kMaxNR - 2; ++i) {
                if (i > 2 * (int)deg - 2) break;
                if ((i & 1) == 0) Ql[i >> 1] = plog(g, X);
                const unsigned top = __builtin_amdgcn_readlane(X, deg - 1);
                X = __shfl_up(X, 1, 64);
                if (lane == 0 || lane >= deg) X = 0;
                if (top) {                                   // x^deg = sum_(m < deg) L_m x^m
                    const unsigned lt = __builtin_amdgcn_readfirstlane(I[top]);
                    if (lane < deg && Ll != A0) X ^= AT[red1(lt + Ll, NN)];
                }
            }
        }
        unsigned Pl[kM];                                     // log form of P_0 .. P_(m-1)
        unsigned P = x1;
#pragma unroll
        for (int kk = 0; kk < kM; ++kk) {
            Pl[kk] = plog(g, P);
            unsigned acc = 0;
#pragma unroll
            for (int j = 0; j < kMaxNR; ++j) {
                if (j >= (int)deg) break;
                const unsigned lp = __builtin_amdgcn_readlane(Pl[kk], j);
                if (lp != A0 && Ql[j] != A0) acc ^= AT[red1(red1(2 * lp, NN) + Ql[j], NN)];
            }
            P = acc;
        }
        count = __ballot(P != x1) ? -1 : 0;
        if (count == 0) {
            if (lane <= deg) pool[lane] = (uint16_t)pexp(g, Ll);
            if (lane == 0) stk[0] = deg << 8;                // off | deg << 8 | first b << 16
            int nstk = 1;
            __builtin_amdgcn_wave_barrier();
            while (nstk > 0) {
                const uint32_t e = stk[--nstk];
                const int off = (int)(e & 255), f = (int)((e >> 8) & 255);
                const unsigned F = (int)lane <= f ? pool[off + lane] : 0u;
                __builtin_amdgcn_wave_barrier();
                if (f == 2) {
                    // x^2 + p x + q, p != 0 (distinct roots): x = p y, y^2 + y = q / p^2, a GF(2)-
                    // linear equation with the precomputed solver; roots p y and p y + p
                    const unsigned q = __builtin_amdgcn_readlane(F, 0), pp = __builtin_amdgcn_readlane(F, 1);
                    if (!pp) { count = -1; break; }
                    const unsigned lp = __builtin_amdgcn_readfirstlane(I[pp]);
                    const unsigned lq = __builtin_amdgcn_readfirstlane(I[q]);
                    const unsigned cv = __builtin_amdgcn_readfirstlane(AT[fold(lq + 2 * (NN - lp), NN, MM)]);
                    unsigned y = 0;
#pragma unroll
                    for (int j = 0; j < kM; ++j) y ^= (cv >> j & 1) ? ea.qsolve[j] : 0u;
                    const unsigned ly = __builtin_amdgcn_readfirstlane(I[y]);
                    const unsigned r1 = AT[red1(lp + ly, NN)], r2 = r1 ^ pp;
                    const unsigned i1 = I[lane == 0 ? r1 : r2];
                    if (lane < 2) roots[count + lane] = i1 ? i1 : NN;
                    count += 2;
                    continue;
                }
                if (f == 1) {
                    const unsigned il = __builtin_amdgcn_readfirstlane(I[__builtin_amdgcn_readlane(F, 0)]);
                    if (lane == 0) roots[count] = il ? il : NN;
                    ++count;
                    continue;
                }
                const unsigned Fl = plog(g, F);              // F is monic
                bool split = false;
                for (unsigned b = e >> 16; b < (unsigned)kM; ++b) {
                    unsigned T = 0, eb = b;                  // Tr(alpha^b x) mod L
#pragma unroll
                    for (int kk = 0; kk < kM; ++kk) {
                        if (Pl[kk] != A0) T ^= AT[red1(Pl[kk] + eb, NN)];
                        eb = red1(2 * eb, NN);
                    }
                    const unsigned R = pmod(g, T, (int)deg - 1, Fl, f, lane);
                    int dg;
                    const unsigned G = pgcd(g, F, R, dg, lane);
                    if (dg > 0 && dg < f) {
                        const unsigned H = pdiv(g, F, f, plog(g, G), dg, lane);
                        if ((int)lane <= dg) pool[off + lane] = (uint16_t)G;
                        if ((int)lane <= f - dg) pool[off + dg + 1 + lane] = (uint16_t)H;
                        if (lane == 0) {
                            stk[nstk] = (uint32_t)off | (uint32_t)dg << 8 | (b + 1) << 16;
                            stk[nstk + 1] = (uint32_t)(off + dg + 1) | (uint32_t)(f - dg) << 8 | (b + 1) << 16;
                        }
                        nstk += 2;
                        __builtin_amdgcn_wave_barrier();
                        split = true;
                        break;
                    }
                }
                if (!split) {                                // unreachable for distinct roots
                    count = -1;
                    break;
                }
            }
        }
        if (count == (int)deg) {                             // ascending order (rank sort)
            __builtin_amdgcn_wave_barrier();
            unsigned v = 0, rank = 0;
            if (lane < (unsigned)count) {
                v = roots[lane];
                for (int s2 = 0; s2 < count; ++s2) rank += roots[s2] < v;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane < (unsigned)count) roots[rank] = v;
            __builtin_amdgcn_wave_barrier();
        }
        if (count != (int)deg || deg == 0) {                // 1577-1595: no corrections
            if (lane == 0) a.result[k] = -1;
            continue;
        }
        // Omega = S Lambda mod x^NR (1596-1604): lane i <= deg - 1
        const unsigned deg_omega = deg - 1;
        if (lane <= deg_omega) {
            unsigned tmp = 0;
            for (unsigned j = 0; j <= lane; ++j) {
                const unsigned sv = slg[lane - j], lv = llg[j];
                if (sv != A0 && lv != A0) tmp ^= AT[red1(sv + lv, NN)];
            }
            omg[lane] = (uint16_t)(tmp ? I[tmp] : A0);
        }
        __builtin_amdgcn_wave_barrier();
        // Forney (1610-1690): lane j handles root j
        bool fail = false, wrote = false;
        unsigned cor = 0, loc = 0;
        if (lane < (unsigned)count) {
            const unsigned rj = roots[lane];
            unsigned num1 = 0;
            for (unsigned i = 0; i <= deg_omega; ++i) {
                const unsigned ov = omg[i];
                if (ov != A0) num1 ^= AT[fold(ov + i * rj, NN, MM)];
            }
            const unsigned num2 = AT[fold(rj * fold(FCR + NN - 1, NN, MM), NN, MM)];
            unsigned den = 0;
            const unsigned top = deg < NR - 1 ? deg : NR - 1;
            for (int i = (int)(top & ~1u); i >= 0; i -= 2) {
                const unsigned lv = llg[i + 1];
                if (lv != A0) den ^= AT[fold(lv + (unsigned)i * rj, NN, MM)];
            }
            loc = fold(rj * c.iprim + NN - 1, NN, MM);
            if (den == 0) fail = true;
            else if (num1 != 0) {
                if (loc < pad) fail = true;
                else {
                    cor = AT[fold(I[num1] + I[num2] + NN - I[den], NN, MM)];
                    wrote = true;
                }
            }
        }
        // the reference walks j = count-1 .. 0 and stops at the first failure: roots above the
        // highest failing one keep their corrections
        const uint64_t fm = __ballot(fail);
        const int jf = fm ? 63 - __builtin_clzll(fm) : -1;
        if ((int)lane <= jf) wrote = false;
        if (wrote) {
            if (loc < NN - NR) data[loc - pad] ^= (uint16_t)cor;
            else parity[loc - (NN - NR)] ^= (uint16_t)cor;
            if (corr) corr[lane] = (uint16_t)cor;
        }
        count = fm ? -1 : count;
        if (pos && count > 0 && lane < (unsigned)count) pos[lane] = loc - pad;
        if (lane == 0) a.result[k] = count;
    }
}

} // namespace wide

// ------------------------------------------------------------------------------------------------
namespace {

template <class C> bool wide_matches(const DevCodec &d) {
    static_assert(C::M == wide::kM, "the wide engine is GF(2^16)");
    return d.mm == C::M && d.poly == C::POLY && d.fcr == C::FCR && d.prim == C::PRIM &&
           d.nroots == C::NR && !d.dual && !d.masked;
}

template <class C> constexpr uint32_t nlp_of() {
    return ((C::NL + wide::kLPW - 1) / wide::kLPW) * wide::kLPW;
}

// Workspace: [queue: 4 + 4 ncw B, rounded to 256] [syn: 64 ncw B] [rem: 32 nlp ncw B]
struct WideWs {
    uint32_t *queue;
    uint16_t *syn;
    uint16_t *rem;
};

WideWs carve(void *ws, size_t ncw) {
    uint8_t *p = static_cast<uint8_t *>(ws);
    WideWs w;
    w.queue = reinterpret_cast<uint32_t *>(p);
    p += ((4 + 4 * ncw) + 255) / 256 * 256;
    w.syn = reinterpret_cast<uint16_t *>(p);
    p += 64 * ncw;
    w.rem = reinterpret_cast<uint16_t *>(p);
    return w;
}

template <class C>
hipError_t launch_rem(const uint8_t *base, size_t stride_bytes, uint32_t n, size_t ncw, uint16_t *rem,
                      hipStream_t s) {
    wide::RemArgs r{base, stride_bytes, n, (uint32_t)ncw, rem, nlp_of<C>()};
    const unsigned grid = (unsigned)((ncw + wide::kRows - 1) / wide::kRows);
    constexpr int NW = (C::NL + wide::kLPW - 1) / wide::kLPW;
    hipLaunchKernelGGL((wide::k_wide_rem<C>), dim3(grid), dim3(64 * NW), 0, s, r);
    return hipGetLastError();
}

} // namespace

int wide_codec_id(const DevCodec &d) {
    int id = 0, found = -1;
#define EZRS_WIDE_MATCH(C) \
    if (found < 0 && wide_matches<wide::WC_##C>(d)) found = id; \
    ++id;
    EZRS_WIDE_CODEC_LIST(EZRS_WIDE_MATCH)
#undef EZRS_WIDE_MATCH
    return found;
}

static uint32_t wide_nlp(int id) {
    int k = 0;
    uint32_t v = 0;
#define EZRS_WIDE_NLP(C) if (k++ == id) v = nlp_of<wide::WC_##C>();
    EZRS_WIDE_CODEC_LIST(EZRS_WIDE_NLP)
#undef EZRS_WIDE_NLP
    return v;
}

size_t wide_ws_bytes(int id, size_t ncw) {
    return ((4 + 4 * ncw) + 255) / 256 * 256 + 64 * ncw + 32 * (size_t)wide_nlp(id) * ncw;
}

// Host tables of a wide codec: leader of each syndrome (same coset rule as gen_wide.py) and
// Q = V^-1 diag(beta^NR) in index form.
// Linear solver of y^2 + y = c over GF(2^mm) (field polynomial poly): y -> y^2 + y is GF(2)-linear
// with kernel {0, 1}; its image (trace-0 elements) gets a reduced echelon basis b_j (pivot bit j)
// with preimages p_j, so for c in the image y = sum over pivot bits j of c_j p_j.
void quad_solver(unsigned poly, unsigned mm, uint16_t out[16]) {
    auto mul = [&](unsigned a, unsigned b) {
        unsigned r = 0;
        for (unsigned i = 0; i < mm; ++i) {
            if (b >> i & 1) r ^= a;
            a <<= 1;
            if (a >> mm & 1) a ^= poly;
        }
        return r;
    };
    unsigned vec[16] = {}, pre[16] = {};                 // indexed by pivot bit
    bool have[16] = {};
    for (unsigned i = 0; i < mm; ++i) {
        unsigned v = mul(1u << i, 1u << i) ^ (1u << i), p = 1u << i;
        for (int b = (int)mm - 1; b >= 0; --b)
            if ((v >> b & 1) && have[b]) { v ^= vec[b]; p ^= pre[b]; }
        if (!v) continue;
        const int hb = 31 - __builtin_clz(v);
        for (int b = 0; b < 16; ++b)                        // keep the basis fully reduced
            if (have[b] && (vec[b] >> hb & 1)) { vec[b] ^= v; pre[b] ^= p; }
        vec[hb] = v; pre[hb] = p; have[hb] = true;
    }
    for (unsigned j = 0; j < 16; ++j) out[j] = (uint16_t)(j < mm && have[j] ? pre[j] : 0);
}

bool wide_build_consts(int id, const CodecMath &m, std::vector<uint16_t> &blob) {
    const unsigned NN = m.nn, NR = m.spec.nroots;
    if (NR > wide::kMaxNR) return false;
    const Field &gf = m.gf;
    // the kernel's slot order of the coset leaders (gen_wide.py: WC_*::LEADER)
    std::vector<unsigned> lead;
    {
        int k = 0;
#define EZRS_WIDE_LEAD(C) \
        if (k++ == id) lead.assign(wide::WC_##C::LEADER, wide::WC_##C::LEADER + wide::WC_##C::NL);
        EZRS_WIDE_CODEC_LIST(EZRS_WIDE_LEAD)
#undef EZRS_WIDE_LEAD
    }
    std::vector<uint8_t> li(NR);
    std::vector<uint16_t> el(NR);
    for (unsigned i = 0; i < NR; ++i) {
        const unsigned e = (unsigned)(((uint64_t)(m.spec.fcr + i) * m.spec.prim) % NN);
        el[i] = (uint16_t)e;
        unsigned mn = e, x = e;
        do { x = (unsigned)((2ull * x) % NN); if (x < mn) mn = x; } while (x != e);
        unsigned slot = 0;
        while (slot < lead.size() && lead[slot] != mn) ++slot;
        if (slot == lead.size()) return false;          // not a coset the kernel evaluates
        li[i] = (uint8_t)slot;
    }
    // V[i][k] = beta_i^(NR-1-k); invert by Gauss-Jordan
    std::vector<unsigned> V(NR * NR), Inv(NR * NR, 0);
    for (unsigned i = 0; i < NR; ++i) {
        for (unsigned k = 0; k < NR; ++k)
            V[i * NR + k] = gf.pow_alpha((unsigned)(((uint64_t)el[i] * (NR - 1 - k)) % NN));
        Inv[i * NR + i] = 1;
    }
    auto inv = [&](unsigned a) { return gf.alpha_to[(NN - gf.index_of[a]) % NN]; };
    for (unsigned col = 0; col < NR; ++col) {
        unsigned piv = col;
        while (piv < NR && !V[piv * NR + col]) ++piv;
        if (piv == NR) return false;
        if (piv != col)
            for (unsigned k = 0; k < NR; ++k) {
                std::swap(V[piv * NR + k], V[col * NR + k]);
                std::swap(Inv[piv * NR + k], Inv[col * NR + k]);
            }
        const unsigned f = inv(V[col * NR + col]);
        for (unsigned k = 0; k < NR; ++k) {
            V[col * NR + k] = gf.mul(V[col * NR + k], f);
            Inv[col * NR + k] = gf.mul(Inv[col * NR + k], f);
        }
        for (unsigned r = 0; r < NR; ++r) {
            if (r == col || !V[r * NR + col]) continue;
            const unsigned g = V[r * NR + col];
            for (unsigned k = 0; k < NR; ++k) {
                V[r * NR + k] ^= gf.mul(g, V[col * NR + k]);
                Inv[r * NR + k] ^= gf.mul(g, Inv[col * NR + k]);
            }
        }
    }
    // blob: leader[32] (as u16) | elog[32] | columns (the device copy): beta_i * 2^b [NR][16], then
    // Q_ki * 2^b [NR][NR][16] with Q = V^-1 diag(beta^NR): parity_k = sum_i Q_ki S_i
    blob.assign(2 * wide::kMaxNR + NR * 16 + NR * NR * 16, 0);
    for (unsigned i = 0; i < NR; ++i) {
        blob[i] = li[i];
        blob[wide::kMaxNR + i] = el[i];
        const unsigned beta = gf.pow_alpha(el[i]);
        for (unsigned b = 0; b < 16; ++b) blob[2 * wide::kMaxNR + i * 16 + b] = (uint16_t)gf.mul(beta, 1u << b);
    }
    uint16_t *qc = blob.data() + 2 * wide::kMaxNR + NR * 16;
    for (unsigned k = 0; k < NR; ++k)
        for (unsigned i = 0; i < NR; ++i) {
            const unsigned bn = gf.pow_alpha((unsigned)(((uint64_t)el[i] * NR) % NN));
            const unsigned q = gf.mul(Inv[k * NR + i], bn);
            for (unsigned b = 0; b < 16; ++b) qc[(k * NR + i) * 16 + b] = (uint16_t)gf.mul(q, 1u << b);
        }
    return true;
}

size_t wide_cols_count(unsigned nroots) { return (size_t)nroots * 16 + (size_t)nroots * nroots * 16; }

static wide::FinishArgs finish_args(const DevCodec &d, int id, const uint16_t *blob_host,
                                    const uint16_t *cols_dev, size_t ncw, uint16_t *rem) {
    wide::FinishArgs f{};
    f.rem = rem;
    f.nlp = wide_nlp(id);
    f.ncw = (uint32_t)ncw;
    f.nr = d.nroots;
    for (unsigned i = 0; i < d.nroots; ++i) f.leader[i] = (uint8_t)blob_host[i];
    f.cols = cols_dev;
    return f;
}

static unsigned finish_grid(const DevCodec &d, size_t ncw) {
    const size_t want = (ncw + wide::kFinGroups - 1) / wide::kFinGroups, cap = (size_t)(d.ncu > 0 ? d.ncu : 256) * 8;
    return (unsigned)(want < cap ? want : cap);
}

bool wide_can_encode(const DevCodec &, const EncodeArgs &a) {
    return a.ncw <= 0xFFFFFFFFu && (a.ncw <= 1 || 2 * a.data_stride * (wide::kRows - 1) < 0x80000000u);
}

bool wide_can_decode(const DevCodec &d, const DecodeArgs &a) {
    const bool inline_par = a.parity == static_cast<uint16_t *>(a.data) + a.len &&
                            a.parity_stride == a.data_stride;
    return inline_par && a.ncw <= 0xFFFFFFFFu &&
           (a.ncw <= 1 || 2 * a.data_stride * (wide::kRows - 1) < 0x80000000u) &&
           (a.ncw <= 1 || a.data_stride >= (size_t)a.len + d.nroots);
}

hipError_t launch_wide_encode(int id, const DevCodec &d, const EncodeArgs &a, const uint16_t *blob_host,
                              const uint16_t *cols_dev, void *ws, hipStream_t s) {
    if (a.ncw == 0) return hipSuccess;
    WideWs w = carve(ws, a.ncw);
    const size_t sb = 2 * (a.ncw > 1 ? a.data_stride : (size_t)a.len);
    int k = 0;
    hipError_t e = hipSuccess;
#define EZRS_WIDE_ENC(C) \
    if (k++ == id) e = launch_rem<wide::WC_##C>(static_cast<const uint8_t *>(a.data), sb, a.len, a.ncw, w.rem, s);
    EZRS_WIDE_CODEC_LIST(EZRS_WIDE_ENC)
#undef EZRS_WIDE_ENC
    if (e != hipSuccess) return e;
    wide::FinishArgs f = finish_args(d, id, blob_host, cols_dev, a.ncw, w.rem);
    f.parity = static_cast<uint16_t *>(a.parity);
    f.pstride = a.parity_stride;
    hipLaunchKernelGGL(wide::k_wide_finish<true>, dim3(finish_grid(d, a.ncw)), dim3(256), 0, s, f);
    return hipGetLastError();
}

hipError_t launch_wide_decode(int id, const DevCodec &d, const DecodeArgs &a, const uint16_t *blob_host,
                              const uint16_t *cols_dev, void *ws, hipStream_t s) {
    if (a.ncw == 0) return hipSuccess;
    WideWs w = carve(ws, a.ncw);
    hipError_t e = hipMemsetAsync(w.queue, 0, 4, s);
    if (e != hipSuccess) return e;
    const size_t sb = 2 * (a.ncw > 1 ? a.data_stride : (size_t)a.len + d.nroots);
    int k = 0;
#define EZRS_WIDE_DEC(C) \
    if (k++ == id) e = launch_rem<wide::WC_##C>(static_cast<const uint8_t *>(a.data), sb, a.len + d.nroots, a.ncw, w.rem, s);
    EZRS_WIDE_CODEC_LIST(EZRS_WIDE_DEC)
#undef EZRS_WIDE_DEC
    if (e != hipSuccess) return e;
    wide::FinishArgs f = finish_args(d, id, blob_host, cols_dev, a.ncw, w.rem);
    f.neras = a.neras;
    f.result = a.result;
    f.syn = w.syn;
    f.queue = w.queue;
    hipLaunchKernelGGL(wide::k_wide_finish<false>, dim3(finish_grid(d, a.ncw)), dim3(256), 0, s, f);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    wide::ErrArgs ea{d, a, w.syn, w.queue, {}};
    quad_solver(d.poly, d.mm, ea.qsolve);
    const size_t smem = (((size_t)d.nn + 7) & ~(size_t)7) * 2 + wide::kErrWaves * wide::kErrScratch * 4;
    const unsigned grid = (unsigned)(d.ncu > 0 ? d.ncu : 256);
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void *>(&wide::k_wide_errors),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(wide::k_wide_errors, dim3(grid), dim3(64 * wide::kErrWaves), smem, s, ea);
    return hipGetLastError();
}

} // namespace ezrs
