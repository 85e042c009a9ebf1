// ezrs_generic.hip -- per-codeword RS encode / decode kernels for every codec (GF(2^2)..GF(2^16)).
//
// One lane owns one codeword and runs the reference algorithm on it verbatim: the systematic LFSR
// of encode_symbols (c++/ezpwd/rs_base:1296-1332) and the syndrome -> erasure locator ->
// Berlekamp-Massey -> Chien -> Omega -> Forney chain of decode_symbols (rs_base:1335-1718), with the
// data-type mapping of encode<INP>/decode<INP> (rs_base:868-904, 1170-1242).  These kernels define
// the engine's semantics for all inputs (shortened codes, erasures, the overwhelmed regime) and are
// the error-path back end of the fast GF(2^8) kernels; they are table-driven (log/antilog in LDS
// for m <= 12, in L2-resident global memory above that).
#include "ezrs_internal.hpp"

namespace ezrs {
namespace {

constexpr int kBlock = 256;
constexpr int kDecBlock = 64;    // generic decode with NR <= 32: LDS working arrays per 64 lanes

// x mod nn for x < 2^32 (Karn's fold, rs_base:648-657).
__device__ __forceinline__ unsigned modnn(unsigned x, unsigned nn, unsigned mm) {
    while (x >= nn) {
        x -= nn;
        x = (x >> mm) + (x & nn);
    }
    return x;
}

template <typename T> struct Tabs {
    const uint16_t *A;   // alpha_to
    const uint16_t *I;   // index_of
    const uint8_t *ID;   // into_dual
    const uint8_t *FD;   // from_dual
};

// Stage the field tables into LDS when they fit (m <= 12: 2 x 8 KiB), else read them from HBM/L2.
template <bool LDS>
__device__ __forceinline__ void stage_tables(const DevCodec &c, uint16_t *smem, const uint16_t *&A,
                                             const uint16_t *&I, const uint8_t *&ID,
                                             const uint8_t *&FD) {
    if (LDS) {
        uint16_t *sA = smem, *sI = smem + (c.nn + 1);
        uint8_t *sD = reinterpret_cast<uint8_t *>(smem + 2 * (c.nn + 1));
        for (unsigned i = threadIdx.x; i <= c.nn; i += blockDim.x) {
            sA[i] = c.alpha_to[i];
            sI[i] = c.index_of[i];
        }
        if (c.dual)
            for (unsigned i = threadIdx.x; i < 256; i += blockDim.x) {
                sD[i] = c.into_dual[i];
                sD[256 + i] = c.from_dual[i];
            }
        __syncthreads();
        A = sA; I = sI; ID = sD; FD = sD + 256;
    } else {
        A = c.alpha_to; I = c.index_of; ID = c.into_dual; FD = c.from_dual;
    }
}

// ------------------------------------------------------------------------------------------------
template <typename T, int MAXR, bool LDS>
__global__ void __launch_bounds__(kBlock) k_encode_generic(DevCodec c, EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    const uint16_t *A, *I;
    const uint8_t *ID, *FD;
    stage_tables<LDS>(c, smem, A, I, ID, FD);
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.ncw) return;
    const T *data;
    T *parity;
    unsigned len;
    row_ptrs<T>(a, k, data, parity, len);
    const unsigned NR = c.nroots, nn = c.nn, mm = c.mm;

    // Circular parity register: logical parity[j] lives at par[(head + j) % NR], so the
    // reference's std::rotate (rs_base:1318) becomes a head increment.  Its data-dependent index
    // keeps it out of VGPRs: in LDS (lanes interleaved) for NR <= 32, private memory above.
    constexpr int PS = MAXR <= 32 ? kBlock : 1;
    __shared__ uint16_t pbuf[MAXR <= 32 ? MAXR * kBlock : 1];
    uint16_t priv[MAXR <= 32 ? 1 : MAXR];
    uint16_t *const par = MAXR <= 32 ? pbuf + threadIdx.x : priv;
    for (unsigned j = 0; j < NR; ++j) par[(j) * PS] = 0;
    unsigned head = 0;
    for (unsigned i = 0; i < len; ++i) {
        unsigned sym = static_cast<unsigned>(data[i]) & nn;        // masked copy (rs_base:893)
        if (c.dual) sym = FD[sym];
        const unsigned fb = I[sym ^ par[(head) * PS]];
        if (fb != nn) {
            unsigned p = head + 1;
            for (unsigned j = 1; j < NR; ++j, ++p) {
                if (p >= NR) p -= NR;
                par[(p) * PS] ^= A[modnn(fb + c.genpoly[NR - j], nn, mm)];
            }
        }
        par[(head) * PS] = fb != nn ? A[modnn(fb + c.genpoly[0], nn, mm)] : 0;
        if (++head == NR) head = 0;
    }
    for (unsigned j = 0, p = head; j < NR; ++j) {
        unsigned v = par[(p) * PS];
        parity[j] = static_cast<T>(c.dual ? ID[v] : v);
        if (++p == NR) p = 0;
    }
}

// ------------------------------------------------------------------------------------------------
// encode_symbols with a 32-lane group per codeword (NR <= 32): lane j holds logical parity[j] of
// the reference's rotating register (rs_base:1296-1332).  One data symbol per step:
//   fb = index_of[sym ^ parity[0]];  parity'[j] = parity[j+1] ^ alpha_to[fb + genpoly[NR-1-j]]
// (parity[NR] = 0; nothing is added when fb = A0), i.e. the reference's XOR-then-rotate with the
// rotation done by a lane shift.  For long codewords (m > 8: up to 65535 symbols) the per-step
// latency is spread over 32x fewer codewords per lane, and 32x more lanes are busy.
constexpr int kLaneGroup = 32;

template <typename T, bool LDS>
__global__ void __launch_bounds__(kBlock) k_encode_lanes(DevCodec c, EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    const uint16_t *A, *I;
    const uint8_t *ID, *FD;
    stage_tables<LDS>(c, smem, A, I, ID, FD);
    const unsigned j = threadIdx.x & (kLaneGroup - 1);
    const size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / kLaneGroup;
    if (k >= a.ncw) return;                 // uniform over the group
    const T *data;
    T *parity;
    unsigned len;
    row_ptrs<T>(a, k, data, parity, len);
    const unsigned NR = c.nroots, nn = c.nn;
    const unsigned g = j < NR ? c.genpoly[NR - 1 - j] : 0;
    unsigned par = 0;
    for (unsigned i0 = 0; i0 < len; i0 += kLaneGroup) {
        unsigned dv = 0;
        if (i0 + j < len) {
            dv = static_cast<unsigned>(data[i0 + j]) & nn;            // masked copy (rs_base:893)
            if (c.dual) dv = FD[dv];
        }
        const unsigned cnt = len - i0 < (unsigned)kLaneGroup ? len - i0 : kLaneGroup;
        for (unsigned s = 0; s < cnt; ++s) {
            const unsigned sym = __shfl(dv, (int)s, kLaneGroup);
            const unsigned p0 = __shfl(par, 0, kLaneGroup);
            unsigned nxt = __shfl_down(par, 1, kLaneGroup);
            nxt = j + 1 < NR ? nxt : 0u;
            const unsigned fb = I[sym ^ p0];
            const unsigned x = fb + g, y = x >= nn ? x - nn : x;
            par = j < NR ? (nxt ^ (fb != nn ? (unsigned)A[y] : 0u)) : 0u;
        }
    }
    if (j < NR) parity[j] = static_cast<T>(c.dual ? ID[par] : par);
}

template <typename T>
hipError_t enc_lanes_launch(const DevCodec &c, const EncodeArgs &a, hipStream_t s) {
    const size_t threads = a.ncw * kLaneGroup;
    const unsigned grid = (unsigned)((threads + kBlock - 1) / kBlock);
    if (c.nn <= 4095) {
        const size_t sm = 2 * (c.nn + 1) * sizeof(uint16_t) + 512;
        hipLaunchKernelGGL((k_encode_lanes<T, true>), dim3(grid), dim3(kBlock), sm, s, c, a);
    } else {
        hipLaunchKernelGGL((k_encode_lanes<T, false>), dim3(grid), dim3(kBlock), 0, s, c, a);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// decode_symbols on one codeword.  Corrections are recorded and applied at the end: for the direct
// path every recorded correction (the reference corrects in place, so partial corrections before a
// failure persist, rs_base:1238-1241), for the masked path only when count > 0 (rs_base:1223-1234).
// Working arrays: private (WS = 0), or -- for the flagged-codeword kernel, whose per-lane arrays
// with data-dependent indices would otherwise sit in waterfall-indexed VGPRs -- in LDS at `lds`,
// element i of a lane's array at lds[i * WS] (lanes interleaved: conflict-free).  W is the element
// type: uint16_t, or uint8_t where every value fits (m = 8: indices, log values and A0 = 255).
// Working arrays per lane: arrays whose live ranges do not overlap share storage (root reuses b after
// BM, omega reuses the Chien registers t, the Forney deltas reuse syn), the Forney "wrote" flags are
// a register bitmask for MAXR <= 32, and fix positions are re-derived from loc.  Fewer bytes per lane
// in LDS means more resident waves for the latency-bound flagged-codeword kernel.
template <int MAXR>
constexpr int kWorkArrays = MAXR <= 32 ? 5 : 6;

template <typename T, int MAXR, int WS = 0, typename W = uint16_t, typename SY = uint8_t>
__device__ int decode_one(const DevCodec &c, const uint16_t *__restrict__ A,
                          const uint16_t *__restrict__ I, const uint8_t *ID, const uint8_t *FD,
                          T *data, unsigned len, T *parity, const uint32_t *eras,
                          unsigned no_eras, uint32_t *pos_out, T *corr_out,
                          const SY *syn_in = nullptr, W *lds = nullptr) {
    const unsigned NR = c.nroots, NN = c.nn, A0 = c.nn, mm = c.mm, LOAD = c.load;
    const unsigned FCR = c.fcr, PRM = c.prim;
    // Karn mode (c.karn): erasures and positions in the full NN frame (decode_rs.h:114, 295), the
    // datum is the symbol (no masked-path rules), and none of ezpwd's extra failure checks
    const bool karn = c.karn != 0, masked = c.masked && !karn;
    if (len == 0 || len > LOAD) return -1;                                    // 1375-1377
    if (no_eras > NR) return -1;                                              // 1380-1382
    // Karn mode: an erasure outside the frame is reported after the zero-syndrome return, the
    // order of libfec's checks (decode_rs.h:108-132; -1 here where libfec's result is undefined)
    bool eras_bad = false;
    for (unsigned i = 0; i < no_eras; ++i)
        if (eras[i] >= (karn ? NN : len + NR)) {                              // 1383-1387
            if (!karn) return -1;
            eras_bad = true;
        }
    if (masked)
        for (unsigned i = 0; i < NR; ++i)
            if (static_cast<unsigned>(parity[i]) & ~NN) return -1;            // 1215-1218
    const unsigned pad = LOAD - len;
    const unsigned epad = karn ? 0u : pad;    // frame offset of an erasure position

    constexpr int kS = WS ? WS : 1;
    constexpr int kW = MAXR + 1;       // elements per working array
    W priv[WS ? 1 : kWorkArrays<MAXR> * kW];
    W *const base = WS ? lds : priv;
    W *syn = base, *lambda = base + kW * kS, *b = base + 2 * kW * kS, *t = base + 3 * kW * kS,
             *corrv = base + 4 * kW * kS;
    W *const root = b, *const omega = t, *const fixv = syn;
    // wrote[j]: corr[j] (and fix j) written by the reference's Forney loop
    W *const wrote = kWorkArrays<MAXR> > 5 ? base + 5 * kW * kS : nullptr;
    // loc[j]: the Chien loop's k for root i = root[j], k = i * iprim - 1 (mod NN) (1562-1575)
    auto locof = [&](unsigned j) -> unsigned {
        return (unsigned)(((uint64_t)root[(j) * kS] * c.iprim + NN - 1) % NN);
    };
    uint32_t wmask = 0;
    auto set_wrote = [&](unsigned j) {
        if constexpr (MAXR <= 32) wmask |= 1u << j; else wrote[j * kS] = 1;
    };
    auto has_wrote = [&](unsigned j) -> bool {
        if constexpr (MAXR <= 32) return wmask >> j & 1; else return wrote[j * kS] != 0;
    };
    unsigned nroot = 0;
    int count = 0;
    unsigned deg_lambda = 0, deg_omega = 0, r = no_eras, el = no_eras;

    auto cnv = [&](unsigned x) -> unsigned {
        x &= NN;
        return c.dual ? FD[x] : x;
    };
    // syndromes by Horner over data then parity (1390-1414), unless the bit-sliced kernel
    // already evaluated them (same values: S_i = r(alpha^((fcr+i)*prim)) in polynomial form)
    if (syn_in) {
        for (unsigned i = 0; i < NR; ++i) syn[(i) * kS] = syn_in[i];
    } else {
        const unsigned s0 = cnv(data[0]);
        for (unsigned i = 0; i < NR; ++i) syn[(i) * kS] = (uint16_t)s0;
        for (unsigned j = 1; j < len + NR; ++j) {
            const unsigned x = cnv(j < len ? static_cast<unsigned>(data[j])
                                           : static_cast<unsigned>(parity[j - len]));
            for (unsigned i = 0; i < NR; ++i)
                syn[(i) * kS] = syn[(i) * kS] == 0 ? (uint16_t)x
                                     : (uint16_t)(x ^ A[modnn(I[syn[(i) * kS]] + (FCR + i) * PRM, NN, mm)]);
        }
    }
    unsigned syn_error = 0;
    for (unsigned i = 0; i < NR; ++i) {
        syn_error |= syn[(i) * kS];
        syn[(i) * kS] = I[syn[(i) * kS]];
    }
    if (!syn_error) return 0;                                                 // 1427-1434
    if (eras_bad) return -1;

    for (unsigned i = 0; i <= NR; ++i) lambda[(i) * kS] = 0;                        // 1436-1450
    lambda[(0) * kS] = 1;
    if (no_eras > 0) {
        lambda[(1) * kS] = A[modnn(PRM * (NN - 1 - (eras[0] + epad)), NN, mm)];
        for (unsigned i = 1; i < no_eras; ++i) {
            const unsigned u = modnn(PRM * (NN - 1 - (eras[i] + epad)), NN, mm);
            for (unsigned j = i + 1; j > 0; --j) {
                const unsigned tmp = I[lambda[(j - 1) * kS]];
                if (tmp != A0) lambda[(j) * kS] ^= A[modnn(u + tmp, NN, mm)];
            }
        }
    }
    for (unsigned i = 0; i <= NR; ++i) b[(i) * kS] = I[lambda[(i) * kS]];

    while (++r <= NR) {                                                       // BM 1507-1546
        // branch-free terms: index_of[0] = A0, and a term with an A0 factor adds 0
        unsigned discr_r = 0;
        for (unsigned i = 0; i < r; ++i) {
            const unsigned li = I[lambda[(i) * kS]], si = syn[(r - i - 1) * kS];
            const unsigned x = li + si, y = x >= NN ? x - NN : x;
            discr_r ^= (li == A0 || si == A0) ? 0u : (unsigned)A[y];
        }
        discr_r = I[discr_r];
        if (discr_r == A0) {
            for (unsigned i = NR; i > 0; --i) b[(i) * kS] = b[(i - 1) * kS];
            b[(0) * kS] = (uint16_t)A0;
        } else {
            t[(0) * kS] = lambda[(0) * kS];
            for (unsigned i = 0; i < NR; ++i) {
                const unsigned bi = b[(i) * kS], x = discr_r + bi, y = x >= NN ? x - NN : x;
                t[(i + 1) * kS] = (W)(lambda[(i + 1) * kS] ^ (bi == A0 ? 0u : (unsigned)A[y]));
            }
            if (2 * el <= r + no_eras - 1) {
                el = r + no_eras - el;
                for (unsigned i = 0; i <= NR; ++i)
                    b[(i) * kS] = lambda[(i) * kS] == 0 ? (uint16_t)A0
                                          : (uint16_t)modnn(I[lambda[(i) * kS]] - discr_r + NN, NN, mm);
            } else {
                for (unsigned i = NR; i > 0; --i) b[(i) * kS] = b[(i - 1) * kS];
                b[(0) * kS] = (uint16_t)A0;
            }
            for (unsigned i = 0; i <= NR; ++i) lambda[(i) * kS] = t[(i) * kS];
        }
    }

    for (unsigned i = 0; i <= NR; ++i) {                                      // 1549-1553
        lambda[(i) * kS] = I[lambda[(i) * kS]];
        if (lambda[(i) * kS] != NN) deg_lambda = i;
    }
    if constexpr (MAXR <= 32) {                                               // Chien 1555-1584
        // the Chien registers live in VGPRs: fully unrolled over j, so every index is a constant;
        // terms above deg_lambda are skipped (wave-uniform in practice), as the reference's loop does
        unsigned rg[MAXR + 1];
#pragma unroll
        for (int j = 1; j <= MAXR; ++j) rg[j] = j <= (int)deg_lambda ? lambda[(j) * kS] : A0;
        count = 0;
        for (unsigned i = 1; i <= NN; ++i) {
            // blocks of 4 terms, branch-free inside (independent table loads can be in flight
            // together): a zero coefficient stays A0 and adds alpha_to[A0] = 0; j <= deg < NN,
            // so one conditional subtract reduces rg + j
            unsigned q = 1;
#pragma unroll
            for (int j0 = 1; j0 <= MAXR; j0 += 4) {
                if (j0 > (int)deg_lambda) break;
#pragma unroll
                for (int j = j0; j < j0 + 4 && j <= MAXR; ++j) {
                    const unsigned x = rg[j] + j, y = x >= NN ? x - NN : x;
                    rg[j] = rg[j] == A0 ? A0 : y;
                    q ^= A[rg[j]];
                }
            }
            if (q != 0) continue;
            root[(count) * kS] = (uint16_t)i;
            if (++count == (int)deg_lambda) break;
        }
    } else {
        W *reg = t;
        for (unsigned i = 0; i <= NR; ++i) reg[(i) * kS] = lambda[(i) * kS];
        count = 0;
        for (unsigned i = 1; i <= NN; ++i) {
            unsigned q = 1;
            for (unsigned j = deg_lambda; j > 0; --j)
                if (reg[(j) * kS] != A0) {
                    reg[(j) * kS] = (uint16_t)modnn(reg[(j) * kS] + j, NN, mm);
                    q ^= A[reg[(j) * kS]];
                }
            if (q != 0) continue;
            root[(count) * kS] = (uint16_t)i;
            if (++count == (int)deg_lambda) break;
        }
    }
    if ((int)deg_lambda != count || (deg_lambda == 0 && !karn)) { count = -1; goto finish; }   // 1577-1595
    if (count == 0) goto finish;              // Karn: deg lambda = 0 decodes to 0 (decode_rs.h:232-240)

    nroot = (unsigned)count;
    if constexpr (MAXR > 32)
        for (unsigned j = 0; j < nroot; ++j) wrote[(j) * kS] = 0;
    deg_omega = deg_lambda - 1;                                               // 1596-1604
    for (unsigned i = 0; i <= deg_omega; ++i) {
        unsigned tmp = 0;
        for (unsigned j = i + 1; j-- > 0;)
            if (syn[(i - j) * kS] != A0 && lambda[(j) * kS] != A0) tmp ^= A[modnn(syn[(i - j) * kS] + lambda[(j) * kS], NN, mm)];
        omega[(i) * kS] = I[tmp];
    }

    for (unsigned j = (unsigned)count; j-- > 0;) {                           // Forney 1610-1690
        const unsigned rj = root[(j) * kS];
        unsigned num1 = 0;
        for (unsigned i = deg_omega + 1; i-- > 0;)
            if (omega[(i) * kS] != A0) num1 ^= A[modnn(omega[(i) * kS] + i * rj, NN, mm)];
        const unsigned num2 = A[modnn(rj * (FCR - 1) + NN, NN, mm)];
        unsigned den = 0;
        const unsigned top = deg_lambda < NR - 1 ? deg_lambda : NR - 1;
        for (int i = (int)(top & ~1u); i >= 0; i -= 2)
            if (lambda[(i + 1) * kS] != A0) den ^= A[modnn(lambda[(i + 1) * kS] + (unsigned)i * rj, NN, mm)];
        // Karn applies den == 0 (its log is A0 = NN: the correction is num1 * num2) and skips a
        // root in the pad (decode_rs.h:277-289); ezpwd fails both (1625-1648)
        if (den == 0 && !karn) { count = -1; goto finish; }
        if (karn && locof(j) < pad) {                 // skipped, as libfec does: no correction, and
            if (corr_out) corr_out[j] = static_cast<T>(0);   // corr 0 whatever the error value
            continue;                                 // (include/ezrs.h)
        }
        if (num1 != 0) {
            if (locof(j) < pad) {
                count = -1;
                goto finish;
            }
            const unsigned cor = A[modnn(I[num1] + I[num2] + NN - I[den], NN, mm)];
            unsigned cv = cor;
            unsigned at, delta = cor;
            if (locof(j) < NN - NR) {
                at = locof(j) - pad;
                if (c.dual) {
                    const unsigned err_dua = static_cast<unsigned>(data[at]) & NN;
                    delta = ID[FD[err_dua] ^ cor] ^ err_dua;
                    cv = delta;
                }
            } else {
                const unsigned pi = locof(j) - (NN - NR);
                at = len + pi;
                if (c.dual) {
                    const unsigned err_dua = static_cast<unsigned>(parity[pi]);
                    const unsigned err_cnv = FD[err_dua];
                    delta = ID[err_cnv ^ cor] ^ err_dua;
                    cv = cor;                                 // fix_cnv ^ err_cnv (1684)
                }
            }
            (void)at;
            corrv[(j) * kS] = (uint16_t)cv;
            fixv[(j) * kS] = (uint16_t)delta;
            set_wrote(j);
        }
    }

finish:
    if (!masked || count > 0)     // roots are distinct, so the fixes commute
        for (unsigned j = 0; j < nroot; ++j) {
            if (!has_wrote(j)) continue;
            const unsigned l = locof(j);
            if (l < NN - NR) data[l - pad] = static_cast<T>(data[l - pad] ^ fixv[(j) * kS]);
            else parity[l - (NN - NR)] = static_cast<T>(parity[l - (NN - NR)] ^ fixv[(j) * kS]);
        }
    if (corr_out)  // corr is passed straight through by decode<INP> in both paths (1222, 1240)
        for (unsigned j = 0; j < nroot; ++j)
            if (has_wrote(j)) corr_out[j] = static_cast<T>(corrv[(j) * kS]);
    if (pos_out && count > 0)
        for (int i = 0; i < count; ++i) pos_out[i] = locof(i) - (karn ? 0u : pad);
    return count;
}

// Wide symbols, NR <= 32: a 32-lane group per codeword evaluates the syndromes (lane i: S_i by
// Horner over data then parity, rs_base:1390-1414, one symbol per step broadcast across the
// group); lane 0 then runs the reference decode on them with its working arrays in LDS.
template <typename T, bool LDS>
__global__ void __launch_bounds__(kBlock) k_decode_lanes(DevCodec c, DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    constexpr int kGroups = kBlock / kLaneGroup;
    __shared__ uint16_t sy[kGroups * kLaneGroup];
    __shared__ uint16_t work[kGroups * kWorkArrays<32> * 33];
    const uint16_t *A, *I;
    const uint8_t *ID, *FD;
    stage_tables<LDS>(c, smem, A, I, ID, FD);
    const unsigned j = threadIdx.x & (kLaneGroup - 1), grp = threadIdx.x / kLaneGroup;
    const size_t k = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / kLaneGroup;
    const bool valid = k < a.ncw;                       // uniform over the group
    const unsigned NR = c.nroots, NN = c.nn;
    unsigned len = a.len;
    T *data = nullptr, *parity = nullptr;
    if (valid) {
        row_ptrs<T>(a, k, data, parity, len);
        const unsigned root = (unsigned)(((uint64_t)(c.fcr + j) * c.prim) % NN);
        const unsigned tot = len + NR;
        unsigned sv = 0;
        for (unsigned i0 = 0; i0 < tot; i0 += kLaneGroup) {
            unsigned dv = 0;
            const unsigned at = i0 + j;
            if (at < tot) {
                dv = static_cast<unsigned>(at < len ? data[at] : parity[at - len]) & NN;
                if (c.dual) dv = FD[dv];
            }
            const unsigned cnt = tot - i0 < (unsigned)kLaneGroup ? tot - i0 : kLaneGroup;
            for (unsigned t = 0; t < cnt; ++t) {
                const unsigned x = __shfl(dv, (int)t, kLaneGroup);
                const unsigned li = I[sv], e = li + root, y = e >= NN ? e - NN : e;
                sv = sv == 0 ? x : x ^ (unsigned)A[y];
            }
        }
        sy[grp * kLaneGroup + j] = (uint16_t)sv;
    }
    __syncthreads();
    if (!valid || j != 0) return;
    const uint32_t *eras = a.eras ? a.eras + k * a.eras_stride : nullptr;
    const unsigned ne = a.neras ? a.neras[k] : 0;
    uint32_t *pos = a.positions ? a.positions + k * a.pos_stride : nullptr;
    T *corr = a.corr ? static_cast<T *>(a.corr) + k * a.corr_stride : nullptr;
    a.result[k] = decode_one<T, 32, 1, uint16_t, uint16_t>(c, A, I, ID, FD, data, len, parity, eras,
                                                          ne, pos, corr, sy + grp * kLaneGroup,
                                                          work + grp * kWorkArrays<32> * 33);
}

template <typename T>
hipError_t dec_lanes_launch(const DevCodec &c, const DecodeArgs &a, hipStream_t s) {
    const size_t threads = a.ncw * kLaneGroup;
    const unsigned grid = (unsigned)((threads + kBlock - 1) / kBlock);
    if (c.nn <= 4095) {
        const size_t sm = 2 * (c.nn + 1) * sizeof(uint16_t) + 512;
        hipLaunchKernelGGL((k_decode_lanes<T, true>), dim3(grid), dim3(kBlock), sm, s, c, a);
    } else {
        hipLaunchKernelGGL((k_decode_lanes<T, false>), dim3(grid), dim3(kBlock), 0, s, c, a);
    }
    return hipGetLastError();
}

template <typename T, int MAXR, bool LDS>
__global__ void __launch_bounds__(kBlock) k_decode_generic(DevCodec c, DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    const uint16_t *A, *I;
    const uint8_t *ID, *FD;
    stage_tables<LDS>(c, smem, A, I, ID, FD);
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.ncw) return;
    T *data, *parity;
    unsigned len;
    row_ptrs<T>(a, k, data, parity, len);
    const uint32_t *eras = a.eras ? a.eras + k * a.eras_stride : nullptr;
    const unsigned ne = a.neras ? a.neras[k] : 0;
    uint32_t *pos = a.positions ? a.positions + k * a.pos_stride : nullptr;
    T *corr = a.corr ? static_cast<T *>(a.corr) + k * a.corr_stride : nullptr;
    if constexpr (MAXR <= 32) {        // working arrays in LDS, lanes interleaved (kDecBlock lanes)
        __shared__ uint16_t work[kWorkArrays<MAXR> * (MAXR + 1) * kDecBlock];
        a.result[k] = decode_one<T, MAXR, kDecBlock>(c, A, I, ID, FD, data, len, parity, eras, ne,
                                                     pos, corr, static_cast<const uint8_t *>(nullptr), work + threadIdx.x);
    } else {
        a.result[k] = decode_one<T, MAXR>(c, A, I, ID, FD, data, len, parity, eras, ne, pos, corr);
    }
}

template <typename T, int MAXR>
hipError_t enc_launch(const DevCodec &c, const EncodeArgs &a, hipStream_t s) {
    const unsigned grid = (unsigned)((a.ncw + kBlock - 1) / kBlock);
    if (c.nn <= 4095) {
        const size_t sm = 2 * (c.nn + 1) * sizeof(uint16_t) + 512;
        hipLaunchKernelGGL((k_encode_generic<T, MAXR, true>), dim3(grid), dim3(kBlock), sm, s, c, a);
    } else {
        hipLaunchKernelGGL((k_encode_generic<T, MAXR, false>), dim3(grid), dim3(kBlock), 0, s, c, a);
    }
    return hipGetLastError();
}

template <typename T, int MAXR>
hipError_t dec_launch(const DevCodec &c, const DecodeArgs &a, hipStream_t s) {
    const unsigned blk = MAXR <= 32 ? kDecBlock : kBlock;
    const unsigned grid = (unsigned)((a.ncw + blk - 1) / blk);
    if (c.nn <= 4095) {
        const size_t sm = 2 * (c.nn + 1) * sizeof(uint16_t) + 512;
        hipLaunchKernelGGL((k_decode_generic<T, MAXR, true>), dim3(grid), dim3(blk), sm, s, c, a);
    } else {
        hipLaunchKernelGGL((k_decode_generic<T, MAXR, false>), dim3(grid), dim3(blk), 0, s, c, a);
    }
    return hipGetLastError();
}

} // namespace

hipError_t launch_encode_generic(const DevCodec &c, const EncodeArgs &a, hipStream_t s) {
    if (a.ncw == 0) return hipSuccess;
    if (c.mm <= 8) return c.nroots <= 32 ? enc_launch<uint8_t, 32>(c, a, s) : enc_launch<uint8_t, 256>(c, a, s);
    // wide symbols (long codewords): a lane group per codeword
    return c.nroots <= 32 ? enc_lanes_launch<uint16_t>(c, a, s) : enc_launch<uint16_t, 256>(c, a, s);
}

hipError_t launch_decode_generic(const DevCodec &c, const DecodeArgs &a, hipStream_t s) {
    if (a.ncw == 0) return hipSuccess;
    if (c.mm <= 8) return c.nroots <= 32 ? dec_launch<uint8_t, 32>(c, a, s) : dec_launch<uint8_t, 256>(c, a, s);
    // wide symbols (long codewords): syndromes by a lane group per codeword
    return c.nroots <= 32 ? dec_lanes_launch<uint16_t>(c, a, s) : dec_launch<uint16_t, 256>(c, a, s);
}

} // namespace ezrs
