// ezrs_errors.hip -- the error path behind the sliced GF(2^8) syndrome kernels: decodes the
// codewords whose syndromes are not all zero (or that carry erasures), starting from the syndromes
// those kernels left in the workspace.
//
// Same algorithm, same branch structure and same outputs as decode_symbols (c++/ezpwd/rs_base:
// 1335-1718): erasure locator (1436-1450), Berlekamp-Massey with the reference's length rule
// (1507-1546), Chien in the reference's root order (1555-1584), Omega (1596-1604), Forney with
// in-place correction and partial fixes kept on failure (1610-1690), positions (1700-1716).
//
// Organisation for CDNA4 (m = 8, NR <= 32):
//  * A persistent grid of one 16-wave workgroup per CU.  Each wavefront screens spans of 256 result
//    slots (a 16-byte load per lane), compacts the flagged ones into an LDS list with ballots, and
//    decodes them 64 at a time, one codeword per lane: a sparse batch keeps every lane busy, a dense
//    one (C3: every codeword flagged) runs at full width.  A workgroup with nothing flagged leaves
//    after the screen, before building any table.
//  * All working polynomials (lambda, B, log lambda, Chien registers, Omega) live in VGPRs: every
//    loop over coefficients is unrolled, so every index is a constant; coefficient blocks of 8 above
//    the current degree bound are skipped (deg lambda, deg B <= r - 1 at BM step r).  Only the
//    syndromes (read at the run-time offset r - 1 - i) and the Chien roots are per-lane LDS arrays.
//  * GF products through a 256-byte antilog table in LDS with a zero class for log(0): any log >= 510
//    marks zero, and a product's index is min(x, x - 255, 255) with alpha_to[255] = 0, so no
//    compare/select per product.
//  * Chien evaluates eight consecutive positions per table read: CH8[j][x] packs lambda_j-term values
//    alpha^x, alpha^(x+j), .., alpha^(x+7j) into 8 bytes (32 KiB for j = 1..16; j = 17..32 use a
//    4-position dword table and two reads), so each register steps by 8j and a zero byte of the XOR
//    marks a root.  That is 32 steps of deg(lambda) reads instead of 255, the LDS-read rate being
//    what bounds this kernel (r05j, C3 decode: 0.686 vs 0.731 ms with four positions per read).
//    Measured and dropped (r05j): corrections applied by the wave in whole 16-byte pieces of the
//    rows (the records of each row gathered per piece): 1.01 vs 0.73 ms.
//  * Phase costs on C3 (timing ablations EZRS_ERR_STOP; the syndrome kernel is 0.095 ms of the
//    decode call).  r05j, call 0.731 ms: screen, syndromes and erasure locator 0.077, Berlekamp-
//    Massey 0.19, Chien 0.22 (four positions per read), Omega and Forney 0.10, corrections 0.05.
//    r05o, call 0.631 ms (eight positions per read; a codeword's loads issued together; the lambda
//    update masked to lanes with a nonzero discrepancy; Omega's syndromes read once): 0.05, 0.166,
//    0.164, 0.103, 0.052.  The LDS -- table reads, half their cycles bank conflicts -- bounds it.
#include "ezrs_internal.hpp"

namespace ezrs {
namespace {

constexpr int32_t kSentinel = INT32_MIN;
#ifndef EZRS_ERR_STOP
#define EZRS_ERR_STOP 0                 // timing ablations (variant builds only): see decode_lane
#endif

constexpr int kSpan = 256;              // result slots screened per wavefront
constexpr int kWaves = 16;              // wavefronts per workgroup (one workgroup per CU)
constexpr unsigned kZ = 1024;           // log(0); every value >= 510 is in the zero class
constexpr int kSrows = 35;              // reversed syndromes: rows 0..31, zero-class padding 32..34
                                        // (BM reads rows up to 32 - r + (r - 1) + 3)

// antilog index of the product of two logs (either may be in the zero class)
__device__ __forceinline__ unsigned pidx(unsigned x) {
    const unsigned y = x - 255u;
    return min(min(x, y), 255u);
}
// (x + y) mod 255 for x, y in [0, 254]
__device__ __forceinline__ unsigned addmod(unsigned x, unsigned y) {
    const unsigned s = x + y;
    return min(s, s - 255u);
}

struct WaveLds {
    uint16_t srev[kSrows * 64];          // [row][lane]: row k holds S_{31-k} (log), rows >= 32 kZ
    uint8_t root[32 * 64];               // [j][lane]: Chien roots in order
    uint16_t list[kSpan];                // flagged slots of the current span
};
struct Lds {
    uint2 CH8[16 * 256];                 // Chien, j = 1..16: CH8[j-1][x] = alpha^(x + k j), k = 0..7, per byte
    uint32_t CH[16 * 256];               // j = 17..32: CH[j-17][x] = alpha^(x + k j), k = 0..3
    uint8_t A[256];                      // alpha_to, A[255] = 0
    uint16_t I[256];                     // index_of, I[0] = kZ
    WaveLds w[kWaves];
};

// Table reads of the decode; gp: the antilog of a sum of two logs (either may be in the zero class).
// Measured and dropped (C3 decode 0.767 ms): 8-byte antilog reads banked mod 64 (60+ VGPRs of
// spills; again in r05 for every product, conflict-free but 45 VGPRs of spills: 0.722 vs 0.630
// ms), a per-bank replicated antilog table (3 more VALU per read: 0.871 ms), an antilog table
// extended over every sum instead of pidx (fewer VALU, more bank conflicts: 0.777 ms), and B
// updates skipped in wave-uniform branches (170+ VGPRs of spills).
__device__ __forceinline__ unsigned ga(const Lds &L, unsigned x) { return L.A[x]; }
__device__ __forceinline__ unsigned gi(const Lds &L, unsigned x) { return L.I[x]; }
__device__ __forceinline__ unsigned gp(const Lds &L, unsigned x) { return L.A[pidx(x)]; }

__device__ __attribute__((always_inline)) int decode_lane(const DevCodec &c, const Lds &L, WaveLds &W,
                                                          const unsigned lane, uint8_t *data, unsigned len,
                                                          uint8_t *parity, const uint32_t *eras,
                                                          unsigned no_eras, unsigned eras_cap, uint32_t *pos_out,
                                                          uint8_t *corr_out, const uint8_t *syn_in,
                                                          unsigned syn_step, bool synz) {
    const unsigned NR = c.nroots, LOAD = c.load, FCR = c.fcr, PRM = c.prim;
    // Karn mode (c.karn): erasures and positions in the full 255 frame (decode_rs.h:114, 295) and
    // none of ezpwd's extra failure checks
    const bool karn = c.karn != 0;
    const unsigned elim = karn ? 255u : len + NR;
    // The codeword's global loads go out together, one memory round trip: its syndromes (also for
    // a slot flagged for erasures only, whose syndromes were not written: then ignored) and its
    // first four erasure positions, before the erasure count (itself still in flight) is looked at.
    // (Issued one at a time behind the checks, r05: C3 decode 0.686 ms; together 0.655.)
    unsigned sv[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) sv[i] = syn_in && i < (int)NR ? syn_in[i * syn_step] : 0u;
    const bool eras_vec = eras != nullptr && (reinterpret_cast<uintptr_t>(eras) & 15) == 0 && eras_cap >= 4;
    uint4 v[8];
    if (eras_vec) __builtin_memcpy(&v[0], eras, 16);
    if (len == 0 || len > LOAD) return -1;                                    // 1375-1377
    if (no_eras > NR) return -1;                                              // 1380-1382
    // erasure positions (1383-1387): loaded four at a time where the row allows (all loads issued
    // before the first use) and kept as bytes in this lane's Chien root column, free until the
    // search, for the erasure locator
    bool eras_bad = false;                    // Karn mode: an erasure outside the frame, reported after
    if (no_eras > 0) {                        // the zero-syndrome return as libfec does
        unsigned bad = 0;
        uint8_t *ep = W.root + lane;
        if (eras_vec && ((no_eras + 3) & ~3u) <= eras_cap) {
#pragma unroll
            for (int c = 1; c < 8; ++c)
                if (4u * c < no_eras) __builtin_memcpy(&v[c], eras + 4 * c, 16);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (4u * c < no_eras) {
                    const unsigned x[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (4u * c + q < no_eras) {
                            bad |= x[q] >= elim;
                            ep[(4 * c + q) * 64] = (uint8_t)x[q];
                        }
                    }
                }
            }
        } else {
            for (unsigned i = 0; i < no_eras; ++i) {
                const unsigned x = eras[i];
                bad |= x >= elim;
                ep[i * 64] = (uint8_t)x;
            }
        }
        if (bad && !karn) return -1;
        if (bad) eras_bad = true;
    }
    const unsigned pad = LOAD - len;
    const unsigned epad = karn ? 0u : pad;    // frame offset of an erasure position
    auto S = [&](int k) -> uint16_t & { return W.srev[k * 64 + lane]; };

    // syndromes (polynomial form from the syndrome kernel; syndrome i at syn_in[i * syn_step]) ->
    // logs, stored reversed (1416-1434)
    unsigned syn_error = 0;
    {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const unsigned x = synz ? 0u : sv[i];
            syn_error |= x;
            S(31 - i) = gi(L, x);
        }
#pragma unroll
        for (int k = 32; k < kSrows; ++k) S(k) = kZ;
    }
    if (!syn_error) return 0;
    if (eras_bad) return -1;                  // (Karn mode only: undefined in libfec, -1 here)

    // erasure locator (1436-1450): lambda in polynomial form, lam[0] == 1
    unsigned lam[33];
#pragma unroll
    for (int i = 0; i <= 32; ++i) lam[i] = i == 0;
    if (no_eras > 0) {
        lam[1] = ga(L, (PRM * (c.nn - 1 - (W.root[lane] + epad))) % 255u);
        for (unsigned e = 1; e < no_eras; ++e) {
            const unsigned u = (PRM * (c.nn - 1 - (W.root[e * 64 + lane] + epad))) % 255u;
            // lam[j] ^= lam[j-1] * alpha^u for j = e+1 .. 1 (lam[j-1] == 0 for j - 1 > e)
#pragma unroll
            for (int j0 = 32; j0 >= 0; j0 -= 4) {
                if ((unsigned)(j0 > 0 ? j0 - 1 : 0) <= e) {
#pragma unroll
                    for (int j = j0 + 3; j >= j0; --j) {
                        if (j < 1 || j > 32) continue;
                        lam[j] ^= gp(L, (u + gi(L, lam[j - 1])));
                    }
                }
            }
        }
    }
    unsigned b[33], l[33];
#pragma unroll
    for (int i = 0; i <= 32; ++i) b[i] = i == 0 ? 0u : gi(L, lam[i]);
#if EZRS_ERR_STOP == 4                  // timing ablation: syndromes and erasure locator only
    { unsigned x = 0; for (int i = 0; i <= 32; ++i) x ^= lam[i]; return (int)(x & 1); }
#endif

    // Berlekamp-Massey (1507-1546).  Before step r, deg lambda <= el and deg B <= r - 1 - el +
    // no_eras (the reference's length rule keeps both; checked exhaustively against a model), so
    // the discrepancy needs coefficients i <= min(r - 1, el) and the update i <= max(el, r - el +
    // no_eras): coefficient blocks of 4 above those per-lane bounds hold zeros and are skipped
    // (whole blocks when every lane of the wave is past them).  l[i] = log lambda_i stays the zero
    // class above el.
#pragma unroll
    for (int i = 0; i <= 32; ++i) l[i] = i == 0 ? 0u : kZ;
    unsigned el = no_eras;
    // l[1 .. lhi] hold log lambda for this lane (reset when its lambda changes): an iteration with a
    // zero discrepancy leaves lambda alone, and the next one reuses the logs
    unsigned lhi = 0;
    for (unsigned r = no_eras + 1; r <= NR; ++r) {
        const int sb = 32 - (int)r;           // row of S_{r-1}; S_{r-1-i} at row sb + i
        const unsigned dmax = min(r - 1, el), umax = max(el, r + no_eras - el);
        unsigned discr = 0;
#pragma unroll
        for (int i0 = 0; i0 <= 32; i0 += 4) {
            if ((unsigned)i0 <= dmax) {
                if ((unsigned)i0 + 3u > lhi) {
#pragma unroll
                    for (int i = i0; i < i0 + 4 && i <= 32; ++i) l[i] = i == 0 ? 0u : gi(L, lam[i]);
                }
#pragma unroll
                for (int i = i0; i < i0 + 4 && i < 32; ++i) discr ^= gp(L, (l[i] + S(sb + i)));
            }
        }
        lhi = max(lhi, (dmax & ~3u) + 3u);
        const unsigned dl = gi(L, discr);
        const bool upd = dl < 510u && 2 * el <= r + no_eras - 1;
        const unsigned ndl = 255u - dl;
        // lambda += Delta x B only in the lanes whose discrepancy is nonzero: the others issue no
        // table reads (a zero discrepancy is the rule past step 2 nu + ne of a decodable word)
        if (dl < 510u) {
#pragma unroll
            for (int i0 = 32; i0 >= 0; i0 -= 4) {
                if ((unsigned)i0 <= umax) {
#pragma unroll
                    for (int i = i0 + 3; i >= i0; --i)
                        if (i > 0 && i <= 32) lam[i] ^= gp(L, (dl + b[i - 1]));
                }
            }
        }
#pragma unroll
        for (int i0 = 32; i0 >= 0; i0 -= 4) {
            if ((unsigned)i0 <= umax) {
#pragma unroll
                for (int i = i0 + 3; i >= i0; --i) {
                    if (i > 32) continue;
                    const unsigned bp = i > 0 ? b[i - 1] : kZ;
                    const unsigned d = l[i] + ndl;
                    const unsigned nb = min(min(d, d - 255u), kZ);
                    b[i] = upd ? nb : bp;
                }
            }
        }
        if (dl < 510u) lhi = 0;               // this lane's lambda changed
        el = upd ? r + no_eras - el : el;
    }
#if EZRS_ERR_STOP == 1                  // timing ablation: up to Berlekamp-Massey
    { unsigned x = 0; for (int i = 0; i <= 32; ++i) x ^= lam[i]; return (int)(x & 1); }
#endif

    // lambda to index form, its degree (1549-1553)
    unsigned deg = 0;
#pragma unroll
    for (int i = 0; i <= 32; ++i) {
        l[i] = i == 0 ? 0u : gi(L, lam[i]);
        if (i > 0 && lam[i] != 0) deg = i;
    }

    // Chien search (1555-1584); lambda_j = 0 keeps rg[j] in the zero class (clamped to entry 255)
    int count = 0;
    if (deg > 0) {
        // eight positions i .. i+7 per step: j <= 16 one 8-byte read of CH8[j-1] (rg[j] = 8 * ((log
        // lambda_j + j*i) mod 255)), j > 16 two 4-byte reads of CH[j-17] (rg[j] = 4 * (...))
        unsigned rg[33];
#pragma unroll
        for (int j = 1; j <= 32; ++j)
            rg[j] = l[j] < 255u ? (j <= 16 ? 8u : 4u) * addmod(l[j], (unsigned)j) : 0x80000000u;
        for (unsigned i = 1; i <= 255; i += 8) {
            unsigned q0 = 0x01010101u, q1 = 0x01010101u;
#pragma unroll
            for (int j0 = 1; j0 <= 32; j0 += 4) {
                if ((unsigned)j0 <= deg) {
#pragma unroll
                    for (int j = j0; j < j0 + 4; ++j) {
                        if (j <= 16) {
                            const uint2 v = *reinterpret_cast<const uint2 *>(
                                reinterpret_cast<const uint8_t *>(L.CH8 + (j - 1) * 256) + min(rg[j], 2040u));
                            q0 ^= v.x;
                            q1 ^= v.y;
                            const unsigned a = rg[j] + 64u * j, z = a - 2040u;
                            rg[j] = min(a, z);
                        } else {
                            const uint8_t *t = reinterpret_cast<const uint8_t *>(L.CH + (j - 17) * 256);
                            q0 ^= *reinterpret_cast<const uint32_t *>(t + min(rg[j], 1020u));
                            const unsigned a = rg[j] + 16u * j, z = a - 1020u, r1 = min(a, z);
                            q1 ^= *reinterpret_cast<const uint32_t *>(t + min(r1, 1020u));
                            const unsigned b2 = r1 + 16u * j, z2 = b2 - 1020u;
                            rg[j] = min(b2, z2);
                        }
                    }
                }
            }
            if (i == 249) q1 |= 0xff000000u;                    // position 256 does not exist
            const bool z0 = ((q0 - 0x01010101u) & ~q0 & 0x80808080u) != 0,
                       z1 = ((q1 - 0x01010101u) & ~q1 & 0x80808080u) != 0;
            if (!z0 && !z1) continue;
            bool done = false;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if ((((k < 4 ? q0 : q1) >> (8 * (k & 3))) & 255u) == 0) {
                    W.root[count * 64 + lane] = (uint8_t)(i + k);
                    if (++count == (int)deg) { done = true; break; }
                }
            }
            if (done) break;
        }
    }
    if ((int)deg != count || (deg == 0 && !karn)) count = -1;                // 1577-1595 (Karn: 0)
#if EZRS_ERR_STOP == 2                  // timing ablation: up to the Chien search
    return count;
#endif

    if (count > 0) {
        // Omega = S * lambda mod x^(deg lambda), index form (1596-1604)
        const unsigned deg_omega = deg - 1;
        unsigned om[32], sl[32];               // sl[k] = log S_k, read once
#pragma unroll
        for (int i0 = 0; i0 < 32; i0 += 4) {
            if ((unsigned)i0 <= deg_omega) {
#pragma unroll
                for (int i = i0; i < i0 + 4; ++i) sl[i] = S(31 - i);
            }
        }
#pragma unroll
        for (int i0 = 0; i0 < 32; i0 += 4) {
            if ((unsigned)i0 <= deg_omega) {
#pragma unroll
                for (int i = i0; i < i0 + 4; ++i) {
                    unsigned t = 0;
                    if ((unsigned)i <= deg_omega) {      // (lanes past their degree read nothing)
#pragma unroll
                        for (int j = 0; j <= i; ++j) t ^= gp(L, (sl[i - j] + l[j]));
                    }
                    om[i] = gi(L, t);
                }
            }
        }
        const unsigned top = (deg < NR - 1 ? deg : NR - 1) & ~1u;
        // Forney, roots in reverse order (1610-1690).  The reference applies each correction as it
        // is found and keeps the ones before a failure; here they are recorded (position, value) in
        // the syndrome rows -- dead once Omega is formed -- and applied afterwards with the row
        // bytes loaded eight at a time, so the byte read-modify-writes of a codeword overlap their
        // global-memory latency instead of paying it once per correction (atomic XORs of the
        // dwords instead: 0.99 against 0.78 ms per C3 decode).  The dual basis (CCSDS) needs each
        // received byte to form its correction and keeps the in-order path.
        unsigned nrec = 0;
        for (int j = count - 1; j >= 0; --j) {
            const unsigned rj = W.root[j * 64 + lane];
            unsigned num1 = 0, den = 0, e = 0;     // e = i * rj (mod 255)
#pragma unroll
            for (int i0 = 0; i0 < 32; i0 += 4) {
                if ((unsigned)i0 <= deg_omega) {
#pragma unroll
                    for (int i = i0; i < i0 + 4; ++i) {
                        if ((unsigned)i <= deg_omega) num1 ^= gp(L, (om[i] + e));
                        if ((i & 1) == 0 && (unsigned)i <= top) den ^= gp(L, (l[i + 1] + e));
                        e = addmod(e, rj);
                    }
                }
            }
            // Karn applies den == 0 (log A0 = NN: the correction is num1 * num2) and skips a root
            // in the pad (decode_rs.h:277-289); ezpwd fails both (1625-1648)
            if (den == 0 && !karn) { count = -1; break; }
            const unsigned loc = (rj * c.iprim + 254u) % 255u;
            if (karn && loc < pad) {                  // skipped, as libfec does: no correction, and
                if (corr_out) corr_out[j] = 0;        // corr 0 whatever the error value
                continue;                             // (include/ezrs.h)
            }
            if (num1 != 0) {
                if (loc < pad) {
                    count = -1;
                    break;
                }
                const unsigned n2 = (unsigned)(((int)rj * ((int)FCR - 1)) % 255 + 255) % 255u;
                const unsigned cor = ga(L, (gi(L, num1) + n2 + (den ? 255u - gi(L, den) : 0u)) % 255u);
                if (!c.dual) {
                    S(nrec++) = (uint16_t)(loc << 8 | cor);
                    if (corr_out) corr_out[j] = (uint8_t)cor;
                    continue;
                }
                unsigned cv = cor, delta = cor;
                uint8_t *at;
                if (loc < 255u - NR) {
                    at = data + (loc - pad);
                    if (c.dual) {
                        const unsigned err_dua = *at;
                        delta = c.into_dual[c.from_dual[err_dua] ^ cor] ^ err_dua;
                        cv = delta;
                    }
                } else {
                    at = parity + (loc - (255u - NR));
                    if (c.dual) {
                        const unsigned err_dua = *at;
                        delta = c.into_dual[c.from_dual[err_dua] ^ cor] ^ err_dua;
                    }
                }
                *at = (uint8_t)(*at ^ delta);
                if (corr_out) corr_out[j] = (uint8_t)cv;
            }
        }
#if EZRS_ERR_STOP == 3                  // timing ablation: no corrections applied
        return (int)nrec;
#endif
        for (unsigned g0 = 0; g0 < nrec; g0 += 8) {
            uint8_t *at[8];
            unsigned v[8], dlt[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (g0 + t < nrec) {
                    const unsigned rec = S(g0 + t), loc = rec >> 8;
                    dlt[t] = rec & 255u;
                    at[t] = loc < 255u - NR ? data + (loc - pad) : parity + (loc - (255u - NR));
                    v[t] = *at[t];
                }
            }
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (g0 + t < nrec) *at[t] = (uint8_t)(v[t] ^ dlt[t]);
        }
    }
    if (pos_out && count > 0)
        for (int i = 0; i < count; ++i)
            pos_out[i] = (W.root[i * 64 + lane] * c.iprim + 254u) % 255u - (karn ? 0u : pad);
    return count;
}

// Screen span `sp`: the flagged slots' offsets into `list` (when given), their number returned.
// A slot is flagged when the syndrome kernel left the sentinel in it (nonzero syndromes) or when
// the codeword carries erasures (the reference validates them before the zero-syndrome return,
// rs_base:1375-1387; a slot holding 0 then means all-zero syndromes).
__device__ __forceinline__ unsigned screen(const DecodeArgs &a, size_t sp, unsigned lane, uint16_t *list) {
    const size_t k0 = sp * kSpan + 4 * lane;
    unsigned mine = 0;
    if (k0 + 4 <= a.ncw && (reinterpret_cast<uintptr_t>(a.result + k0) & 15) == 0) {
        int4 r;
        __builtin_memcpy(&r, a.result + k0, 16);
        mine = (r.x == kSentinel) | (r.y == kSentinel) << 1 | (r.z == kSentinel) << 2 |
               (r.w == kSentinel) << 3;
    } else {
        for (int i = 0; i < 4; ++i)
            if (k0 + i < a.ncw && a.result[k0 + i] == kSentinel) mine |= 1u << i;
    }
    if (a.neras) {
        if (k0 + 4 <= a.ncw && (reinterpret_cast<uintptr_t>(a.neras + k0) & 15) == 0) {
            uint4 e;
            __builtin_memcpy(&e, a.neras + k0, 16);
            mine |= (e.x != 0) | (e.y != 0) << 1 | (e.z != 0) << 2 | (e.w != 0) << 3;
        } else {
            for (int i = 0; i < 4; ++i)
                if (k0 + i < a.ncw && a.neras[k0 + i]) mine |= 1u << i;
        }
    }
    // entry (lane, bit) goes to base_bit + (lanes below with that bit)
    unsigned nflag = 0;
#pragma unroll
    for (int bit = 0; bit < 4; ++bit) {
        const uint64_t m = __ballot((mine >> bit) & 1);
        if (list && ((mine >> bit) & 1)) {
            const unsigned below = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            list[nflag + below] = (uint16_t)(4 * lane + bit);
        }
        nflag += (unsigned)__popcll(m);
    }
    return nflag;
}

__global__ void __launch_bounds__(64 * kWaves) k_decode_errors(DevCodec c, DecodeArgs a, const uint8_t *syn_ws,
                                                              SynLayout layout) {
    __shared__ __attribute__((aligned(16))) Lds L;
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // nothing flagged by this call's syndrome kernel and no erasures: no screen (C2 decode)
    if (a.flag_word && !a.neras && *reinterpret_cast<volatile const uint32_t *>(a.flag_word) != a.flag_gen) return;
    const size_t nspan = (a.ncw + kSpan - 1) / kSpan, step = (size_t)gridDim.x * kWaves;
    unsigned any = 0;
    for (size_t sp = (size_t)blockIdx.x * kWaves + wave; sp < nspan; sp += step)
        any |= screen(a, sp, lane, nullptr);
    if (!__syncthreads_or(any != 0)) return;      // the common case: nothing flagged here

    for (unsigned i = threadIdx.x; i < 256; i += 64 * kWaves) {
        L.A[i] = (uint8_t)c.alpha_to[i];          // alpha_to[255] = 0 (A0)
        L.I[i] = i == 0 ? (uint16_t)kZ : c.index_of[i];
    }
    __syncthreads();
    for (unsigned t = threadIdx.x; t < 16 * 256; t += 64 * kWaves) {
        const unsigned j = t / 256 + 1, x = t % 256;
        uint32_t v0 = 0, v1 = 0;
        if (x < 255)
            for (unsigned k = 0; k < 4; ++k) {
                v0 |= (uint32_t)L.A[(x + k * j) % 255u] << (8 * k);
                v1 |= (uint32_t)L.A[(x + (k + 4) * j) % 255u] << (8 * k);
            }
        L.CH8[t] = make_uint2(v0, v1);
    }
    for (unsigned t = threadIdx.x; t < 16 * 256; t += 64 * kWaves) {
        const unsigned j = t / 256 + 17, x = t % 256;
        uint32_t v = 0;
        if (x < 255)
            for (unsigned k = 0; k < 4; ++k) v |= (uint32_t)L.A[(x + k * j) % 255u] << (8 * k);
        L.CH[t] = v;
    }
    __syncthreads();

    WaveLds &W = L.w[wave];
    for (size_t sp = (size_t)blockIdx.x * kWaves + wave; sp < nspan; sp += step) {
        const unsigned n = screen(a, sp, lane, W.list);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // list entries of other lanes
        for (unsigned c0 = 0; c0 < n; c0 += 64) {
            if (c0 + lane < n) {
                const size_t k = sp * kSpan + W.list[c0 + lane];
                uint8_t *data, *parity;
                unsigned len;
                row_ptrs<uint8_t>(a, k, data, parity, len);
                const uint32_t *eras = a.eras ? a.eras + k * a.eras_stride : nullptr;
                const unsigned ne = a.neras ? a.neras[k] : 0;
                uint32_t *pos = a.positions ? a.positions + k * a.pos_stride : nullptr;
                uint8_t *corr = a.corr ? static_cast<uint8_t *>(a.corr) + k * a.corr_stride : nullptr;
                // a slot that does not hold the sentinel was flagged for its erasures only: its
                // syndromes are zero and were not written
                const bool synz = a.result[k] != kSentinel;
                const bool tiled = layout == SynLayout::Tiled;
                const uint8_t *syn = tiled ? syn_ws + k / 256 * kSynTile + k % 256 : syn_ws + k * 32;
                const unsigned cap = !eras ? 0u : a.eras_stride < 32 ? (unsigned)a.eras_stride : 32u;
                a.result[k] = decode_lane(c, L, W, lane, data, len, parity, eras, ne, cap, pos, corr,
                                          syn_ws ? syn : nullptr, tiled ? 256u : 1u, synz);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // list reads done before the next span
    }
}

} // namespace

hipError_t launch_decode_flagged(const DevCodec &c, const DecodeArgs &a, const uint8_t *syn_ws,
                                 SynLayout layout, hipStream_t s) {
    if (a.ncw == 0) return hipSuccess;
    if (c.mm != 8 || c.nroots > 32 || c.masked) return hipErrorInvalidValue;
    const size_t nspan = (a.ncw + kSpan - 1) / kSpan;
    const size_t want = (nspan + kWaves - 1) / kWaves;
    const size_t ncu = c.ncu > 0 ? (size_t)c.ncu : 256;    // attribute query failed: assume 256
    const unsigned grid = (unsigned)(want < ncu ? want : ncu);
    hipLaunchKernelGGL(k_decode_errors, dim3(grid), dim3(64 * kWaves), 0, s, c, a, syn_ws, layout);
    return hipGetLastError();
}

} // namespace ezrs
