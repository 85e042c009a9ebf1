/*
 * ezrs_oracle.c -- CPU restatement of the ezpwd Reed-Solomon codec (TEST INFRASTRUCTURE ONLY).
 *
 * Checker, never product: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load this library.  See ezrs_oracle.h for the parity status (pinned against oracle/_ref and
 * tests/golden/).
 *
 * Every function below restates one piece of c++/ezpwd/rs_base (reference VERSION 2.2.0) with
 * runtime codec parameters instead of template parameters.  The arithmetic is kept literally
 * identical (same branch structure, same order of in-place corrections) because the decoder's
 * behaviour in the overwhelmed regime (return -1, partial corrections) depends on it.
 */
#include "ezrs_oracle.h"

#include <stdlib.h>
#include <string.h>

struct ezo_codec {
    unsigned mm;        /* bits per symbol                          (rs_base:570) */
    unsigned nn;        /* symbols per block, 2^mm - 1 == A0        (rs_base:571-573) */
    unsigned poly;      /* field generator polynomial               (rs_base:537-557) */
    unsigned fcr;       /* first consecutive root, index form       (rs_base:683) */
    unsigned prim;      /* primitive element, index form            (rs_base:684) */
    unsigned iprim;     /* prim-th root of 1, index form            (rs_base:630-634) */
    unsigned nroots;    /* parity symbols                           (rs_base:723) */
    int dual;           /* Berlekamp dual basis (mm == 8 only)      (rs_base:696-700) */
    unsigned datum;     /* bytes per datum: 1 (uint8_t) or 2 (uint16_t) (rs:75-89) */
    uint16_t *alpha_to; /* nn+1 entries; alpha_to[nn] = 0           (rs_base:613-621) */
    uint16_t *index_of; /* nn+1 entries; index_of[0] = nn (A0)      (rs_base:613-621) */
    uint16_t *genpoly;  /* nroots+1 entries, index form             (rs_base:1263-1285) */
    int karn;           /* decode with libfec's semantics (ezo_set_karn)               */
};

/* ------------------------------------------------------------------------------------------ */
/* Berlekamp dual basis.  rs_base:109-146 lists the two 256-entry maps; both are GF(2)-linear, so
 * they are generated here from the images of the eight basis bytes (the columns of the CCSDS
 * 131.0-B Annex F transform) and the inverse is found by inverting the map.  tests/ check the
 * generated maps entry-for-entry against the reference's own tables via oracle/_ref. */
static uint8_t g_into_dual[256], g_from_dual[256];
static int g_dual_ready;
static void dual_init(void) {
    static const uint8_t col[8] = {0x7b, 0xaf, 0x99, 0xfa, 0x86, 0xec, 0xef, 0x8d};
    if (g_dual_ready) return;
    for (unsigned x = 0; x < 256; ++x) {
        uint8_t y = 0;
        for (unsigned b = 0; b < 8; ++b)
            if (x >> b & 1) y ^= col[b];
        g_into_dual[x] = y;
    }
    for (unsigned x = 0; x < 256; ++x) g_from_dual[g_into_dual[x]] = (uint8_t)x;
    g_dual_ready = 1;
}
const uint8_t *ezo_into_dual(void) { dual_init(); return g_into_dual; }
const uint8_t *ezo_from_dual(void) { dual_init(); return g_from_dual; }

/* modnn (rs_base:648-669): the fold-and-table reduction always lands on x mod NN. */
static inline unsigned modnn(const ezo_codec *c, unsigned x) { return x % c->nn; }

/* ------------------------------------------------------------------------------------------ */
ezo_codec *ezo_create(unsigned mm, unsigned poly, unsigned fcr, unsigned prim, unsigned nroots,
                      int dual) {
    if (mm < 2 || mm > 16 || prim == 0) return NULL;
    unsigned nn = (1u << mm) - 1;
    if (nroots == 0 || nroots >= nn) return NULL;          /* rs_base:1254-1256 */
    if (dual && mm != 8) return NULL;                       /* rs_base:1188-1190 */
    ezo_codec *c = (ezo_codec *)calloc(1, sizeof *c);
    c->mm = mm; c->nn = nn; c->poly = poly; c->fcr = fcr; c->prim = prim;
    c->nroots = nroots; c->dual = dual; c->datum = mm <= 8 ? 1 : 2;
    c->alpha_to = (uint16_t *)calloc(nn + 1, sizeof(uint16_t));
    c->index_of = (uint16_t *)calloc(nn + 1, sizeof(uint16_t));
    c->genpoly = (uint16_t *)calloc(nroots + 1, sizeof(uint16_t));

    /* Field tables: successive powers of alpha via the gfpoly shift register (rs_base:537-557,
     * 612-621). */
    c->index_of[0] = (uint16_t)nn;
    c->alpha_to[nn] = 0;
    unsigned sr = 1;
    for (unsigned i = 0; i < nn; ++i) {
        c->index_of[sr] = (uint16_t)i;
        c->alpha_to[i] = (uint16_t)sr;
        sr <<= 1;
        if (sr & (1u << mm)) sr ^= poly;
        sr &= nn;
    }
    if (sr != c->alpha_to[0]) { ezo_destroy(c); return NULL; }   /* rs_base:623-625 */

    unsigned iptmp = 1;                                          /* rs_base:631-634 */
    while (iptmp % prim != 0) iptmp += nn;
    c->iprim = iptmp / prim;

    /* Generator polynomial from its roots alpha^((fcr+i)*prim) (rs_base:1263-1285). */
    uint16_t *tp = (uint16_t *)calloc(nroots + 1, sizeof(uint16_t));
    tp[0] = 1;
    for (unsigned i = 0, root = fcr * prim; i < nroots; i++, root += prim) {
        tp[i + 1] = 1;
        for (unsigned j = i; j > 0; j--) {
            if (tp[j] != 0)
                tp[j] = tp[j - 1] ^ c->alpha_to[modnn(c, c->index_of[tp[j]] + root)];
            else
                tp[j] = tp[j - 1];
        }
        tp[0] = c->alpha_to[modnn(c, c->index_of[tp[0]] + root)];
    }
    for (unsigned i = 0; i <= nroots; ++i) c->genpoly[i] = c->index_of[tp[i]];
    free(tp);
    if (dual) dual_init();
    return c;
}

void ezo_destroy(ezo_codec *c) {
    if (!c) return;
    free(c->alpha_to); free(c->index_of); free(c->genpoly); free(c);
}

unsigned ezo_size(const ezo_codec *c) { return c->nn; }
unsigned ezo_nroots(const ezo_codec *c) { return c->nroots; }
unsigned ezo_load(const ezo_codec *c) { return c->nn - c->nroots; }
unsigned ezo_datum_bytes(const ezo_codec *c) { return c->datum; }
unsigned ezo_iprim(const ezo_codec *c) { return c->iprim; }
void ezo_tables(const ezo_codec *c, uint16_t *a, uint16_t *i, uint16_t *g) {
    if (a) memcpy(a, c->alpha_to, (c->nn + 1) * sizeof(uint16_t));
    if (i) memcpy(i, c->index_of, (c->nn + 1) * sizeof(uint16_t));
    if (g) memcpy(g, c->genpoly, (c->nroots + 1) * sizeof(uint16_t));
}

/* ------------------------------------------------------------------------------------------ */
/* encode_symbols (rs_base:1296-1332): systematic LFSR division by g(x). */
static int encode_symbols(const ezo_codec *c, const uint16_t *data, unsigned len,
                          uint16_t *parity) {
    const unsigned NR = c->nroots, A0 = c->nn;
    if (len == 0 || len > c->nn - NR) return -1;
    for (unsigned i = 0; i < NR; i++) parity[i] = 0;
    for (unsigned i = 0; i < len; i++) {
        unsigned sym = c->dual ? g_from_dual[data[i]] : data[i];
        unsigned fb = c->index_of[sym ^ parity[0]];
        if (fb != A0)
            for (unsigned j = 1; j < NR; j++)
                parity[j] ^= c->alpha_to[modnn(c, fb + c->genpoly[NR - j])];
        memmove(parity, parity + 1, (NR - 1) * sizeof(uint16_t));   /* std::rotate left by 1 */
        parity[NR - 1] = fb != A0 ? c->alpha_to[modnn(c, fb + c->genpoly[0])] : 0;
    }
    if (c->dual)
        for (unsigned i = 0; i < NR; ++i) parity[i] = g_into_dual[parity[i]];
    return (int)NR;
}

/* decode_symbols (rs_base:1335-1718): syndromes -> erasure locator -> Berlekamp-Massey ->
 * Chien -> Omega -> Forney, with ezpwd's extra failure checks and in-place corrections. */
static int decode_symbols(const ezo_codec *c, uint16_t *data, unsigned len, uint16_t *parity,
                          unsigned *eras_pos, unsigned no_eras, uint16_t *corr) {
    const unsigned NR = c->nroots, NN = c->nn, A0 = c->nn, LOAD = c->nn - c->nroots;
    const unsigned FCR = c->fcr, PRM = c->prim;
    const uint16_t *alpha_to = c->alpha_to, *index_of = c->index_of;
    const int DUAL = c->dual;
    /* Karn mode (fec-3.0.1/decode_rs.h:71-298): erasures and positions in the full NN frame
     * (decode_rs.h:114, 295); none of ezpwd's checks of deg lambda = 0, den = 0 and roots in the
     * pad (decode_rs.h:232-289) */
    const int KARN = c->karn;
    if (len == 0 || len > LOAD) return -1;                               /* 1375-1377 */
    unsigned pad = LOAD - len, epad = KARN ? 0 : pad;
    if (no_eras) {                                                       /* 1379-1388 */
        if (no_eras > NR) return -1;
        for (unsigned i = 0; i < no_eras; ++i)
            if (eras_pos[i] >= (KARN ? NN : len + NR)) return -1;
    }

    /* scratch: lambda, b, t, omega, reg (NR+1 each), syn (NR), root, loc (NR unsigned) */
    uint16_t sbuf[6 * 257];
    unsigned ubuf[2 * 256];
    uint16_t *s16 = NR <= 256 ? sbuf : (uint16_t *)malloc(6 * (NR + 1) * sizeof(uint16_t));
    unsigned *u32 = NR <= 256 ? ubuf : (unsigned *)malloc(2 * NR * sizeof(unsigned));
    uint16_t *lambda = s16, *b = s16 + (NR + 1), *t = s16 + 2 * (NR + 1);
    uint16_t *omega = s16 + 3 * (NR + 1), *reg = s16 + 4 * (NR + 1), *syn = s16 + 5 * (NR + 1);
    unsigned *root = u32, *loc = u32 + NR;
    memset(lambda, 0, (NR + 1) * sizeof(uint16_t));
    memset(root, 0, NR * sizeof(unsigned));
    memset(loc, 0, NR * sizeof(unsigned));
    int count = 0;

#define CNV(x) (DUAL ? g_from_dual[(x)] : (x))
    /* syndromes by Horner over data then parity (1390-1414) */
    for (unsigned i = 0; i < NR; i++) syn[i] = CNV(data[0]);
    for (unsigned j = 1; j < len; j++)
        for (unsigned i = 0; i < NR; i++)
            syn[i] = syn[i] == 0 ? CNV(data[j])
                                 : CNV(data[j]) ^ alpha_to[modnn(c, index_of[syn[i]] + (FCR + i) * PRM)];
    for (unsigned j = 0; j < NR; j++)
        for (unsigned i = 0; i < NR; i++)
            syn[i] = syn[i] == 0 ? CNV(parity[j])
                                 : CNV(parity[j]) ^ alpha_to[modnn(c, index_of[syn[i]] + (FCR + i) * PRM)];

    unsigned syn_error = 0;                                              /* 1416-1421 */
    for (unsigned i = 0; i < NR; i++) { syn_error |= syn[i]; syn[i] = index_of[syn[i]]; }

    unsigned deg_lambda = 0, deg_omega = 0, r = no_eras, el = no_eras;
    if (!syn_error) { count = 0; goto finish; }                          /* 1427-1434 */

    lambda[0] = 1;                                                       /* 1436-1450 */
    if (no_eras > 0) {
        lambda[1] = alpha_to[modnn(c, PRM * (NN - 1 - (eras_pos[0] + epad)))];
        for (unsigned i = 1; i < no_eras; i++) {
            uint16_t u = (uint16_t)modnn(c, PRM * (NN - 1 - (eras_pos[i] + epad)));
            for (unsigned j = i + 1; j > 0; j--) {
                uint16_t tmp = index_of[lambda[j - 1]];
                if (tmp != A0) lambda[j] ^= alpha_to[modnn(c, u + tmp)];
            }
        }
    }
    for (unsigned i = 0; i < NR + 1; i++) b[i] = index_of[lambda[i]];    /* 1501-1502 */

    while (++r <= NR) {                                                  /* BM, 1507-1546 */
        unsigned discr_r = 0;
        for (unsigned i = 0; i < r; i++)
            if (lambda[i] != 0 && syn[r - i - 1] != A0)
                discr_r ^= alpha_to[modnn(c, index_of[lambda[i]] + syn[r - i - 1])];
        discr_r = index_of[discr_r];
        if (discr_r == A0) {
            memmove(b + 1, b, NR * sizeof(uint16_t));                    /* B(x) <- x*B(x) */
            b[0] = (uint16_t)A0;
        } else {
            t[0] = lambda[0];
            for (unsigned i = 0; i < NR; i++)
                t[i + 1] = b[i] != A0 ? lambda[i + 1] ^ alpha_to[modnn(c, discr_r + b[i])]
                                      : lambda[i + 1];
            if (2 * el <= r + no_eras - 1) {
                el = r + no_eras - el;
                for (unsigned i = 0; i <= NR; i++)
                    b[i] = lambda[i] == 0 ? (uint16_t)A0
                                          : (uint16_t)modnn(c, index_of[lambda[i]] - discr_r + NN);
            } else {
                memmove(b + 1, b, NR * sizeof(uint16_t));
                b[0] = (uint16_t)A0;
            }
            memcpy(lambda, t, (NR + 1) * sizeof(uint16_t));
        }
    }

    for (unsigned i = 0; i < NR + 1; i++) {                              /* 1549-1553 */
        lambda[i] = index_of[lambda[i]];
        if (lambda[i] != NN) deg_lambda = i;
    }
    memcpy(reg, lambda, (NR + 1) * sizeof(uint16_t));                    /* Chien, 1555-1584 */
    count = 0;
    for (unsigned i = 1, k = c->iprim - 1; i <= NN; i++, k = modnn(c, k + c->iprim)) {
        unsigned q = 1;
        for (unsigned j = deg_lambda; j > 0; j--)
            if (reg[j] != A0) {
                reg[j] = (uint16_t)modnn(c, reg[j] + j);
                q ^= alpha_to[reg[j]];
            }
        if (q != 0) continue;
        root[count] = i;
        loc[count] = k;
        if (++count == (int)deg_lambda) break;
    }
    if ((int)deg_lambda != count) { count = -1; goto finish; }
    if (deg_lambda == 0) { count = KARN ? 0 : -1; goto finish; }         /* 1589-1595 */

    deg_omega = deg_lambda - 1;                                          /* 1596-1604 */
    for (unsigned i = 0; i <= deg_omega; i++) {
        unsigned tmp = 0;
        for (unsigned j = i + 1; j-- > 0;)
            if (syn[i - j] != A0 && lambda[j] != A0)
                tmp ^= alpha_to[modnn(c, syn[i - j] + lambda[j])];
        omega[i] = index_of[tmp];
    }

    for (unsigned j = (unsigned)count; j-- > 0;) {                      /* Forney, 1610-1690 */
        unsigned num1 = 0;
        for (unsigned i = deg_omega + 1; i-- > 0;)
            if (omega[i] != A0) num1 ^= alpha_to[modnn(c, omega[i] + i * root[j])];
        unsigned num2 = alpha_to[modnn(c, root[j] * (FCR - 1) + NN)];
        unsigned den = 0;
        unsigned top = deg_lambda < NR - 1 ? deg_lambda : NR - 1;
        for (int i = (int)(top & ~1u); i >= 0; i -= 2)
            if (lambda[i + 1] != A0) den ^= alpha_to[modnn(c, lambda[i + 1] + (unsigned)i * root[j])];
        if (den == 0 && !KARN) { count = -1; goto finish; }   /* Karn: index_of[0] = A0 = NN */
        if (num1 != 0) {
            if (loc[j] < pad) {
                if (KARN) continue;                                      /* not corrected */
                count = -1;
                goto finish;
            }
            uint16_t cor = alpha_to[modnn(c, index_of[num1] + index_of[num2] + NN - index_of[den])];
            if (corr) corr[j] = cor;
            if (loc[j] < NN - NR) {
                unsigned di = loc[j] - pad;
                if (DUAL) {
                    uint16_t err_dua = data[di];
                    uint16_t fix_dua = g_into_dual[g_from_dual[err_dua] ^ cor];
                    data[di] = fix_dua;
                    if (corr) corr[j] = fix_dua ^ err_dua;
                } else {
                    data[di] ^= cor;
                }
            } else if (loc[j] < NN) {
                unsigned pi = loc[j] - (NN - NR);
                if (DUAL) {
                    uint16_t err_cnv = g_from_dual[parity[pi]];
                    uint16_t fix_cnv = err_cnv ^ cor;
                    parity[pi] = g_into_dual[fix_cnv];
                    if (corr) corr[j] = fix_cnv ^ err_cnv;
                } else {
                    parity[pi] ^= cor;
                }
            }
        }
    }
#undef CNV

finish:                                                                  /* 1713-1717 */
    if (eras_pos != NULL)
        for (int i = 0; i < count; i++) eras_pos[i] = loc[i] - (KARN ? 0 : pad);
    if (s16 != sbuf) free(s16);
    if (u32 != ubuf) free(u32);
    return count;
}

/* ------------------------------------------------------------------------------------------ */
/* Data type mapping layer: encode<INP> (rs_base:868-904) and decode<INP> (rs_base:1170-1242)
 * with INP == TYP.  The masked copy path is taken when the symbol is narrower than the datum
 * (RS<31,.> in uint8_t, RS<1023,.> in uint16_t, ...). */
static inline unsigned ld(const void *p, unsigned w, size_t i) {
    return w == 1 ? ((const uint8_t *)p)[i] : ((const uint16_t *)p)[i];
}
static inline void st(void *p, unsigned w, size_t i, unsigned v) {
    if (w == 1) ((uint8_t *)p)[i] = (uint8_t)v; else ((uint16_t *)p)[i] = (uint16_t)v;
}

int ezo_encode(const ezo_codec *c, const void *data, unsigned len, void *parity) {
    const unsigned NR = c->nroots, LOAD = c->nn - c->nroots, w = c->datum;
    if (len < 1 || len > LOAD) return -1;                                /* 875-877 */
    const unsigned symmask = c->nn;  /* ~msk: the low SYMBOL bits */
    uint16_t tmp[65536];
    uint16_t *sym = tmp, *par = tmp + LOAD;
    /* Both paths compute encode_symbols on the (masked) symbols; the masked path copies. */
    for (unsigned i = 0; i < len; ++i) sym[i] = (uint16_t)(ld(data, w, i) & symmask);
    int r = encode_symbols(c, sym, len, par);
    for (unsigned i = 0; i < NR; ++i) st(parity, w, i, par[i]);
    return r;
}

int ezo_decode(const ezo_codec *c, void *data, unsigned len, void *parity, unsigned *eras_pos,
               unsigned no_eras, void *corr) {
    const unsigned NR = c->nroots, LOAD = c->nn - c->nroots, w = c->datum;
    if (len < 1 || parity == NULL) return -1;                            /* 1180-1182 */
    const int masked = c->mm != 8 * w && !c->karn;                       /* 1194 */
    uint16_t tmp[65536], ctmp[65536];
    if (len > LOAD) return -1;  /* decode_symbols rejects it; never index tmp past LOAD */
    uint16_t *dp = tmp, *pp = tmp + len;
    const unsigned symmask = c->nn;
    for (unsigned i = 0; i < len; ++i) dp[i] = (uint16_t)(ld(data, w, i) & symmask);
    for (unsigned i = 0; i < NR; ++i) {
        unsigned v = ld(parity, w, i);
        if (masked && (v & ~symmask)) return -1;                         /* 1215-1218 */
        pp[i] = (uint16_t)v;
    }
    /* corr is passed straight through to decode_symbols in both paths (1222, 1240), which
     * writes only the entries it reaches: copy the caller's entries in and all of them back. */
    if (corr)
        for (unsigned i = 0; i < NR; ++i) ctmp[i] = (uint16_t)ld(corr, w, i);
    int res = decode_symbols(c, dp, len, pp, eras_pos, no_eras, corr ? ctmp : NULL);
    /* Masked path copies back only when corrections were reported (1223-1234); the direct path
     * operates in place, so partial corrections made before a -1 stay visible (1238-1241). */
    if (!masked || res > 0) {
        for (unsigned i = 0; i < len; ++i) {
            unsigned hi = masked ? (ld(data, w, i) & ~symmask) : 0;
            st(data, w, i, hi | dp[i]);
        }
        for (unsigned i = 0; i < NR; ++i) st(parity, w, i, pp[i]);
    }
    if (corr)
        for (unsigned i = 0; i < NR; ++i) st(corr, w, i, ctmp[i]);
    return res;
}

/* ------------------------------------------------------------------------------------------ */
int ezo_encode_batch(const ezo_codec *c, const void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, size_t ncw, int nthreads) {
    const unsigned w = c->datum;
    int bad = 0;
    (void)nthreads;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1) reduction(|:bad)
    for (long long k = 0; k < (long long)ncw; ++k) {
        const char *d = (const char *)data + (size_t)k * data_stride * w;
        char *p = parity ? (char *)parity + (size_t)k * parity_stride * w
                         : (char *)data + ((size_t)k * data_stride + len) * w;
        bad |= ezo_encode(c, d, len, p) < 0;
    }
    return bad ? -1 : 0;
}

int ezo_decode_batch(const ezo_codec *c, void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                     const uint32_t *neras, int32_t *result, uint32_t *positions,
                     size_t pos_stride, void *corr, size_t corr_stride, size_t ncw, int nthreads) {
    const unsigned w = c->datum, NR = c->nroots;
    (void)nthreads;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (long long k = 0; k < (long long)ncw; ++k) {
        char *d = (char *)data + (size_t)k * data_stride * w;
        char *p = parity ? (char *)parity + (size_t)k * parity_stride * w
                         : (char *)data + ((size_t)k * data_stride + len) * w;
        unsigned ne = neras ? neras[k] : 0;
        unsigned pos[65536];
        unsigned cap = ne > NR ? ne : NR;
        for (unsigned i = 0; i < ne && i < cap; ++i) pos[i] = eras[(size_t)k * eras_stride + i];
        int r = ezo_decode(c, d, len, p, pos, ne, corr ? (char *)corr + (size_t)k * corr_stride * w : NULL);
        result[k] = r;
        if (positions)
            for (int i = 0; i < r; ++i) positions[(size_t)k * pos_stride + i] = pos[i];
    }
    return 0;
}

/* Karn mode on (1) / off (0): decode with fec-3.0.1's semantics (see decode_symbols). */
void ezo_set_karn(ezo_codec *c, int karn) { c->karn = karn ? 1 : 0; }
