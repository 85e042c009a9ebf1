/*
 * ezbch_oracle.c -- TEST INFRASTRUCTURE ONLY: clean-room CPU restatement of the binary BCH codec the
 * reference wraps as ezpwd::bch_base / ezpwd::bch<N,T> / ezpwd::BCH<N,K,T> (c++/ezpwd/bch:48-463)
 * with ezpwd::correct_bch (c++/ezpwd/bch_base:168-199).  The algorithm underneath is Ivan Djelic's
 * Linux lib/bch.c (init_bch / encode_bch / decode_bch); in the reference it is an EMPTY git
 * submodule (djelic/, .gitmodules:1-9), so it is restated here from the published algorithm and
 * the conventions the reference's own call sites and fixtures fix:
 *
 *   - GF(2^m), m = 5..15, default primitive polynomial per m (lib/bch.c prim_poly_tab);
 *     init fails unless t >= 1 and m*t < 2^m - 1 (bch_base:49-69)
 *   - g(x) = product of the minimal polynomials of alpha, alpha^3, ..., alpha^(2t-1);
 *     ecc_bits = deg g, ecc_bytes = ceil(m*t / 8) (bch_base:35-36)
 *   - ECC = d(x) x^ecc_bits mod g(x): data bits MSB first (bit 7 of data[0] is the highest power),
 *     remainder stored left-justified and big-endian, unused trailing bits 0
 *     (README.org:1173-1188 vector; bch_itron.C:159-177 record layout)
 *   - decode: -EINVAL if 8*len > n - ecc_bits; 0 if the received ECC equals the computed one; else
 *     syndromes S_1..S_2t of the difference (only its ecc_bits significant bits), Berlekamp-Massey
 *     (the binary form: odd steps), roots of the locator; a locator degree > t, a root count that
 *     differs from the degree, or a root outside the codeword's nbits = 8*len + ecc_bits bits is
 *     -EBADMSG; a root at polynomial power p is reported as e = nbits-1-p with its bit order
 *     reversed within the byte, so that data[e/8] bit (e%8) is the bit (bch_base:116-123)
 *
 * Roots are found here by a Chien search over the whole field (the GPU path uses closed forms, so
 * the two are independent).  Parity status: pinned by the reference's fixtures only (see
 * tests/test_bch_oracle.py); the order of reported locations is unpinned -- ascending here.
 */
#include "ezbch_oracle.h"

#include <stdlib.h>
#include <string.h>

#define EZB_EINVAL 22   /* Linux errno values, returned negated as decode_bch does */
#define EZB_EBADMSG 74

struct ezb {
    int m, n, t, ecc_bits, ecc_bytes;
    unsigned poly;
    int *ex;      /* ex[i] = alpha^i, i in [0, 2n) */
    int *lg;      /* lg[x] = log x, lg[0] = -1 */
    uint8_t *g;   /* generator, g[i] = coefficient of x^i, i = 0..ecc_bits */
};

/* init_bch's default primitive polynomials for m = 5..15 */
static const unsigned kPrim[11] = {0x25, 0x43, 0x83, 0x11d, 0x211, 0x409,
                                   0x805, 0x1053, 0x201b, 0x402b, 0x8003};

static int gmul(const ezb_t *b, int x, int y) { return (x && y) ? b->ex[b->lg[x] + b->lg[y]] : 0; }
static int gdiv(const ezb_t *b, int x, int y) { return x ? b->ex[b->lg[x] + b->n - b->lg[y]] : 0; }

void ezb_destroy(ezb_t *b) {
    if (!b) return;
    free(b->ex);
    free(b->lg);
    free(b->g);
    free(b);
}

ezb_t *ezb_create(int m, int t, unsigned poly) {
    if (m < 5 || m > 15) return NULL;
    const int n = (1 << m) - 1;
    if (t < 1 || m * t >= n) return NULL;
    if (!poly) poly = kPrim[m - 5];
    if ((poly >> m) != 1) return NULL;
    ezb_t *b = calloc(1, sizeof *b);
    int *gc = calloc((size_t)n + 1, sizeof(int));
    char *root = calloc((size_t)n, 1);
    if (!b || !gc || !root) goto fail;
    b->m = m; b->n = n; b->t = t; b->poly = poly;
    b->ex = malloc(sizeof(int) * 2 * (size_t)n);
    b->lg = malloc(sizeof(int) * ((size_t)n + 1));
    if (!b->ex || !b->lg) goto fail;
    for (int i = 0; i <= n; ++i) b->lg[i] = -1;
    for (int i = 0, x = 1; i < n; ++i) {
        if (b->lg[x] >= 0) goto fail;                 /* not primitive */
        b->ex[i] = b->ex[i + n] = x;
        b->lg[x] = i;
        x <<= 1;
        if (x >> m) x ^= (int)poly;
    }
    /* roots alpha^j, j in the cyclotomic cosets of 1, 3, ..., 2t-1 */
    for (int i = 0; i < t; ++i)
        for (int k = 0, j = 2 * i + 1; k < m; ++k, j = (2 * j) % n) root[j] = 1;
    int deg = 0;
    gc[0] = 1;
    for (int j = 0; j < n; ++j) {
        if (!root[j]) continue;
        const int r = b->ex[j];                        /* g *= (x + alpha^j) */
        for (int k = deg + 1; k > 0; --k) gc[k] = gc[k - 1] ^ gmul(b, gc[k], r);
        gc[0] = gmul(b, gc[0], r);
        ++deg;
    }
    b->g = malloc((size_t)deg + 1);
    if (!b->g) goto fail;
    for (int k = 0; k <= deg; ++k) {
        if (gc[k] > 1) goto fail;                      /* a product of minimal polynomials is binary */
        b->g[k] = (uint8_t)gc[k];
    }
    b->ecc_bits = deg;
    b->ecc_bytes = (m * t + 7) / 8;
    free(gc);
    free(root);
    return b;
fail:
    free(gc);
    free(root);
    ezb_destroy(b);
    return NULL;
}

void ezb_info(const ezb_t *b, unsigned *o) {
    o[0] = (unsigned)b->m; o[1] = (unsigned)b->n; o[2] = (unsigned)b->t;
    o[3] = (unsigned)b->ecc_bits; o[4] = (unsigned)b->ecc_bytes; o[5] = b->poly;
}

void ezb_genpoly(const ezb_t *b, uint8_t *coef) { memcpy(coef, b->g, (size_t)b->ecc_bits + 1); }

/* r[0..E) = coefficients of d(x) x^E mod g(x), by the bitwise LFSR, data MSB first */
static void lfsr_remainder(const ezb_t *b, const uint8_t *data, unsigned len, uint8_t *r) {
    const int E = b->ecc_bits;
    memset(r, 0, (size_t)E);
    for (unsigned i = 0; i < len; ++i)
        for (int k = 7; k >= 0; --k) {
            const uint8_t fb = (uint8_t)(((data[i] >> k) & 1) ^ r[E - 1]);
            for (int j = E - 1; j > 0; --j) r[j] = (uint8_t)(r[j - 1] ^ (fb & b->g[j]));
            r[0] = (uint8_t)(fb & b->g[0]);
        }
}

/* left-justified, big-endian: x^(E-1) is bit 7 of ecc[0] */
static void pack(const ezb_t *b, const uint8_t *r, uint8_t *ecc) {
    memset(ecc, 0, (size_t)b->ecc_bytes);
    for (int i = 0; i < b->ecc_bits; ++i)
        if (r[b->ecc_bits - 1 - i]) ecc[i >> 3] |= (uint8_t)(0x80u >> (i & 7));
}

void ezb_encode(const ezb_t *b, const uint8_t *data, unsigned len, uint8_t *ecc) {
    uint8_t *r = malloc((size_t)b->ecc_bits);
    lfsr_remainder(b, data, len, r);
    pack(b, r, ecc);
    free(r);
}

/* S[1..2t] of the received codeword; returns 0 when recv equals the computed ECC (no syndromes) */
static int syndromes(const ezb_t *b, const uint8_t *data, unsigned len, const uint8_t *recv, int *S) {
    const int n = b->n, t = b->t, E = b->ecc_bits;
    uint8_t *r = malloc((size_t)E), *diff = malloc((size_t)b->ecc_bytes);
    lfsr_remainder(b, data, len, r);
    pack(b, r, diff);
    int any = 0;
    for (int i = 0; i < b->ecc_bytes; ++i) {
        diff[i] ^= recv[i];
        any |= diff[i];
    }
    memset(S, 0, sizeof(int) * (2 * (size_t)t + 1));
    /* S_j = diff(alpha^j) over the ecc_bits significant bits; bit i (MSB first) is x^(E-1-i) */
    for (int i = 0; i < E && any; ++i) {
        if (!((diff[i >> 3] >> (7 - (i & 7))) & 1)) continue;
        const long long p = E - 1 - i;
        for (int j = 1; j < 2 * t; j += 2) S[j] ^= b->ex[(j * p) % n];
    }
    for (int j = 1; j <= t; ++j) S[2 * j] = gmul(b, S[j], S[j]);
    free(r);
    free(diff);
    return any;
}

/* decode_bch's syndrome form (bch_base:96-114, "by providing syndrome results @syn"): the error
 * locations from S_1..S_2t = syn[0..2t) alone */
static int decode_from_syndromes(const ezb_t *b, unsigned len, const int *S, unsigned *errloc);

int ezb_syndromes(const ezb_t *b, const uint8_t *data, unsigned len, const uint8_t *recv,
                  unsigned *syn) {
    int *S = calloc(2 * (size_t)b->t + 1, sizeof(int));
    syndromes(b, data, len, recv, S);
    for (int j = 1; j <= 2 * b->t; ++j) syn[j - 1] = (unsigned)S[j];
    free(S);
    return 0;
}

int ezb_decode_syn(const ezb_t *b, unsigned len, const unsigned *syn, unsigned *errloc) {
    if (8ull * len > (unsigned long long)(b->n - b->ecc_bits)) return -EZB_EINVAL;
    int *S = calloc(2 * (size_t)b->t + 1, sizeof(int));
    for (int j = 1; j <= 2 * b->t; ++j) S[j] = (int)syn[j - 1];
    const int r = decode_from_syndromes(b, len, S, errloc);
    free(S);
    return r;
}

int ezb_decode(const ezb_t *b, const uint8_t *data, unsigned len, const uint8_t *recv,
               unsigned *errloc) {
    if (8ull * len > (unsigned long long)(b->n - b->ecc_bits)) return -EZB_EINVAL;
    int *S = calloc(2 * (size_t)b->t + 1, sizeof(int));
    const int any = syndromes(b, data, len, recv, S);
    const int r = any ? decode_from_syndromes(b, len, S, errloc) : 0;
    free(S);
    return r;
}

static int decode_from_syndromes(const ezb_t *b, unsigned len, const int *S, unsigned *errloc) {
    const int n = b->n, t = b->t, E = b->ecc_bits;
    const int W = 4 * t + 2;
    int *elp = calloc((size_t)W, sizeof(int)), *pelp = calloc((size_t)W, sizeof(int)),
        *cpy = calloc((size_t)W, sizeof(int));
    unsigned *loc = calloc((size_t)t + 1, sizeof(unsigned));
    int ret;
    /* Berlekamp-Massey, binary form: elp(x) = 1 + ... ; pelp = x^k-shifted previous elp */
    int edeg = 0, pdeg = 0, pp = -1, pd = 1, d = S[1];
    elp[0] = pelp[0] = 1;
    for (int i = 0; i < t && edeg <= t; ++i) {
        if (d) {
            const int k = 2 * i - pp, cdeg = edeg, q = gdiv(b, d, pd);
            memcpy(cpy, elp, sizeof(int) * (size_t)W);
            for (int j = 0; j <= pdeg; ++j)
                if (pelp[j]) elp[j + k] ^= gmul(b, q, pelp[j]);
            if (pdeg + k > edeg) {
                edeg = pdeg + k;
                memcpy(pelp, cpy, sizeof(int) * (size_t)W);
                pdeg = cdeg;
                pd = d;
                pp = 2 * i;
            }
        }
        if (i < t - 1) {
            d = S[2 * i + 3];
            for (int j = 1; j <= edeg; ++j) d ^= gmul(b, elp[j], S[2 * i + 3 - j]);
        }
    }
    if (edeg > t || edeg == 0) { ret = edeg ? -EZB_EBADMSG : 0; goto out; }
    /* Chien over the whole field: X = alpha^p is a locator iff elp(alpha^-p) = 0 */
    int cnt = 0;
    for (int p = 0; p < n && cnt <= edeg; ++p) {
        int v = 0;
        for (int j = 0; j <= edeg; ++j)
            if (elp[j]) v ^= b->ex[(b->lg[elp[j]] + (long long)j * (n - p)) % n];
        if (!v) {
            if (cnt < edeg) loc[cnt] = (unsigned)p;
            ++cnt;
        }
    }
    if (cnt != edeg) { ret = -EZB_EBADMSG; goto out; }
    const unsigned nbits = 8 * len + (unsigned)E;
    for (int i = 0; i < cnt; ++i) {
        if (loc[i] >= nbits) { ret = -EZB_EBADMSG; goto out; }
        const unsigned e = nbits - 1 - loc[i];
        loc[i] = (e & ~7u) | (7u - (e & 7u));
    }
    for (int i = 1; i < cnt; ++i)                      /* ascending */
        for (int j = i; j > 0 && loc[j - 1] > loc[j]; --j) {
            const unsigned x = loc[j];
            loc[j] = loc[j - 1];
            loc[j - 1] = x;
        }
    if (errloc) memcpy(errloc, loc, sizeof(unsigned) * (size_t)cnt);
    ret = cnt;
out:
    free(elp); free(pelp); free(cpy); free(loc);
    return ret;
}

int ezb_correct(const ezb_t *b, uint8_t *data, unsigned len, uint8_t *ecc, unsigned *errloc) {
    unsigned *loc = malloc(sizeof(unsigned) * ((size_t)b->t + 1));
    const int r = ezb_decode(b, data, len, ecc, loc);
    for (int i = 0; i < r; ++i) {
        const unsigned e = loc[i];
        if (e < 8 * len) data[e >> 3] ^= (uint8_t)(1u << (e & 7));
        else if (e < 8 * len + 8 * (unsigned)b->ecc_bytes) ecc[(e >> 3) - len] ^= (uint8_t)(1u << (e & 7));
    }
    if (errloc && r > 0) memcpy(errloc, loc, sizeof(unsigned) * (size_t)r);
    free(loc);
    return r;
}

void ezb_encode_batch(const ezb_t *b, const uint8_t *data, size_t dstride, unsigned len,
                      uint8_t *ecc, size_t estride, size_t ncw, int nthreads) {
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
    for (size_t k = 0; k < ncw; ++k) {
        const uint8_t *d = data + k * dstride;
        uint8_t *e = ecc ? ecc + k * estride : (uint8_t *)d + len;
        ezb_encode(b, d, len, e);
    }
}

void ezb_decode_batch(const ezb_t *b, uint8_t *data, size_t dstride, unsigned len, uint8_t *ecc,
                      size_t estride, int32_t *result, uint32_t *errloc, size_t lstride,
                      size_t ncw, int nthreads) {
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
    for (size_t k = 0; k < ncw; ++k) {
        uint8_t *d = data + k * dstride;
        uint8_t *e = ecc ? ecc + k * estride : d + len;
        result[k] = ezb_correct(b, d, len, e, errloc ? errloc + k * lstride : NULL);
    }
}
