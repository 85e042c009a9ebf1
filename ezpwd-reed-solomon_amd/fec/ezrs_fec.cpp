// ezrs_fec.cpp -- Phil Karn's libfec RS ABI (include/ezrs_fec.h) over the MI355X engine.
//
// Each Karn codec is an engine codec in EZRS_SEM_KARN mode (full-NN-frame positions, Karn's
// failure rules: fec-3.0.1/decode_rs.h:71-298), created by init_rs_*; the encode / decode calls
// are the engine's host-memory batch forms over one codeword (or a whole batch, *_batch).  Nothing
// here computes a code symbol: the host side only checks arguments, converts containers (int
// symbols, symbols narrower than their container) and copies results.
#include "ezrs_fec.h"

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace {

// fec-3.0.1/rs-common.h:7-19 layout first: callers read nn, nroots and pad through it.
struct KarnRs {
    int mm;
    int nn;
    void *alpha_to;
    void *index_of;
    void *genpoly;
    int nroots;
    int fcr;
    int prim;
    int iprim;
    int pad;
    // engine side
    ezrs_codec *codec;
    int int_symbols;    // created by init_rs_int (unsigned int containers)
};

[[noreturn]] void die(const char *what, int rc) {
    std::fprintf(stderr, "ezrs_fec: %s failed (errno %d): %s\n", what, -rc, ezrs_last_error());
    std::abort();
}

int fec_device() {
    const char *e = std::getenv("EZRS_FEC_DEVICE");
    return e ? std::atoi(e) : 0;
}

// init_rs.h:48-101 argument rules, then the engine codec in Karn mode.
KarnRs *make_rs(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad, bool ints, bool dual) {
    if (symsize < 2 || symsize > (ints ? 16 : 8)) return nullptr;
    const int nn = (1 << symsize) - 1;
    if (fcr < 0 || fcr >= (1 << symsize)) return nullptr;
    if (prim <= 0 || prim >= (1 << symsize)) return nullptr;
    if (nroots < 1 || nroots >= (1 << symsize)) return nullptr;
    if (pad < 0 || pad >= nn - nroots) return nullptr;
    ezrs_codec *c = nullptr;
    if (ezrs_create(&c, (unsigned)symsize, (unsigned)gfpoly, (unsigned)fcr, (unsigned)prim,
                    (unsigned)nroots, dual ? 1 : 0, fec_device()) != 0)
        return nullptr;                      // invalid polynomial / no GPU: init fails, as Karn's
    if (ezrs_set_semantics(c, EZRS_SEM_KARN) != 0) {
        ezrs_destroy(c);
        return nullptr;
    }
    KarnRs *rs = new (std::nothrow) KarnRs{};
    if (!rs) {
        ezrs_destroy(c);
        return nullptr;
    }
    rs->mm = symsize;
    rs->nn = nn;
    rs->nroots = nroots;
    rs->fcr = fcr;
    rs->prim = prim;
    int iprim = 1;                           // prim-th root of 1 (init_rs.h:96-98)
    while (iprim % prim != 0) iprim += nn;
    rs->iprim = iprim / prim;
    rs->pad = pad;
    rs->codec = c;
    rs->int_symbols = ints ? 1 : 0;
    return rs;
}

void free_rs(void *p) {
    KarnRs *rs = static_cast<KarnRs *>(p);
    if (!rs) return;
    ezrs_destroy(rs->codec);
    delete rs;
}

// Encode ncw codewords of src (container C, stride in elements) -> parity.
template <typename C>
int encode_batch(KarnRs *rs, const C *data, size_t stride, C *parity, size_t pstride, size_t ncw) {
    if (!rs || !data || !parity) return -EINVAL;
    if (!ncw) return 0;
    const unsigned len = (unsigned)(rs->nn - rs->nroots - rs->pad), NR = (unsigned)rs->nroots;
    const unsigned mask = (unsigned)rs->nn;
    if (!stride) stride = len;               // single-codeword calls pass 0
    if (!pstride) pstride = NR;
    // Karn's tables index with the symbol as given: values must fit the symbol; the engine's
    // containers are uint8_t (m <= 8) / uint16_t (m > 8)
    if (rs->mm <= 8 && sizeof(C) == 1 && rs->mm == 8)
        return ezrs_encode_host(rs->codec, data, stride, len, parity, pstride, ncw, 0);
    if (rs->mm <= 8) {
        std::vector<uint8_t> d((size_t)ncw * len), p((size_t)ncw * NR);
        for (size_t k = 0; k < ncw; ++k)
            for (unsigned i = 0; i < len; ++i) d[k * len + i] = (uint8_t)(data[k * stride + i] & mask);
        const int r = ezrs_encode_host(rs->codec, d.data(), len, len, p.data(), NR, ncw, 0);
        if (r) return r;
        for (size_t k = 0; k < ncw; ++k)
            for (unsigned i = 0; i < NR; ++i) parity[k * pstride + i] = (C)p[k * NR + i];
        return 0;
    }
    std::vector<uint16_t> d((size_t)ncw * len), p((size_t)ncw * NR);
    for (size_t k = 0; k < ncw; ++k)
        for (unsigned i = 0; i < len; ++i) d[k * len + i] = (uint16_t)(data[k * stride + i] & mask);
    const int r = ezrs_encode_host(rs->codec, d.data(), len, len, p.data(), NR, ncw, 0);
    if (r) return r;
    for (size_t k = 0; k < ncw; ++k)
        for (unsigned i = 0; i < NR; ++i) parity[k * pstride + i] = (C)p[k * NR + i];
    return 0;
}

// Decode ncw rows of NN-PAD symbols in place (Karn's data[]).
template <typename C>
int decode_batch(KarnRs *rs, C *data, size_t stride, int *eras_pos, size_t eras_stride, const int *no_eras,
                 int *result, size_t ncw) {
    if (!rs || !data || !result) return -EINVAL;
    if (!ncw) return 0;
    const unsigned NR = (unsigned)rs->nroots, len = (unsigned)(rs->nn - rs->nroots - rs->pad), row = len + NR;
    const unsigned mask = (unsigned)rs->nn;
    if (!stride) stride = row;               // single-codeword calls pass 0
    if (!eras_stride) eras_stride = NR;
    const bool have_eras = eras_pos && no_eras;
    std::vector<uint32_t> eras(have_eras ? ncw * NR : 0), ne(have_eras ? ncw : 0), pos(eras_pos ? ncw * NR : 0);
    if (have_eras)
        for (size_t k = 0; k < ncw; ++k) {
            const int n = no_eras[k] < 0 ? 0 : no_eras[k];
            ne[k] = (uint32_t)n;
            for (int i = 0; i < n && i < (int)NR; ++i) eras[k * NR + i] = (uint32_t)eras_pos[k * eras_stride + i];
        }
    std::vector<int32_t> res(ncw);
    int r;
    if (rs->mm == 8 && sizeof(C) == 1) {
        // the caller's rows in place: only rows whose result is nonzero are written back
        r = ezrs_decode_host(rs->codec, data, stride, len, reinterpret_cast<uint8_t *>(data) + len, stride,
                             have_eras ? eras.data() : nullptr, NR, have_eras ? ne.data() : nullptr, res.data(),
                             eras_pos ? pos.data() : nullptr, NR, nullptr, 0, ncw, 0);
    } else {
        // narrower symbols (masked copy; only the symbols the decode changed are written back, so
        // container bits above the symbol survive) or int containers
        const bool wide = rs->mm > 8;
        std::vector<uint8_t> b8(wide ? 0 : (size_t)ncw * row), o8;
        std::vector<uint16_t> b16(wide ? (size_t)ncw * row : 0), o16;
        for (size_t k = 0; k < ncw; ++k)
            for (unsigned i = 0; i < row; ++i) {
                const unsigned v = (unsigned)data[k * stride + i] & mask;
                if (wide) b16[k * row + i] = (uint16_t)v; else b8[k * row + i] = (uint8_t)v;
            }
        o8 = b8;
        o16 = b16;
        void *buf = wide ? (void *)b16.data() : (void *)b8.data();
        void *par = wide ? (void *)(b16.data() + len) : (void *)(b8.data() + len);
        r = ezrs_decode_host(rs->codec, buf, row, len, par, row, have_eras ? eras.data() : nullptr, NR,
                             have_eras ? ne.data() : nullptr, res.data(), eras_pos ? pos.data() : nullptr, NR,
                             nullptr, 0, ncw, 0);
        if (!r)
            for (size_t k = 0; k < ncw; ++k)
                for (unsigned i = 0; i < row; ++i) {
                    const size_t j = k * row + i;
                    const unsigned d = wide ? (unsigned)(b16[j] ^ o16[j]) : (unsigned)(b8[j] ^ o8[j]);
                    if (d) data[k * stride + i] = (C)(data[k * stride + i] ^ d);
                }
    }
    if (r) return r;
    for (size_t k = 0; k < ncw; ++k) {
        result[k] = res[k];
        if (eras_pos)    // decode_rs.h:292-296: loc[0..count) into eras_pos
            for (int i = 0; i < res[k]; ++i) eras_pos[k * eras_stride + i] = (int)pos[k * NR + i];
    }
    return 0;
}

// The fixed CCSDS codecs (0x187, fcr 112, prim 11, 32 roots), pad per call: one engine codec each.
KarnRs *fixed_codec(bool dual) {
    static std::once_flag once[2];
    static KarnRs *codec[2] = {nullptr, nullptr};
    const int i = dual ? 1 : 0;
    std::call_once(once[i], [&] { codec[i] = make_rs(8, 0x187, 112, 11, 32, 0, false, dual); });
    if (!codec[i]) die(dual ? "init of the CCSDS dual-basis codec" : "init of the CCSDS codec", -ENODEV);
    return codec[i];
}

// A copy of a fixed codec's handle with this call's pad (the engine codec is shared).
KarnRs with_pad(KarnRs *rs, int pad) {
    KarnRs t = *rs;
    t.pad = pad;
    return t;
}

} // namespace

extern "C" {

void *init_rs_char(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad) {
    return make_rs(symsize, gfpoly, fcr, prim, nroots, pad, false, false);
}
void *init_rs_int(int symsize, int gfpoly, int fcr, int prim, int nroots, int pad) {
    return make_rs(symsize, gfpoly, fcr, prim, nroots, pad, true, false);
}
void free_rs_char(void *rs) { free_rs(rs); }
void free_rs_int(void *rs) { free_rs(rs); }

void encode_rs_char(void *p, unsigned char *data, unsigned char *parity) {
    if (int r = encode_batch(static_cast<KarnRs *>(p), data, 0, parity, 0, 1)) die("encode_rs_char", r);
}
int decode_rs_char(void *p, unsigned char *data, int *eras_pos, int no_eras) {
    int result = -1;
    if (int r = decode_batch(static_cast<KarnRs *>(p), data, 0, eras_pos, 0, eras_pos ? &no_eras : nullptr,
                             &result, 1))
        die("decode_rs_char", r);
    return result;
}
void encode_rs_int(void *p, unsigned int *data, unsigned int *parity) {
    if (int r = encode_batch(static_cast<KarnRs *>(p), data, 0, parity, 0, 1)) die("encode_rs_int", r);
}
int decode_rs_int(void *p, unsigned int *data, int *eras_pos, int no_eras) {
    int result = -1;
    if (int r = decode_batch(static_cast<KarnRs *>(p), data, 0, eras_pos, 0, eras_pos ? &no_eras : nullptr,
                             &result, 1))
        die("decode_rs_int", r);
    return result;
}

void encode_rs_8(unsigned char *data, unsigned char *parity, int pad) {
    if (pad < 0 || pad >= 223) die("encode_rs_8 (pad out of range)", -EINVAL);
    KarnRs t = with_pad(fixed_codec(false), pad);
    if (int r = encode_batch(&t, data, 0, parity, 0, 1)) die("encode_rs_8", r);
}
int decode_rs_8(unsigned char *data, int *eras_pos, int no_eras, int pad) {
    if (pad < 0 || pad >= 223) return -1;
    KarnRs t = with_pad(fixed_codec(false), pad);
    int result = -1;
    if (int r = decode_batch(&t, data, 0, eras_pos, 0, eras_pos ? &no_eras : nullptr, &result, 1))
        die("decode_rs_8", r);
    return result;
}
void encode_rs_ccsds(unsigned char *data, unsigned char *parity, int pad) {
    if (pad < 0 || pad >= 223) die("encode_rs_ccsds (pad out of range)", -EINVAL);
    KarnRs t = with_pad(fixed_codec(true), pad);
    if (int r = encode_batch(&t, data, 0, parity, 0, 1)) die("encode_rs_ccsds", r);
}
int decode_rs_ccsds(unsigned char *data, int *eras_pos, int no_eras, int pad) {
    if (pad < 0 || pad >= 223) return -1;
    KarnRs t = with_pad(fixed_codec(true), pad);
    int result = -1;
    if (int r = decode_batch(&t, data, 0, eras_pos, 0, eras_pos ? &no_eras : nullptr, &result, 1))
        die("decode_rs_ccsds", r);
    return result;
}

void *pad_rs_char(void *p, int pad) {
    KarnRs *rs = static_cast<KarnRs *>(p);
    if (!rs || pad < 0 || pad >= rs->nn - rs->nroots) return nullptr;   // pad_rs.c:15-17
    rs->pad = pad;
    return p;
}
void *pad_rs_int(void *p, int pad) { return pad_rs_char(p, pad); }

int encode_rs_char_batch(void *rs, const unsigned char *data, size_t stride, unsigned char *parity,
                         size_t parity_stride, size_t ncw) {
    return encode_batch(static_cast<KarnRs *>(rs), data, stride, parity, parity_stride, ncw);
}
int decode_rs_char_batch(void *rs, unsigned char *data, size_t stride, int *eras_pos, size_t eras_stride,
                         const int *no_eras, int *result, size_t ncw) {
    return decode_batch(static_cast<KarnRs *>(rs), data, stride, eras_pos, eras_stride, no_eras, result, ncw);
}
int encode_rs_int_batch(void *rs, const unsigned int *data, size_t stride, unsigned int *parity,
                        size_t parity_stride, size_t ncw) {
    return encode_batch(static_cast<KarnRs *>(rs), data, stride, parity, parity_stride, ncw);
}
int decode_rs_int_batch(void *rs, unsigned int *data, size_t stride, int *eras_pos, size_t eras_stride,
                        const int *no_eras, int *result, size_t ncw) {
    return decode_batch(static_cast<KarnRs *>(rs), data, stride, eras_pos, eras_stride, no_eras, result, ncw);
}

ezrs_codec *ezrs_fec_codec(void *rs) { return rs ? static_cast<KarnRs *>(rs)->codec : nullptr; }

} // extern "C"
