// ezrs_stream.hip -- the rsencode streaming wire format over the batch host forms (include/ezrs.h).
//
// rsencode.C:93-163 cuts its input into chunks of `chunk` data symbols (the last one may be
// shorter) and writes each chunk followed by its NROOTS parity symbols; symbols wider than 8 bits
// are serialized big-endian (rsencode.C:52-85).  Decoding reads chunk + NROOTS symbols at a time,
// corrects in place (a failed chunk keeps whatever the decoder left, rsencode.C:145-156) and drops
// the parity.  The reference does this one codeword per call; here a whole buffer of chunks becomes
// one batch: rows of (chunk + NROOTS) symbols in host memory, ezrs_encode_rows_host /
// ezrs_decode_host over all full chunks, a second call for a shorter last chunk.
#include <cerrno>
#include <cstring>
#include <vector>

#include "../../include/ezrs.h"

namespace {

struct Shape {
    unsigned w, nr;
    size_t load;
};

bool shape_of(const ezrs_codec *c, Shape &s) {
    ezrs_info info;
    if (!c || ezrs_get_info(c, &info) != 0) return false;
    s.w = info.datum_bytes;
    s.nr = info.nroots;
    s.load = info.load;
    return true;
}

// big-endian wire <-> host 16-bit symbols
void be_to_u16(const uint8_t *src, uint16_t *dst, size_t n) {
    for (size_t i = 0; i < n; ++i) dst[i] = (uint16_t)(src[2 * i] << 8 | src[2 * i + 1]);
}
void u16_to_be(const uint16_t *src, uint8_t *dst, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        dst[2 * i] = (uint8_t)(src[i] >> 8);
        dst[2 * i + 1] = (uint8_t)src[i];
    }
}

} // namespace

extern "C" {

size_t ezrs_stream_encoded_bound(const ezrs_codec *c, size_t in_bytes, unsigned chunk) {
    Shape s;
    if (!shape_of(c, s) || chunk == 0) return 0;
    const size_t cb = (size_t)chunk * s.w;
    const size_t nchunks = (in_bytes + cb - 1) / cb;
    return in_bytes + nchunks * s.nr * s.w;
}

int ezrs_stream_encode(ezrs_codec *c, const void *in, size_t in_bytes, unsigned chunk, void *out,
                       size_t out_cap, size_t *out_bytes) {
    Shape s;
    if (out_bytes) *out_bytes = 0;
    if (!shape_of(c, s) || (!in && in_bytes) || !out_bytes) return -EINVAL;
    if (chunk == 0 || chunk > s.load) return -EINVAL;
    if (in_bytes == 0) return 0;
    if (!out || out_cap < ezrs_stream_encoded_bound(c, in_bytes, chunk)) return -ENOSPC;
    const uint8_t *src = static_cast<const uint8_t *>(in);
    uint8_t *dst = static_cast<uint8_t *>(out);
    const size_t cb = (size_t)chunk * s.w, row = (size_t)(chunk + s.nr) * s.w;
    const size_t nfull = in_bytes / cb, tail = in_bytes - nfull * cb;
    const size_t ntail_sym = tail / s.w;
    const bool bad_tail = tail % s.w != 0;               // rsencode.C:110-111
    const size_t nrows = nfull + (tail && !bad_tail ? 1 : 0);
    if (s.w == 1) {
        // the output buffer is the row array: data copied in, parity written in place
        for (size_t k = 0; k < nfull; ++k) std::memcpy(dst + k * row, src + k * cb, cb);
        int r = ezrs_encode_rows_host(c, dst, row, chunk, nfull, 0);
        if (r) return r;
        if (nrows > nfull) {
            std::memcpy(dst + nfull * row, src + nfull * cb, ntail_sym);
            if ((r = ezrs_encode_rows_host(c, dst + nfull * row, ntail_sym + s.nr,
                                           (unsigned)ntail_sym, 1, 0)))
                return r;
        }
    } else {
        std::vector<uint16_t> rows((nfull + 1) * (chunk + s.nr));
        for (size_t k = 0; k < nfull; ++k) be_to_u16(src + k * cb, &rows[k * (chunk + s.nr)], chunk);
        int r = ezrs_encode_rows_host(c, rows.data(), chunk + s.nr, chunk, nfull, 0);
        if (r) return r;
        u16_to_be(rows.data(), dst, nfull * (chunk + s.nr));
        if (nrows > nfull) {
            uint16_t *t = &rows[nfull * (chunk + s.nr)];
            be_to_u16(src + nfull * cb, t, ntail_sym);
            if ((r = ezrs_encode_rows_host(c, t, ntail_sym + s.nr, (unsigned)ntail_sym, 1, 0))) return r;
            u16_to_be(t, dst + nfull * row, ntail_sym + s.nr);
        }
    }
    *out_bytes = nfull * row + (nrows > nfull ? (ntail_sym + s.nr) * s.w : 0);
    return bad_tail ? -EMSGSIZE : 0;
}

int ezrs_stream_decode(ezrs_codec *c, const void *in, size_t in_bytes, unsigned chunk, void *out,
                       size_t out_cap, size_t *out_bytes, size_t *n_failed) {
    Shape s;
    if (out_bytes) *out_bytes = 0;
    if (n_failed) *n_failed = 0;
    if (!shape_of(c, s) || (!in && in_bytes) || !out_bytes) return -EINVAL;
    if (chunk == 0 || chunk > s.load) return -EINVAL;
    if (in_bytes == 0) return 0;
    if (!out || out_cap < in_bytes) return -ENOSPC;
    const uint8_t *src = static_cast<const uint8_t *>(in);
    uint8_t *dst = static_cast<uint8_t *>(out);
    const size_t rs = chunk + s.nr, row = rs * s.w;
    const size_t nfull = in_bytes / row, tail = in_bytes - nfull * row;
    // rsencode.C:140-141: a chunk needs more than NROOTS whole symbols
    const bool bad_tail = tail != 0 && (tail < (size_t)(s.nr + 1) * s.w || tail % s.w != 0);
    const size_t ntail_sym = tail / s.w;
    const size_t nrows = nfull + (tail && !bad_tail ? 1 : 0);
    std::vector<int32_t> res(nrows ? nrows : 1);
    size_t failed = 0;
    if (s.w == 1) {
        std::vector<uint8_t> rows(src, src + nfull * row + (nrows > nfull ? tail : 0));
        int r = ezrs_decode_host(c, rows.data(), row, chunk, nullptr, 0, nullptr, 0, nullptr,
                                 res.data(), nullptr, 0, nullptr, 0, nfull, 0);
        if (r) return r;
        if (nrows > nfull &&
            (r = ezrs_decode_host(c, rows.data() + nfull * row, tail, (unsigned)(ntail_sym - s.nr),
                                  nullptr, 0, nullptr, 0, nullptr, &res[nfull], nullptr, 0,
                                  nullptr, 0, 1, 0)))
            return r;
        for (size_t k = 0; k < nfull; ++k) std::memcpy(dst + k * chunk, rows.data() + k * row, chunk);
        if (nrows > nfull)
            std::memcpy(dst + nfull * chunk, rows.data() + nfull * row, ntail_sym - s.nr);
    } else {
        std::vector<uint16_t> rows(nfull * rs + (nrows > nfull ? ntail_sym : 0));
        be_to_u16(src, rows.data(), rows.size());
        int r = ezrs_decode_host(c, rows.data(), rs, chunk, nullptr, 0, nullptr, 0, nullptr,
                                 res.data(), nullptr, 0, nullptr, 0, nfull, 0);
        if (r) return r;
        if (nrows > nfull &&
            (r = ezrs_decode_host(c, rows.data() + nfull * rs, ntail_sym,
                                  (unsigned)(ntail_sym - s.nr), nullptr, 0, nullptr, 0, nullptr,
                                  &res[nfull], nullptr, 0, nullptr, 0, 1, 0)))
            return r;
        for (size_t k = 0; k < nfull; ++k) u16_to_be(&rows[k * rs], dst + k * chunk * 2, chunk);
        if (nrows > nfull) u16_to_be(&rows[nfull * rs], dst + nfull * chunk * 2, ntail_sym - s.nr);
    }
    for (size_t k = 0; k < nrows; ++k) failed += res[k] < 0;
    if (n_failed) *n_failed = failed;
    *out_bytes = (nfull * chunk + (nrows > nfull ? ntail_sym - s.nr : 0)) * s.w;
    return bad_tail ? -EMSGSIZE : 0;
}

} // extern "C"
