// ezrs_capi.hip -- the C ABI of the MI355X RS engine (include/ezrs.h).
//
// Codec objects own their device-resident tables (built once, like the reference's static
// reed_solomon_tabs / genpoly, rs_base:599-635, 1248-1286) and a decode workspace.  Batch entry
// points validate arguments the way the reference's encode<INP>/decode<INP> do
// (rs_base:868-904, 1170-1242) and dispatch to the fastest kernel that is bit-exact for the codec:
// the bit-sliced GF(2^8) kernels where they apply, the generic per-codeword kernels otherwise.
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/ezrs.h"
#include "ezrs_internal.hpp"

using namespace ezrs;

struct ezrs_codec {
    CodecMath math;
    int device = 0;
    DevCodec dev{};
    uint16_t *d_tabs = nullptr;   // alpha_to | index_of | genpoly
    uint8_t *d_dual = nullptr;    // into_dual | from_dual
    std::mutex mu;                // guards the lazily grown host-pipeline buffers
    void *h_stage[2] = {nullptr, nullptr};
    void *d_stage[2] = {nullptr, nullptr};
    size_t stage_bytes = 0;
    hipStream_t streams[2] = {nullptr, nullptr};
    int bs_id = -1;               // bit-sliced GF(2^8) kernel set, -1 if none
    uint8_t *d_syn = nullptr;     // decode workspace: syndromes of flagged codewords, [ncw][32]
    size_t syn_cap = 0;           // codewords the workspace can hold
};

namespace {

thread_local std::string g_last_error;

int hip_fail(hipError_t e, const char *what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return -ENODEV;
    return -EIO;
}

#define HIP_TRY(expr)                                          \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) return hip_fail(e_, #expr);      \
    } while (0)

// Standard field polynomial per symbol size (rs:75-89).
unsigned std_poly(unsigned mm) {
    static const unsigned p[17] = {0, 0, 0x7, 0xb, 0x13, 0x25, 0x43, 0x89, 0x11d, 0x211, 0x409,
                                   0x805, 0x1053, 0x201b, 0x4443, 0x8003, 0x1100b};
    return mm <= 16 ? p[mm] : 0;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

} // namespace

extern "C" {

int ezrs_abi_version(void) { return EZRS_ABI_VERSION; }

int ezrs_device_count(void) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    return n;
}

const char *ezrs_last_error(void) { return g_last_error.c_str(); }

int ezrs_create(ezrs_codec **out, unsigned symbol_bits, unsigned poly, unsigned fcr,
                unsigned prim, unsigned nroots, int dual, int device) {
    if (!out) return -EINVAL;
    *out = nullptr;
    CodecSpec spec{symbol_bits, poly, fcr, prim, nroots, dual ? 1 : 0};
    ezrs_codec *c = new (std::nothrow) ezrs_codec;
    if (!c) return -ENOMEM;
    if (!c->math.build(spec)) {
        delete c;
        g_last_error = "invalid RS codec parameters";
        return -EINVAL;
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0 || device < 0 || device >= ndev) {
        delete c;
        g_last_error = "no usable HIP device";
        return -ENODEV;
    }
    c->device = device;
    DeviceGuard g(device);
    const CodecMath &m = c->math;
    const size_t ntab = 2 * (size_t)(m.nn + 1) + (m.spec.nroots + 1);
    if ((e = hipMalloc(&c->d_tabs, ntab * sizeof(uint16_t))) != hipSuccess ||
        (e = hipMalloc(&c->d_dual, 512)) != hipSuccess) {
        ezrs_destroy(c);
        return hip_fail(e, "hipMalloc(tables)");
    }
    std::vector<uint16_t> h(ntab);
    std::copy(m.gf.alpha_to.begin(), m.gf.alpha_to.end(), h.begin());
    std::copy(m.gf.index_of.begin(), m.gf.index_of.end(), h.begin() + (m.nn + 1));
    std::copy(m.genpoly.begin(), m.genpoly.end(), h.begin() + 2 * (m.nn + 1));
    uint8_t dm[512];
    std::memcpy(dm, m.into_dual, 256);
    std::memcpy(dm + 256, m.from_dual, 256);
    if ((e = hipMemcpy(c->d_tabs, h.data(), ntab * sizeof(uint16_t), hipMemcpyHostToDevice)) !=
            hipSuccess ||
        (e = hipMemcpy(c->d_dual, dm, 512, hipMemcpyHostToDevice)) != hipSuccess) {
        ezrs_destroy(c);
        return hip_fail(e, "hipMemcpy(tables)");
    }
    DevCodec &d = c->dev;
    d.mm = m.spec.mm; d.nn = m.nn; d.nroots = m.spec.nroots; d.load = m.load;
    d.fcr = m.spec.fcr; d.prim = m.spec.prim; d.iprim = m.iprim; d.dual = m.spec.dual;
    d.poly = m.spec.poly;
    d.masked = m.spec.mm != (m.spec.mm <= 8 ? 8u : 16u);
    d.alpha_to = c->d_tabs;
    d.index_of = c->d_tabs + (m.nn + 1);
    d.genpoly = c->d_tabs + 2 * (m.nn + 1);
    d.into_dual = c->d_dual;
    d.from_dual = c->d_dual + 256;
    if (hipDeviceGetAttribute(&d.ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        d.ncu = 0;
    c->bs_id = bitslice_codec_id(d);
    *out = c;
    return 0;
}

int ezrs_create_rs(ezrs_codec **out, unsigned n, unsigned k, int device) {
    unsigned mm = 0;
    while (mm < 17 && ((1u << mm) - 1) < n) ++mm;
    if (mm < 2 || mm > 16 || ((1u << mm) - 1) != n || k == 0 || k >= n) {
        if (out) *out = nullptr;
        g_last_error = "RS<N,K>: N must be 2^m-1 (m = 2..16) and 0 < K < N";
        return -EINVAL;
    }
    return ezrs_create(out, mm, std_poly(mm), 1, 1, n - k, 0, device);
}

int ezrs_create_ccsds(ezrs_codec **out, unsigned k, int dual, int device) {
    if (k == 0 || k >= 255 || ((255 - k) & 1)) {
        if (out) *out = nullptr;
        g_last_error = "RS_CCSDS<255,K>: K must leave an even number of parity symbols";
        return -EINVAL;
    }
    return ezrs_create(out, 8, 0x187, 128 - (255 - k) / 2, 11, 255 - k, dual ? 1 : 0, device);
}

int ezrs_destroy(ezrs_codec *c) {
    if (!c) return 0;
    DeviceGuard g(c->device);
    (void)hipFree(c->d_tabs);
    (void)hipFree(c->d_dual);
    if (c->d_syn) (void)hipFree(c->d_syn);
    for (int i = 0; i < 2; ++i) {
        if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
        if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
        if (c->streams[i]) (void)hipStreamDestroy(c->streams[i]);
    }
    delete c;
    return 0;
}

int ezrs_get_info(const ezrs_codec *c, ezrs_info *info) {
    if (!c || !info) return -EINVAL;
    const CodecMath &m = c->math;
    info->symbol_bits = m.spec.mm;
    info->size = m.nn;
    info->nroots = m.spec.nroots;
    info->load = m.load;
    info->poly = m.spec.poly;
    info->fcr = m.spec.fcr;
    info->prim = m.spec.prim;
    info->datum_bytes = m.spec.mm <= 8 ? 1 : 2;
    info->dual = m.spec.dual;
    info->device = c->device;
    return 0;
}

namespace {

// Grow the flagged-codeword syndrome workspace (bit-sliced decode path only).
int reserve_syn(ezrs_codec *c, size_t ncw) {
    if (c->bs_id < 0 || ncw <= c->syn_cap) return 0;
    DeviceGuard g(c->device);
    if (c->d_syn) {
        HIP_TRY(hipDeviceSynchronize());
        (void)hipFree(c->d_syn);
        c->d_syn = nullptr;
        c->syn_cap = 0;
    }
    HIP_TRY(hipMalloc(&c->d_syn, bs_encode_ws_bytes(ncw)));   // >= ncw * 32 (decode's need)
    c->syn_cap = ncw;
    return 0;
}

} // namespace

namespace {

// The one place that picks kernels: every entry point (device or host-memory) goes through these.
// ws: bs_encode_ws_bytes(ncw) bytes (bit-sliced path only).
hipError_t dispatch_encode(const ezrs_codec *c, const EncodeArgs &a, void *ws, hipStream_t st) {
    return c->bs_id >= 0 ? launch_bs_encode(c->bs_id, c->dev, a, ws, st) : launch_encode_generic(c->dev, a, st);
}

// syn_ws: [ncw][32] bytes (bit-sliced path only).
hipError_t dispatch_decode(const ezrs_codec *c, const DecodeArgs &a, uint8_t *syn_ws,
                           hipStream_t st) {
    const unsigned w = c->dev.mm <= 8 ? 1 : 2;
    const bool contiguous = a.parity == static_cast<char *>(a.data) + (size_t)a.len * w &&
                            a.parity_stride == a.data_stride;
    if (c->bs_id >= 0 && contiguous) {
        // Bit-sliced syndromes for the whole batch; the reference algorithm only for the codewords
        // that are not valid as received (or carry erasures to validate).
        hipError_t e = launch_bs_syndromes(c->bs_id, c->dev, a, syn_ws, st);
        if (e == hipSuccess) e = launch_decode_flagged(c->dev, a, syn_ws, st);
        return e;
    }
    return launch_decode_generic(c->dev, a, st);
}

} // namespace

int ezrs_reserve(ezrs_codec *c, size_t ncw) {
    if (!c) return -EINVAL;
    return reserve_syn(c, ncw);
}

int ezrs_encode(const ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
                void *parity, size_t parity_stride, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!data) return -EINVAL;
    const unsigned w = c->dev.mm <= 8 ? 1 : 2;
    if (len < 1 || len > c->dev.load) return -EINVAL;                 // rs_base:875-877
    if (!parity) {
        parity = static_cast<char *>(const_cast<void *>(data)) + (size_t)len * w;
        parity_stride = data_stride;
        if (data_stride < (size_t)len + c->dev.nroots && ncw > 1) return -EINVAL;
    } else if (ncw > 1 && parity_stride < c->dev.nroots) {
        return -EINVAL;
    }
    if (ncw > 1 && data_stride < len) return -EINVAL;
    DeviceGuard g(c->device);
    EncodeArgs a{data, data_stride, len, parity, parity_stride, ncw};
    if (int r = reserve_syn(const_cast<ezrs_codec *>(c), ncw)) return r;
    hipError_t e = dispatch_encode(c, a, c->d_syn, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "encode launch");
    return 0;
}

int ezrs_decode(const ezrs_codec *c, void *data, size_t data_stride, unsigned len, void *parity,
                size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                const uint32_t *neras, int32_t *result, uint32_t *positions, size_t pos_stride,
                void *corr, size_t corr_stride, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!data || !result) return -EINVAL;
    const unsigned w = c->dev.mm <= 8 ? 1 : 2;
    const unsigned NR = c->dev.nroots;
    if (len < 1 || len > c->dev.load) return -EINVAL;
    if (!parity) {
        parity = static_cast<char *>(data) + (size_t)len * w;
        parity_stride = data_stride;
        if (ncw > 1 && data_stride < (size_t)len + NR) return -EINVAL;
    } else if (ncw > 1 && parity_stride < NR) {
        return -EINVAL;
    }
    if (ncw > 1 && data_stride < len) return -EINVAL;
    if (neras && !eras) return -EINVAL;
    if (positions && ncw > 1 && pos_stride < NR) return -EINVAL;
    if (corr && ncw > 1 && corr_stride < NR) return -EINVAL;
    DeviceGuard g(c->device);
    DecodeArgs a{data, data_stride, len, parity, parity_stride, eras, eras_stride, neras,
                 result, positions, pos_stride, corr, corr_stride, ncw};
    if (int r = reserve_syn(const_cast<ezrs_codec *>(c), ncw)) return r;
    hipError_t e = dispatch_decode(c, a, c->d_syn, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "decode launch");
    return 0;
}

// ---- host-memory pipeline ---------------------------------------------------------------------
namespace {

int ensure_stage(ezrs_codec *c, size_t bytes) {
    if (!c->streams[0])
        for (int i = 0; i < 2; ++i)
            HIP_TRY(hipStreamCreateWithFlags(&c->streams[i], hipStreamNonBlocking));
    if (c->stage_bytes >= bytes) return 0;
    for (int i = 0; i < 2; ++i) {
        if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
        c->d_stage[i] = nullptr;
    }
    c->stage_bytes = 0;
    for (int i = 0; i < 2; ++i) HIP_TRY(hipMalloc(&c->d_stage[i], bytes));
    c->stage_bytes = bytes;
    return 0;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t default_chunk(size_t row_bytes) {
    const size_t target = (size_t)64 << 20;  // 64 MiB of codewords per chunk
    size_t n = target / (row_bytes ? row_bytes : 1);
    return n ? n : 1;
}

} // namespace

int ezrs_encode_host(ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, size_t ncw, size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!data) return -EINVAL;
    const unsigned w = c->dev.mm <= 8 ? 1 : 2, NR = c->dev.nroots;
    if (len < 1 || len > c->dev.load) return -EINVAL;
    if (!parity) {
        parity = static_cast<char *>(const_cast<void *>(data)) + (size_t)len * w;
        parity_stride = data_stride;
    }
    if (ncw > 1 && (data_stride < len || parity_stride < NR)) return -EINVAL;
    // Parity inside the row (the common RS<N,K> layout): move whole rows with one linear copy per
    // chunk instead of a 2-D copy of ncw short rows (2-D copies from pageable memory go row by row).
    const bool inline_par = parity_stride == data_stride && data_stride >= (size_t)len + NR &&
                            static_cast<const char *>(parity) ==
                                static_cast<const char *>(data) + (size_t)len * w;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const size_t drow = inline_par ? data_stride : len;      // device row stride, symbols
    if (!chunk) chunk = default_chunk((size_t)(len + NR) * w);
    if (chunk > ncw) chunk = ncw;
    const size_t dbytes = align_up(chunk * drow * w), pbytes = align_up(chunk * NR * w),
                 wbytes = c->bs_id >= 0 ? align_up(bs_encode_ws_bytes(chunk)) : 0;
    if (int r = ensure_stage(c, dbytes + pbytes + wbytes)) return r;
    for (size_t i = 0, k0 = 0; k0 < ncw; ++i, k0 += chunk) {
        const int s = (int)(i & 1);
        hipStream_t st = c->streams[s];
        const size_t n = ncw - k0 < chunk ? ncw - k0 : chunk;
        if (i >= 2) HIP_TRY(hipStreamSynchronize(st));
        char *dd = static_cast<char *>(c->d_stage[s]), *dp = dd + dbytes;
        const char *hd = static_cast<const char *>(data) + k0 * data_stride * w;
        char *hp = static_cast<char *>(parity) + k0 * parity_stride * w;
        if (inline_par) {
            // the last row's tail past its parity may lie outside the caller's buffer
            HIP_TRY(hipMemcpyAsync(dd, hd, ((n - 1) * data_stride + len + NR) * w,
                                   hipMemcpyHostToDevice, st));
            EncodeArgs a{dd, data_stride, len, dd + (size_t)len * w, data_stride, n};
            HIP_TRY(dispatch_encode(c, a, dp + pbytes, st));
            // Rows go back whole: a 2-D copy of NR-symbol pieces at row pitch runs row by row
            // (6.8 s for 1M RS(255,223) rows, pinned or not); the data bytes written back are
            // the ones just read, unchanged.
            HIP_TRY(hipMemcpyAsync(const_cast<char *>(hd), dd, ((n - 1) * data_stride + len + NR) * w,
                                   hipMemcpyDeviceToHost, st));
            continue;
        }
        HIP_TRY(ezrs::copy2d(dd, (size_t)len * w, hd, data_stride * w, (size_t)len * w, n,
                                 hipMemcpyHostToDevice, st));
        EncodeArgs a{dd, len, len, dp, NR, n};
        HIP_TRY(dispatch_encode(c, a, dp + pbytes, st));
        HIP_TRY(ezrs::copy2d(hp, parity_stride * w, dp, (size_t)NR * w, (size_t)NR * w, n,
                                 hipMemcpyDeviceToHost, st));
    }
    for (int s = 0; s < 2; ++s) HIP_TRY(hipStreamSynchronize(c->streams[s]));
    return 0;
}

int ezrs_decode_host(ezrs_codec *c, void *data, size_t data_stride, unsigned len, void *parity,
                     size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                     const uint32_t *neras, int32_t *result, uint32_t *positions,
                     size_t pos_stride, void *corr, size_t corr_stride, size_t ncw, size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (!data || !result) return -EINVAL;
    const unsigned w = c->dev.mm <= 8 ? 1 : 2, NR = c->dev.nroots;
    if (len < 1 || len > c->dev.load) return -EINVAL;
    if (!parity) {
        parity = static_cast<char *>(data) + (size_t)len * w;
        parity_stride = data_stride;
    }
    if (ncw > 1 && (data_stride < len || parity_stride < NR)) return -EINVAL;
    if (neras && !eras) return -EINVAL;
    if (positions && ncw > 1 && pos_stride < NR) return -EINVAL;
    if (corr && ncw > 1 && corr_stride < NR) return -EINVAL;
    const size_t ecols = eras ? (eras_stride < NR ? eras_stride : NR) : 0;
    if (eras && ecols == 0 && ncw > 1) return -EINVAL;
    const bool inline_par = parity_stride == data_stride && data_stride >= (size_t)len + NR &&
                            static_cast<const char *>(parity) ==
                                static_cast<const char *>(data) + (size_t)len * w;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    // device row: the caller's whole row when parity is inline (one linear copy each way)
    const size_t row = inline_par ? data_stride * w : (size_t)(len + NR) * w;
    if (!chunk) chunk = default_chunk(row);
    if (chunk > ncw) chunk = ncw;
    const size_t b_cw = align_up(chunk * row), b_er = align_up(chunk * ecols * 4),
                 b_ne = align_up(neras ? chunk * 4 : 0), b_rs = align_up(chunk * 4),
                 b_ps = align_up(positions ? chunk * NR * 4 : 0),
                 b_co = align_up(corr ? chunk * NR * w : 0),
                 b_sy = align_up(c->bs_id >= 0 ? chunk * 32 : 0);
    if (int r = ensure_stage(c, b_cw + b_er + b_ne + b_rs + b_ps + b_co + b_sy)) return r;
    for (size_t i = 0, k0 = 0; k0 < ncw; ++i, k0 += chunk) {
        const int s = (int)(i & 1);
        hipStream_t st = c->streams[s];
        const size_t n = ncw - k0 < chunk ? ncw - k0 : chunk;
        if (i >= 2) HIP_TRY(hipStreamSynchronize(st));
        char *base = static_cast<char *>(c->d_stage[s]);
        char *dcw = base, *der = dcw + b_cw, *dne = der + b_er, *drs = dne + b_ne, *dps = drs + b_rs,
             *dco = dps + b_ps, *dsy = dco + b_co;
        char *hd = static_cast<char *>(data) + k0 * data_stride * w;
        char *hp = static_cast<char *>(parity) + k0 * parity_stride * w;
        const size_t span = ((n - 1) * data_stride + len + NR) * w;
        if (inline_par) {
            HIP_TRY(hipMemcpyAsync(dcw, hd, span, hipMemcpyHostToDevice, st));
        } else {
            HIP_TRY(ezrs::copy2d(dcw, row, hd, data_stride * w, (size_t)len * w, n,
                                     hipMemcpyHostToDevice, st));
            HIP_TRY(ezrs::copy2d(dcw + (size_t)len * w, row, hp, parity_stride * w,
                                     (size_t)NR * w, n, hipMemcpyHostToDevice, st));
        }
        if (eras)
            HIP_TRY(ezrs::copy2d(der, ecols * 4, eras + k0 * eras_stride, eras_stride * 4,
                                     ecols * 4, n, hipMemcpyHostToDevice, st));
        if (neras) HIP_TRY(hipMemcpyAsync(dne, neras + k0, n * 4, hipMemcpyHostToDevice, st));
        if (positions)
            HIP_TRY(ezrs::copy2d(dps, (size_t)NR * 4, positions + k0 * pos_stride,
                                     pos_stride * 4, (size_t)NR * 4, n, hipMemcpyHostToDevice, st));
        if (corr)   // corr is copy-in/copy-out: entries the decode does not write keep their value
            HIP_TRY(ezrs::copy2d(dco, (size_t)NR * w, static_cast<char *>(corr) + k0 * corr_stride * w,
                                     corr_stride * w, (size_t)NR * w, n, hipMemcpyHostToDevice, st));
        const size_t ds = row / w;
        DecodeArgs a{dcw, ds, len, dcw + (size_t)len * w, ds,
                     eras ? reinterpret_cast<uint32_t *>(der) : nullptr, ecols,
                     neras ? reinterpret_cast<uint32_t *>(dne) : nullptr,
                     reinterpret_cast<int32_t *>(drs),
                     positions ? reinterpret_cast<uint32_t *>(dps) : nullptr, NR,
                     corr ? dco : nullptr, NR, n};
        HIP_TRY(dispatch_decode(c, a, reinterpret_cast<uint8_t *>(dsy), st));
        if (inline_par) {
            HIP_TRY(hipMemcpyAsync(hd, dcw, span, hipMemcpyDeviceToHost, st));
        } else {
            HIP_TRY(ezrs::copy2d(hd, data_stride * w, dcw, row, (size_t)len * w, n,
                                     hipMemcpyDeviceToHost, st));
            HIP_TRY(ezrs::copy2d(hp, parity_stride * w, dcw + (size_t)len * w, row,
                                     (size_t)NR * w, n, hipMemcpyDeviceToHost, st));
        }
        HIP_TRY(hipMemcpyAsync(result + k0, drs, n * 4, hipMemcpyDeviceToHost, st));
        if (positions)
            HIP_TRY(ezrs::copy2d(positions + k0 * pos_stride, pos_stride * 4, dps,
                                     (size_t)NR * 4, (size_t)NR * 4, n, hipMemcpyDeviceToHost, st));
        if (corr)
            HIP_TRY(ezrs::copy2d(static_cast<char *>(corr) + k0 * corr_stride * w, corr_stride * w,
                                     dco, (size_t)NR * w, (size_t)NR * w, n, hipMemcpyDeviceToHost, st));
    }
    for (int s = 0; s < 2; ++s) HIP_TRY(hipStreamSynchronize(c->streams[s]));
    return 0;
}

int ezrs_host_alloc(void **ptr, size_t bytes) {
    if (!ptr) return -EINVAL;
    HIP_TRY(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
    return 0;
}

int ezrs_host_free(void *ptr) {
    if (ptr) HIP_TRY(hipHostFree(ptr));
    return 0;
}

} // extern "C"
