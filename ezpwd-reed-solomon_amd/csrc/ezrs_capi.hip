// ezrs_capi.hip -- the C ABI of the MI355X RS engine (include/ezrs.h).
//
// Codec objects own their device-resident tables (built once, like the reference's static
// reed_solomon_tabs / genpoly, rs_base:599-635, 1248-1286) and a decode workspace.  Batch entry
// points validate arguments the way the reference's encode<INP>/decode<INP> do
// (rs_base:868-904, 1170-1242) and dispatch to the fastest kernel that is bit-exact for the codec:
// the bit-sliced GF(2^8) kernels where they apply, the generic per-codeword kernels otherwise.
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

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
    size_t stage_bytes = 0;       // device bytes of each d_stage buffer
    size_t hstage_bytes = 0;      // pinned host bytes of each h_stage buffer
    hipStream_t streams[2] = {nullptr, nullptr};
    int bs_id = -1;               // bit-sliced GF(2^8) kernel set, -1 if none
    int ps_id = -1;               // plane-sliced GF(2^8) kernel set, -1 if none
    int wide_id = -1;             // GF(2^16) remainder kernel set, -1 if none
    mutable std::atomic<uint32_t> decode_gen{0};   // plane-sliced decode calls (DecodeArgs::flag_gen)
    std::vector<uint16_t> wide_blob;   // host: leader slots | log beta | column tables
    uint16_t *d_wcols = nullptr;  // device copy of the column tables (constant multipliers)
    // Device workspaces of the batch entry points, one per HIP stream: calls on different streams
    // never share scratch memory, calls on one stream are ordered by the stream.  A workspace only
    // grows; the buffer it replaces is kept until ezrs_destroy, so work already queued (or a
    // captured graph) that still points at it stays valid.  No entry point synchronises the device.
    struct Ws {
        void *p = nullptr;
        size_t bytes = 0;
    };
    mutable std::mutex ws_mu;
    mutable std::unordered_map<void *, Ws> ws;
    mutable std::vector<void *> ws_retired;
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
    if (symbol_bits > 8 && nroots > 256) {
        // the wide-symbol kernels keep at most 256 parity symbols' working state per lane
        delete c;
        g_last_error = "RS codecs with symbols wider than 8 bits support at most 256 parity symbols";
        return -ENOTSUP;
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
    // EZRS_NO_PLANESLICE=1 keeps the per-symbol bit-sliced kernels (A/B measurements)
    const char *nops = getenv("EZRS_NO_PLANESLICE");
    c->ps_id = (nops && *nops == '1') ? -1 : planeslice_codec_id(d);
    // EZRS_NO_WIDE=1 keeps the lane-group GF(2^16) kernels (A/B measurements)
    const char *now = getenv("EZRS_NO_WIDE");
    c->wide_id = (now && *now == '1') ? -1 : wide_codec_id(d);
    if (c->wide_id >= 0) {
        if (!wide_build_consts(c->wide_id, m, c->wide_blob)) {
            c->wide_id = -1;
        } else {
            const size_t qn = wide_cols_count(m.spec.nroots);
            if ((e = hipMalloc(&c->d_wcols, qn * sizeof(uint16_t))) != hipSuccess ||
                (e = hipMemcpy(c->d_wcols, c->wide_blob.data() + 64, qn * sizeof(uint16_t),
                               hipMemcpyHostToDevice)) != hipSuccess) {
                ezrs_destroy(c);
                return hip_fail(e, "hipMalloc(wide tables)");
            }
        }
    }
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
    if (c->d_wcols) (void)hipFree(c->d_wcols);
    for (auto &kv : c->ws) (void)hipFree(kv.second.p);
    for (void *p : c->ws_retired) (void)hipFree(p);
    for (int i = 0; i < 2; ++i) {
        if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
        if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
        if (c->streams[i]) (void)hipStreamDestroy(c->streams[i]);
    }
    delete c;
    return 0;
}

int ezrs_set_semantics(ezrs_codec *c, int semantics) {
    if (!c || (semantics != EZRS_SEM_EZPWD && semantics != EZRS_SEM_KARN)) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->dev.karn = semantics == EZRS_SEM_KARN;
    return 0;
}

int ezrs_set_launch_rows(ezrs_codec *c, size_t rows) {
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    c->dev.launch_rows = rows;
    return 0;
}

int ezrs_get_semantics(const ezrs_codec *c) {
    if (!c) return -EINVAL;
    return c->dev.karn ? EZRS_SEM_KARN : EZRS_SEM_EZPWD;
}

int ezrs_kernel_path(const ezrs_codec *c) {
    if (!c) return -EINVAL;
    if (c->ps_id >= 0) return EZRS_PATH_PLANESLICE;
    if (c->wide_id >= 0) return EZRS_PATH_WIDE;
    if (c->bs_id >= 0) return EZRS_PATH_BITSLICE;
    return EZRS_PATH_GENERIC;
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

// Device scratch bytes one batch call of ncw codewords needs (encode and decode alike).
size_t ws_bytes_for(const ezrs_codec *c, size_t ncw) {
    size_t b = 0;                                          // both >= ncw * 32 (decode's need)
    if (c->bs_id >= 0) b = bs_encode_ws_bytes(ncw);
    if (c->ps_id >= 0 && ps_ws_bytes(ncw) + 256 > b) b = ps_ws_bytes(ncw) + 256;   // + the flag word
    if (c->wide_id >= 0 && wide_ws_bytes(c->wide_id, ncw) > b) b = wide_ws_bytes(c->wide_id, ncw);
    return b;
}

// The calling stream's workspace, grown to at least `bytes` (see ezrs_codec::Ws).
int stream_ws(const ezrs_codec *c, void *stream, size_t bytes, void **out) {
    *out = nullptr;
    if (!bytes) return 0;
    std::lock_guard<std::mutex> lk(c->ws_mu);
    ezrs_codec::Ws &w = c->ws[stream];
    if (w.bytes < bytes) {
        const size_t grow = w.bytes + w.bytes / 2 > bytes ? w.bytes + w.bytes / 2 : bytes;
        void *p = nullptr;
        HIP_TRY(hipMalloc(&p, grow));
        if (w.p) c->ws_retired.push_back(w.p);
        w.p = p;
        w.bytes = grow;
    }
    *out = w.p;
    return 0;
}

} // namespace

namespace {

// The one place that picks kernels: every entry point (device or host-memory) goes through these.
// ws: bs_encode_ws_bytes(ncw) bytes (bit-sliced path only).
hipError_t dispatch_encode(const ezrs_codec *c, const EncodeArgs &a, void *ws, hipStream_t st) {
    if (c->ps_id >= 0 && ps_can_encode(c->dev, a)) return launch_ps_encode(c->ps_id, c->dev, a, ws, st);
    if (a.sh.rows) return launch_encode_generic(c->dev, a, st);     // shard rows: per-codeword kernels
    if (c->wide_id >= 0 && wide_can_encode(c->dev, a))
        return launch_wide_encode(c->wide_id, c->dev, a, c->wide_blob.data(), c->d_wcols, ws, st);
    return c->bs_id >= 0 ? launch_bs_encode(c->bs_id, c->dev, a, ws, st) : launch_encode_generic(c->dev, a, st);
}

// syn_ws: the sliced paths' syndrome workspace (ws_bytes_for).
hipError_t dispatch_decode(const ezrs_codec *c, const DecodeArgs &a, uint8_t *syn_ws,
                           hipStream_t st) {
    const unsigned w = c->dev.mm <= 8 ? 1 : 2;
    const bool contiguous = a.parity == static_cast<char *>(a.data) + (size_t)a.len * w &&
                            a.parity_stride == a.data_stride;
    if (c->ps_id >= 0 && ps_can_decode(c->dev, a)) {
        // the call's flag word (after the tiled syndromes) and a value no earlier call stored there
        // (a stale match only costs the error path's full screen)
        DecodeArgs b = a;
        b.flag_word = reinterpret_cast<uint32_t *>(syn_ws + ps_ws_bytes(a.ncw));
        b.flag_gen = c->decode_gen.fetch_add(1, std::memory_order_relaxed) + 1;
        hipError_t e = launch_ps_syndromes(c->ps_id, c->dev, b, syn_ws, st);
        if (e == hipSuccess) e = launch_decode_flagged(c->dev, b, syn_ws, SynLayout::Tiled, st);
        return e;
    }
    if (a.sh.rows) return launch_decode_generic(c->dev, a, st);     // shard rows: per-codeword kernels
    // the GF(2^16) error path keeps ezpwd's semantics only: Karn-mode codecs decode on the
    // per-codeword kernels (same syndromes, Karn's frame and checks)
    if (c->wide_id >= 0 && !c->dev.karn && wide_can_decode(c->dev, a))
        return launch_wide_decode(c->wide_id, c->dev, a, c->wide_blob.data(), c->d_wcols, syn_ws, st);
    if (c->bs_id >= 0 && contiguous) {
        // Bit-sliced syndromes for the whole batch; the reference algorithm only for the codewords
        // that are not valid as received (or carry erasures to validate).
        hipError_t e = launch_bs_syndromes(c->bs_id, c->dev, a, syn_ws, st);
        if (e == hipSuccess) e = launch_decode_flagged(c->dev, a, syn_ws, SynLayout::Rows, st);
        return e;
    }
    return launch_decode_generic(c->dev, a, st);
}

} // namespace

int ezrs_reserve(ezrs_codec *c, size_t ncw) { return ezrs_reserve_stream(c, ncw, nullptr); }

int ezrs_reserve_stream(const ezrs_codec *c, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    DeviceGuard g(c->device);
    void *p;
    return stream_ws(c, stream, ws_bytes_for(c, ncw), &p);
}

size_t ezrs_workspace_bytes(const ezrs_codec *c, size_t ncw) {
    return c ? ws_bytes_for(c, ncw) : 0;
}

namespace {

// Argument checks of encode<INP> (rs_base:868-904) for a batch with a separate parity array.
int check_encode(const ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
                 const void *parity, size_t parity_stride, size_t ncw) {
    if (!c || !data || !parity) return -EINVAL;
    if (len < 1 || len > c->dev.load) return -EINVAL;                 // rs_base:875-877
    if (ncw > 1 && (parity_stride < c->dev.nroots || data_stride < len)) return -EINVAL;
    return 0;
}

// Row form (rs_base:778-790): the parity follows the data in each row.
int check_rows(const ezrs_codec *c, const void *rows, size_t stride, unsigned len, size_t ncw) {
    if (!c || !rows) return -EINVAL;
    if (len < 1 || len > c->dev.load) return -EINVAL;
    if (ncw > 1 && stride < (size_t)len + c->dev.nroots) return -EINVAL;
    return 0;
}

int encode_dev(const ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
               void *parity, size_t parity_stride, size_t ncw, void *ws, size_t ws_bytes,
               void *stream) {
    if (ws_bytes < ws_bytes_for(c, ncw) || (ws_bytes && !ws)) return -EINVAL;
    DeviceGuard g(c->device);
    EncodeArgs a{data, data_stride, len, parity, parity_stride, ncw};
    hipError_t e = dispatch_encode(c, a, ws, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "encode launch");
    return 0;
}

int check_decode(const ezrs_codec *c, void *data, size_t data_stride, unsigned len,
                 void *&parity, size_t &parity_stride, const uint32_t *eras, size_t eras_stride,
                 const uint32_t *neras, int32_t *result, uint32_t *positions, size_t pos_stride,
                 void *corr, size_t corr_stride, size_t ncw) {
    if (!c || !data || !result) return -EINVAL;
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
    if (eras && ncw > 1 && eras_stride == 0) return -EINVAL;
    if (positions && ncw > 1 && pos_stride < NR) return -EINVAL;
    if (corr && ncw > 1 && corr_stride < NR) return -EINVAL;
    return 0;
}

} // namespace

int ezrs_encode_ws(const ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
                   void *parity, size_t parity_stride, size_t ncw, void *ws, size_t ws_bytes,
                   void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_encode(c, data, data_stride, len, parity, parity_stride, ncw)) return r;
    return encode_dev(c, data, data_stride, len, parity, parity_stride, ncw, ws, ws_bytes, stream);
}

int ezrs_encode(const ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
                void *parity, size_t parity_stride, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_encode(c, data, data_stride, len, parity, parity_stride, ncw)) return r;
    DeviceGuard g(c->device);
    const size_t need = ws_bytes_for(c, ncw);
    void *ws = nullptr;
    if (int r = stream_ws(c, stream, need, &ws)) return r;
    return encode_dev(c, data, data_stride, len, parity, parity_stride, ncw, ws, need, stream);
}

int ezrs_encode_rows_ws(const ezrs_codec *c, void *rows, size_t stride, unsigned len, size_t ncw,
                        void *ws, size_t ws_bytes, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_rows(c, rows, stride, len, ncw)) return r;
    char *r0 = static_cast<char *>(rows);
    const size_t w = c->dev.mm <= 8 ? 1 : 2;
    return encode_dev(c, r0, stride, len, r0 + (size_t)len * w, stride, ncw, ws, ws_bytes, stream);
}

int ezrs_encode_rows(const ezrs_codec *c, void *rows, size_t stride, unsigned len, size_t ncw,
                     void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_rows(c, rows, stride, len, ncw)) return r;
    DeviceGuard g(c->device);
    const size_t need = ws_bytes_for(c, ncw);
    void *ws = nullptr;
    if (int r = stream_ws(c, stream, need, &ws)) return r;
    return ezrs_encode_rows_ws(c, rows, stride, len, ncw, ws, need, stream);
}

int ezrs_decode_ws(const ezrs_codec *c, void *data, size_t data_stride, unsigned len,
                   void *parity, size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                   const uint32_t *neras, int32_t *result, uint32_t *positions, size_t pos_stride,
                   void *corr, size_t corr_stride, size_t ncw, void *ws, size_t ws_bytes,
                   void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_decode(c, data, data_stride, len, parity, parity_stride, eras, eras_stride,
                             neras, result, positions, pos_stride, corr, corr_stride, ncw))
        return r;
    if (ws_bytes < ws_bytes_for(c, ncw) || (ws_bytes && !ws)) return -EINVAL;
    DeviceGuard g(c->device);
    // one codeword: a zero eras_stride is harmless (row 0 only)
    DecodeArgs a{data, data_stride, len, parity, parity_stride, eras, eras_stride, neras,
                 result, positions, pos_stride, corr, corr_stride, ncw};
    hipError_t e = dispatch_decode(c, a, static_cast<uint8_t *>(ws), static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "decode launch");
    return 0;
}

int ezrs_decode(const ezrs_codec *c, void *data, size_t data_stride, unsigned len, void *parity,
                size_t parity_stride, const uint32_t *eras, size_t eras_stride,
                const uint32_t *neras, int32_t *result, uint32_t *positions, size_t pos_stride,
                void *corr, size_t corr_stride, size_t ncw, void *stream) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    DeviceGuard g(c->device);
    const size_t need = ws_bytes_for(c, ncw);
    void *ws = nullptr;
    if (int r = stream_ws(c, stream, need, &ws)) return r;
    return ezrs_decode_ws(c, data, data_stride, len, parity, parity_stride, eras, eras_stride,
                          neras, result, positions, pos_stride, corr, corr_stride, ncw, ws, need,
                          stream);
}

// ---- shard batches -----------------------------------------------------------------------------
namespace {

// Rows per shard and the geometry of a shard batch (rsencode layout); false on bad arguments.
bool shard_geom(const ezrs_codec *c, size_t shard_len, unsigned chunk, size_t shard_pitch, Shards &g) {
    if (!c || shard_len == 0 || chunk == 0 || chunk > c->dev.load) return false;
    const size_t R = (shard_len + chunk - 1) / chunk;
    if (R > 0xFFFFFFFFu) return false;
    const size_t enc = shard_len + R * c->dev.nroots;
    if (shard_pitch < enc) return false;
    g.rows = (uint32_t)R;
    g.tail = (uint32_t)(shard_len - (R - 1) * chunk);
    g.pitch = shard_pitch;
    return true;
}

} // namespace

size_t ezrs_shard_codewords(const ezrs_codec *c, size_t shard_len, unsigned chunk) {
    if (!c || shard_len == 0 || chunk == 0 || chunk > c->dev.load) return 0;
    return (shard_len + chunk - 1) / chunk;
}

size_t ezrs_shard_encoded_len(const ezrs_codec *c, size_t shard_len, unsigned chunk) {
    const size_t R = ezrs_shard_codewords(c, shard_len, chunk);
    return R ? shard_len + R * c->dev.nroots : 0;
}

int ezrs_encode_shards(const ezrs_codec *c, void *shards, size_t shard_pitch, size_t shard_len,
                       unsigned chunk, size_t nshards, void *stream) {
    Shards g;
    if (!c || !shards || !shard_geom(c, shard_len, chunk, shard_pitch, g)) return -EINVAL;
    if (nshards == 0) return 0;
    const size_t w = c->dev.mm <= 8 ? 1 : 2, ncw = nshards * g.rows;
    DeviceGuard dg(c->device);
    const size_t need = ws_bytes_for(c, ncw);
    void *ws = nullptr;
    if (int r = stream_ws(c, stream, need, &ws)) return r;
    char *r0 = static_cast<char *>(shards);
    EncodeArgs a{r0, (size_t)chunk + c->dev.nroots, chunk, r0 + (size_t)chunk * w,
                 (size_t)chunk + c->dev.nroots, ncw, g};
    hipError_t e = dispatch_encode(c, a, ws, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "encode launch");
    return 0;
}

int ezrs_decode_shards(const ezrs_codec *c, void *shards, size_t shard_pitch, size_t shard_len,
                       unsigned chunk, size_t nshards, const uint32_t *eras, size_t eras_stride,
                       const uint32_t *neras, int32_t *result, uint32_t *positions,
                       size_t pos_stride, void *corr, size_t corr_stride, void *stream) {
    Shards g;
    if (!c || !shards || !result || !shard_geom(c, shard_len, chunk, shard_pitch, g)) return -EINVAL;
    if (nshards == 0) return 0;
    const unsigned NR = c->dev.nroots;
    const size_t w = c->dev.mm <= 8 ? 1 : 2, ncw = nshards * g.rows;
    if (neras && !eras) return -EINVAL;
    if (eras && ncw > 1 && eras_stride == 0) return -EINVAL;
    if (positions && ncw > 1 && pos_stride < NR) return -EINVAL;
    if (corr && ncw > 1 && corr_stride < NR) return -EINVAL;
    DeviceGuard dg(c->device);
    const size_t need = ws_bytes_for(c, ncw);
    void *ws = nullptr;
    if (int r = stream_ws(c, stream, need, &ws)) return r;
    char *r0 = static_cast<char *>(shards);
    DecodeArgs a{r0, (size_t)chunk + NR, chunk, r0 + (size_t)chunk * w, (size_t)chunk + NR, eras,
                 eras_stride, neras, result, positions, pos_stride, corr, corr_stride, ncw, g};
    hipError_t e = dispatch_decode(c, a, static_cast<uint8_t *>(ws), static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "decode launch");
    return 0;
}

// ---- host-memory pipeline ---------------------------------------------------------------------
namespace {

// Rows whose decode result is nonzero, compacted straight into pinned host memory (the kernel's
// stores cross PCIe; nothing to copy back afterwards): *cnt (device) counts them, hix[j] = chunk-
// relative row index of compacted row j (in no particular order), hout + j * pitch = its bytes,
// pitch = row_bytes rounded up to 16.  *cnt must be zero on entry.
__global__ void __launch_bounds__(256) k_compact_rows(const int32_t *result, size_t n, const char *rows,
                                                      size_t row_bytes, uint32_t *cnt, uint32_t *hix,
                                                      char *hout, size_t pitch) {
    __shared__ uint32_t slot[256];
    const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
    const bool mine = k < n && result[k] != 0;
    slot[threadIdx.x] = mine ? atomicAdd(cnt, 1u) : 0xFFFFFFFFu;
    if (mine) hix[slot[threadIdx.x]] = (uint32_t)k;
    __syncthreads();
    // the block copies its flagged rows, one row per wavefront at a time, 16 bytes per lane (byte
    // loads: rows of any length and alignment; one 16-byte store into the padded host row)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int t = wave; t < 256; t += 4) {
        const uint32_t sl = slot[t];
        if (sl == 0xFFFFFFFFu) continue;
        const unsigned char *src = reinterpret_cast<const unsigned char *>(rows) + ((size_t)blockIdx.x * 256 + t) * row_bytes;
        char *dst = hout + (size_t)sl * pitch;
        for (size_t b = 16 * (size_t)lane; b < row_bytes; b += 16 * 64) {
            uint32_t v[4] = {0, 0, 0, 0};
            if (b + 16 <= row_bytes) {
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q >> 2] |= (uint32_t)src[b + q] << (8 * (q & 3));
            } else {
                for (size_t q = 0; b + q < row_bytes; ++q) v[q >> 2] |= (uint32_t)src[b + q] << (8 * (q & 3));
            }
            *reinterpret_cast<uint4 *>(dst + b) = make_uint4(v[0], v[1], v[2], v[3]);
        }
    }
}

hipError_t launch_compact_rows(const int32_t *result, size_t n, const char *rows, size_t row_bytes,
                               uint32_t *cnt, uint32_t *hix, char *hout, size_t pitch, hipStream_t st) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_compact_rows, dim3(grid), dim3(256), 0, st, result, n, rows, row_bytes, cnt, hix,
                       hout, pitch);
    return hipGetLastError();
}

// Device and pinned-host staging of the host-memory forms: two sets (one per pipeline stream).
int ensure_stage(ezrs_codec *c, size_t dbytes, size_t hbytes) {
    if (!c->streams[0])
        for (int i = 0; i < 2; ++i)
            HIP_TRY(hipStreamCreateWithFlags(&c->streams[i], hipStreamNonBlocking));
    if (c->stage_bytes < dbytes) {
        for (int i = 0; i < 2; ++i) {
            if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
            c->d_stage[i] = nullptr;
        }
        c->stage_bytes = 0;
        for (int i = 0; i < 2; ++i) HIP_TRY(hipMalloc(&c->d_stage[i], dbytes));
        c->stage_bytes = dbytes;
    }
    if (c->hstage_bytes < hbytes) {
        for (int i = 0; i < 2; ++i) {
            if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
            c->h_stage[i] = nullptr;
        }
        c->hstage_bytes = 0;
        for (int i = 0; i < 2; ++i) HIP_TRY(hipHostMalloc(&c->h_stage[i], hbytes, hipHostMallocMapped));   // device-visible: k_compact_rows writes here
        c->hstage_bytes = hbytes;
    }
    return 0;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Host threads for the CPU-side scatters of the host-memory forms (EZRS_HOST_THREADS, default 8).
size_t host_threads() {
    static const size_t n = [] {
        const char *e = getenv("EZRS_HOST_THREADS");
        const long v = e ? atol(e) : 8;
        return (size_t)(v < 1 ? 1 : v > 64 ? 64 : v);
    }();
    return n;
}

// Pinned (page-locked) host memory?  Pageable copies go through the runtime's own staging, which
// pipelines badly on single large copies: they get smaller chunks.
bool host_pinned(const void *p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

size_t default_chunk(size_t row_bytes, bool pinned = true) {
    // staged rows per chunk: 64 MiB from pinned memory, 32 MiB from pageable (measured, 1 M
    // RS(255,223) rows: pageable decode 17.5 ms at 64 MiB, 6.6 ms at 32 MiB; pinned 5.4 / 6.9)
    const size_t target = (size_t)(pinned ? 64 : 32) << 20;
    size_t n = target / (row_bytes ? row_bytes : 1);
    return n ? n : 1;
}

// Encode of host rows.  PCIe traffic: the rows' data symbols go to the device (one linear copy
// of the rows' span when the row pitch is at most twice what a row needs, otherwise a CPU gather
// into pinned staging first), the kernel writes the parity as one compact [n][NR] block, and only
// that block comes back (a linear copy; a CPU scatter puts each row's NR symbols in place unless
// the caller's parity array is itself compact).  The caller's data symbols are never written.
//   rows != NULL: the rs_base:778-790 row form, parity at rows + len (data is rows)
int encode_host_core(ezrs_codec *c, const char *data, size_t data_stride, unsigned len,
                     char *parity, size_t parity_stride, size_t ncw, size_t chunk) {
    const size_t w = c->dev.mm <= 8 ? 1 : 2, NR = c->dev.nroots;
    const size_t need = (size_t)len;                               // symbols a row must carry over
    const bool span = ncw == 1 || data_stride <= 2 * need + NR;    // linear copy of the rows' span
    // device row pitch (symbols); a single row is staged at pitch len whatever its stride (a stride
    // below len, 0 included, is legal for one codeword and must not size the staging)
    const size_t drow = ncw == 1 ? need : span ? data_stride : need;
    const bool par_direct = parity_stride == NR || ncw == 1;       // caller's parity is compact
    if (!chunk) chunk = default_chunk(drow * w, host_pinned(data));
    if (chunk > ncw) chunk = ncw;
    const size_t b_in = align_up(chunk * drow * w), b_par = align_up(chunk * NR * w),
                 b_ws = align_up(ws_bytes_for(c, chunk));
    const size_t h_in = span ? 0 : align_up(chunk * need * w), h_par = par_direct ? 0 : b_par;
    if (int r = ensure_stage(c, b_in + b_par + b_ws, h_in + h_par + 256)) return r;
    struct Pending { size_t k0 = 0, n = 0; bool live = false; } pend[2];
    // scatter of a chunk's compact parity into the caller's rows: split over host threads (a
    // single thread writing 32-byte pieces into 1 M rows takes ~5 ms, 2x the copy itself)
    auto scatter = [&](int s) {
        if (!pend[s].live || par_direct) return;
        const char *src = static_cast<const char *>(c->h_stage[s]) + h_in;
        const size_t n = pend[s].n, k0 = pend[s].k0;
        auto part = [&](size_t r0, size_t r1) {
            for (size_t r = r0; r < r1; ++r)
                std::memcpy(parity + (k0 + r) * parity_stride * w, src + r * NR * w, NR * w);
        };
        const size_t nt = n >= 65536 ? host_threads() : 1;
        if (nt <= 1) {
            part(0, n);
            return;
        }
        std::vector<std::thread> th;
        for (size_t t = 1; t < nt; ++t) th.emplace_back(part, n * t / nt, n * (t + 1) / nt);
        part(0, n / nt);
        for (auto &x : th) x.join();
    };
    for (size_t i = 0, k0 = 0; k0 < ncw; ++i, k0 += chunk) {
        const int s = (int)(i & 1);
        hipStream_t st = c->streams[s];
        const size_t n = ncw - k0 < chunk ? ncw - k0 : chunk;
        if (pend[s].live) {
            HIP_TRY(hipStreamSynchronize(st));
            scatter(s);
            pend[s].live = false;
        }
        char *d_in = static_cast<char *>(c->d_stage[s]), *d_par = d_in + b_in, *d_ws = d_par + b_par;
        char *hs = static_cast<char *>(c->h_stage[s]);
        const char *hd = data + k0 * data_stride * w;
        if (span) {
            HIP_TRY(hipMemcpyAsync(d_in, hd, ((n - 1) * data_stride + need) * w,
                                   hipMemcpyHostToDevice, st));
        } else {
            for (size_t r = 0; r < n; ++r) std::memcpy(hs + r * need * w, hd + r * data_stride * w, need * w);
            HIP_TRY(hipMemcpyAsync(d_in, hs, n * need * w, hipMemcpyHostToDevice, st));
        }
        EncodeArgs a{d_in, drow, len, d_par, NR, n};
        HIP_TRY(dispatch_encode(c, a, d_ws, st));
        if (par_direct)
            HIP_TRY(hipMemcpyAsync(parity + k0 * NR * w, d_par, n * NR * w, hipMemcpyDeviceToHost, st));
        else
            HIP_TRY(hipMemcpyAsync(hs + h_in, d_par, n * NR * w, hipMemcpyDeviceToHost, st));
        pend[s] = {k0, n, true};
    }
    for (int s = 0; s < 2; ++s) {
        HIP_TRY(hipStreamSynchronize(c->streams[s]));
        scatter(s);
    }
    return 0;
}

} // namespace

int ezrs_encode_host(ezrs_codec *c, const void *data, size_t data_stride, unsigned len,
                     void *parity, size_t parity_stride, size_t ncw, size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r = check_encode(c, data, data_stride, len, parity, parity_stride, ncw)) {
        if (!parity)
            g_last_error = "ezrs_encode_host: parity is required (rows that carry their own parity: "
                           "ezrs_encode_rows_host)";
        return r;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    return encode_host_core(c, static_cast<const char *>(data), data_stride, len,
                            static_cast<char *>(parity), parity_stride, ncw, chunk);
}

int ezrs_encode_rows_host(ezrs_codec *c, void *rows, size_t stride, unsigned len, size_t ncw,
                          size_t chunk) {
    if (!c) return -EINVAL;
    if (ncw == 0) return 0;
    if (int r0 = check_rows(c, rows, stride, len, ncw)) return r0;
    const size_t w = c->dev.mm <= 8 ? 1 : 2;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    char *r = static_cast<char *>(rows);
    return encode_host_core(c, r, stride, len, r + (size_t)len * w, stride, ncw, chunk);
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
    // erasure columns to stage: the row stride (capped at NR); a single codeword may pass
    // eras_stride 0, and then carries neras[0] entries
    size_t ecols = eras ? (eras_stride < NR ? eras_stride : NR) : 0;
    if (eras && ncw == 1 && eras_stride == 0) ecols = neras ? (neras[0] < NR ? neras[0] : NR) : 0;
    if (eras && ecols == 0 && ncw > 1) return -EINVAL;
    if (eras && ecols == 0) eras = nullptr, neras = nullptr;
    const bool inline_par = parity_stride == data_stride && data_stride >= (size_t)len + NR &&
                            static_cast<const char *>(parity) ==
                                static_cast<const char *>(data) + (size_t)len * w;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    // device row: the caller's whole row when parity is inline (one linear copy in)
    const size_t row = inline_par ? data_stride * w : (size_t)(len + NR) * w;
    if (!chunk) chunk = default_chunk(row, host_pinned(data));
    if (chunk > ncw) chunk = ncw;
    const size_t b_cw = align_up(chunk * row), b_er = align_up(chunk * ecols * 4),
                 b_ne = align_up(neras ? chunk * 4 : 0), b_rs = align_up(chunk * 4),
                 b_ps = align_up(positions ? chunk * NR * 4 : 0),
                 b_co = align_up(corr ? chunk * NR * w : 0),
                 b_sy = align_up(ws_bytes_for(c, chunk)), b_ct = 256;
    // pinned host staging: the compacted rows (16-byte pitch), their indices, the count
    const size_t pitch = (row + 15) & ~(size_t)15;
    const size_t h_cp = align_up(chunk * pitch), h_ix = align_up(chunk * 4), h_ct = 256;
    if (int r = ensure_stage(c, b_cw + b_er + b_ne + b_rs + b_ps + b_co + b_sy + b_ct, h_cp + h_ix + h_ct)) return r;
    // Only the codewords whose result is nonzero can differ from what was sent (a clean codeword is
    // never written; -1 may leave partial corrections, rs_base:1238-1241): the device compacts those
    // rows straight into pinned host memory, and only the results and the count are copied back, so
    // a chunk needs one synchronisation before its rows are scattered.
    struct Pending { size_t k0 = 0; bool live = false; } pend[2];
    auto finish = [&](int s) -> int {
        if (!pend[s].live) return 0;
        pend[s].live = false;
        HIP_TRY(hipStreamSynchronize(c->streams[s]));           // rows, indices, results, count
        const char *hb = static_cast<const char *>(c->h_stage[s]);
        const uint32_t *hix = reinterpret_cast<const uint32_t *>(hb + h_cp);
        const uint32_t cnt = *reinterpret_cast<const uint32_t *>(hb + h_cp + h_ix);
        const size_t k0 = pend[s].k0;
        for (uint32_t j = 0; j < cnt; ++j) {
            const size_t k = k0 + hix[j];
            const char *src = hb + (size_t)j * pitch;
            if (inline_par) {
                std::memcpy(static_cast<char *>(data) + k * data_stride * w, src, (size_t)(len + NR) * w);
            } else {
                std::memcpy(static_cast<char *>(data) + k * data_stride * w, src, (size_t)len * w);
                std::memcpy(static_cast<char *>(parity) + k * parity_stride * w, src + (size_t)len * w,
                            (size_t)NR * w);
            }
        }
        return 0;
    };
    for (size_t i = 0, k0 = 0; k0 < ncw; ++i, k0 += chunk) {
        const int s = (int)(i & 1);
        hipStream_t st = c->streams[s];
        const size_t n = ncw - k0 < chunk ? ncw - k0 : chunk;
        if (int r = finish(s)) return r;                        // chunk i-2 (this stream's buffers)
        char *base = static_cast<char *>(c->d_stage[s]);
        char *dcw = base, *der = dcw + b_cw, *dne = der + b_er, *drs = dne + b_ne, *dps = drs + b_rs,
             *dco = dps + b_ps, *dsy = dco + b_co, *dct = dsy + b_sy;
        char *hb = static_cast<char *>(c->h_stage[s]), *dhb = nullptr;
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&dhb), hb, 0));
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
        HIP_TRY(hipMemsetAsync(dct, 0, 4, st));
        HIP_TRY(launch_compact_rows(reinterpret_cast<const int32_t *>(drs), n, dcw, row,
                                    reinterpret_cast<uint32_t *>(dct), reinterpret_cast<uint32_t *>(dhb + h_cp),
                                    dhb, pitch, st));
        HIP_TRY(hipMemcpyAsync(result + k0, drs, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(hb + h_cp + h_ix, dct, 4, hipMemcpyDeviceToHost, st));
        if (positions)
            HIP_TRY(ezrs::copy2d(positions + k0 * pos_stride, pos_stride * 4, dps,
                                 (size_t)NR * 4, (size_t)NR * 4, n, hipMemcpyDeviceToHost, st));
        if (corr)
            HIP_TRY(ezrs::copy2d(static_cast<char *>(corr) + k0 * corr_stride * w, corr_stride * w,
                                 dco, (size_t)NR * w, (size_t)NR * w, n, hipMemcpyDeviceToHost, st));
        pend[s] = {k0, true};
    }
    for (int s = 0; s < 2; ++s)
        if (int r = finish(s)) return r;
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
