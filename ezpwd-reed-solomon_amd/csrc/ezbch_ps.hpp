// Plane-sliced BCH remainder kernels (ezbch_ps.hip), used by ezbch.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ezrs {

struct BpsArgs {
    const uint8_t *base;        // row 0
    uint32_t span;              // bytes readable from base (all offsets 32-bit)
    uint32_t stride;            // row pitch, <= 128
    uint32_t ncw;
    uint32_t ntiles;            // 256-row tiles
    int fb;                     // frame position of a row's first byte: F - len (encode),
                                // F - (len + ecc_bytes) (decode)
    uint8_t *ecc;               // encode: ECC of row k at ecc + k * estride
    size_t estride;
    uint32_t espan;             // encode: bytes writable from ecc ((ncw - 1) * estride + ECC bytes)
};

// Codec id of the plane-sliced path for init_bch(m, t) with its default polynomial, -1 if none.
int bps_codec_id(int m, int t, int ecc_bits);
int bps_frame(int id);          // frame bytes F: rows of at most F bytes read
hipError_t launch_bps(int id, const BpsArgs &a, int ncu, hipStream_t s);   // encode

} // namespace ezrs
