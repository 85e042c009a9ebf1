// Plane-sliced BCH remainder kernels (ezbch_ps.hip), used by ezbch.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ezrs {

constexpr int32_t kBpsFlag = INT32_MIN;       // decode: the remainder differs (the error path's slot)

struct BpsArgs {
    const uint8_t *base;        // row 0
    uint32_t span;              // bytes readable from base (all offsets 32-bit)
    uint32_t stride;            // row pitch, <= 128
    uint32_t ncw;
    uint32_t ntiles;            // 256-row tiles
    int fb;                     // frame position of a row's first byte: F - (len + ecc_bytes)
    uint8_t *ecc;               // encode: ECC of row k at ecc + k * estride
    size_t estride;
    uint64_t *rem;              // decode: remainder XOR received ECC, left-justified (as data_remainder)
    int32_t *result;            // decode: 0 where that is zero, else kBpsFlag
};

// Codec id of the plane-sliced path for init_bch(m, t) with its default polynomial, -1 if none.
int bps_codec_id(int m, int t, int ecc_bits);
int bps_frame(int id);          // frame bytes F: rows of at most F bytes (data + ECC)
hipError_t launch_bps(int id, bool dec, const BpsArgs &a, int ncu, hipStream_t s);

} // namespace ezrs
