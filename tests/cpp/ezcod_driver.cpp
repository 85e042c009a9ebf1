// ezcod_driver.cpp -- exercises the reference's ezcod C API (ezcod.h: ezcod_3_{10,11,12}_{encode,
// decode}, implemented in the reference's ezcod.C over ezpwd::RS<31,31-P>).  Built twice:
// against the reference's own headers (oracle/_ref/ezcod_ref: the fixture generator) and against
// this repository's include/ (tests/cpp/_bin/ezcod_gpu: ezcod.C unchanged, its RS on the GPU).
// Prints one line per call; the two builds must print the same lines.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "ezcod.h"

typedef int (*enc_t)(double, double, char *, size_t, size_t);
typedef int (*dec_t)(char *, size_t, double *, double *, double *);

int main() {
    const enc_t enc[3] = {ezcod_3_10_encode, ezcod_3_11_encode, ezcod_3_12_encode};
    const dec_t dec[3] = {ezcod_3_10_decode, ezcod_3_11_decode, ezcod_3_12_decode};
    uint64_t s = 0x5EED0005ull;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); };
    for (int v = 0; v < 3; ++v) {
        for (int n = 0; n < 120; ++n) {
            const double lat = -90.0 + 180.0 * (rnd() / 2147483648.0);
            const double lon = -180.0 + 360.0 * (rnd() / 2147483648.0);
            char buf[64];
            std::memset(buf, 0, sizeof buf);
            const int rc = enc[v](lat, lon, buf, sizeof buf, n % 3 ? 3 : 0);
            std::printf("E %d %d %s\n", v, rc, rc > 0 ? buf : "-");
            if (rc <= 0) continue;
            for (int k = 0; k < 4; ++k) {                 // clean, then 1..3 corrupted characters
                char t[64];
                std::memcpy(t, buf, sizeof t);
                const int L = (int)std::strlen(t);
                for (int e = 0; e < k; ++e) {
                    const int at = (int)(rnd() % (unsigned)L);
                    if (t[at] == '.' || t[at] == '!') continue;
                    t[at] = "0123456789ABCDEFGHJKMNPQRTUVWXYZ"[rnd() % 32];
                }
                double la = 0, lo = 0, ac = 0;
                const int r = dec[v](t, sizeof t, &la, &lo, &ac);
                std::printf("D %d %d %d %.9f %.9f %.3f %s\n", v, k, r, r >= 0 ? la : 0.0,
                            r >= 0 ? lo : 0.0, r >= 0 ? ac : 0.0, r >= 0 ? "" : t);
            }
        }
    }
    return 0;
}
