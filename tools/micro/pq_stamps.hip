// Per-phase timing of the 4-wave tile kernel k_pq_lin (timing-only build of ezrs_ps.hip with
// EZRS_PS_STAMPS): s_memtime at each phase boundary of the first tiles of the first workgroups,
// averaged over workgroups 0..15 and tiles 1..6.  Usage: pq_stamps [enc]
#define EZRS_PS_STAMPS 1
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip"
#include <cstdio>
using namespace ezrs;
int main(int argc, char **argv) {
    const int enc = argc > 1 ? atoi(argv[1]) : 0;
    const size_t ncw = 1u << 20;
    uint8_t *d, *ws; int32_t *res;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&ws, ncw * 32 + 65536); (void)hipMalloc(&res, ncw * 4);
    (void)hipMemset(d, 0, ncw * 255);
    int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    ps::PsArgs p{};
    p.base = d; p.span = ncw * 255 - (enc ? 32 : 0); p.stride = 255; p.ncw = ncw; p.ntiles = ncw / 256;
    p.lo = 0; p.result = res; p.ws = ws; p.ws_pitch = enc ? (ncw + 2047) / 2048 * 2048 : 0;
    unsigned grid = 2 * ncu;
    for (int rep = 0; rep < 4; ++rep) {
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        if (enc) hipLaunchKernelGGL((ps::pq::k_pq_lin<ps::PQ_RS_255_223, true, false, true>), dim3(grid), dim3(256), 0, 0, p);
        else hipLaunchKernelGGL((ps::pq::k_pq_lin<ps::PQ_RS_255_223, false, false, true>), dim3(grid), dim3(256), 0, 0, p);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("%s: %.1f us\n", enc ? "encode syndromes" : "decode", ms * 1e3);
    }
    static unsigned long long st[16][4][8][8];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(ps::g_pq_stamps), sizeof st);
    const char *names[] = {"dma+bar", "main", "bar", "xchg", "fold", "st", "next"};
    double acc[4][7] = {};
    int n = 0;
    for (int wg = 0; wg < 16; ++wg)
        for (int it = 1; it < 7; ++it) {
            ++n;
            for (int w = 0; w < 4; ++w) {
                for (int ph = 0; ph < 6; ++ph) acc[w][ph] += (double)(st[wg][w][it][ph + 1] - st[wg][w][it][ph]);
                acc[w][6] += (double)(st[wg][w][it + 1][0] - st[wg][w][it][6]);
            }
        }
    printf("ticks per tile (s_memtime), mean over %d tiles:\n", n);
    for (int w = 0; w < 4; ++w) {
        printf(" wave %d:", w);
        double tot = 0;
        for (int ph = 0; ph < 7; ++ph) { printf(" %s %6.0f", names[ph], acc[w][ph] / n); tot += acc[w][ph] / n; }
        printf("  | total %6.0f\n", tot);
    }
    return 0;
}
