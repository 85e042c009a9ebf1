// Per-phase timing of the group syndrome kernel (timing-only build of ezrs_ps.hip with
// EZRS_PS_STAMPS): s_memtime at phase boundaries of the first tiles of the first workgroups.
#define EZRS_PS_STAMPS 1
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip"
#include <cstdio>
using namespace ezrs;
int main(int argc, char **argv) {
    const int enc = argc > 1 ? atoi(argv[1]) : 1;
    const int per_cu = argc > 2 ? atoi(argv[2]) : 2;
    const size_t ncw = argc > 3 ? (size_t)atol(argv[3]) : (1u << 20);
    uint8_t *d; uint8_t *ws; int32_t *res;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&ws, ncw * 32 + 65536); (void)hipMalloc(&res, ncw * 4);
    (void)hipMemset(d, 0x37, ncw * 255);
    int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    ps::PsArgs p{};
    p.base = d; p.span = ncw * 255; p.stride = 255; p.ncw = ncw; p.ntiles = ncw / 256;
    p.lo = 0; p.hi = enc ? 223 : 255; p.result = res; p.ws = ws; p.ws_pitch = (ncw + 2047) / 2048 * 2048;
    unsigned grid = per_cu * ncu < p.ntiles ? per_cu * ncu : p.ntiles;
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        if (enc) hipLaunchKernelGGL((ps::k_pg_syndromes<ps::PG4_RS_255_223, true>), dim3(grid), dim3(256), 0, 0, p);
        else hipLaunchKernelGGL((ps::k_pg_syndromes<ps::PG4_RS_255_223, false>), dim3(grid), dim3(256), 0, 0, p);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("%s wg/CU %d ncw %zu: %.1f us\n", enc ? "encode" : "decode", per_cu, ncw, ms * 1e3);
    }
    static unsigned long long st[16][8][16][8];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(ps::g_pg_stamps), sizeof st);
    // 0 top, 1 own DMA done, 2 barrier (tile landed), 3 compute done, 4 barrier, 5 exchange done, 6 epilogue done
    const char *names[] = {"vmwait", "bar1", "comp", "bar2", "xchg", "epi"};
    const int ntile = (int)((p.ntiles + grid - 1) / grid) < 16 ? (int)((p.ntiles + grid - 1) / grid) : 16;
    for (int wg = 0; wg < 3; ++wg) {
        printf("wg %d\n", wg);
        for (int it = 0; it < ntile; ++it) {
            printf(" t%-2d", it);
            for (int q = 0; q < 4; ++q) {
                printf(" w%d[", q);
                for (int ph = 0; ph < 6; ++ph) printf("%s%llu", ph ? " " : "", st[wg][q][it][ph + 1] - st[wg][q][it][ph]);
                printf("|%lld]", it + 1 < ntile ? (long long)(st[wg][q][it + 1][0] - st[wg][q][it][6]) : 0ll);
            }
            printf("\n");
        }
    }
    return 0;
}
