// Per-phase timing of the plane-sliced syndrome kernel (timing-only build of ezrs_ps.hip with
// EZRS_PS_STAMPS): for the first workgroups, s_memtime at each phase boundary of every tile.
#define EZRS_PS_STAMPS 1
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip"
#include <cstdio>
#include <vector>
using namespace ezrs;
__global__ void k_clock(unsigned long long *o, int spin) {
    // s_memtime (shader clock) against s_memrealtime (constant 100 MHz) over a busy loop
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (int i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; o[2] = x; }
}
int main(int argc, char **argv) {
    const int enc = argc > 1 ? atoi(argv[1]) : 1;
    const int per_cu = argc > 2 ? atoi(argv[2]) : 2;
    const size_t ncw = 1 << 20;
    uint8_t *d; uint8_t *ws; int32_t *res;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&ws, ncw * 32 + 65536); (void)hipMalloc(&res, ncw * 4);
    (void)hipMemset(d, 0x37, ncw * 255);
    int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    ps::PsArgs p{};
    p.base = d; p.span = ncw * 255; p.stride = 255; p.ncw = ncw; p.ntiles = ncw / 256;
    p.lo = 0; p.hi = enc ? 223 : 255; p.result = res; p.ws = ws; p.ws_pitch = ncw;
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        if (enc) hipLaunchKernelGGL((ps::k_ps_syndromes<ps::PS_RS_255_223, true>), dim3(per_cu * ncu), dim3(512), 0, 0, p);
        else hipLaunchKernelGGL((ps::k_ps_syndromes<ps::PS_RS_255_223, false>), dim3(per_cu * ncu), dim3(512), 0, 0, p);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("%s wg/CU %d: %.1f us\n", enc ? "encode" : "decode", per_cu, ms * 1e3);
    }
    {
        unsigned long long *o; (void)hipMalloc(&o, 64);
        hipLaunchKernelGGL(k_clock, dim3(1024), dim3(256), 0, 0, o, 2000000);
        unsigned long long h[3]; (void)hipMemcpy(h, o, 24, hipMemcpyDeviceToHost);
        printf("clock: %llu memtime ticks in %llu realtime ticks (100 MHz) -> %.0f MHz\n", h[0], h[1], h[0] * 100.0 / h[1]);
    }
    if (argc > 3) return 0;
    static unsigned long long st[8][8][16][8];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(ps::g_ps_stamps), sizeof st);
    // phases: 0 top, 1 after B1 (tile landed), 2 main loop done, 3 after B2, 4 reduce done + DMA
    // issued, 5 epilogue done; memtime ticks (100 MHz on gfx9 = 10 ns)... printed raw deltas
    const char *names[] = {"wait+B1", "main", "B2", "reduce", "epilogue", "flags/next"};
    for (int wg = 0; wg < 2; ++wg) {
        printf("wg %d\n", wg);
        for (int it = 0; it < 8; ++it) {
            printf(" tile %d:", it);
            for (int w = 0; w < 8; w += 3) {
                printf(" w%d[", w);
                for (int ph = 0; ph < 5; ++ph) printf("%s%llu", ph ? " " : "", st[wg][w][it][ph + 1] - st[wg][w][it][ph]);
                printf(" | %llu]", it + 1 < 8 ? st[wg][w][it + 1][0] - st[wg][w][it][5] : 0ull);
            }
            printf("\n");
        }
    }
    return 0;
}
