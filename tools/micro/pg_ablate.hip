// Phase ablation of the 4-wave group syndrome kernel: kernel time with parts switched off
// (PsArgs::ablate), to price each phase under the real concurrency.  Results are garbage.
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip"
#include <cstdio>
using namespace ezrs;
int main(int argc, char **argv) {
    const size_t ncw = 1u << 20;
    uint8_t *d; uint8_t *ws; int32_t *res;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&ws, ncw * 32 + 65536); (void)hipMalloc(&res, ncw * 4);
    (void)hipMemset(d, 0x37, ncw * 255);
    int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    ps::PsArgs p{};
    p.base = d; p.span = ncw * 255; p.stride = 255; p.ncw = ncw; p.ntiles = ncw / 256;
    p.lo = 0; p.result = res; p.ws = ws; p.ws_pitch = ncw;
    unsigned grid = 2 * ncu;
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const char *names[] = {"full", "no-main", "no-xchg", "no-main-xchg", "no-epi", "no-main-epi", "no-xchg-epi",
                           "dma-only", "no-dma", "no-dma-main", "", "", "no-dma-epi"};
    for (int enc = 1; enc >= 1; --enc)
        for (int ab : {0, 16, 13, 29, 15, 31, 7, 23, 8, 24}) {
            p.ablate = ab;
            p.hi = enc ? 223 : 255;
            float best = 1e9;
            for (int rep = 0; rep < 4; ++rep) {
                (void)hipEventRecord(a);
                if (enc) hipLaunchKernelGGL((ps::k_pg_syndromes<ps::PG4_RS_255_223, true>), dim3(grid), dim3(256), 0, 0, p);
                else hipLaunchKernelGGL((ps::k_pg_syndromes<ps::PG4_RS_255_223, false>), dim3(grid), dim3(256), 0, 0, p);
                (void)hipEventRecord(b); (void)hipEventSynchronize(b);
                float ms; (void)hipEventElapsedTime(&ms, a, b);
                if (rep && ms < best) best = ms;
            }
            printf("%s ablate %2d %-14s %7.1f us\n", enc ? "encode" : "decode", ab, ab < 13 ? names[ab] : "?", best * 1e3);
        }
    return 0;
}
