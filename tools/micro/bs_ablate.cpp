// Timing-only ablation driver for the bit-sliced syndrome kernel (RS(255,223), 1M codewords).
// Built three times: full, -DEZRS_BS_ABLATE_DMA (no HBM stream), -DEZRS_BS_ABLATE_COMPUTE (no XOR
// networks).  Outputs of the ablated builds are meaningless; only their times matter.
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_bitslice.hip"
#include <cstdio>
#include <vector>
int main(int argc, char **argv) {
    using namespace ezrs;
    const size_t ncw = 1 << 20;
    uint8_t *d, *syn; int32_t *res;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&syn, ncw * 32); (void)hipMalloc(&res, ncw * 4);
    (void)hipMemset(d, 0x5a, ncw * 255);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const unsigned grid = (unsigned)(ncw / bs::kTile);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL(bs::k_bs_syndromes<bs::BS_RS_255_223>, dim3(grid), dim3(bs::kThreads), 0, 0,
                           d, (size_t)255, 255u, ncw, (const uint32_t *)nullptr, res, syn);
    (void)hipEventRecord(a);
    const int it = 20;
    for (int i = 0; i < it; ++i)
        hipLaunchKernelGGL(bs::k_bs_syndromes<bs::BS_RS_255_223>, dim3(grid), dim3(bs::kThreads), 0, 0,
                           d, (size_t)255, 255u, ncw, (const uint32_t *)nullptr, res, syn);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    printf("%s: %.1f us per launch\n", argc > 1 ? argv[1] : "variant", ms * 1000 / it);
    return 0;
}
