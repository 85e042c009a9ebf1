// Timing-only ablation driver for the bit-sliced kernels (RS(255,223), 1M codewords).
// Built once per variant: full, -DEZRS_BS_ABLATE_DMA (no HBM stream), -DEZRS_BS_ABLATE_COMPUTE (no
// XOR networks), -DEZRS_BS_ABLATE_TRANSPOSE (no bit transposition).  Outputs of the ablated builds
// are meaningless; only their times matter.
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_bitslice.hip"
#include <cstdio>
#include <vector>
int main(int argc, char **argv) {
    using namespace ezrs;
    const size_t ncw = 1 << 20;
    uint8_t *d, *syn; int32_t *res; uint32_t *ws;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&syn, ncw * 32); (void)hipMalloc(&res, ncw * 4);
    (void)hipMalloc(&ws, bs_encode_ws_bytes(ncw));
    (void)hipMemset(d, 0x5a, ncw * 255);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const unsigned grid = (unsigned)(ncw / bs::kTile);
    const int it = 20;
    const char *names[3] = {"syndromes", "encode_syn", "parity"};
    for (int which = 0; which < 3; ++which) {
        for (int i = -3; i < it; ++i) {
            if (i == 0) (void)hipEventRecord(a);
            if (which == 0)
                hipLaunchKernelGGL(bs::k_bs_syndromes<bs::BS_RS_255_223>, dim3(grid), dim3(bs::kThreads), 0, 0,
                                   d, (size_t)255, 255u, ncw, (const uint32_t *)nullptr, res, syn);
            else if (which == 1)
                hipLaunchKernelGGL(bs::k_bs_encode_syn<bs::BS_RS_255_223>, dim3(grid), dim3(bs::kThreads), 0, 0,
                                   d, (size_t)255, 223u, ncw, ws);
            else
                hipLaunchKernelGGL(bs::k_bs_parity<bs::BS_RS_255_223>, dim3((ncw + bs::kParCw - 1) / bs::kParCw), dim3(256), 0, 0,
                                   ws, d + 223, (size_t)255, ncw);
        }
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("%-8s %-10s: %7.1f us per launch\n", argc > 1 ? argv[1] : "variant", names[which], ms * 1000 / it);
    }
    return 0;
}
