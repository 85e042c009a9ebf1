// VALU-rate probe: the generated RS(255,223) role-0 Horner networks (LDS plane reads + xor3 networks)
// in a loop with no HBM traffic and no barriers, at 1..4 workgroups (of 4 waves) per CU (occupancy set
// by a dynamic LDS pad).  Reports wave-instructions per SIMD-cycle implied by the XOR-network count.
#include <hip/hip_runtime.h>
#include "../../ezpwd-reed-solomon_amd/csrc/gen/ezrs_bs_tables.inc"
#include <cstdio>
using namespace ezrs::bs;

template <int R>
__global__ void __launch_bounds__(256) k_rate(uint32_t *out, int iters) {
    extern __shared__ uint32_t lds[];
    for (int i = threadIdx.x; i < 64 * 257; i += 256) lds[i] = i * 0x9E3779B9u;
    __syncthreads();
    uint32_t S[16][8];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) S[i][q] = threadIdx.x * (i + 1) + q;
    const int lane = threadIdx.x & 63;
    const uint32_t *p = lds + lane * 257;
    for (int it = 0; it < iters; ++it) {
        BS_RS_255_223::horner_half<R, 0>(S, p);
        BS_RS_255_223::horner_half<R, 1>(S, p + 8);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) x ^= S[i][q];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 4096 * 256 * 4);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const int iters = 64;
    for (int wg_per_cu = 1; wg_per_cu <= 4; ++wg_per_cu) {
        const size_t lds = 160 * 1024 / wg_per_cu - 1024;
        (void)hipFuncSetAttribute((const void *)k_rate<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        const int grid = 256 * wg_per_cu * 4;
        for (int r = 0; r < 2; ++r) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k_rate<0>, dim3(grid), dim3(256), lds, 0, out, iters);
            (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        }
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        // per wave: iters x 16 y-steps x (22 combos + 64 xor3) network instructions
        const double winst = (double)grid * 4 * iters * 16 * 86;
        const double per_simd_cycle = winst / (ms * 1e-3) / (1024 * 2.4e9);
        printf("wg/CU %d: %.1f us, network wave-instr per SIMD per cycle @2.4GHz: %.3f (ideal 0.5)\n",
               wg_per_cu, ms * 1e3, per_simd_cycle);
    }
    return 0;
}
