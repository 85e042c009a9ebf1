// Probe: does global_load_lds_dwordx4 accept byte-unaligned global addresses on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
__global__ void k(const uint8_t* src, uint32_t* out, int shift) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[64 * 4];
    const int lane = threadIdx.x;
    const uint8_t* g = src + lane * 16 + shift;
    __builtin_amdgcn_global_load_lds((const void*)g, (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = 0; i < 4; ++i) out[lane * 4 + i] = lds[lane * 4 + i];
}
int main() {
    std::vector<uint8_t> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t* d; uint32_t* o;
    hipMalloc(&d, 4096); hipMalloc(&o, 4096);
    hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int shift = 0; shift < 16; ++shift) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, shift);
        std::vector<uint8_t> r(1024);
        hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 1024; ++i) bad += r[i] != h[i + shift];
        printf("shift %2d: %s (%d bad bytes)\n", shift, bad ? "MISMATCH" : "ok", bad);
        bad_total += bad;
    }
    printf("glds_unaligned: %s\n", bad_total ? "UNALIGNED NOT SUPPORTED" : "all shifts ok");
    return 0;
}
