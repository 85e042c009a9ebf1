// Probe: the pair kernel's window DMA (128 positions x 256 rows, 8 consecutive rows x 128 B per
// instruction, XOR-swizzled pieces) with a synthetic compute phase of SPIN dependent VALU ops per
// wave per window, for several workgroup shapes: WAVES waves per workgroup, D window buffers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int rsrc_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

template <int WAVES, int D, int W = 128>
__global__ void __launch_bounds__(64 * WAVES) k_py_dma(const unsigned char *base, unsigned span, unsigned ncw,
                                                      unsigned *out, int spin) {
    constexpr int LPR = W / 16;                     // lanes per row
    constexpr int RPI = 64 / LPR;                   // consecutive rows per instruction
    constexpr int NWIN = 256 / W;                   // windows per tile
    __shared__ __attribute__((aligned(16))) unsigned char buf[D][256 * W];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t p = (uint64_t)(uintptr_t)base;
    rsrc_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(p >> 32) & 0xFFFFu));
    r.z = __builtin_amdgcn_readfirstlane((int)span);
    r.w = 0x00020000;
    const unsigned ntiles = (ncw + 255) / 256;
    const unsigned nsteps = ((ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x) * NWIN;
    auto issue = [&](unsigned s, int b) {
        const unsigned tile = blockIdx.x + (s / NWIN) * gridDim.x, w = s % NWIN;
        const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr(buf[b]));
        const uint32_t dslot = lane / LPR;
        for (int i = wave; i < W / 4; i += WAVES) {
            const int rows0 = i * RPI;
            const uint32_t pc = lane % LPR;
            const uint32_t off = tile * 65280u + (rows0 + dslot) * 255u + W * w + 16 * pc;
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
                         :: "s"(__builtin_amdgcn_readfirstlane(lb + i * 1024)), "v"(off), "s"(r) : "memory", "m0");
        }
    };
    uint32_t acc = lane;
    for (unsigned s = 0; s < D - 1 && s < nsteps; ++s) issue(s, s % D);
    for (unsigned s = 0; s < nsteps; ++s) {
        if (D == 1) {
            if (s == 0) issue(0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (s + D - 1 < nsteps) issue(s + D - 1, (s + D - 1) % D);
        }
        uint4 v;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(lds_addr(buf[s % D]) + 16 * (threadIdx.x & 255)) : "memory");
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
        for (int i = 0; i < spin; ++i) acc = __builtin_amdgcn_bitop3_b32(acc, acc >> 1, (uint32_t)i, 0x96);
        __syncthreads();
        if (D == 1 && s + 1 < nsteps) issue(s + 1, 0);
    }
    out[blockIdx.x * 64 * WAVES + threadIdx.x] = acc;
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned ncw = 1u << 20;
    unsigned char *d; unsigned *out;
    (void)hipMalloc(&d, (size_t)ncw * 255 + 65536);
    (void)hipMalloc(&out, 1 << 24);
    (void)hipMemset(d, 0x5a, (size_t)ncw * 255 + 65536);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    auto timeit = [&](auto launch) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(a); launch(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b);
            if (rep && ms < best) best = ms;
        }
        return best;
    };
    const unsigned span = ncw * 255u, ntiles = ncw / 256;
    const double gb = span / 1e9;
#define RUN(WV, D, PC, WIN)                                                                            \
    for (int spin : {0}) {                                                                             \
        unsigned grid = ncu * PC < ntiles ? ncu * PC : ntiles;                                         \
        float ms = timeit([&] { hipLaunchKernelGGL((k_py_dma<WV, D, WIN>), dim3(grid), dim3(64 * WV), 0, 0, d, span, ncw, out, spin); }); \
        printf("W=%3d waves/WG %d D=%d WG/CU %d spin %4d: %7.1f us %5.2f TB/s\n", WIN, WV, D, PC, spin, ms * 1e3, gb / ms); }
    RUN(4, 1, 2, 256) RUN(8, 1, 1, 256) RUN(8, 2, 1, 256) RUN(2, 1, 2, 256) RUN(4, 2, 1, 256) RUN(4, 1, 2, 128) RUN(2, 1, 4, 128)
    return 0;
}
