// Streaming-pattern probe #2: how the per-instruction shape of the LDS-DMA row gather sets the
// bandwidth.  255-byte rows, tiles of 256 rows per workgroup (4 waves), persistent grid.
//   mode G<L>: window of W positions, each DMA instruction = 64/L rows x L lanes x 16 B (L*16 B
//              contiguous per row), D windows in flight
//   mode T   : whole tiles (65,280 contiguous bytes) by 1-KiB linear DMA instructions, double
//              buffered, 1 workgroup per CU
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>
typedef __attribute__((address_space(3))) void lds_void;

template <int W, int D>
__global__ void __launch_bounds__(256) k_gather(const unsigned char *base, unsigned span, unsigned ncw,
                                                unsigned *out) {
    constexpr int L = W / 16;                 // lanes per row
    constexpr int RPI = 64 / L;               // rows per instruction
    constexpr int NI = 256 / RPI;             // instructions per window (whole WG)
    constexpr int WIN = 256 / W;
    __shared__ __attribute__((aligned(16))) unsigned char lds[D][256 * W];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)span, 0x00020000);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned ntiles = (ncw + 255) / 256;
    unsigned acc = 0;
    auto issue = [&](unsigned tile, int w, int b) {
        for (int i = wave; i < NI; i += 4) {
            unsigned row = tile * 256 + i * RPI + lane / L;
            if (row >= ncw) row = ncw - 1;
            const unsigned off = row * 255u + w * W + 16 * (lane % L);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&lds[b][i * 1024], 16, off, 0, 0, 0);
        }
    };
    // flat sequence of (tile, window) steps for this workgroup
    const unsigned nsteps = ((ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x) * WIN;
    auto step_tw = [&](unsigned s, unsigned &t, int &w) { t = blockIdx.x + (s / WIN) * gridDim.x; w = s % WIN; };
    for (unsigned s = 0; s < D - 1 && s < nsteps; ++s) { unsigned t; int w; step_tw(s, t, w); issue(t, w, s % D); }
    for (unsigned s = 0; s < nsteps; ++s) {
        if (s + D - 1 < nsteps) {
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"((D - 2) * (NI / 4)) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (s + D - 1 < nsteps) { unsigned t; int w; step_tw(s + D - 1, t, w); issue(t, w, (s + D - 1) % D); }
        const unsigned *p = reinterpret_cast<const unsigned *>(lds[s % D]);
        for (int k = threadIdx.x; k < 64 * W; k += 256) acc ^= p[k];
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(512) k_tiles(const unsigned char *base, unsigned span, unsigned ncw, unsigned *out) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][65536];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)span, 0x00020000);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;   // 8 waves
    const unsigned ntiles = (ncw + 255) / 256;
    unsigned acc = 0;
    auto issue = [&](unsigned tile, int b) {
        for (int i = wave; i < 64; i += 8) {   // 64 x 1 KiB = 64 KiB >= 65,280 B
            const unsigned off = tile * 65280u + i * 1024 + 16 * lane;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&lds[b][i * 1024], 16, off, 0, 0, 0);
        }
    };
    unsigned tile = blockIdx.x;
    int b = 0;
    if (tile < ntiles) issue(tile, 0);
    for (; tile < ntiles; tile += gridDim.x) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tile + gridDim.x < ntiles) issue(tile + gridDim.x, b ^ 1);
        const unsigned *p = reinterpret_cast<const unsigned *>(lds[b]);
        for (int k = threadIdx.x; k < 16320; k += 512) acc ^= p[k];
        b ^= 1;
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t maxcw = 4u << 20;
    unsigned char *d; unsigned *out;
    (void)hipMalloc(&d, maxcw * 255 + 65536);
    (void)hipMalloc(&out, 1 << 24);
    (void)hipMemset(d, 0x5a, maxcw * 255 + 65536);
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
    const char *only = argc > 1 ? argv[1] : nullptr;
    for (unsigned ncw : {1u << 20, 4u << 20}) {
        const unsigned span = ncw * 255u;
        const double gb = span / 1e9;
#define G(W, D, PC)                                                                                  \
        if (!only || std::string(only) == "G" #W "_" #D "_" #PC) {                                   \
            float ms = timeit([&] { hipLaunchKernelGGL((k_gather<W, D>), dim3(ncu * PC), dim3(256), 0, 0, d, span, ncw, out); }); \
            printf("ncw %7u gather W=%3d D=%d wg/CU=%d: %7.1f us %5.2f TB/s\n", ncw, W, D, PC, ms * 1e3, gb / ms); }
        G(64, 2, 2) G(64, 3, 2) G(64, 4, 2) G(128, 2, 2) G(128, 3, 1) G(128, 2, 1) G(256, 2, 1)
        if (!only || std::string(only) == "T") {
            float ms = timeit([&] { hipLaunchKernelGGL(k_tiles, dim3(ncu), dim3(512), 0, 0, d, span, ncw, out); });
            printf("ncw %7u whole tiles 1/CU double-buffered: %7.1f us %5.2f TB/s\n", ncw, ms * 1e3, gb / ms);
        }
    }
    return 0;
}
