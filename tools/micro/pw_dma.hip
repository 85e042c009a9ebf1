// Probe: per-wave window streaming of 255-byte rows (the k_pw_syndromes access pattern) without
// the arithmetic.  One single-wave workgroup owns tiles of 256 rows and walks them in windows of W
// positions; each LDS-DMA instruction moves 16 B per lane, L consecutive lanes per row (16 L bytes
// contiguous per row, 64 / L rows per instruction); D window buffers per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
typedef __attribute__((address_space(3))) void lds_void;

template <int W, int L, int D>
__global__ void __launch_bounds__(64) k_win(const unsigned char *base, unsigned span, unsigned ncw, unsigned *out) {
    constexpr int RPI = 64 / L;                   // rows per instruction
    constexpr int HALVES = W / (16 * L);          // instructions per row group
    constexpr int NI = (256 / RPI) * HALVES;      // instructions per window
    constexpr int WIN = (255 + W - 1) / W;
    __shared__ __attribute__((aligned(16))) unsigned char lds[D][256 * W];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)span, 0x00020000);
    const int lane = threadIdx.x;
    const unsigned ntiles = (ncw + 255) / 256;
    unsigned acc = 0;
    auto issue = [&](unsigned tile, int w, int b) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int g = i / HALVES, h = i % HALVES;
            const unsigned row = tile * 256 + g * RPI + lane / L;
            const unsigned off = row * 255u + w * W + 16 * (L * h + lane % L);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&lds[b][i * 1024], 16, off, 0, 0, 0);
        }
    };
    const unsigned nsteps = ((ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x) * WIN;
    auto step_tw = [&](unsigned s, unsigned &t, int &w) { t = blockIdx.x + (s / WIN) * gridDim.x; w = s % WIN; };
    for (unsigned s = 0; s < D - 1 && s < nsteps; ++s) { unsigned t; int w; step_tw(s, t, w); issue(t, w, s % D); }
    for (unsigned s = 0; s < nsteps; ++s) {
        if (s + D - 1 < nsteps) { unsigned t; int w; step_tw(s + D - 1, t, w); issue(t, w, (s + D - 1) % D); }
        if (s + D - 1 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" :: "n"((D - 1) * NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint4 *p = reinterpret_cast<const uint4 *>(lds[s % D]);
#pragma unroll 4
        for (int k = lane; k < 16 * W; k += 64) { const uint4 v = p[k]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

// Same as k_win<32, 1, 2> plus an L2 prefetch of the next 128-position chunk of the tile's rows
// (both lines of each row's 128-byte span, 4-byte LDS-DMA into a scratch area), issued with the
// first window of each chunk.
template <int PF>
__global__ void __launch_bounds__(64) k_win_pf(const unsigned char *base, unsigned span, unsigned ncw, unsigned *out) {
    constexpr int W = 32, NI = 8, WIN = 8;
    __shared__ __attribute__((aligned(16))) unsigned char lds[2][256 * W];
    __shared__ __attribute__((aligned(16))) unsigned char scratch[256];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)span, 0x00020000);
    const int lane = threadIdx.x;
    const unsigned ntiles = (ncw + 255) / 256;
    unsigned acc = 0;
    auto issue = [&](unsigned tile, int w, int b) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int k = i >> 1, h = i & 1;
            const unsigned row = tile * 256 + 4 * lane + k;
            const unsigned off = row * 255u + w * W + 16 * h;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&lds[b][i * 1024], 16, off, 0, 0, 0);
        }
    };
    auto prefetch = [&](unsigned tile, int c) {     // chunk c: positions 128c..128c+127
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const unsigned row = tile * 256 + 4 * lane + (i & 3);
            const unsigned off = row * 255u + 128 * c + ((i >> 2) ? 124 : 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)scratch, 4, off, 0, 0, 0);
        }
    };
    const unsigned nsteps = ((ntiles - blockIdx.x + gridDim.x - 1) / gridDim.x) * WIN;
    auto step_tw = [&](unsigned s, unsigned &t, int &w) { t = blockIdx.x + (s / WIN) * gridDim.x; w = s % WIN; };
    if (PF) { prefetch(blockIdx.x, 0); prefetch(blockIdx.x, 1); }
    issue(blockIdx.x, 0, 0);
    for (unsigned s = 0; s < nsteps; ++s) {
        unsigned t; int w; step_tw(s, t, w);
        if (s + 1 < nsteps) {
            if (PF && (w & 3) == 0) {
                // prefetch the chunk after the next one (same tile or the next tile's chunk 0/1)
                const int c = (w >> 2) + 2;
                if (c < 2) prefetch(t, c); else if (t + gridDim.x < ntiles) prefetch(t + gridDim.x, c - 2);
                unsigned t1; int w1; step_tw(s + 1, t1, w1); issue(t1, w1, (s + 1) & 1);
                asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            } else {
                unsigned t1; int w1; step_tw(s + 1, t1, w1); issue(t1, w1, (s + 1) & 1);
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            }
        } else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint4 *p = reinterpret_cast<const uint4 *>(lds[s & 1]);
#pragma unroll 4
        for (int k = lane; k < 16 * W; k += 64) { const uint4 v = p[k]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

int main(int argc, char **argv) {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t maxcw = 4u << 20;
    unsigned char *d; unsigned *out;
    (void)hipMalloc(&d, maxcw * 255 + 65536);
    (void)hipMalloc(&out, 1 << 26);
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
    for (unsigned ncw : {1u << 20, 4u << 20}) {
        const unsigned span = ncw * 255u;
        const double gb = span / 1e9;
        const unsigned ntiles = (ncw + 255) / 256;
#define P(W, L, D, PC)                                                                               \
        {                                                                                            \
            unsigned grid = ncu * PC < ntiles ? ncu * PC : ntiles;                                   \
            float ms = timeit([&] { hipLaunchKernelGGL((k_win<W, L, D>), dim3(grid), dim3(64), 0, 0, d, span, ncw, out); }); \
            printf("ncw %7u W=%3d L=%d D=%d waves/CU=%2d: %7.1f us %5.2f TB/s\n", ncw, W, L, D, PC, ms * 1e3, gb / ms); }
        P(32, 1, 2, 8) P(32, 2, 2, 8) P(32, 2, 3, 6) P(32, 2, 4, 4) P(64, 4, 2, 4) P(64, 2, 2, 4) P(64, 4, 2, 5)
        P(32, 1, 2, 4) P(32, 2, 2, 4) P(32, 2, 2, 6)
        for (int pc : {8, 6, 4}) {
            unsigned grid = ncu * pc < ntiles ? ncu * pc : ntiles;
            float ms0 = timeit([&] { hipLaunchKernelGGL((k_win_pf<0>), dim3(grid), dim3(64), 0, 0, d, span, ncw, out); });
            float ms1 = timeit([&] { hipLaunchKernelGGL((k_win_pf<1>), dim3(grid), dim3(64), 0, 0, d, span, ncw, out); });
            printf("ncw %7u W=32 pf-variant waves/CU=%d: no-pf %7.1f us %5.2f TB/s | pf %7.1f us %5.2f TB/s\n", ncw, pc, ms0 * 1e3, gb / ms0, ms1 * 1e3, gb / ms1);
        }
    }
    return 0;
}
