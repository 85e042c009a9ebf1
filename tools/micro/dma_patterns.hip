// Memory-pattern probe: how fast can a workgroup stream a [512 rows x 255 B] tile into LDS when
// the rows are consumed chunk by chunk (positions [P*k, P*k+P) of every row per step)?
// Each variant only moves data (global_load_lds_dwordx4 into two LDS buffers + barriers).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void lds_void;
constexpr int kTile = 512;

// P = chunk bytes per row (16..128); rows per DMA instruction = 64*16/P.
template <int P, bool ALT>
__global__ void __launch_bounds__(128) k_chunks(const uint8_t* base, size_t ncw, uint32_t* sink) {
    constexpr int kBuf = kTile * P / 4 + 64;           // dwords per buffer
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * kBuf];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const size_t cw0 = (size_t)blockIdx.x * kTile;
    constexpr int lanes_per_row = P / 16, rows_per_inst = 64 / lanes_per_row;
    constexpr int insts = kTile / rows_per_inst;        // per chunk
    const int nch = (255 + P - 1) / P;
    uint32_t acc = 0;
    for (int k = 0; k < nch; ++k) {
        uint32_t* buf = lds + (k & 1) * kBuf;
        for (int i = wave; i < insts; i += 2) {
            const int row = i * rows_per_inst + lane / lanes_per_row;
            size_t cw = cw0 + row; if (cw >= ncw) cw = ncw - 1;
            int kk = ALT && (row & 1) ? nch - 1 - k : k;
            long off = (long)cw * 255 + (long)kk * P + 16 * (lane % lanes_per_row);
            if (off + 16 > (long)ncw * 255) off = (long)ncw * 255 - 16;
            __builtin_amdgcn_global_load_lds((const void*)(base + off), (lds_void*)(buf + i * 256), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        acc ^= buf[threadIdx.x];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// Reference: the same bytes as one contiguous stream (1 KB per wave-instruction).
__global__ void __launch_bounds__(128) k_contig(const uint8_t* base, size_t ncw, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * 8192];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const size_t b0 = (size_t)blockIdx.x * kTile * 255;
    const int total = kTile * 255 / 1024;               // 127 full KB pieces
    uint32_t acc = 0;
    for (int k = 0; k < 4; ++k) {
        uint32_t* buf = lds + (k & 1) * 8192;
        for (int i = wave + 2 * 16 * k; i < total && i < 32 * (k + 1); i += 2)
            __builtin_amdgcn_global_load_lds((const void*)(base + b0 + (size_t)i * 1024 + lane * 16),
                                             (lds_void*)(buf + (i % 32) * 256), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        acc ^= buf[threadIdx.x];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    (void)hipEventRecord(a);
    for (int i = 0; i < 20; ++i) f();
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000 / 20;
}

int main() {
    const size_t ncw = 1 << 20;
    uint8_t* d; uint32_t* s;
    (void)hipMalloc(&d, ncw * 255 + 4096); (void)hipMalloc(&s, 64);
    (void)hipMemset(d, 1, ncw * 255 + 4096);
    const unsigned grid = ncw / kTile;
    const double mb = ncw * 255.0 / 1e6;
    auto rep = [&](const char* n, float us) { printf("%-28s %8.1f us  %7.2f TB/s\n", n, us, mb / us); };
    rep("contiguous 1KB/inst", timeit([&] { hipLaunchKernelGGL(k_contig, dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    rep("chunk 16B/row", timeit([&] { hipLaunchKernelGGL((k_chunks<16, false>), dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    rep("chunk 32B/row", timeit([&] { hipLaunchKernelGGL((k_chunks<32, false>), dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    rep("chunk 32B/row alt-dir", timeit([&] { hipLaunchKernelGGL((k_chunks<32, true>), dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    rep("chunk 64B/row", timeit([&] { hipLaunchKernelGGL((k_chunks<64, false>), dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    rep("chunk 64B/row alt-dir", timeit([&] { hipLaunchKernelGGL((k_chunks<64, true>), dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    rep("chunk 128B/row", timeit([&] { hipLaunchKernelGGL((k_chunks<128, false>), dim3(grid), dim3(128), 0, 0, d, ncw, s); }));
    return 0;
}
