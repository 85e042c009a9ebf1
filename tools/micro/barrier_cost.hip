// Probe: cost of s_barrier for 2/4/8-wave workgroups with 1-4 workgroups per CU (empty loop vs
// barrier loop), plus an LDS write/read round trip per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void k(unsigned *out, int iters) {
    __shared__ unsigned lds[512 * 4];
    unsigned acc = threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 1) __syncthreads();
        if (MODE == 2) {
            lds[threadIdx.x] = acc;
            __syncthreads();
            acc += lds[(threadIdx.x + 64) % blockDim.x];
            __syncthreads();
        }
        acc = acc * 1664525u + 1013904223u;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
    int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *out; (void)hipMalloc(&out, 1 << 24);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    const int iters = 20000;
    for (int waves : {2, 4, 8})
        for (int per_cu : {1, 2, 4}) {
            if (waves * per_cu > 16) continue;
            float t[3];
            for (int mode = 0; mode < 3; ++mode) {
                float best = 1e9;
                for (int rep = 0; rep < 3; ++rep) {
                    (void)hipEventRecord(a);
                    if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(ncu * per_cu), dim3(64 * waves), 0, 0, out, iters);
                    if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(ncu * per_cu), dim3(64 * waves), 0, 0, out, iters);
                    if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(ncu * per_cu), dim3(64 * waves), 0, 0, out, iters);
                    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
                    float ms; (void)hipEventElapsedTime(&ms, a, b);
                    if (ms < best) best = ms;
                }
                t[mode] = best;
            }
            printf("waves/WG %d WG/CU %d: loop %.1f ns/iter, +barrier %.1f ns, +lds round trip (2 barriers) %.1f ns\n",
                   waves, per_cu, t[0] * 1e6 / iters, (t[1] - t[0]) * 1e6 / iters, (t[2] - t[0]) * 1e6 / iters);
        }
    return 0;
}
