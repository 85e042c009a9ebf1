// Per-phase timing of the encode parity kernel k_ps_parity8 (timing-only build of ezrs_ps.hip with
// EZRS_PS_STAMPS): s_memtime at each phase boundary of blocks 0..63, every wave, on the C2 shape
// (1M codewords, parity written in place at column 223 of 255-byte rows).  Usage: par_stamps
#define EZRS_PS_STAMPS 1
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip"
#include <cstdio>
using namespace ezrs;
int main() {
    const size_t ncw = 1u << 20, pitch = (ncw + 2047) / 2048 * 2048;
    uint8_t *rows, *ws;
    (void)hipMalloc(&rows, ncw * 255); (void)hipMalloc(&ws, 32 * pitch);
    (void)hipMemset(ws, 0x5a, 32 * pitch);
    const unsigned grid = (unsigned)((ncw + ps::kParCw - 1) / ps::kParCw);
    for (int rep = 0; rep < 4; ++rep) {
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((ps::k_ps_parity8<ps::PS_RS_255_223>), dim3(grid), dim3(512), 0, 0, ws, pitch, rows + 223,
                           (size_t)255, ncw, Shards{}, 223u);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        printf("parity8: %.1f us\n", ms * 1e3);
    }
    static unsigned long long st[64][8][8];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(ps::g_par_stamps), sizeof st);
    const char *names[] = {"load+tr", "bar", "map", "bar", "stage", "bar", "store"};
    double acc[8][7] = {};
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int blk = 0; blk < 64; ++blk)
        for (int w = 0; w < 8; ++w) {
            for (int ph = 0; ph < 7; ++ph) acc[w][ph] += (double)(st[blk][w][ph + 1] - st[blk][w][ph]);
            t0 = st[blk][w][0] < t0 ? st[blk][w][0] : t0;
            t1 = st[blk][w][7] > t1 ? st[blk][w][7] : t1;
        }
    printf("ticks per block (s_memtime), mean over 64 blocks; first start .. last end %llu\n", t1 - t0);
    for (int w = 0; w < 8; ++w) {
        printf(" wave %d:", w);
        double tot = 0;
        for (int ph = 0; ph < 7; ++ph) { printf(" %s %6.0f", names[ph], acc[w][ph] / 64); tot += acc[w][ph] / 64; }
        printf("  | total %6.0f\n", tot);
    }
    static unsigned long long rt[4096][2];
    static unsigned hw[4096];
    (void)hipMemcpyFromSymbol(rt, HIP_SYMBOL(ps::g_par_rt), sizeof rt);
    (void)hipMemcpyFromSymbol(hw, HIP_SYMBOL(ps::g_par_hw), sizeof hw);
    unsigned long long r0 = ~0ull, r1 = 0;
    for (unsigned b = 0; b < grid; ++b) { r0 = rt[b][0] < r0 ? rt[b][0] : r0; r1 = rt[b][1] > r1 ? rt[b][1] : r1; }
    printf("realtime (100 MHz ticks = 10 ns): first start .. last end %llu ticks\n", r1 - r0);
    int hist_s[64] = {}, hist_d[64] = {};
    double dsum = 0;
    for (unsigned b = 0; b < grid; ++b) {
        const unsigned long long s_ = (rt[b][0] - r0) / 100, d = (rt[b][1] - rt[b][0]) / 100;  // us
        hist_s[s_ < 63 ? s_ : 63]++;
        hist_d[d < 63 ? d : 63]++;
        dsum += (double)(rt[b][1] - rt[b][0]) / 100.0;
    }
    printf("block durations: mean %.2f us\nstart-time histogram (us: count):", dsum / grid);
    for (int i = 0; i < 64; ++i) if (hist_s[i]) printf(" %d:%d", i, hist_s[i]);
    printf("\nduration histogram (us: count):");
    for (int i = 0; i < 64; ++i) if (hist_d[i]) printf(" %d:%d", i, hist_d[i]);
    printf("\nHW_ID of blocks 0..15:");
    for (int b = 0; b < 16; ++b) printf(" %08x", hw[b]);
    printf("\n");
    unsigned long long s0[64];
    for (int blk = 0; blk < 64; ++blk) s0[blk] = st[blk][0][0] - t0;
    printf("block start offsets:");
    for (int blk = 0; blk < 64; blk += 4) printf(" %llu", s0[blk]);
    printf("\n");
    return 0;
}
