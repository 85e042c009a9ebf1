// Per-phase timing of the 4-wave tile kernel k_pq_lin (timing-only build of ezrs_ps.hip with
// EZRS_PS_STAMPS): s_memtime at each phase boundary of every workgroup's first 9 tiles, and
// s_memrealtime + s_memtime at each workgroup's start and end (its clock).  Decode runs on 1 M valid
// RS(255,223) codewords (random data encoded on the host: the clean C2 case); encode on random data.
// Usage: pq_stamps [enc]
#define EZRS_PS_STAMPS 1
#include "../../ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>
using namespace ezrs;

// host RS(255,223) over 0x11d, fcr 1, prim 1: parity = x^32 d(x) mod g(x) (rs_base:1296-1332)
static void host_encode(uint8_t *cw, const uint8_t *A, const uint8_t *L, const uint8_t *g) {
    uint8_t par[32] = {0};
    for (int i = 0; i < 223; ++i) {
        const uint8_t fb = cw[i] ^ par[0];
        for (int j = 0; j < 31; ++j) par[j] = par[j + 1] ^ (fb && g[31 - j] ? A[(L[fb] + L[g[31 - j]]) % 255] : 0);
        par[31] = fb && g[0] ? A[(L[fb] + L[g[0]]) % 255] : 0;
    }
    for (int j = 0; j < 32; ++j) cw[223 + j] = par[j];
}

int main(int argc, char **argv) {
    const int enc = argc > 1 ? atoi(argv[1]) : 0;
    const size_t ncw = 1u << 20;
    uint8_t A[256], L[256];
    for (int i = 0, x = 1; i < 255; ++i) { A[i] = (uint8_t)x; L[x] = (uint8_t)i; x <<= 1; if (x & 256) x ^= 0x11d; }
    // g(x) = prod_{i=1..32} (x - alpha^i), coefficients g[0] (x^0) .. g[32] = 1
    uint8_t g[33] = {1};
    for (int i = 1; i <= 32; ++i) {
        uint8_t ng[33] = {0};
        for (int k = 0; k <= 32; ++k) {
            if (k > 0) ng[k] ^= g[k - 1];
            if (g[k]) ng[k] ^= A[(L[g[k]] + i) % 255];
        }
        std::copy(ng, ng + 33, g);
    }
    std::vector<uint8_t> h(ncw * 255);
    uint64_t st = 0x5EED;
    for (auto &b : h) { st = st * 6364136223846793005ull + 1442695040888963407ull; b = (uint8_t)(st >> 56); }
    if (!enc) {   // 4096 distinct valid codewords, tiled over the batch
        for (size_t k = 0; k < 4096; ++k) host_encode(&h[k * 255], A, L, g);
        for (size_t k = 4096; k < ncw; ++k) std::copy(&h[(k % 4096) * 255], &h[(k % 4096) * 255] + 255, &h[k * 255]);
    }
    uint8_t *d, *ws; int32_t *res;
    (void)hipMalloc(&d, ncw * 255); (void)hipMalloc(&ws, ncw * 32 + 65536); (void)hipMalloc(&res, ncw * 4);
    (void)hipMemcpy(d, h.data(), ncw * 255, hipMemcpyHostToDevice);
    int ncu = 0; (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    ps::PsArgs p{};
    p.base = d; p.span = ncw * 255 - (enc ? 32 : 0); p.stride = 255; p.ncw = ncw; p.ntiles = ncw / 256;
    p.lo = 0; p.result = res; p.ws = ws; p.ws_pitch = enc ? (ncw + 2047) / 2048 * 2048 : 0;
    unsigned grid = 2 * ncu;
    float best = 1e9f;
    for (int rep = 0; rep < 60; ++rep) {
        hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        if (enc) hipLaunchKernelGGL((ps::pq::k_pq_lin<ps::PQ_RS_255_223, true, false, true>), dim3(grid), dim3(256), 0, 0, p);
        else hipLaunchKernelGGL((ps::pq::k_pq_lin<ps::PQ_RS_255_223, false, false, true>), dim3(grid), dim3(256), 0, 0, p);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
        if (rep % 20 == 19) printf("%s: %.1f us (best %.1f)\n", enc ? "encode syndromes" : "decode", ms * 1e3, best * 1e3);
    }
    if (!enc) {
        std::vector<int32_t> r(ncw);
        (void)hipMemcpy(r.data(), res, ncw * 4, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (auto x : r) bad += x != 0;
        printf("flagged codewords: %zu (expect 0)\n", bad);
    }
    static unsigned long long stp[512][4][9][8], rt[512][4];
    (void)hipMemcpyFromSymbol(stp, HIP_SYMBOL(ps::g_pq_stamps), sizeof stp);
    (void)hipMemcpyFromSymbol(rt, HIP_SYMBOL(ps::g_pq_rt), sizeof rt);
    const char *names[] = {"dma+bar", "main", "bar", "xchg", "fold", "st", "next", ""};
    const int nph = 6;                                            // phases within a tile
    // per-workgroup duration and clock
    std::vector<double> dur, clk;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int wg = 0; wg < (int)grid && wg < 512; ++wg) {
        dur.push_back((rt[wg][2] - rt[wg][0]) * 0.01);                 // us (100 MHz)
        clk.push_back((double)(rt[wg][3] - rt[wg][1]) / (double)(rt[wg][2] - rt[wg][0]) * 0.1);   // GHz
        t0 = std::min(t0, rt[wg][0]); t1 = std::max(t1, rt[wg][2]);
    }
    std::vector<double> sd = dur, sc = clk;
    std::sort(sd.begin(), sd.end()); std::sort(sc.begin(), sc.end());
    printf("workgroup duration us: min %.1f med %.1f max %.1f; first start -> last end %.1f us\n",
           sd.front(), sd[sd.size() / 2], sd.back(), (t1 - t0) * 0.01);
    printf("workgroup clock GHz: min %.3f med %.3f max %.3f\n", sc.front(), sc[sc.size() / 2], sc.back());
    // start skew
    std::vector<double> s0;
    for (int wg = 0; wg < (int)grid && wg < 512; ++wg) s0.push_back((rt[wg][0] - t0) * 0.01);
    std::sort(s0.begin(), s0.end());
    printf("start skew us: med %.2f max %.2f\n", s0[s0.size() / 2], s0.back());
    // co-residency: workgroups sharing a CU (HW_ID cu/sh/se + XCC_ID), the phase offset of the pair
    static unsigned hw[512][2];
    (void)hipMemcpyFromSymbol(hw, HIP_SYMBOL(ps::g_pq_hw), sizeof hw);
    {
        std::vector<std::pair<unsigned, int>> key;
        for (int wg = 0; wg < (int)grid && wg < 512; ++wg) {
            const unsigned h = hw[wg][0], cu = (h >> 8) & 15, sh = (h >> 12) & 1, se = (h >> 13) & 7;
            key.push_back({(hw[wg][1] & 15) << 8 | se << 5 | sh << 4 | cu, wg});
        }
        std::sort(key.begin(), key.end());
        int pairs = 0, bplus = 0;
        double off = 0;
        for (size_t i = 0; i + 1 < key.size(); ++i)
            if (key[i].first == key[i + 1].first) {
                ++pairs;
                const int a = key[i].second, b = key[i + 1].second;
                bplus += std::abs(a - b) == (int)grid / 2;
                // phase offset of the pair's tile-1 main-loop starts, in ticks
                off += std::fabs((double)stp[a][0][1][1] - (double)stp[b][0][1][1]);
                if (pairs <= 6) printf("  pair wg %d + wg %d (cu key %x)\n", a, b, key[i].first);
            }
        printf("co-resident pairs: %d, of which b and b+grid/2: %d; mean |tile-1 start offset| %.0f ticks\n", pairs, bplus,
               pairs ? off / pairs : 0.0);
    }
    const int ntile = std::min<int>(9, (int)((ncw / 256 + grid - 1) / grid));
    for (int it = 0; it < ntile; ++it) {
        double acc[8] = {};
        int n = 0;
        for (int wg = 0; wg < (int)grid && wg < 512; ++wg)
            for (int w = 0; w < 4; ++w) {
                ++n;
                for (int ph = 0; ph < nph; ++ph) acc[ph] += (double)(stp[wg][w][it][ph + 1] - stp[wg][w][it][ph]);
                if (it + 1 < ntile) acc[nph] += (double)(stp[wg][w][it + 1][0] - stp[wg][w][it][nph]);
            }
        printf(" tile %d:", it);
        double tot = 0;
        for (int ph = 0; ph <= nph; ++ph) { printf(" %s %6.0f", names[ph], acc[ph] / n); tot += acc[ph] / n; }
        printf("  | total %6.0f\n", tot);
    }
    return 0;
}
