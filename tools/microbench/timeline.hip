// Wave timeline of the production staged seal kernel on the C2 shape
// (64Ki x 1400 B, one key): per wave start/end (s_memrealtime, 100 MHz) and
// hardware placement (HW_ID, XCC_ID).  Answers: how long the dispatch ramp
// is, how long one wave runs, how many waves a SIMD holds over time, and
// how much of the kernel is tail.
#include "../../noise-c_amd/csrc/chachapoly.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
using namespace na;

struct Stamp { uint64_t t0, t1, c0, c1; uint32_t hw, xcc; };

template <int K, int MODE>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void timed(UniformArgs a, Stamp *st)
{
    __shared__ uint4 tiles[4][512];
    __shared__ FinSlot fin[4];
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (MODE == 0) seal_il_staged<K, true>(a, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6]);
    else open_il_staged<K, true>(a, tiles[threadIdx.x >> 6]);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = (blockIdx.x * 256u + threadIdx.x) >> 6;
        st[w] = Stamp{t0, t1, c0, c1, (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)),
                      (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11))};
    }
}

template <int K, int MODE>
static void run(const char *name, UniformArgs a, uint32_t N)
{
    const uint32_t waves = (N * K + 63) / 64, blocks = (waves + 3) / 4;
    Stamp *d;
    hipMalloc(&d, sizeof(Stamp) * blocks * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((timed<K, MODE>), dim3(blocks), dim3(256), 0, 0, a, d);
    hipEventRecord(e0);
    hipLaunchKernelGGL((timed<K, MODE>), dim3(blocks), dim3(256), 0, 0, a, d);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<Stamp> h(waves);
    hipMemcpy(h.data(), d, sizeof(Stamp) * waves, hipMemcpyDeviceToHost);
    uint64_t tmin = ~0ull, tmax = 0;
    for (auto &s : h) { tmin = std::min(tmin, s.t0); tmax = std::max(tmax, s.t1); }
    std::vector<double> dur, start, end;
    for (auto &s : h) {
        dur.push_back((s.t1 - s.t0) * 0.01);
        start.push_back((s.t0 - tmin) * 0.01);
        end.push_back((s.t1 - tmin) * 0.01);
    }
    auto pct = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
    printf("%s K=%d: event %.2f us, waves %u, span %.2f us\n", name, K, ms * 1e3, waves, (tmax - tmin) * 0.01);
    printf("  start  p0 %.2f p50 %.2f p90 %.2f p100 %.2f us\n", pct(start, 0), pct(start, .5), pct(start, .9), pct(start, 1));
    printf("  end    p0 %.2f p10 %.2f p50 %.2f p90 %.2f p100 %.2f us\n", pct(end, 0), pct(end, .1), pct(end, .5), pct(end, .9), pct(end, 1));
    printf("  dur    p0 %.2f p10 %.2f p50 %.2f p90 %.2f p100 %.2f us\n", pct(dur, 0), pct(dur, .1), pct(dur, .5), pct(dur, .9), pct(dur, 1));
    // waves per SIMD resident over time (XCC, SE, CU, SIMD -> key)
    std::vector<int> per(8 * 8 * 16 * 4 * 2, 0);
    int maxres = 0;
    for (auto &s : h) {
        const uint32_t simd = (s.hw >> 4) & 3, cu = (s.hw >> 8) & 15, sh = (s.hw >> 12) & 1, se = (s.hw >> 13) & 7;
        const uint32_t key = ((((s.xcc & 7) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd;
        if (key < per.size()) maxres = std::max(maxres, ++per[key]);
    }
    int used = 0; for (int c : per) used += c > 0;
    double clk = 0; int nclk = 0;
    for (auto &s : h) if (s.t1 - s.t0 > 500) { clk += (double)(s.c1 - s.c0) / ((s.t1 - s.t0) * 0.01); ++nclk; }
    printf("  s_memtime rate %.0f MHz (mean over waves)\n", nclk ? clk / nclk : 0.0);
    printf("  SIMDs used %d, waves per SIMD max %d\n", used, maxres);
    // concurrency histogram: resident waves at 10 instants
    for (int q = 1; q <= 9; ++q) {
        const double t = (tmax - tmin) * 0.01 * q / 10;
        int live = 0; for (size_t i = 0; i < h.size(); ++i) live += start[i] <= t && end[i] > t;
        printf("  t=%5.1f us resident %d\n", t, live);
    }
    hipFree(d);
}

int main()
{
    const uint32_t N = 65536, L = 1400, SI = 1408, SO = 1424;
    uint8_t *in, *out, *key; uint64_t *nb;
    hipMalloc(&in, (size_t)N * SO + 4096); hipMalloc(&out, (size_t)N * SO + 4096);
    hipMalloc(&key, 32); hipMalloc(&nb, 8);
    hipMemset(in, 0x5a, (size_t)N * SO); hipMemset(key, 7, 32); hipMemset(nb, 0, 8);
    UniformArgs a{key, nb, in, out, nullptr, nullptr, SI, SO, 0, N, N, L, 0};
    run<4, 0>("seal", a, N);
    run<8, 0>("seal", a, N);
    // open of the sealed records (all verify)
    hipLaunchKernelGGL((chachapoly_seal_staged<4, true>), dim3(N * 4 / 256), dim3(256), 0, 0, a);
    uint8_t *st; hipMalloc(&st, N);
    UniformArgs o{key, nb, out, in, nullptr, st, SO, SI, 0, N, N, L, 0};
    run<4, 1>("open", o, N);
    return 0;
}
