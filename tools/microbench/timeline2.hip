// Wave timelines of the production ChaChaPoly kernels on the C2 shape (64Ki x
// 1400 B, one key): seal, open (of ciphertext sealed into a second buffer set)
// and the duplex launch (seal set A while opening set B).  Per wave: start/end
// (s_memrealtime, 100 MHz), the shader clock (s_memtime) and its hardware
// place (HW_ID, XCC_ID).  Reports the dispatch ramp, the kernel event time vs
// the waves' span, and per SIMD how long it held 4, 3, 2, 1 waves — where a
// one-generation launch loses issue rate to its own tail.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../noise-c_amd/csrc timeline2.hip -o timeline2
#include "../../noise-c_amd/csrc/chachapoly.hip"
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>
using namespace na;

struct Stamp { uint64_t t0, t1, c0, c1; uint32_t hw, xcc, kind, pad; };

NA_DEV void stamp_out(Stamp *st, uint64_t t0, uint64_t c0, uint32_t kind)
{
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = (blockIdx.x * 256u + threadIdx.x) >> 6;
        Stamp s;
        s.t0 = t0; s.t1 = t1; s.c0 = c0; s.c1 = c1;
        s.hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        s.xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));
        s.kind = kind; s.pad = 0;
        st[w] = s;
    }
}

/* MODE 0 seal, 1 open, 2 duplex (blocks alternate as chachapoly_duplex_staged) */
template <int MODE>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void timed(UniformArgs s, UniformArgs o, uint32_t sb,
                                                            uint32_t ob, Stamp *st)
{
    __shared__ uint4 tiles[4][512];
    __shared__ FinSlot fin[4];
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t b = blockIdx.x;
    bool open = MODE == 1;
    if (MODE == 2) {
        const uint32_t n = min(sb, ob);
        if (b < 2 * n) { open = b & 1; b >>= 1; }
        else { open = ob > sb; b -= n; }
    }
    if (open) open_il_staged<4, true>(o, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], b);
    else seal_il_staged<4, true>(s, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], b);
    stamp_out(st, t0, c0, open ? 1u : 0u);
}

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[(size_t)(p * (v.size() - 1))];
}

template <int MODE>
static void run(const char *name, UniformArgs s, UniformArgs o, uint32_t sb, uint32_t ob)
{
    const uint32_t blocks = MODE == 0 ? sb : (MODE == 1 ? ob : sb + ob), waves = blocks * 4;
    Stamp *d;
    hipMalloc(&d, sizeof(Stamp) * waves);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((timed<MODE>), dim3(blocks), dim3(256), 0, 0, s, o, sb, ob, d);
    hipEventRecord(e0);
    hipLaunchKernelGGL((timed<MODE>), dim3(blocks), dim3(256), 0, 0, s, o, sb, ob, d);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<Stamp> h(waves);
    hipMemcpy(h.data(), d, sizeof(Stamp) * waves, hipMemcpyDeviceToHost);
    uint64_t tmin = ~0ull, tmax = 0;
    for (auto &x : h) { tmin = std::min(tmin, x.t0); tmax = std::max(tmax, x.t1); }
    std::vector<double> dur[2], start, end;
    double clk = 0; int nclk = 0;
    for (auto &x : h) {
        dur[x.kind & 1].push_back((x.t1 - x.t0) * 0.01);
        start.push_back((x.t0 - tmin) * 0.01);
        end.push_back((x.t1 - tmin) * 0.01);
        if (x.t1 - x.t0 > 500) { clk += (double)(x.c1 - x.c0) / ((x.t1 - x.t0) * 0.01); ++nclk; }
    }
    const double span = (tmax - tmin) * 0.01;
    printf("%s: event %.2f us, waves %u, span %.2f us, shader clock %.0f MHz\n", name, ms * 1e3, waves,
           span, nclk ? clk / nclk : 0.0);
    printf("  start p50 %.2f p90 %.2f p100 %.2f | end p0 %.2f p50 %.2f p100 %.2f us\n", pct(start, .5),
           pct(start, .9), pct(start, 1), pct(end, 0), pct(end, .5), pct(end, 1));
    for (int k = 0; k < 2; ++k)
        if (!dur[k].empty())
            printf("  %s waves: dur p0 %.2f p50 %.2f p100 %.2f mean %.2f us\n", k ? "open" : "seal",
                   pct(dur[k], 0), pct(dur[k], .5), pct(dur[k], 1),
                   [&] { double t = 0; for (double v : dur[k]) t += v; return t / dur[k].size(); }());
    // per SIMD: time holding n resident waves (event sweep)
    std::map<uint32_t, std::vector<std::pair<double, int>>> ev;
    for (size_t i = 0; i < h.size(); ++i) {
        const uint32_t simd = (h[i].hw >> 4) & 3, cu = (h[i].hw >> 8) & 15, sh = (h[i].hw >> 12) & 1,
                       se = (h[i].hw >> 13) & 7;
        const uint32_t key = ((((h[i].xcc & 7) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd;
        ev[key].push_back({start[i], +1});
        ev[key].push_back({end[i], -1});
    }
    double occ_t[9] = {0}, simd_span = 0;
    for (auto &kv : ev) {
        auto &v = kv.second;
        std::sort(v.begin(), v.end());
        int live = 0;
        double last = v.front().first;
        simd_span += v.back().first - v.front().first;
        for (auto &p : v) {
            occ_t[std::min(live, 8)] += p.first - last;
            last = p.first;
            live += p.second;
        }
    }
    const double ns = (double)ev.size();
    printf("  SIMDs %zu, mean SIMD span %.2f us; mean time with n waves:", ev.size(), simd_span / ns);
    for (int n = 1; n <= 8; ++n)
        if (occ_t[n] > 0) printf(" %d:%.2f", n, occ_t[n] / ns);
    printf(" us\n");
    hipFree(d);
}

int main()
{
    const uint32_t N = 65536, L = 1400, SI = 1408, SO = 1424;
    uint8_t *pa, *ca, *pb, *cb, *back, *key, *st;
    uint64_t *nb;
    hipMalloc(&pa, (size_t)N * SO + 4096); hipMalloc(&ca, (size_t)N * SO + 4096);
    hipMalloc(&pb, (size_t)N * SO + 4096); hipMalloc(&cb, (size_t)N * SO + 4096);
    hipMalloc(&back, (size_t)N * SO + 4096);
    hipMalloc(&key, 32); hipMalloc(&nb, 8); hipMalloc(&st, N);
    hipMemset(pa, 0x5a, (size_t)N * SO); hipMemset(pb, 0x33, (size_t)N * SO);
    hipMemset(key, 7, 32); hipMemset(nb, 0, 8);
    UniformArgs sa{key, nb, pa, ca, nullptr, nullptr, SI, SO, 0, N, N, L, 0, 0};
    UniformArgs sbj{key, nb, pb, cb, nullptr, nullptr, SI, SO, 0, N, N, L, 0, 0};
    const uint32_t blocks = N * 4 / 256;
    hipLaunchKernelGGL((chachapoly_seal_staged<4, true>), dim3(blocks), dim3(256), 0, 0, sbj);
    UniformArgs ob{key, nb, cb, back, nullptr, st, SO, SI, 0, N, N, L, 0, 0};
    hipDeviceSynchronize();
    run<0>("seal", sa, ob, blocks, blocks);
    sa.balance = 1;
    run<0>("seal+prio", sa, ob, blocks, blocks);
    sa.balance = 0;
    run<1>("open", sa, ob, blocks, blocks);
    ob.balance = 1;
    run<1>("open+prio", sa, ob, blocks, blocks);
    ob.balance = 0;
    run<2>("duplex", sa, ob, blocks, blocks);
    sa.balance = ob.balance = 1;
    run<2>("duplex+prio", sa, ob, blocks, blocks);
    return 0;
}
