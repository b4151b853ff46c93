// Where a C2 duplex launch spends its time, in the bench's sustained regime
// (round 3).  Per wave: start/end (s_memrealtime, 100 MHz), the shader clock
// (s_memtime) and its SIMD (HW_ID, XCC_ID).  For the C2 shape (64 Ki records
// per job, 8192 waves: two generations on the 1024 SIMDs) and a C4-like shape
// (512 Ki records per job, 16 generations), after WARM back-to-back launches:
// event time, wave span, launch ramp (first wave start) and tail (event end -
// last wave end), per-SIMD span spread, time with n waves resident, and the
// SIMD cycles per VALU instruction (VALU_PER_WAVE from the PMC profile).
// Modes: plain duplex (chachapoly_duplex_staged's block mapping) and a
// persistent grid with static wave-jobs (each resident wave takes wave-jobs
// w, w + W, ...).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../noise-c_amd/csrc timeline3.hip -o timeline3
#include "../../noise-c_amd/csrc/chachapoly.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
using namespace na;

struct Stamp { uint64_t t0, t1, c0, c1; uint32_t hw, xcc, kind, jobs; };

NA_DEV void stamp_out(Stamp *st, uint32_t w, uint64_t t0, uint64_t c0, uint32_t kind, uint32_t jobs)
{
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        Stamp s;
        s.t0 = t0; s.t1 = t1; s.c0 = c0; s.c1 = c1;
        s.hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        s.xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));
        s.kind = kind; s.jobs = jobs;
        st[w] = s;
    }
}

/* MODE 0: plain duplex (one wave-job per wave, blocks alternate seal/open);
   MODE 1: persistent static (grid of `grid` blocks, wave w runs wave-jobs
   w, w + W, ... of the interleaved seal/open ticket order) */
template <int MODE>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void timed(UniformArgs s, UniformArgs o, uint32_t sj,
                                                            uint32_t oj, Stamp *st)
{
    __shared__ uint4 tiles[4][512];
    __shared__ FinSlot fin[4];
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t w = threadIdx.x >> 6, gw = blockIdx.x * 4 + w;
    const uint32_t n = min(sj, oj), total = sj + oj;
    uint32_t kind = 0, jobs = 0;
    if (MODE == 0) {
        uint32_t b = blockIdx.x;
        const uint32_t nb = n / 4;
        bool open;
        if (b < 2 * nb) { open = b & 1; b >>= 1; }
        else { open = oj > sj; b -= nb; }
        if (open) open_il_staged<4, true>(o, tiles[w], &fin[w], wave_of(b));
        else seal_il_staged<4, true>(s, tiles[w], &fin[w], wave_of(b));
        kind = open; jobs = 1;
    } else {
        const uint32_t W = gridDim.x * 4;
        for (uint32_t t = gw; t < total; t += W) {
            bool open;
            uint32_t j;
            if (t < 2 * n) { open = t & 1; j = t >> 1; }
            else { open = oj > sj; j = t - n; }
            __builtin_amdgcn_wave_barrier();
            if (open) open_il_staged<4, true>(o, tiles[w], &fin[w], j);
            else seal_il_staged<4, true>(s, tiles[w], &fin[w], j);
            kind |= open ? 2u : 1u;
            ++jobs;
        }
    }
    stamp_out(st, gw, t0, c0, kind, jobs);
}

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[(size_t)(p * (v.size() - 1))];
}

template <int MODE>
static void run(const char *name, UniformArgs s, UniformArgs o, uint32_t sj, uint32_t oj, uint32_t grid,
                int warm, double valu_per_job)
{
    const uint32_t waves = grid * 4;
    Stamp *d;
    hipMalloc(&d, sizeof(Stamp) * waves);
    hipMemset(d, 0, sizeof(Stamp) * waves);
    hipEvent_t e[8];
    for (auto &x : e) hipEventCreate(&x);
    for (int i = 0; i < warm; ++i) hipLaunchKernelGGL((timed<MODE>), dim3(grid), dim3(256), 0, 0, s, o, sj, oj, d);
    hipEventRecord(e[0]);
    for (int i = 0; i < 5; ++i) {
        hipLaunchKernelGGL((timed<MODE>), dim3(grid), dim3(256), 0, 0, s, o, sj, oj, d);
        hipEventRecord(e[i + 1]);
    }
    hipEventSynchronize(e[5]);
    float ms[5];
    for (int i = 0; i < 5; ++i) hipEventElapsedTime(&ms[i], e[i], e[i + 1]);
    std::vector<Stamp> h(waves);
    hipMemcpy(h.data(), d, sizeof(Stamp) * waves, hipMemcpyDeviceToHost);
    uint64_t tmin = ~0ull, tmax = 0;
    for (auto &x : h) { tmin = std::min(tmin, x.t0); tmax = std::max(tmax, x.t1); }
    std::vector<double> start, end;
    double clk = 0; int nclk = 0;
    for (auto &x : h) {
        start.push_back((x.t0 - tmin) * 0.01);
        end.push_back((x.t1 - tmin) * 0.01);
        if (x.t1 - x.t0 > 500) { clk += (double)(x.c1 - x.c0) / ((x.t1 - x.t0) * 0.01); ++nclk; }
    }
    const double span = (tmax - tmin) * 0.01, mhz = nclk ? clk / nclk : 0.0;
    printf("%s (warm %d): events %.1f %.1f %.1f %.1f %.1f us; last: span %.2f us, clock %.0f MHz\n", name, warm,
           ms[0] * 1e3, ms[1] * 1e3, ms[2] * 1e3, ms[3] * 1e3, ms[4] * 1e3, span, mhz);
    printf("  start p50 %.2f p90 %.2f p100 %.2f | end p0 %.2f p50 %.2f p100 %.2f us; event - span %.2f us\n",
           pct(start, .5), pct(start, .9), pct(start, 1), pct(end, 0), pct(end, .5), pct(end, 1),
           ms[4] * 1e3 - span);
    std::map<uint32_t, std::vector<std::pair<double, int>>> ev;
    std::map<uint32_t, uint32_t> jobs_of;
    for (size_t i = 0; i < h.size(); ++i) {
        const uint32_t simd = (h[i].hw >> 4) & 3, cu = (h[i].hw >> 8) & 15, sh = (h[i].hw >> 12) & 1,
                       se = (h[i].hw >> 13) & 7;
        const uint32_t key = ((((h[i].xcc & 7) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd;
        ev[key].push_back({start[i], +1});
        ev[key].push_back({end[i], -1});
        jobs_of[key] += h[i].jobs;
    }
    double occ_t[9] = {0};
    std::vector<double> spans, ends, cpi;
    for (auto &kv : ev) {
        auto &v = kv.second;
        std::sort(v.begin(), v.end());
        int live = 0;
        double last = v.front().first;
        const double sp = v.back().first - v.front().first;
        spans.push_back(sp);
        ends.push_back(v.back().first);
        cpi.push_back(sp * mhz / (jobs_of[kv.first] * valu_per_job));
        for (auto &p : v) {
            occ_t[std::min(live, 8)] += p.first - last;
            last = p.first;
            live += p.second;
        }
    }
    const double ns = (double)ev.size();
    printf("  SIMDs %zu: span p0 %.2f p50 %.2f p100 %.2f us, end p50 %.2f p100 %.2f; cycles/VALU p50 %.3f; n waves:",
           ev.size(), pct(spans, 0), pct(spans, .5), pct(spans, 1), pct(ends, .5), pct(ends, 1), pct(cpi, .5));
    for (int k = 1; k <= 8; ++k)
        if (occ_t[k] > 0) printf(" %d:%.1f", k, occ_t[k] / ns);
    printf(" us\n");
    hipFree(d);
}

int main(int argc, char **argv)
{
    const int warm = argc > 1 ? atoi(argv[1]) : 40;
    const uint32_t only = argc > 2 ? (uint32_t)atoi(argv[2]) : 0; /* 0: both shapes */
    const bool persist = argc > 3 ? atoi(argv[3]) != 0 : true;
    const double valu = 8192.0; /* SQ_INSTS_VALU per wave-job (profiles/traffic_c2.json) */
    const uint32_t L = 1400, SI = 1408, SO = 1536;
    const bool big_first = argc > 4 && atoi(argv[4]) != 0; /* clock hysteresis check */
    const uint32_t order[2] = {big_first ? 524288u : 65536u, big_first ? 65536u : 524288u};
    for (uint32_t N : order) {
        if (only && N != only) continue;
        uint8_t *pa, *ca, *cb, *back, *key, *st;
        uint64_t *nb;
        hipMalloc(&pa, (size_t)N * SI + 4096); hipMalloc(&ca, (size_t)N * SO + 4096);
        hipMalloc(&cb, (size_t)N * SO + 4096); hipMalloc(&back, (size_t)N * SI + 4096);
        hipMalloc(&key, 32); hipMalloc(&nb, 8); hipMalloc(&st, N);
        hipMemset(pa, 0x5a, (size_t)N * SI); hipMemset(key, 7, 32); hipMemset(nb, 0, 8);
        UniformArgs sa{key, nb, pa, ca, nullptr, nullptr, SI, SO, 0, N, N, L, 0, 0, 0};
        UniformArgs sb{key, nb, pa, cb, nullptr, nullptr, SI, SO, 0, N, N, L, 0, 0, 0};
        hipLaunchKernelGGL((chachapoly_seal_staged<4, true>), dim3(N * 4 / 256), dim3(256), 0, 0, sb);
        UniformArgs ob{key, nb, cb, back, nullptr, st, SO, SI, 0, N, N, L, 0, 0, 0};
        hipDeviceSynchronize();
        const uint32_t jobs = N / 16;
        char name[64];
        snprintf(name, sizeof name, "N=%u plain", N);
        run<0>(name, sa, ob, jobs, jobs, 2 * jobs / 4, warm, valu);
        snprintf(name, sizeof name, "N=%u persist-static", N);
        if (persist) run<1>(name, sa, ob, jobs, jobs, 1024, warm, valu);
        hipFree(pa); hipFree(ca); hipFree(cb); hipFree(back); hipFree(key); hipFree(nb); hipFree(st);
    }
    return 0;
}
