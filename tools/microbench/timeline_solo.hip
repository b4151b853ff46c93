// Where a C2 duplex launch of the one-lane kernels spends its time (round 4):
// chachapoly_duplex_solo's block mapping (seal/open runs of the CU count, or
// block-by-block with RUN=0), the open one-pass or verify-first.  Per wave:
// start, the open's end of authentication (verify-first: the AUTH pass;
// one-pass: the whole pass), end (s_memrealtime, 100 MHz), and its SIMD.
// Reports per kind the start/end/AUTH distributions, how SIMDs pair the
// kinds, and the time the SIMDs spend with 0/1/2 waves resident.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../noise-c_amd/csrc timeline_solo.hip -o timeline_solo
#include <cstdint>
__device__ uint64_t g_auth_t[8192];
#define NA_SOLO_AUTH_HOOK() do { if ((threadIdx.x & 63) == 0) g_auth_t[blockIdx.x * 4 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#include "../../noise-c_amd/csrc/chachapoly.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
using namespace na;

struct Stamp { uint64_t t0, t1; uint32_t hw, xcc, kind, pad; };

__global__ __launch_bounds__(256) NA_SOLO_OCC void timed(UniformArgs s, UniformArgs o, uint32_t sb, uint32_t ob,
                                                         uint32_t C, Stamp *st)
{
    __shared__ uint4 tiles[4][2 * SOLO_TILE];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t n = min(sb, ob);
    const uint32_t full = C ? n / C * C : 0;
    uint32_t b = blockIdx.x;
    bool open;
    if (b < 2 * full) {
        const uint32_t run = b / C;
        open = run & 1;
        b = (run >> 1) * C + b % C;
    } else if (b < 2 * n) {
        b -= 2 * full;
        open = b & 1;
        b = full + (b >> 1);
    } else {
        open = ob > sb;
        b -= n;
    }
    if (open) open_solo_staged<true, true>(o, tiles[threadIdx.x >> 6], wave_of(b));
    else seal_solo_staged<true, true>(s, tiles[threadIdx.x >> 6], wave_of(b));
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        Stamp x;
        x.t0 = t0; x.t1 = t1;
        x.hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        x.xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));
        x.kind = open; x.pad = 0;
        st[blockIdx.x * 4 + (threadIdx.x >> 6)] = x;
    }
}

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char **argv)
{
    const int vf = argc > 1 ? atoi(argv[1]) : 0;
    const uint32_t C = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
    const int warm = argc > 3 ? atoi(argv[3]) : 2000;
    /* sets > 1: launch i seals and opens set i mod sets (4 sets: > 1.5 GB,
       beyond the 256 MB MALL, as the bench's rotating sets) */
    const int sets = argc > 4 ? atoi(argv[4]) : 1;
    const uint32_t N = 65536, L = 1400, SI = 1408, SO = 1536;
    uint8_t *key, *stt;
    uint64_t *nb;
    hipMalloc(&key, 32); hipMalloc(&nb, 8); hipMalloc(&stt, N);
    hipMemset(key, 7, 32); hipMemset(nb, 0, 8);
    std::vector<UniformArgs> SA, OB;
    for (int k = 0; k < sets; ++k) {
        uint8_t *pa, *ca, *cb, *back;
        hipMalloc(&pa, (size_t)N * SI + 4096); hipMalloc(&ca, (size_t)N * SO + 4096);
        hipMalloc(&cb, (size_t)N * SO + 4096); hipMalloc(&back, (size_t)N * SI + 4096);
        hipMemset(pa, 0x5a + k, (size_t)N * SI);
        UniformArgs sa{key, nb, pa, ca, nullptr, nullptr, SI, SO, 0, N, N, L, 0, 1, 0}; /* balance: one generation, as the library sets it */
        UniformArgs sb{key, nb, pa, cb, nullptr, nullptr, SI, SO, 0, N, N, L, 0, 0, 0};
        hipLaunchKernelGGL((chachapoly_seal_solo<true, true>), dim3(N / 256), dim3(256), 0, 0, sb);
        UniformArgs ob{key, nb, cb, back, nullptr, stt, SO, SI, 0, N, N, L, 0, 1, (uint32_t)vf};
        SA.push_back(sa);
        OB.push_back(ob);
    }
    hipDeviceSynchronize();
    const UniformArgs &sa = SA[0], &ob = OB[0];
    const uint32_t blocks = N / 256, grid = 2 * blocks, waves = grid * 4;
    Stamp *d;
    hipMalloc(&d, sizeof(Stamp) * waves);
    for (int i = 0; i < warm; ++i)
        hipLaunchKernelGGL(timed, dim3(grid), dim3(256), 0, 0, SA[(i + 1) % sets], OB[(i + 1) % sets], blocks, blocks,
                           C, d);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    if (argc > 5 && atoi(argv[5])) { /* the library's own kernel, 20 launches after the same warmup */
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i)
            hipLaunchKernelGGL((chachapoly_duplex_solo<true>), dim3(grid), dim3(256), 0, 0, SA[i % sets],
                               OB[i % sets], blocks, blocks, C);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float lib_ms = 0;
        hipEventElapsedTime(&lib_ms, e0, e1);
        printf("library chachapoly_duplex_solo<true>: %.1f us per launch (20 launches)\n", lib_ms * 1e3 / 20);
    }
    /* 20 launches timed together (the stamps are the last one's, set 0) */
    hipEventRecord(e0);
    for (int i = 19; i >= 0; --i)
        hipLaunchKernelGGL(timed, dim3(grid), dim3(256), 0, 0, SA[i % sets], OB[i % sets], blocks, blocks, C, d);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    std::vector<Stamp> h(waves);
    std::vector<uint64_t> au(waves);
    hipMemcpy(h.data(), d, sizeof(Stamp) * waves, hipMemcpyDeviceToHost);
    hipMemcpyFromSymbol(au.data(), HIP_SYMBOL(g_auth_t), sizeof(uint64_t) * waves);
    uint64_t tmin = ~0ull, tmax = 0;
    for (auto &x : h) { tmin = std::min(tmin, x.t0); tmax = std::max(tmax, x.t1); }
    std::vector<double> s0[2], s1[2], dur[2], auth;
    for (uint32_t i = 0; i < waves; ++i) {
        const int k = (int)h[i].kind;
        s0[k].push_back((h[i].t0 - tmin) * 0.01);
        s1[k].push_back((h[i].t1 - tmin) * 0.01);
        dur[k].push_back((h[i].t1 - h[i].t0) * 0.01);
        if (k) auth.push_back((au[i] - h[i].t0) * 0.01);
    }
    printf("sets=%d vf=%d C=%u: event %.1f us (mean of 20), span %.1f us\n", sets, vf, C, ms * 1e3, (tmax - tmin) * 0.01);
    for (int k = 0; k < 2; ++k)
        printf("  %s: start p50 %.1f p100 %.1f | end p0 %.1f p50 %.1f p100 %.1f | duration p50 %.1f p100 %.1f us\n",
               k ? "open" : "seal", pct(s0[k], .5), pct(s0[k], 1), pct(s1[k], 0), pct(s1[k], .5), pct(s1[k], 1),
               pct(dur[k], .5), pct(dur[k], 1));
    printf("  open: authenticated after p0 %.1f p50 %.1f p100 %.1f us of its run\n", pct(auth, 0), pct(auth, .5),
           pct(auth, 1));
    std::map<uint32_t, std::vector<int>> kinds;
    std::map<uint32_t, std::vector<std::pair<double, int>>> ev;
    for (uint32_t i = 0; i < waves; ++i) {
        const uint32_t simd = (h[i].hw >> 4) & 3, cu = (h[i].hw >> 8) & 15, sh = (h[i].hw >> 12) & 1,
                       se = (h[i].hw >> 13) & 7;
        const uint32_t key2 = ((((h[i].xcc & 7) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd;
        kinds[key2].push_back((int)h[i].kind);
        ev[key2].push_back({(h[i].t0 - tmin) * 0.01, +1});
        ev[key2].push_back({(h[i].t1 - tmin) * 0.01, -1});
    }
    int mix[3] = {0, 0, 0};
    for (auto &kv : kinds) {
        int o = 0;
        for (int k : kv.second) o += k;
        mix[std::min(o, 2)] += kv.second.size() == 2;
    }
    double occ[3] = {0, 0, 0};
    for (auto &kv : ev) {
        auto &v = kv.second;
        std::sort(v.begin(), v.end());
        int live = 0;
        double last = v.front().first;
        for (auto &p : v) {
            occ[std::min(live, 2)] += p.first - last;
            last = p.first;
            live += p.second;
        }
    }
    printf("  SIMDs %zu: pairs seal+seal %d, seal+open %d, open+open %d; mean time with 1 / 2 waves %.1f / %.1f us\n",
           kinds.size(), mix[0], mix[1], mix[2], occ[1] / kinds.size(), occ[2] / kinds.size());
    return 0;
}
