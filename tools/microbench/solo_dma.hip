// The one-lane kernels' memory pattern alone (round 4): a C2 duplex launch
// shape (64 Ki records per job, 128-B slots, 2048 waves, two per SIMD) that
// moves every record through the LDS tiles exactly as chachapoly_duplex_solo
// does — LDS-DMA of 8 records x 128 B per instruction, owner reads, the
// coalesced 16-B stores — with the ChaCha20/Poly1305 arithmetic replaced by
// one XOR.  Its rate is the HBM ceiling of that access pattern.
// arg: 0 reads only, 1 reads + stores (the kernel's pattern), 2 stores only
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../noise-c_amd/csrc solo_dma.hip -o solo_dma
#include "../../noise-c_amd/csrc/chachapoly.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace na;

__global__ __launch_bounds__(256) NA_SOLO_OCC void dma_only(UniformArgs s, UniformArgs o, uint32_t blocks, int stores)
{
    __shared__ uint4 tiles[4][2 * SOLO_TILE];
    uint32_t b = blockIdx.x;
    const bool second = b >= blocks; /* runs of the CU count as in the duplex: here seal run, open run */
    if (second) b -= blocks;
    const UniformArgs &a = second ? o : s;
    const SoloRec q = solo_rec(a, wave_of(b));
    uint4 *t = tiles[threadIdx.x >> 6];
    const bool reads = stores != 2;
    if (q.S && reads) solo_dma(a, q.rec0, q.lane, 0, q.lim, t);
    uint32_t acc = 0;
    for (uint32_t m = 0; m < q.S; ++m) {
        uint4 *cur = t + SOLO_TILE * (m & 1), *nxt = t + SOLO_TILE * ((m + 1) & 1);
        uint32_t wu[2][16];
        solo_wait();
        solo_get(cur, q.lane, 0, wu[0]);
        solo_get(cur, q.lane, 1, wu[1]);
        if (stores && m >= 1) solo_store(a, q.rec0, q.lane, m - 1, q.full_lim, nxt, 0xffu);
        __builtin_amdgcn_wave_barrier();
        if (m + 1 < q.S && reads) solo_dma(a, q.rec0, q.lane, m + 1, q.lim, nxt);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int i = 0; i < 16; ++i) { wu[u][i] ^= 0x9e3779b9u; acc += wu[u][i]; }
            if (stores) solo_put(cur, q.lane, u, wu[u]);
        }
    }
    if (stores && q.S) {
        __builtin_amdgcn_wave_barrier();
        solo_store(a, q.rec0, q.lane, q.S - 1, q.full_lim, t + SOLO_TILE * ((q.S - 1) & 1), 0xffu);
    }
    if (acc == 0x12345678u) a.status[0] = 1; /* keep the reads */
}

int main(int argc, char **argv)
{
    const int stores = argc > 1 ? atoi(argv[1]) : 1;
    const int sets = 4, warm = 1000;
    const uint32_t N = 65536, L = 1400, SI = 1408, SO = 1536;
    uint8_t *key, *stt;
    uint64_t *nb;
    hipMalloc(&key, 32); hipMalloc(&nb, 8); hipMalloc(&stt, N);
    std::vector<UniformArgs> S, O;
    for (int k = 0; k < sets; ++k) {
        uint8_t *pa, *ca, *cb, *back;
        hipMalloc(&pa, (size_t)N * SI + 4096); hipMalloc(&ca, (size_t)N * SO + 4096);
        hipMalloc(&cb, (size_t)N * SO + 4096); hipMalloc(&back, (size_t)N * SI + 4096);
        hipMemset(pa, 1, (size_t)N * SI); hipMemset(cb, 2, (size_t)N * SO);
        S.push_back(UniformArgs{key, nb, pa, ca, nullptr, stt, SI, SO, 0, N, N, L, 0, 0, 0});
        O.push_back(UniformArgs{key, nb, cb, back, nullptr, stt, SO, SI, 0, N, N, L, 0, 0, 0});
    }
    const uint32_t blocks = N / 256;
    for (int i = 0; i < warm; ++i)
        hipLaunchKernelGGL(dma_only, dim3(2 * blocks), dim3(256), 0, 0, S[i % sets], O[i % sets], blocks, stores);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 40; ++i)
        hipLaunchKernelGGL(dma_only, dim3(2 * blocks), dim3(256), 0, 0, S[i % sets], O[i % sets], blocks, stores);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 40;
    const double bytes = stores == 1 ? 2.0 * N * (2.0 * L + 16) : 2.0 * N * (L + 8.0);
    printf("stores=%d: %.1f us per launch, %.2f TB/s of algorithmic bytes (%.0f MB)\n", stores, us,
           bytes / (us * 1e-6) / 1e12, bytes / 1e6);
    return 0;
}
