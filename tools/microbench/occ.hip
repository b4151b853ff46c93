// Issue rate of the hot loops vs resident waves per SIMD: W waves on each of
// the 1024 SIMDs, every lane runs NB iterations of (a) the ChaCha20 block,
// (b) a radix-2^26 Poly1305 multiply (fe_mul), (c) a radix-2^32 Poly1305
// block (p32_block).  Prints wall time and cycles per wave-iteration per SIMD
// at the nominal 2.4 GHz.
#include "../../noise-c_amd/csrc/aead_device.h"
#include <cstdio>
using namespace na;

template <int OP>
__global__ __launch_bounds__(256) void spin(uint32_t nb, uint32_t seed, uint32_t *sink)
{
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    uint32_t acc = 0;
    if constexpr (OP == 0) {
        uint32_t key[8];
        for (int i = 0; i < 8; ++i) key[i] = seed * (i + 1) ^ t;
        for (uint32_t b = 0; b < nb; ++b) {
            uint32_t x[16];
            chacha20_block(key, b, 0, t, seed, x);
            for (int i = 0; i < 16; ++i) acc += x[i];
        }
    } else if constexpr (OP == 1) {
        Fe h = Fe{t, seed, t ^ 5, 7, 1};
        const Mul m = mk_mul(fe_clamp_r(seed, t, seed ^ t, 3));
        for (uint32_t b = 0; b < nb; ++b) {
            h = fe_mul(h, m);
            fe_add_block(h, b, t, b ^ t, seed);
        }
        acc = h.l0 ^ h.l1 ^ h.l2 ^ h.l3 ^ h.l4;
    } else {
        P32 h = P32{t, seed, t ^ 5, 7, 1};
        const R32 r = r32_from_key(seed, t, seed ^ t, 3);
        for (uint32_t b = 0; b < nb; ++b) p32_block(h, r, b, t, b ^ t, seed);
        acc = h.h0 ^ h.h1 ^ h.h2 ^ h.h3 ^ h.h4;
    }
    if (acc == 0x9e3779b9u) sink[t] = acc;
}

template <int OP>
static void run(const char *name, uint32_t nb)
{
    uint32_t *sink;
    hipMalloc(&sink, 256u * 64 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int W : {1, 2, 3, 4, 6, 8}) {
        const uint32_t blocks = 256u * W; /* 4 waves per block, one per SIMD of a CU */
        hipLaunchKernelGGL(spin<OP>, dim3(blocks), dim3(256), 0, 0, nb, 12345u, sink);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(spin<OP>, dim3(blocks), dim3(256), 0, 0, nb, 12345u, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double cyc = ms * 1e-3 * 2.4e9 / ((double)W * nb);
        printf("%-10s W=%d  %8.2f us  %7.1f cycles per wave-iteration per SIMD\n", name, W, ms * 1e3, cyc);
    }
    hipFree(sink);
}

int main()
{
    run<0>("chacha", 256);
    run<1>("fe_mul26", 2048);
    run<2>("p32_block", 2048);
    return 0;
}
