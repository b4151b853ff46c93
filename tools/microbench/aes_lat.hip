// Latency of ONE AES-256 block on one lane (the single-record path's
// E_K(J0) and the wide record's CTR blocks): a chain of dependent blocks,
// timed with s_memtime inside the kernel.
//
//   aes_lat
//
// Variants: the library's aes256_block (one T-table with rotates, te/sb/rk in
// LDS), and the same with the four rotated tables in LDS (no rotates).
#define NA_NO_SETUP_KERNELS
#include "../../noise-c_amd/csrc/aesgcm.hip"
#include <cstdio>
#include <cstdlib>

using namespace na;

constexpr int CHAIN = 64;

/* four tables, te_k = rotr(te0, 8k) */
NA_DEV void aes256_block4(const uint32_t *__restrict__ rk, const uint32_t (*T)[256], const uint32_t *sb,
                          uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3)
{
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const uint32_t t0 = T[0][s0 >> 24] ^ T[1][(s1 >> 16) & 255] ^ T[2][(s2 >> 8) & 255] ^ T[3][s3 & 255] ^ rk[4 * r];
        const uint32_t t1 = T[0][s1 >> 24] ^ T[1][(s2 >> 16) & 255] ^ T[2][(s3 >> 8) & 255] ^ T[3][s0 & 255] ^ rk[4 * r + 1];
        const uint32_t t2 = T[0][s2 >> 24] ^ T[1][(s3 >> 16) & 255] ^ T[2][(s0 >> 8) & 255] ^ T[3][s1 & 255] ^ rk[4 * r + 2];
        const uint32_t t3 = T[0][s3 >> 24] ^ T[1][(s0 >> 16) & 255] ^ T[2][(s1 >> 8) & 255] ^ T[3][s2 & 255] ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint32_t o0 = (sb[s0 >> 24] << 24) | (sb[(s1 >> 16) & 255] << 16) | (sb[(s2 >> 8) & 255] << 8) | sb[s3 & 255];
    const uint32_t o1 = (sb[s1 >> 24] << 24) | (sb[(s2 >> 16) & 255] << 16) | (sb[(s3 >> 8) & 255] << 8) | sb[s0 & 255];
    const uint32_t o2 = (sb[s2 >> 24] << 24) | (sb[(s3 >> 16) & 255] << 16) | (sb[(s0 >> 8) & 255] << 8) | sb[s1 & 255];
    const uint32_t o3 = (sb[s3 >> 24] << 24) | (sb[(s0 >> 16) & 255] << 16) | (sb[(s1 >> 8) & 255] << 8) | sb[s2 & 255];
    s0 = o0 ^ rk[56]; s1 = o1 ^ rk[57]; s2 = o2 ^ rk[58]; s3 = o3 ^ rk[59];
}

template <int V>
__global__ __launch_bounds__(256) void lat(const uint32_t *rk_g, uint32_t *out, uint32_t *cyc, int lanes)
{
    __shared__ uint32_t te[256], sb[256], rk[60];
    __shared__ uint32_t T[4][256];
    const uint32_t t = threadIdx.x;
    aes_table_entry(t, sb[t], te[t]);
    __syncthreads();
    for (int k = 0; k < 4; ++k) T[k][t] = rotr(te[t], 8 * k);
    if (t < 60) rk[t] = rk_g[t];
    __syncthreads();
    if ((int)t < lanes) {
        uint32_t s0 = t, s1 = 1, s2 = 2, s3 = 3;
        const uint64_t c0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < CHAIN; ++i) {
            if (V == 0) aes256_block(rk, te, sb, s0, s1, s2, s3);
            else aes256_block4(rk, T, sb, s0, s1, s2, s3);
        }
        const uint64_t c1 = __builtin_amdgcn_s_memtime();
        out[4 * t] = s0; out[4 * t + 1] = s1; out[4 * t + 2] = s2; out[4 * t + 3] = s3;
        if (t == 0) cyc[0] = (uint32_t)(c1 - c0);
    }
}

int main()
{
    uint32_t *rk, *out, *cyc;
    (void)hipMalloc(&rk, 60 * 4);
    (void)hipMalloc(&out, 256 * 16);
    (void)hipMalloc(&cyc, 4);
    uint32_t h[60];
    for (int i = 0; i < 60; ++i) h[i] = 0x9E3779B9u * (i + 1);
    (void)hipMemcpy(rk, h, sizeof h, hipMemcpyHostToDevice);
    uint32_t r0[4], r1[4];
    for (int lanes : {1, 64}) {
        for (int v = 0; v < 2; ++v) {
            uint32_t best = ~0u;
            for (int rep = 0; rep < 20; ++rep) {
                if (v == 0) hipLaunchKernelGGL(lat<0>, dim3(1), dim3(256), 0, 0, rk, out, cyc, lanes);
                else hipLaunchKernelGGL(lat<1>, dim3(1), dim3(256), 0, 0, rk, out, cyc, lanes);
                uint32_t c;
                (void)hipMemcpy(&c, cyc, 4, hipMemcpyDeviceToHost);
                if (c < best) best = c;
            }
            (void)hipMemcpy(v == 0 ? r0 : r1, out, 16, hipMemcpyDeviceToHost);
            printf("{\"aes_block_latency\": \"%s\", \"lanes\": %d, \"cycles_per_block\": %.0f}\n",
                   v == 0 ? "te0+rotates" : "four tables", lanes, (double)best / CHAIN);
        }
    }
    printf("same output: %s\n", (r0[0] == r1[0] && r0[1] == r1[1] && r0[2] == r1[2] && r0[3] == r1[3]) ? "yes" : "NO");
    return 0;
}
