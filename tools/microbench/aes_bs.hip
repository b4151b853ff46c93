// Bitsliced AES-256-CTR on gfx950 against the library's LDS T-table path
// (round 3, VERDICT r2 "decide AES-GCM's structure with a measurement").
//
// Bitsliced: each lane encrypts 32 consecutive counter blocks at once; the
// state is 128 VGPRs, register 8b+k holding bit (7-k) of state byte b for the
// lane's 32 blocks (bit i = block i).  SubBytes is the published Boyar-Peralta
// (2012) S-box circuit (XOR/AND only), ShiftRows is register renaming,
// MixColumns is XORs, AddRoundKey XORs 0/~0 masks of the round-key bits that
// are wave-uniform (SGPR operands).  Every round is fast-class VALU only (no
// shift, permute or LDS).  The keystream is transposed back to byte order by
// four 32x32 bit transposes.  CTR inputs: 0^32 || BE64(n) || BE32(ctr), the
// lane's 32 counters one 32-aligned run, so only the counter's 5 low bits
// differ between its blocks (fixed bit patterns).
//
// T-table: aesgcm.hip's aes_ctr_pre (replicated LDS T-tables, v_perm
// addresses, counter-mode caching) in 1024-thread workgroups, one per CU.
//
// Output: correctness of both against a host AES-256, then blocks/s and
// SIMD-cycles per block (at the in-kernel clock) for each.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include -I../../noise-c_amd/csrc aes_bs.hip -o aes_bs
#include "../../noise-c_amd/csrc/aesgcm.hip"
#include "aes_bs.h" /* the bitsliced circuit (the round-4 A/B kernels' shared code) */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#ifndef BS_OCC
#define BS_OCC __attribute__((amdgpu_waves_per_eu(2)))
#endif
#ifndef BS_FUSED
#define BS_FUSED 1
#endif
#ifndef BS_UNROLL
#define BS_UNROLL 1
#endif
using namespace na;

/* ------------------------------------------------------------ host AES */
static uint8_t H_SB[256];
static uint8_t hx(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
static uint8_t hmul(uint8_t a, uint8_t b)
{
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) { if (b & 1) p ^= a; a = hx(a); b >>= 1; }
    return p;
}
static void h_init()
{
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && x; ++y) if (hmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv;
        for (int i = 1; i <= 4; ++i) s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
        H_SB[x] = s ^ 0x63;
    }
}
/* round keys as bytes rk[r][16] */
static void h_expand(const uint8_t key[32], uint8_t rk[15][16])
{
    uint8_t w[60][4];
    for (int i = 0; i < 8; ++i) memcpy(w[i], key + 4 * i, 4);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4];
        memcpy(t, w[i - 1], 4);
        if (i % 8 == 0) {
            uint8_t a = t[0]; t[0] = t[1]; t[1] = t[2]; t[2] = t[3]; t[3] = a;
            for (int j = 0; j < 4; ++j) t[j] = H_SB[t[j]];
            t[0] ^= rcon; rcon = hx(rcon);
        } else if (i % 8 == 4) {
            for (int j = 0; j < 4; ++j) t[j] = H_SB[t[j]];
        }
        for (int j = 0; j < 4; ++j) w[i][j] = w[i - 8][j] ^ t[j];
    }
    for (int r = 0; r < 15; ++r) for (int j = 0; j < 16; ++j) rk[r][j] = w[4 * r + j / 4][j % 4];
}
static void h_encrypt(const uint8_t rk[15][16], uint8_t s[16])
{
    for (int j = 0; j < 16; ++j) s[j] ^= rk[0][j];
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int j = 0; j < 16; ++j) t[j] = H_SB[s[j]];
        for (int c = 0; c < 4; ++c) for (int row = 0; row < 4; ++row) s[4 * c + row] = t[4 * ((c + row) % 4) + row];
        if (r < 14)
            for (int c = 0; c < 4; ++c) {
                uint8_t a[4];
                memcpy(a, s + 4 * c, 4);
                for (int row = 0; row < 4; ++row)
                    s[4 * c + row] = hx(a[row]) ^ hx(a[(row + 1) % 4]) ^ a[(row + 1) % 4] ^ a[(row + 2) % 4] ^ a[(row + 3) % 4];
            }
        for (int j = 0; j < 16; ++j) s[j] ^= rk[r][j];
    }
}

/* ------------------------------------------------------------ bitsliced */
struct BsKey { uint32_t m[15][128]; };

/* bs_sbox, bs_x3, bs2_round, bs_partner, bs_transpose32: tools/microbench/aes_bs.h
   (included through aesgcm.hip) */

#define BS_SBOX(q, b) bs_sbox(q[8 * (b)], q[8 * (b) + 1], q[8 * (b) + 2], q[8 * (b) + 3], q[8 * (b) + 4], \
                              q[8 * (b) + 5], q[8 * (b) + 6], q[8 * (b) + 7])

/* one round: SubBytes, ShiftRows, MixColumns (MIX), AddRoundKey with the
   round's 128 masks m (LDS, wave-uniform address: broadcast reads).  Output
   column c takes the S-box outputs of bytes (r, c + r), so each column's four
   S-boxes run just before it and their inputs die there. */
NA_DEV void bs_round(uint32_t q[128], const uint32_t *m, bool MIX)
{
    uint32_t o[128];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        /* a_r = byte (r, c) after ShiftRows = byte (r, c + r) before */
        uint32_t *a[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            a[r] = &q[8 * (4 * ((c + r) & 3) + r)];
            bs_sbox(a[r][0], a[r][1], a[r][2], a[r][3], a[r][4], a[r][5], a[r][6], a[r][7]);
        }
        uint32_t mk[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint4 v = ((const uint4 *)m)[8 * c + i];
            mk[4 * i] = v.x; mk[4 * i + 1] = v.y; mk[4 * i + 2] = v.z; mk[4 * i + 3] = v.w;
        }
        if (!MIX) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int k = 0; k < 8; ++k) o[8 * (4 * c + r) + k] = a[r][k] ^ mk[8 * r + k];
            continue;
        }
        /* out_r = xtime(a_r ^ a_r+1) ^ (a_r+1 ^ a_r+2 ^ a_r+3) ^ key
                 = xtime(t_r) ^ (s ^ a_r ^ key),  s = a_0 ^ a_1 ^ a_2 ^ a_3:
           two 3-input XORs (v_bitop3) per output bit */
        uint32_t sx[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) sx[k] = bs_x3(a[0][k], a[1][k], a[2][k]) ^ a[3][k];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t *A = a[r], *B = a[(r + 1) & 3];
            uint32_t t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = A[k] ^ B[k];
            uint32_t *O = &o[8 * (4 * c + r)];
            const uint32_t *M = &mk[8 * r];
            /* xtime(t), k from the MSB: bits 7..0 = t6..t0,0 with t7 into bits 4,3,1,0 */
            O[0] = bs_x3(t[1], sx[0], A[0] ^ M[0]);
            O[1] = bs_x3(t[2], sx[1], A[1] ^ M[1]);
            O[2] = bs_x3(t[3], sx[2], A[2] ^ M[2]);
            O[3] = bs_x3(t[4], t[0], bs_x3(sx[3], A[3], M[3]));
            O[4] = bs_x3(t[5], t[0], bs_x3(sx[4], A[4], M[4]));
            O[5] = bs_x3(t[6], sx[5], A[5] ^ M[5]);
            O[6] = bs_x3(t[7], t[0], bs_x3(sx[6], A[6], M[6]));
            O[7] = bs_x3(t[0], sx[7], A[7] ^ M[7]);
        }
    }
#pragma unroll
    for (int i = 0; i < 128; ++i) q[i] = o[i];
}

/* keystream of the lane's 32 counters ctr0 + i (ctr0 % 32 == 0); MODE 0
   writes them (block-major, 4 LE words each), MODE 1 XOR-accumulates */
template <int MODE>
__global__ __launch_bounds__(256) BS_OCC void bs_ctr(const BsKey *__restrict__ K, uint32_t n_hi, uint32_t n_lo,
                                              uint32_t ctr_base, uint32_t *out, int iters, uint64_t *clk)
{
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    __shared__ __align__(16) uint32_t km[15][128];
    for (int i = threadIdx.x; i < 15 * 128; i += blockDim.x) km[i / 128][i % 128] = K->m[i / 128][i % 128];
    __syncthreads();
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    (void)iters; /* one pass: a loop over passes would keep the round-0 state
                    of the constant nonce bytes live across it (hoisted) */
    {
        const uint32_t ctr0 = ctr_base + 32u * g;
        uint8_t iv[16];
        uint32_t q[128];
        /* bytes 0-3 zero, 4-11 BE64(n), 12-15 BE32(ctr0) */
        const uint32_t w[4] = {0u, n_hi, n_lo, ctr0};
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            const uint32_t byte = (w[b >> 2] >> (24 - 8 * (b & 3))) & 255u;
#pragma unroll
            for (int k = 0; k < 8; ++k) q[8 * b + k] = 0u - ((byte >> (7 - k)) & 1u);
        }
        /* counter bits 0..4 (byte 15, k = 7 - p) run over the 32 blocks */
        q[8 * 15 + 7] = 0xAAAAAAAAu; q[8 * 15 + 6] = 0xCCCCCCCCu; q[8 * 15 + 5] = 0xF0F0F0F0u;
        q[8 * 15 + 4] = 0xFF00FF00u; q[8 * 15 + 3] = 0xFFFF0000u;
        (void)iv;
#pragma unroll
        for (int i = 0; i < 128; ++i) q[i] ^= km[0][i];
#pragma unroll BS_UNROLL
        for (int r = 1; r < 15; ++r) bs_round(q, km[r], r < 14);
        /* group g = state word g (bytes 4g..4g+3): feed bit p = 8*rb + (7-k)
           of the LE word from byte 4g+rb, bit k */
#pragma unroll
        for (int gw = 0; gw < 4; ++gw) {
            uint32_t r[32];
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
#pragma unroll
                for (int k = 0; k < 8; ++k) r[8 * rb + (7 - k)] = q[8 * (4 * gw + rb) + k];
            bs_transpose32(r);
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                if (MODE == 0) out[((size_t)g * 32 + i) * 4 + gw] = r[i];
                else acc ^= r[i];
            }
        }
    }
    if (MODE == 1) out[g] = acc;
    if (clk && threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

/* ------------------------------------------------ bitsliced, two lanes
 * The same 32-block bitsliced state split over a lane pair: lane L holds
 * state columns 2L and 2L+1 (64 VGPRs: local byte 4j + r, j = local column),
 * so 128 VGPRs are enough for four waves per SIMD.  ShiftRows moves 4 of a
 * lane's 8 bytes to its partner and back: with local column j the exchange
 * is symmetric (both lanes want the partner's (1,0), (2,0), (2,1), (3,1)),
 * one quad_perm [1,0,3,2] DPP per register.  Round-key masks depend on the
 * lane's columns: read from LDS per lane. */
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void bs2_ctr(
    const BsKey *__restrict__ K, uint32_t n_hi, uint32_t n_lo, uint32_t ctr_base, uint32_t *out, uint64_t *clk)
{
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    /* masks by lane half: km[round][L][64] (columns 2L, 2L+1) */
    __shared__ __align__(16) uint32_t km[15][2][64];
    for (int i = threadIdx.x; i < 15 * 128; i += blockDim.x) {
        const int rr = i / 128, b = (i % 128) / 8, k = i % 8; /* global byte b, bit k */
        const int c = b / 4, r = b % 4, L = c / 2, j = c % 2;
        km[rr][L][8 * (4 * j + r) + k] = K->m[rr][i % 128];
    }
    __syncthreads();
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t L = g & 1, pair = g >> 1;
    const uint32_t ctr0 = ctr_base + 32u * pair;
    /* this lane's bytes: global columns 2L, 2L+1 = state words 2L, 2L+1 */
    const uint32_t wv[4] = {0u, n_hi, n_lo, ctr0};
    uint32_t h[64];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t word = L ? wv[2 + j] : wv[j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t byte = (word >> (24 - 8 * r)) & 255u;
#pragma unroll
            for (int k = 0; k < 8; ++k) h[8 * (4 * j + r) + k] = 0u - ((byte >> (7 - k)) & 1u);
        }
    }
    if (L) { /* byte 15 = (row 3, column 3): lane 1, local (3, j = 1) */
        uint32_t *q = &h[8 * (4 * 1 + 3)];
        q[7] = 0xAAAAAAAAu; q[6] = 0xCCCCCCCCu; q[5] = 0xF0F0F0F0u; q[4] = 0xFF00FF00u; q[3] = 0xFFFF0000u;
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) h[i] ^= km[0][L][i];
#pragma unroll 1
    for (int rr = 1; rr < 14; ++rr) bs2_round<true>(h, km[rr][L]);
    bs2_round<false>(h, km[14][L]);
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        uint32_t r32[32];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int k = 0; k < 8; ++k) r32[8 * rb + (7 - k)] = h[8 * (4 * j + rb) + k];
        bs_transpose32(r32);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (MODE == 0) out[((size_t)pair * 32 + i) * 4 + 2 * L + j] = r32[i];
            else acc ^= r32[i];
        }
    }
    if (MODE == 1) out[g] = acc;
    if (clk && threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

/* ------------------------------------------------------------ T-table */
__global__ __launch_bounds__(GCM_WG) void tt_ctr(const uint32_t *__restrict__ rk_g, uint32_t n_hi, uint32_t n_lo,
                                                 uint32_t blocks_per_lane, uint32_t *out, int mode, uint64_t *clk)
{
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    extern __shared__ __align__(16) uint8_t smem[];
    GcmLds &L = *(GcmLds *)smem;
    const int t = threadIdx.x;
    for (int q = t; q < 2 * 256 * 16; q += GCM_WG) {
        const int reg = q >> 12, row = (q >> 4) & 255, quad = q & 15;
        const int tab = 2 * reg + (quad >> 3);
        const uint32_t v = rotr(g_te0[row], 8 * tab);
        ((uint4 *)&L.te[reg][row][0])[quad] = make_uint4(v, v, v, v);
    }
    if (t < 60) L.rk[t] = rk_g[t];
    __syncthreads();
    const uint32_t lane = t & 63;
    const uint32_t tpl = (1u << 16) | ((128u + 4u * (lane & 31)) << 8) | (4u * (lane & 31));
    const uint8_t *TE = (const uint8_t *)&L.te[0][0][0];
    const uint32_t g = blockIdx.x * GCM_WG + t;
    /* each lane: its own record nonce (n + g), counters 2 .. 2 + blocks */
    const uint64_t n = (((uint64_t)n_hi << 32) | n_lo) + g;
    const AesPre pre = aes_pre_lds(TE, L.rk, tpl, (uint32_t)(n >> 32), (uint32_t)n);
    uint32_t acc = 0;
#pragma unroll 1
    for (uint32_t d = 0; d < blocks_per_lane; ++d) {
        uint32_t ks[4];
        aes_ctr_pre(TE, L.rk, tpl, pre, 2 + d, ks);
        if (mode == 0) {
            for (int w = 0; w < 4; ++w) out[((size_t)g * blocks_per_lane + d) * 4 + w] = ks[w];
        } else {
            acc ^= ks[0] ^ ks[1] ^ ks[2] ^ ks[3];
        }
    }
    if (mode == 1) out[g] = acc;
    if (clk && threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

__global__ void clock_probe(uint64_t *o, int spin)
{
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (int i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = c1 - c0; o[1] = t1 - t0; o[2] = x; }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    h_init();
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 3);
    uint8_t rkb[15][16];
    h_expand(key, rkb);
    BsKey hk;
    for (int r = 0; r < 15; ++r)
        for (int b = 0; b < 16; ++b)
            for (int k = 0; k < 8; ++k) hk.m[r][8 * b + k] = ((rkb[r][b] >> (7 - k)) & 1) ? ~0u : 0u;
    uint32_t rkw[60];
    for (int i = 0; i < 60; ++i)
        rkw[i] = ((uint32_t)rkb[i / 4][4 * (i % 4)] << 24) | ((uint32_t)rkb[i / 4][4 * (i % 4) + 1] << 16) |
                 ((uint32_t)rkb[i / 4][4 * (i % 4) + 2] << 8) | rkb[i / 4][4 * (i % 4) + 3];
    const uint32_t n_hi = 0x01020304u, n_lo = 0xA0B0C0D0u;

    BsKey *dk; uint32_t *drk, *dout; uint64_t *dclk;
    CK(hipMalloc(&dk, sizeof hk)); CK(hipMalloc(&drk, 240));
    CK(hipMemcpy(dk, &hk, sizeof hk, hipMemcpyHostToDevice));
    CK(hipMemcpy(drk, rkw, 240, hipMemcpyHostToDevice));
    const size_t out_words = 64u << 20;
    CK(hipMalloc(&dout, out_words * 4)); CK(hipMalloc(&dclk, 24));
    hipLaunchKernelGGL(aes_tables_init, dim3(1), dim3(256), 0, 0);
    CK(hipFuncSetAttribute((const void *)tt_ctr, hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(GcmLds)));

    /* correctness: 64 lanes x 32 blocks (bitsliced), 1024 lanes x 8 blocks (T-table) */
    {
        const uint32_t cb = 64;
        hipLaunchKernelGGL((bs_ctr<0>), dim3(1), dim3(64), 0, 0, dk, n_hi, n_lo, cb, dout, 1, nullptr);
        std::vector<uint32_t> h(64 * 32 * 4);
        CK(hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost));
        int bad = 0;
        for (uint32_t blk = 0; blk < 64 * 32; ++blk) {
            uint8_t s[16] = {0, 0, 0, 0};
            const uint32_t ctr = cb + blk;
            for (int j = 0; j < 4; ++j) { s[4 + j] = (uint8_t)(n_hi >> (24 - 8 * j)); s[8 + j] = (uint8_t)(n_lo >> (24 - 8 * j)); s[12 + j] = (uint8_t)(ctr >> (24 - 8 * j)); }
            h_encrypt(rkb, s);
            uint32_t e[4];
            memcpy(e, s, 16);
            if (memcmp(e, &h[blk * 4], 16)) { if (bad++ < 3) printf("bitsliced mismatch block %u: %08x vs %08x\n", blk, h[blk * 4], e[0]); }
        }
        printf("bitsliced check: %s (%d bad of %d)\n", bad ? "FAIL" : "ok", bad, 64 * 32);
        hipLaunchKernelGGL((bs2_ctr<0>), dim3(1), dim3(64), 0, 0, dk, n_hi, n_lo, cb, dout, nullptr);
        CK(hipMemcpy(h.data(), dout, 32 * 32 * 4 * 4, hipMemcpyDeviceToHost));
        int bad3 = 0;
        for (uint32_t blk = 0; blk < 32 * 32; ++blk) {
            uint8_t s2[16] = {0, 0, 0, 0};
            const uint32_t ctr = cb + blk;
            for (int j = 0; j < 4; ++j) { s2[4 + j] = (uint8_t)(n_hi >> (24 - 8 * j)); s2[8 + j] = (uint8_t)(n_lo >> (24 - 8 * j)); s2[12 + j] = (uint8_t)(ctr >> (24 - 8 * j)); }
            h_encrypt(rkb, s2);
            uint32_t e[4];
            memcpy(e, s2, 16);
            if (memcmp(e, &h[blk * 4], 16)) { if (bad3++ < 3) printf("bitsliced-2 mismatch block %u: %08x vs %08x\n", blk, h[blk * 4], e[0]); }
        }
        printf("bitsliced two-lane check: %s (%d bad of %d)\n", bad3 ? "FAIL" : "ok", bad3, 32 * 32);
        bad += bad3;
        const uint32_t bpl = 8;
        hipLaunchKernelGGL(tt_ctr, dim3(1), dim3(GCM_WG), sizeof(GcmLds), 0, drk, n_hi, n_lo, bpl, dout, 0, nullptr);
        std::vector<uint32_t> t(GCM_WG * bpl * 4);
        CK(hipMemcpy(t.data(), dout, t.size() * 4, hipMemcpyDeviceToHost));
        int bad2 = 0;
        for (uint32_t g = 0; g < GCM_WG; ++g)
            for (uint32_t d = 0; d < bpl; ++d) {
                const uint64_t n = (((uint64_t)n_hi << 32) | n_lo) + g;
                uint8_t s[16] = {0, 0, 0, 0};
                const uint32_t ctr = 2 + d;
                for (int j = 0; j < 8; ++j) s[4 + j] = (uint8_t)(n >> (56 - 8 * j));
                for (int j = 0; j < 4; ++j) s[12 + j] = (uint8_t)(ctr >> (24 - 8 * j));
                h_encrypt(rkb, s);
                if (memcmp(s, &t[(g * bpl + d) * 4], 16)) ++bad2;
            }
        printf("t-table check: %s (%d bad)\n", bad2 ? "FAIL" : "ok", bad2);
        if (bad || bad2) return 2;
    }

    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    uint64_t *dck;
    CK(hipMalloc(&dck, 2 * 16384 * sizeof(uint64_t)));
    /* each kernel: ~0.4 s back to back first (the sustained-load clock,
       profiles/r03/clock_vs_warmup.log), then `reps` timed launches; the
       clock from s_memtime / s_memrealtime over every block of the last one */
    auto clock_of = [&](int nblk) {
        std::vector<uint64_t> h(2 * nblk);
        hipMemcpy(h.data(), dck, h.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> f;
        for (int b = 0; b < nblk; ++b)
            if (h[2 * b + 1] > 100) f.push_back((double)h[2 * b] / (h[2 * b + 1] * 0.01));
        std::sort(f.begin(), f.end());
        return f.empty() ? 0.0 : f[f.size() / 2];
    };
    {
        const int grid = 8192, iters = 1;
        const double blocks1 = (double)grid * 256 * 32 * iters;
        for (int w = 0; w < 400; ++w) hipLaunchKernelGGL((bs_ctr<1>), dim3(grid), dim3(256), 0, 0, dk, n_hi, n_lo, 0u, dout, iters, nullptr);
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((bs_ctr<1>), dim3(grid), dim3(256), 0, 0, dk, n_hi, n_lo, 0u, dout, iters, dck);
        hipEventRecord(e1);
        CK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double bps = blocks1 * reps / (ms * 1e-3), mhz = clock_of(grid);
        printf("bitsliced: %.3f ms/launch, %.2f G blocks/s = %.1f GB/s keystream; %.2f SIMD-cycles/block at %.0f MHz (in-kernel)\n",
               ms / reps, bps * 1e-9, bps * 16e-9, 1024.0 * mhz * 1e6 / bps, mhz);
    }
    {
        const int grid = 16384; /* 2 lanes per 32 blocks */
        const double blocks1 = (double)grid * 256 / 2 * 32;
        for (int w = 0; w < 400; ++w) hipLaunchKernelGGL((bs2_ctr<1>), dim3(grid), dim3(256), 0, 0, dk, n_hi, n_lo, 0u, dout, nullptr);
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((bs2_ctr<1>), dim3(grid), dim3(256), 0, 0, dk, n_hi, n_lo, 0u, dout, dck);
        hipEventRecord(e1);
        CK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double bps = blocks1 * reps / (ms * 1e-3), mhz = clock_of(grid);
        printf("bitsliced two-lane: %.3f ms/launch, %.2f G blocks/s; %.2f SIMD-cycles/block at %.0f MHz (in-kernel)\n",
               ms / reps, bps * 1e-9, 1024.0 * mhz * 1e6 / bps, mhz);
    }
    {
        const int grid = 256 * 4; const uint32_t bpl = 256;
        const double blocks1 = (double)grid * GCM_WG * bpl;
        for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(tt_ctr, dim3(grid), dim3(GCM_WG), sizeof(GcmLds), 0, drk, n_hi, n_lo, bpl, dout, 1, nullptr);
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(tt_ctr, dim3(grid), dim3(GCM_WG), sizeof(GcmLds), 0, drk, n_hi, n_lo, bpl, dout, 1, dck);
        hipEventRecord(e1);
        CK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double bps = blocks1 * reps / (ms * 1e-3), mhz = clock_of(grid);
        printf("t-table:   %.3f ms/launch, %.2f G blocks/s = %.1f GB/s keystream; %.2f SIMD-cycles/block at %.0f MHz (in-kernel)\n",
               ms / reps, bps * 1e-9, bps * 16e-9, 1024.0 * mhz * 1e6 / bps, mhz);
    }
    return 0;
}
