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

/* Boyar-Peralta S-box, x0 = MSB of the byte (in place) */
NA_DEV void bs_sbox(uint32_t &q0, uint32_t &q1, uint32_t &q2, uint32_t &q3, uint32_t &q4, uint32_t &q5,
                    uint32_t &q6, uint32_t &q7)
{
    const uint32_t x0 = q0, x1 = q1, x2 = q2, x3 = q3, x4 = q4, x5 = q5, x6 = q6, x7 = q7;
#if BS_FUSED
    /* the circuit with single-use gates folded into 3-input v_bitop3
       (84 operations; generated and checked over all 256 inputs) */
    const uint32_t y14 = __builtin_amdgcn_bitop3_b32(x3, x5, 0u, 0x3c);
    const uint32_t y13 = __builtin_amdgcn_bitop3_b32(x0, x6, 0u, 0x3c);
    const uint32_t y9 = __builtin_amdgcn_bitop3_b32(x0, x3, 0u, 0x3c);
    const uint32_t y8 = __builtin_amdgcn_bitop3_b32(x0, x5, 0u, 0x3c);
    const uint32_t t0 = __builtin_amdgcn_bitop3_b32(x1, x2, 0u, 0x3c);
    const uint32_t y1 = __builtin_amdgcn_bitop3_b32(t0, x7, 0u, 0x3c);
    const uint32_t y4 = __builtin_amdgcn_bitop3_b32(x3, y1, 0u, 0x3c);
    const uint32_t y12 = __builtin_amdgcn_bitop3_b32(y13, y14, 0u, 0x3c);
    const uint32_t y2 = __builtin_amdgcn_bitop3_b32(x0, y1, 0u, 0x3c);
    const uint32_t y5 = __builtin_amdgcn_bitop3_b32(x6, y1, 0u, 0x3c);
    const uint32_t y3 = __builtin_amdgcn_bitop3_b32(y5, y8, 0u, 0x3c);
    const uint32_t t1 = __builtin_amdgcn_bitop3_b32(x4, y12, 0u, 0x3c);
    const uint32_t y15 = __builtin_amdgcn_bitop3_b32(t1, x5, 0u, 0x3c);
    const uint32_t y20 = __builtin_amdgcn_bitop3_b32(t1, x1, 0u, 0x3c);
    const uint32_t y6 = __builtin_amdgcn_bitop3_b32(x7, y15, 0u, 0x3c);
    const uint32_t y10 = __builtin_amdgcn_bitop3_b32(t0, y15, 0u, 0x3c);
    const uint32_t y11 = __builtin_amdgcn_bitop3_b32(y20, y9, 0u, 0x3c);
    const uint32_t y7 = __builtin_amdgcn_bitop3_b32(x7, y11, 0u, 0x3c);
    const uint32_t y17 = __builtin_amdgcn_bitop3_b32(y10, y11, 0u, 0x3c);
    const uint32_t y19 = __builtin_amdgcn_bitop3_b32(y10, y8, 0u, 0x3c);
    const uint32_t y16 = __builtin_amdgcn_bitop3_b32(t0, y11, 0u, 0x3c);
    const uint32_t y21 = __builtin_amdgcn_bitop3_b32(y13, y16, 0u, 0x3c);
    const uint32_t y18 = __builtin_amdgcn_bitop3_b32(x0, y16, 0u, 0x3c);
    const uint32_t t2 = __builtin_amdgcn_bitop3_b32(y12, y15, 0u, 0xc0);
    const uint32_t t4 = __builtin_amdgcn_bitop3_b32(t2, y3, y6, 0x78);
    const uint32_t t6 = __builtin_amdgcn_bitop3_b32(t2, x7, y4, 0x78);
    const uint32_t t7 = __builtin_amdgcn_bitop3_b32(y13, y16, 0u, 0xc0);
    const uint32_t t9 = __builtin_amdgcn_bitop3_b32(t7, y1, y5, 0x78);
    const uint32_t t11 = __builtin_amdgcn_bitop3_b32(t7, y2, y7, 0x78);
    const uint32_t t12 = __builtin_amdgcn_bitop3_b32(y11, y9, 0u, 0xc0);
    const uint32_t t14 = __builtin_amdgcn_bitop3_b32(t12, y14, y17, 0x78);
    const uint32_t t16 = __builtin_amdgcn_bitop3_b32(t12, y10, y8, 0x78);
    const uint32_t t21 = __builtin_amdgcn_bitop3_b32(t14, t4, y20, 0x96);
    const uint32_t t22 = __builtin_amdgcn_bitop3_b32(t16, t6, y19, 0x96);
    const uint32_t t23 = __builtin_amdgcn_bitop3_b32(t14, t9, y21, 0x96);
    const uint32_t t24 = __builtin_amdgcn_bitop3_b32(t11, t16, y18, 0x96);
    const uint32_t t25 = __builtin_amdgcn_bitop3_b32(t21, t22, 0u, 0x3c);
    const uint32_t t26 = __builtin_amdgcn_bitop3_b32(t21, t23, 0u, 0xc0);
    const uint32_t t27 = __builtin_amdgcn_bitop3_b32(t24, t26, 0u, 0x3c);
    const uint32_t t29 = __builtin_amdgcn_bitop3_b32(t22, t25, t27, 0x78);
    const uint32_t t31 = __builtin_amdgcn_bitop3_b32(t22, t26, 0u, 0x3c);
    const uint32_t t33 = __builtin_amdgcn_bitop3_b32(t23, t24, t31, 0xe4);
    const uint32_t t36 = __builtin_amdgcn_bitop3_b32(t24, t27, t33, 0x60);
    const uint32_t t37 = __builtin_amdgcn_bitop3_b32(t23, t33, t36, 0x96);
    const uint32_t t39 = __builtin_amdgcn_bitop3_b32(t27, t29, t36, 0x48);
    const uint32_t t40 = __builtin_amdgcn_bitop3_b32(t25, t39, 0u, 0x3c);
    const uint32_t t41 = __builtin_amdgcn_bitop3_b32(t37, t40, 0u, 0x3c);
    const uint32_t t42 = __builtin_amdgcn_bitop3_b32(t29, t33, 0u, 0x3c);
    const uint32_t t43 = __builtin_amdgcn_bitop3_b32(t29, t40, 0u, 0x3c);
    const uint32_t t44 = __builtin_amdgcn_bitop3_b32(t33, t37, 0u, 0x3c);
    const uint32_t t45 = __builtin_amdgcn_bitop3_b32(t41, t42, 0u, 0x3c);
    const uint32_t z2 = __builtin_amdgcn_bitop3_b32(t33, x7, 0u, 0xc0);
    const uint32_t z3 = __builtin_amdgcn_bitop3_b32(t43, y16, 0u, 0xc0);
    const uint32_t z4 = __builtin_amdgcn_bitop3_b32(t40, y1, 0u, 0xc0);
    const uint32_t z5 = __builtin_amdgcn_bitop3_b32(t29, y7, 0u, 0xc0);
    const uint32_t z7 = __builtin_amdgcn_bitop3_b32(t45, y17, 0u, 0xc0);
    const uint32_t z10 = __builtin_amdgcn_bitop3_b32(t37, y3, 0u, 0xc0);
    const uint32_t z12 = __builtin_amdgcn_bitop3_b32(t43, y13, 0u, 0xc0);
    const uint32_t z16 = __builtin_amdgcn_bitop3_b32(t45, y14, 0u, 0xc0);
    const uint32_t t46 = __builtin_amdgcn_bitop3_b32(t42, y9, z16, 0x6a);
    const uint32_t t47 = __builtin_amdgcn_bitop3_b32(t33, y4, z10, 0x6a);
    const uint32_t t48 = __builtin_amdgcn_bitop3_b32(t40, y5, z5, 0x6a);
    const uint32_t t49 = __builtin_amdgcn_bitop3_b32(t44, y12, z10, 0x6a);
    const uint32_t t52 = __builtin_amdgcn_bitop3_b32(t41, y10, z7, 0x6a);
    const uint32_t t53 = __builtin_amdgcn_bitop3_b32(t44, y15, z3, 0x6a);
    const uint32_t t54 = __builtin_amdgcn_bitop3_b32(t42, y11, z7, 0x6a);
    const uint32_t t55 = __builtin_amdgcn_bitop3_b32(t41, y8, z16, 0x6a);
    const uint32_t t57 = __builtin_amdgcn_bitop3_b32(t53, z12, z2, 0x96);
    const uint32_t t58 = __builtin_amdgcn_bitop3_b32(t46, z4, 0u, 0x3c);
    const uint32_t t59 = __builtin_amdgcn_bitop3_b32(t54, z3, 0u, 0x3c);
    const uint32_t t61 = __builtin_amdgcn_bitop3_b32(t29, t57, y2, 0x6c);
    const uint32_t t62 = __builtin_amdgcn_bitop3_b32(t52, t58, 0u, 0x3c);
    const uint32_t t63 = __builtin_amdgcn_bitop3_b32(t49, t58, 0u, 0x3c);
    const uint32_t t64 = __builtin_amdgcn_bitop3_b32(t59, z4, 0u, 0x3c);
    const uint32_t t65 = __builtin_amdgcn_bitop3_b32(t61, t62, 0u, 0x3c);
    const uint32_t t66 = __builtin_amdgcn_bitop3_b32(t37, t63, y6, 0x6c);
    const uint32_t s0 = __builtin_amdgcn_bitop3_b32(t59, t63, 0u, 0x3c);
    const uint32_t s6 = __builtin_amdgcn_bitop3_b32(t48, t62, z12, 0x69);
    const uint32_t s7 = __builtin_amdgcn_bitop3_b32(t46, t48, t57, 0x69);
    const uint32_t s3 = __builtin_amdgcn_bitop3_b32(t53, t66, 0u, 0x3c);
    const uint32_t s4 = __builtin_amdgcn_bitop3_b32(t66, z2, z5, 0x96);
    const uint32_t s5 = __builtin_amdgcn_bitop3_b32(t47, t65, 0u, 0x3c);
    const uint32_t s1 = __builtin_amdgcn_bitop3_b32(s3, t64, 0u, 0xc3);
    const uint32_t s2 = __builtin_amdgcn_bitop3_b32(t55, t64, t65, 0x69);
#else
    const uint32_t y14 = x3 ^ x5, y13 = x0 ^ x6, y9 = x0 ^ x3, y8 = x0 ^ x5, t0 = x1 ^ x2;
    const uint32_t y1 = t0 ^ x7, y4 = y1 ^ x3, y12 = y13 ^ y14, y2 = y1 ^ x0, y5 = y1 ^ x6;
    const uint32_t y3 = y5 ^ y8, t1 = x4 ^ y12, y15 = t1 ^ x5, y20 = t1 ^ x1, y6 = y15 ^ x7;
    const uint32_t y10 = y15 ^ t0, y11 = y20 ^ y9, y7 = x7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8;
    const uint32_t y16 = t0 ^ y11, y21 = y13 ^ y16, y18 = x0 ^ y16;
    const uint32_t t2 = y12 & y15, t3 = y3 & y6, t4 = t3 ^ t2, t5 = y4 & x7, t6 = t5 ^ t2;
    const uint32_t t7 = y13 & y16, t8 = y5 & y1, t9 = t8 ^ t7, t10 = y2 & y7, t11 = t10 ^ t7;
    const uint32_t t12 = y9 & y11, t13 = y14 & y17, t14 = t13 ^ t12, t15 = y8 & y10, t16 = t15 ^ t12;
    const uint32_t t17 = t4 ^ t14, t18 = t6 ^ t16, t19 = t9 ^ t14, t20 = t11 ^ t16;
    const uint32_t t21 = t17 ^ y20, t22 = t18 ^ y19, t23 = t19 ^ y21, t24 = t20 ^ y18;
    const uint32_t t25 = t21 ^ t22, t26 = t21 & t23, t27 = t24 ^ t26, t28 = t25 & t27, t29 = t28 ^ t22;
    const uint32_t t30 = t23 ^ t24, t31 = t22 ^ t26, t32 = t31 & t30, t33 = t32 ^ t24, t34 = t23 ^ t33;
    const uint32_t t35 = t27 ^ t33, t36 = t24 & t35, t37 = t36 ^ t34, t38 = t27 ^ t36, t39 = t29 & t38;
    const uint32_t t40 = t25 ^ t39;
    const uint32_t t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40, t44 = t33 ^ t37, t45 = t42 ^ t41;
    const uint32_t z0 = t44 & y15, z1 = t37 & y6, z2 = t33 & x7, z3 = t43 & y16, z4 = t40 & y1;
    const uint32_t z5 = t29 & y7, z6 = t42 & y11, z7 = t45 & y17, z8 = t41 & y10, z9 = t44 & y12;
    const uint32_t z10 = t37 & y3, z11 = t33 & y4, z12 = t43 & y13, z13 = t40 & y5, z14 = t29 & y2;
    const uint32_t z15 = t42 & y9, z16 = t45 & y14, z17 = t41 & y8;
    const uint32_t t46 = z15 ^ z16, t47 = z10 ^ z11, t48 = z5 ^ z13, t49 = z9 ^ z10, t50 = z2 ^ z12;
    const uint32_t t51 = z2 ^ z5, t52 = z7 ^ z8, t53 = z0 ^ z3, t54 = z6 ^ z7, t55 = z16 ^ z17;
    const uint32_t t56 = z12 ^ t48, t57 = t50 ^ t53, t58 = z4 ^ t46, t59 = z3 ^ t54, t60 = t46 ^ t57;
    const uint32_t t61 = z14 ^ t57, t62 = t52 ^ t58, t63 = t49 ^ t58, t64 = z4 ^ t59, t65 = t61 ^ t62;
    const uint32_t t66 = z1 ^ t63;
    const uint32_t s0 = t59 ^ t63, s6 = t56 ^ ~t62, s7 = t48 ^ ~t60, t67 = t64 ^ t65;
    const uint32_t s3 = t53 ^ t66, s4 = t51 ^ t66, s5 = t47 ^ t65, s1 = t64 ^ ~s3, s2 = t55 ^ ~t67;
#endif
    q0 = s0; q1 = s1; q2 = s2; q3 = s3; q4 = s4; q5 = s5; q6 = s6; q7 = s7;
}

NA_DEV uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

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

/* swap step of a bit-matrix transpose: exchange a's bits [w, 2w) blocks with
   b's [0, w) blocks under mask */
NA_DEV void tswap(uint32_t &a, uint32_t &b, int w, uint32_t mask)
{
    const uint32_t t = ((a >> w) ^ b) & mask;
    b ^= t;
    a ^= t << w;
}

/* 32x32 bit transpose of r[0..31] in place: bit i of r[p] <-> bit p of r[i] */
NA_DEV void transpose32(uint32_t r[32])
{
    const uint32_t masks[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int w = 16 >> s;
#pragma unroll
        for (int p = 0; p < 32; ++p)
            if (!(p & w)) tswap(r[p], r[p | w], w, masks[s]);
    }
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
            transpose32(r);
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
NA_DEV uint32_t partner(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false); }

/* one round on the lane's half state h[64]; mk: this lane's 64 masks */
NA_DEV void bs2_round(uint32_t h[64], const uint32_t *mk, bool MIX)
{
#pragma unroll
    for (int b = 0; b < 8; ++b) bs_sbox(h[8 * b], h[8 * b + 1], h[8 * b + 2], h[8 * b + 3], h[8 * b + 4],
                                       h[8 * b + 5], h[8 * b + 6], h[8 * b + 7]);
    /* the partner's (1,0), (2,0), (2,1), (3,1): local bytes 1, 2, 6, 7 */
    uint32_t px[4][8];
    const int pb[4] = {1, 2, 6, 7};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) px[i][k] = partner(h[8 * pb[i] + k]);
    uint32_t o[64];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        /* a_r = byte (r, c + r) before ShiftRows, c = 2L + j */
        const uint32_t *a[4];
        a[0] = &h[8 * (4 * j + 0)];
        a[1] = j == 0 ? &h[8 * (4 * 1 + 1)] : px[0];                 /* (1,1) own / (1,0) partner */
        a[2] = j == 0 ? px[1] : px[2];                               /* (2,0) / (2,1) partner */
        a[3] = j == 0 ? px[3] : &h[8 * (4 * 0 + 3)];                 /* (3,1) partner / (3,0) own */
        uint32_t mkc[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) mkc[i] = mk[32 * j + i];
        if (!MIX) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int k = 0; k < 8; ++k) o[8 * (4 * j + r) + k] = a[r][k] ^ mkc[8 * r + k];
            continue;
        }
        uint32_t sx[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) sx[k] = bs_x3(a[0][k], a[1][k], a[2][k]) ^ a[3][k];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t *A = a[r], *B = a[(r + 1) & 3];
            uint32_t t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = A[k] ^ B[k];
            uint32_t *O = &o[8 * (4 * j + r)];
            const uint32_t *M = &mkc[8 * r];
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
    for (int i = 0; i < 64; ++i) h[i] = o[i];
}

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
    for (int rr = 1; rr < 15; ++rr) bs2_round(h, km[rr][L], rr < 14);
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        uint32_t r32[32];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int k = 0; k < 8; ++k) r32[8 * rb + (7 - k)] = h[8 * (4 * j + rb) + k];
        transpose32(r32);
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
