/*
 * aes_bs.h — bitsliced AES-256 for gfx950 (round 4; designed and timed as a
 * microbenchmark in round 3, tools/microbench/aes_bs.hip).
 *
 * The AES of src/crypto/aes/rijndael-alg-fst.c:854-1033 without tables: 32
 * counter blocks at once on a lane pair.  Register 8*(4j + r) + k of lane L
 * holds bit 7-k of state byte (row r, column 2L + j) for the pair's 32
 * blocks (bit i of the register = block i).  SubBytes is the Boyar-Peralta
 * (2012) circuit, XOR/AND only, folded into 84 three-input v_bitop3
 * operations; ShiftRows exchanges four of a lane's eight bytes with its
 * partner (one DPP quad_perm move per register); MixColumns is 3-input XORs;
 * AddRoundKey XORs 0/~0 masks of the round-key bits.  Every round is
 * fast-class VALU (no shift, permute or table), and no data-dependent
 * address is ever formed: the AES is constant-time, unlike a T-table AES.
 */
#pragma once
#include "aead_device.h"

namespace na {

/* Boyar-Peralta S-box, x0 = MSB of the byte (in place) */
NA_DEV void bs_sbox(uint32_t &q0, uint32_t &q1, uint32_t &q2, uint32_t &q3, uint32_t &q4, uint32_t &q5,
                    uint32_t &q6, uint32_t &q7)
{
    const uint32_t x0 = q0, x1 = q1, x2 = q2, x3 = q3, x4 = q4, x5 = q5, x6 = q6, x7 = q7;
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
    q0 = s0; q1 = s1; q2 = s2; q3 = s3; q4 = s4; q5 = s5; q6 = s6; q7 = s7;
}

NA_DEV uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

/* the partner lane's value (lanes 2p and 2p+1 swap): DPP quad_perm [1,0,3,2] */
NA_DEV uint32_t bs_partner(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false); }

/* MixColumns + AddRoundKey of one output column from its four ShiftRows
   inputs a[0..3] (bit-planes, MSB first) and the column's 32 masks mk:
   out_r = xtime(a_r ^ a_r+1) ^ (s ^ a_r ^ key), s = a_0 ^ a_1 ^ a_2 ^ a_3
   (MIX), or a_r ^ key (the last round). */
template <bool MIX>
NA_DEV void bs2_column(const uint32_t *a0, const uint32_t *a1, const uint32_t *a2, const uint32_t *a3,
                       const uint32_t *mk, uint32_t *o)
{
    const uint32_t *a[4] = {a0, a1, a2, a3};
    if constexpr (!MIX) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint4 m0 = ((const uint4 *)mk)[2 * r], m1 = ((const uint4 *)mk)[2 * r + 1];
            const uint32_t M[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) o[8 * r + k] = a[r][k] ^ M[k];
        }
        return;
    }
    uint32_t sx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sx[k] = bs_x3(a[0][k], a[1][k], a[2][k]) ^ a[3][k];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t *A = a[r], *B = a[(r + 1) & 3];
        const uint4 m0 = ((const uint4 *)mk)[2 * r], m1 = ((const uint4 *)mk)[2 * r + 1];
        const uint32_t M[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
        uint32_t t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = A[k] ^ B[k];
        uint32_t *O = &o[8 * r];
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

#define NA_BS_SBOX(q, b) bs_sbox(q[8 * (b)], q[8 * (b) + 1], q[8 * (b) + 2], q[8 * (b) + 3], q[8 * (b) + 4], \
                                 q[8 * (b) + 5], q[8 * (b) + 6], q[8 * (b) + 7])

/* One round on the lane's half state h[64] (SubBytes, ShiftRows, MixColumns
   when MIX, AddRoundKey with this lane's 64 masks mk), in three phases so
   that at most ~100 values are live (four waves per SIMD allow 128 VGPRs):
   the four bytes the partner needs (local 1, 2, 6, 7) go through their
   S-boxes and across first; then output column 0 (own bytes 0 and 5 — (0,0)
   and (1,1) — with the partner's (2,0) and (3,1)); then column 1 (own 4 and
   3 — (0,1) and (3,0) — with the partner's (1,0) and (2,1)).  Local byte
   4j + r is (row r, local column j). */
template <bool MIX>
NA_DEV void bs2_round(uint32_t h[64], const uint32_t *mk)
{
    NA_BS_SBOX(h, 1); NA_BS_SBOX(h, 2); NA_BS_SBOX(h, 6); NA_BS_SBOX(h, 7);
    uint32_t px[4][8]; /* the partner's local bytes 1, 2, 6, 7 */
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        px[0][k] = bs_partner(h[8 + k]);
        px[1][k] = bs_partner(h[16 + k]);
        px[2][k] = bs_partner(h[48 + k]);
        px[3][k] = bs_partner(h[56 + k]);
    }
    __builtin_amdgcn_sched_barrier(0);
    NA_BS_SBOX(h, 0); NA_BS_SBOX(h, 5);
    uint32_t o0[32];
    bs2_column<MIX>(&h[0], &h[40], px[1], px[3], mk, o0);
    __builtin_amdgcn_sched_barrier(0);
    NA_BS_SBOX(h, 4); NA_BS_SBOX(h, 3);
    uint32_t o1[32];
    bs2_column<MIX>(&h[32], px[0], px[2], &h[24], mk + 32, o1);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        h[i] = o0[i];
        h[32 + i] = o1[i];
    }
}

/* swap step of a bit-matrix transpose: exchange a's bits [w, 2w) blocks with
   b's [0, w) blocks under mask */
NA_DEV void bs_tswap(uint32_t &a, uint32_t &b, int w, uint32_t mask)
{
    const uint32_t t = ((a >> w) ^ b) & mask;
    b ^= t;
    a ^= t << w;
}

/* 32x32 bit transpose of r[0..31] in place: bit i of r[p] <-> bit p of r[i] */
NA_DEV void bs_transpose32(uint32_t r[32])
{
    const uint32_t masks[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int w = 16 >> s;
#pragma unroll
        for (int p = 0; p < 32; ++p)
            if (!(p & w)) bs_tswap(r[p], r[p | w], w, masks[s]);
    }
}

/* Round-key masks of one lane half: km[rnd][L][8*(4j + r) + k] = ~0 when bit
   7-k of round-key byte (r, 2L + j) of round rnd is set (rk: the 60 BE words
   of rijndaelKeySetupEnc, rijndael-alg-fst.c:728-807).  Entry e of 1920. */
NA_DEV uint32_t bs_mask_entry(const uint32_t *rk, uint32_t e)
{
    const uint32_t rnd = e / 128, L = (e / 64) & 1, loc = e & 63;
    const uint32_t j = loc >> 5, r = (loc >> 3) & 3, k = loc & 7;
    const uint32_t c = 2 * L + j;
    const uint32_t byte = (rk[4 * rnd + c] >> (24 - 8 * r)) & 255u;
    return 0u - ((byte >> (7 - k)) & 1u);
}

/* Keystream of counter blocks 0^32 || BE64(n) || BE32(32g + i), i = 0..31,
   on a lane pair (lane L = lane & 1), from the masks km (15 x 2 x 64 words in
   LDS): kw[j][i] = little-endian memory word 2L + j of block i. */
NA_DEV void bs2_ctr_group(const uint32_t *km, uint32_t L, uint32_t n_hi, uint32_t n_lo, uint32_t g,
                          uint32_t kw[2][32])
{
    const uint32_t ctr0 = 32u * g;
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
    if (L) { /* byte 15 (row 3, column 3): counter bits 0..4 run over the 32 blocks */
        uint32_t *q = &h[8 * (4 * 1 + 3)];
        q[7] = 0xAAAAAAAAu; q[6] = 0xCCCCCCCCu; q[5] = 0xF0F0F0F0u; q[4] = 0xFF00FF00u; q[3] = 0xFFFF0000u;
    }
    const uint32_t *k0 = km + 64 * L;
#pragma unroll
    for (int i = 0; i < 64; ++i) h[i] ^= k0[i];
#pragma unroll 1
    for (int rr = 1; rr < 14; ++rr) bs2_round<true>(h, km + 128 * rr + 64 * L);
    bs2_round<false>(h, km + 128 * 14 + 64 * L);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        uint32_t *r32 = kw[j];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int k = 0; k < 8; ++k) r32[8 * rb + (7 - k)] = h[8 * (4 * j + rb) + k];
        bs_transpose32(r32);
    }
}

} // namespace na
