/*
 * aesgcm.hip — AES-256-GCM ("AESGCM") transport AEAD for gfx950.
 *
 * Replaces, for batches of records, the per-record CPU path
 *   noise_cipherstate_{en,de}crypt_with_ad     (src/protocol/cipherstate.c:293-410)
 *   -> noise_aesgcm_{encrypt,decrypt}         (src/backend/ref/cipher-aesgcm.c:156-188)
 *   -> rijndaelEncrypt                        (src/crypto/aes/rijndael-alg-fst.c:854-1033)
 *   -> ghash_update / GF128_mul               (src/crypto/ghash/ghash.c:78-206)
 * bit for bit: J0 = 0^32 || BE64(n) || 0x00000001, data counters J0+1.., tag =
 * E_K(J0) xor GHASH_H(AD || pad || CT || pad || BE64(8|AD|) || BE64(8|CT|)),
 * H = E_K(0^128) (cipher-aesgcm.c:38-50, 70-90, 99-154).
 *
 * Decomposition: GCM_LANES = 4 lanes per record.  The record's GHASH blocks
 * i = 0..n-1 (AD, CT, length block) are dealt round-robin, end-aligned, so
 * lane l owns i == l + n (mod 4) and its last block has exponent 4 - l.  Each
 * lane runs Horner with H^4, scales by H^(4-l), and the group XOR-reduces.
 * GHASH multiplies by a per-key constant use 4-bit positional tables (32
 * nibble positions x 16 entries per multiplier) built once per key by
 * gcm_prepare.  The lane that owns data block d also runs its CTR block.
 *
 * Note: table-driven GHASH/AES on LDS/L1 is not constant-time, unlike the
 * reference's bit-serial GF128_mul (ghash.c:85-87); see DESIGN.md.
 */
#include "aead_device.h"
#include "aead_kernels.h"

namespace na {

/* per translation unit (static): launch_aes.hip's kernels read these; the
   resident worker (worker.hip) builds its own copy in LDS */
static __device__ uint32_t g_te0[256]; /* T-table: BE word (2s, s, s, 3s) */
static __device__ uint32_t g_sbox[256];

NA_DEV uint32_t xtime8(uint32_t a) { return ((a << 1) ^ ((a & 0x80) ? 0x1b : 0)) & 0xff; }

NA_DEV uint32_t gf8_mul(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        a = xtime8(a);
        b >>= 1;
    }
    return p;
}

/* FIPS-197 S-box entry x and T-table entry (inverse = x^254). */
NA_DEV void aes_table_entry(uint32_t x, uint32_t &sbox, uint32_t &te0)
{
    uint32_t inv = 1, base = x;
    for (int e = 254; e; e >>= 1) {
        if (e & 1) inv = gf8_mul(inv, base);
        base = gf8_mul(base, base);
    }
    if (x == 0) inv = 0;
    uint32_t s = inv;
    for (int i = 1; i <= 4; ++i) s ^= ((inv << i) | (inv >> (8 - i))) & 0xff;
    s ^= 0x63;
    sbox = s;
    const uint32_t s2 = xtime8(s), s3 = s2 ^ s;
    te0 = (s2 << 24) | (s << 16) | (s << 8) | s3;
}

#ifndef NA_NO_SETUP_KERNELS /* worker.hip includes only the device functions */
/* The tables, generated on the device once (launch_aes.hip ensure_aes_tables). */
__global__ void aes_tables_init()
{
    const uint32_t x = threadIdx.x;
    aes_table_entry(x, g_sbox[x], g_te0[x]);
}
#endif

NA_DEV uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

/* AES-256 encryption of one block in big-endian-word form (the GETU32/PUTU32
   convention of rijndael-alg-fst.c:718-721). te/sb live in LDS. */
NA_DEV void aes256_block(const uint32_t *__restrict__ rk, const uint32_t *te, const uint32_t *sb,
                         uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3)
{
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        /* the round's 16 lookups are independent: issue them all, then one
           wait (the empty asm keeps the scheduler from trading them for
           registers one load at a time: 2x the block's latency in the
           256-VGPR resident worker, tools/microbench/aes_lat.hip) */
        uint32_t a0 = te[s0 >> 24], a1 = te[(s1 >> 16) & 255], a2 = te[(s2 >> 8) & 255], a3 = te[s3 & 255];
        uint32_t b0 = te[s1 >> 24], b1 = te[(s2 >> 16) & 255], b2 = te[(s3 >> 8) & 255], b3 = te[s0 & 255];
        uint32_t c0 = te[s2 >> 24], c1 = te[(s3 >> 16) & 255], c2 = te[(s0 >> 8) & 255], c3 = te[s1 & 255];
        uint32_t d0 = te[s3 >> 24], d1 = te[(s0 >> 16) & 255], d2 = te[(s1 >> 8) & 255], d3 = te[s2 & 255];
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3),
                          "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
        s0 = a0 ^ rotr(a1, 8) ^ rotr(a2, 16) ^ rotr(a3, 24) ^ rk[4 * r];
        s1 = b0 ^ rotr(b1, 8) ^ rotr(b2, 16) ^ rotr(b3, 24) ^ rk[4 * r + 1];
        s2 = c0 ^ rotr(c1, 8) ^ rotr(c2, 16) ^ rotr(c3, 24) ^ rk[4 * r + 2];
        s3 = d0 ^ rotr(d1, 8) ^ rotr(d2, 16) ^ rotr(d3, 24) ^ rk[4 * r + 3];
    }
    const uint32_t o0 = (sb[s0 >> 24] << 24) | (sb[(s1 >> 16) & 255] << 16) |
                        (sb[(s2 >> 8) & 255] << 8) | sb[s3 & 255];
    const uint32_t o1 = (sb[s1 >> 24] << 24) | (sb[(s2 >> 16) & 255] << 16) |
                        (sb[(s3 >> 8) & 255] << 8) | sb[s0 & 255];
    const uint32_t o2 = (sb[s2 >> 24] << 24) | (sb[(s3 >> 16) & 255] << 16) |
                        (sb[(s0 >> 8) & 255] << 8) | sb[s1 & 255];
    const uint32_t o3 = (sb[s3 >> 24] << 24) | (sb[(s0 >> 16) & 255] << 16) |
                        (sb[(s1 >> 8) & 255] << 8) | sb[s2 & 255];
    s0 = o0 ^ rk[56]; s1 = o1 ^ rk[57]; s2 = o2 ^ rk[58]; s3 = o3 ^ rk[59];
}

/* E_K(0^32 || BE64(n) || BE32(ctr)) as little-endian memory words. */
NA_DEV void aes_ctr_block(const uint32_t *rk, const uint32_t *te, const uint32_t *sb,
                          uint64_t n, uint32_t ctr, uint32_t ks[4])
{
    uint32_t s0 = 0, s1 = (uint32_t)(n >> 32), s2 = (uint32_t)n, s3 = ctr;
    aes256_block(rk, te, sb, s0, s1, s2, s3);
    ks[0] = __builtin_bswap32(s0); ks[1] = __builtin_bswap32(s1);
    ks[2] = __builtin_bswap32(s2); ks[3] = __builtin_bswap32(s3);
}

/* y <- y * Y where tab is Y's 4-bit positional table (LE-word layout). */
NA_DEV void gh_mul(uint32_t y[4], const uint4 *__restrict__ tab)
{
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        const int b = p >> 1;
        const int sh = 8 * (b & 3) + ((p & 1) ? 0 : 4);
        const uint32_t v = (y[b >> 2] >> sh) & 15u;
        const uint4 e = tab[p * 16 + v];
        r0 ^= e.x; r1 ^= e.y; r2 ^= e.z; r3 ^= e.w;
    }
    y[0] = r0; y[1] = r1; y[2] = r2; y[3] = r3;
}

NA_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

/* ------------------------------------------- constant-time GHASH (opt-in)
 *
 * NOISE_AEAD_FLAG_CT_GHASH: the GHASH multiplies touch no table — the
 * property the reference's bit-serial GF128_mul has (ghash.c:85-108).  The
 * field element is held in the natural polynomial domain (bit i of the
 * 128-bit word vector = coefficient of x^i): a GCM block loaded as LE words
 * maps there by reversing the bits of each byte (bswap . bfrev, its own
 * inverse).  The product is a carry-less 128x128 multiply — two levels of
 * Karatsuba over nine 32x32 products — reduced by x^128 + x^7 + x^2 + x + 1.
 * A 32x32 carry-less product comes from integer multiplies: split each
 * operand into four parts holding every 4th bit; an integer product of two
 * parts has at most 8 terms on any bit position of its class, so the carries
 * stay in the three positions above it, which the class mask drops (the
 * BearSSL "ctmul" construction).  ≈ 620 VALU per block multiply, no LDS. */
NA_DEV uint32_t gh_nat(uint32_t w) { return __builtin_bswap32(__builtin_bitreverse32(w)); }

NA_DEV uint64_t clmul32(uint32_t a, uint32_t b)
{
    const uint32_t a0 = a & 0x11111111u, a1 = a & 0x22222222u, a2 = a & 0x44444444u,
                   a3 = a & 0x88888888u;
    const uint32_t b0 = b & 0x11111111u, b1 = b & 0x22222222u, b2 = b & 0x44444444u,
                   b3 = b & 0x88888888u;
    const uint64_t z0 = ((uint64_t)a0 * b0) ^ ((uint64_t)a1 * b3) ^ ((uint64_t)a2 * b2) ^ ((uint64_t)a3 * b1);
    const uint64_t z1 = ((uint64_t)a0 * b1) ^ ((uint64_t)a1 * b0) ^ ((uint64_t)a2 * b3) ^ ((uint64_t)a3 * b2);
    const uint64_t z2 = ((uint64_t)a0 * b2) ^ ((uint64_t)a1 * b1) ^ ((uint64_t)a2 * b0) ^ ((uint64_t)a3 * b3);
    const uint64_t z3 = ((uint64_t)a0 * b3) ^ ((uint64_t)a1 * b2) ^ ((uint64_t)a2 * b1) ^ ((uint64_t)a3 * b0);
    return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) |
           (z2 & 0x4444444444444444ull) | (z3 & 0x8888888888888888ull);
}

/* 64x64 -> 128 carry-less (Karatsuba): r[0..3] */
NA_DEV void clmul64(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1, uint32_t r[4])
{
    const uint64_t lo = clmul32(a0, b0), hi = clmul32(a1, b1);
    const uint64_t mid = clmul32(a0 ^ a1, b0 ^ b1) ^ lo ^ hi;
    r[0] = (uint32_t)lo;
    r[1] = (uint32_t)(lo >> 32) ^ (uint32_t)mid;
    r[2] = (uint32_t)hi ^ (uint32_t)(mid >> 32);
    r[3] = (uint32_t)(hi >> 32);
}

/* y <- y * h in GF(2^128), both in the natural domain */
NA_DEV void gh_mul_ct(uint32_t y[4], const uint32_t h[4])
{
    uint32_t lo[4], hi[4], mid[4];
    clmul64(y[0], y[1], h[0], h[1], lo);
    clmul64(y[2], y[3], h[2], h[3], hi);
    clmul64(y[0] ^ y[2], y[1] ^ y[3], h[0] ^ h[2], h[1] ^ h[3], mid);
#pragma unroll
    for (int i = 0; i < 4; ++i) mid[i] = xor3(mid[i], lo[i], hi[i]);
    /* P = hi x^128 + mid x^64 + lo: 256-bit words p0..p7 */
    const uint32_t p0 = lo[0], p1 = lo[1], p2 = lo[2] ^ mid[0], p3 = lo[3] ^ mid[1];
    const uint32_t p4 = hi[0] ^ mid[2], p5 = hi[1] ^ mid[3], p6 = hi[2], p7 = hi[3];
    /* p4..p7 x^128 = (p4..p7)(x^7 + x^2 + x + 1): shift-XOR, then fold the
       bits shifted past x^127 (degree <= 6) the same way */
    const uint32_t t0 = xor3(p4, p4 << 1, p4 << 2) ^ (p4 << 7);
    const uint32_t t1 = xor3(p5, __builtin_amdgcn_alignbit(p5, p4, 31), __builtin_amdgcn_alignbit(p5, p4, 30)) ^
                        __builtin_amdgcn_alignbit(p5, p4, 25);
    const uint32_t t2 = xor3(p6, __builtin_amdgcn_alignbit(p6, p5, 31), __builtin_amdgcn_alignbit(p6, p5, 30)) ^
                        __builtin_amdgcn_alignbit(p6, p5, 25);
    const uint32_t t3 = xor3(p7, __builtin_amdgcn_alignbit(p7, p6, 31), __builtin_amdgcn_alignbit(p7, p6, 30)) ^
                        __builtin_amdgcn_alignbit(p7, p6, 25);
    const uint32_t o = xor3(p7 >> 31, p7 >> 30, p7 >> 25);
    const uint32_t f = xor3(o, o << 1, o << 2) ^ (o << 7);
    y[0] = xor3(p0, t0, f);
    y[1] = p1 ^ t1;
    y[2] = p2 ^ t2;
    y[3] = p3 ^ t3;
}

/* GCM-domain LE words <-> natural domain (the map is an involution) */
NA_DEV void gh_to_nat(uint32_t x[4])
{
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = gh_nat(x[i]);
}



/* gh_mul with the table in LDS: lookups taken in pairs so every accumulate is
   one 3-input XOR */
NA_DEV void gh_mul_lds(uint32_t y[4], const uint4 *tab)
{
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
    for (int p = 0; p < 32; p += 2) {
        const int b = p >> 1; /* byte b: high nibble is position p, low nibble p+1 */
        const uint32_t byte = (y[b >> 2] >> (8 * (b & 3))) & 255u;
        const uint4 e = tab[p * 16 + (byte >> 4)];
        const uint4 f = tab[(p + 1) * 16 + (byte & 15)];
        r0 = xor3(r0, e.x, f.x); r1 = xor3(r1, e.y, f.y);
        r2 = xor3(r2, e.z, f.z); r3 = xor3(r3, e.w, f.w);
    }
    y[0] = r0; y[1] = r1; y[2] = r2; y[3] = r3;
}

/* gh_mul_lds for one wave's latency (the wide record's few GHASH lanes):
   the lookups in two batches of 16, each issued whole before one wait */
NA_DEV void gh_mul_lds_lat(uint32_t y[4], const uint4 *tab)
{
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u *t4 = (const v4u *)tab;
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        v4u e[16];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p = 16 * half + 2 * j, b = p >> 1;
            const uint32_t byte = (y[b >> 2] >> (8 * (b & 3))) & 255u;
            e[2 * j] = t4[p * 16 + (byte >> 4)];
            e[2 * j + 1] = t4[(p + 1) * 16 + (byte & 15)];
        }
        asm volatile("" : "+v"(e[0]), "+v"(e[1]), "+v"(e[2]), "+v"(e[3]), "+v"(e[4]), "+v"(e[5]), "+v"(e[6]),
                          "+v"(e[7]), "+v"(e[8]), "+v"(e[9]), "+v"(e[10]), "+v"(e[11]), "+v"(e[12]), "+v"(e[13]),
                          "+v"(e[14]), "+v"(e[15]));
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
            r0 = xor3(r0, e[j].x, e[j + 1].x); r1 = xor3(r1, e[j].y, e[j + 1].y);
            r2 = xor3(r2, e[j].z, e[j + 1].z); r3 = xor3(r3, e[j].w, e[j + 1].w);
        }
    }
    y[0] = r0; y[1] = r1; y[2] = r2; y[3] = r3;
}

/* The Horner step y <- y * H^4 (tables in LDS, or constant-time: y and the
   blocks in the natural domain, hn4 = H^4 there) and the final scale
   y <- y * H^(m+1) (the context's tables in global memory, or CT). */
template <bool CT>
NA_DEV void gh_step(uint32_t y[4], const uint4 *tab_lds, const uint32_t hn4[4])
{
    if constexpr (CT) gh_mul_ct(y, hn4);
    else gh_mul_lds(y, tab_lds);
}

template <bool CT>
NA_DEV void gh_scale1(uint32_t y[4], const AesCtx *ctx, int m)
{
    if constexpr (CT) {
        uint32_t h[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) h[w] = ctx->hn[m][w];
        gh_mul_ct(y, h);
    } else {
        gh_mul(y, (const uint4 *)ctx->tab[m]);
    }
}

/* y <- y * H^(m+1), m < K (lanes per record): K = 8 lanes 0..3 take
   H^(m+1) = H^4 * H^(m-3) */
template <bool CT, int K = GCM_LANES>
NA_DEV void gh_scale(uint32_t y[4], const AesCtx *ctx, int m)
{
    if (K > GCM_LANES && m >= GCM_LANES) {
        gh_scale1<CT>(y, ctx, GCM_LANES - 1);
        m -= GCM_LANES;
    }
    gh_scale1<CT>(y, ctx, m);
}

/* ----------------------------------------------------------- key prepare */

/* Byte-serial GF(2^128) helpers for the (once per key) table build. */
NA_DEV void gf_mulx(uint8_t v[16])
{
    const uint8_t carry = v[15] & 1;
    for (int j = 15; j > 0; --j) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
    v[0] >>= 1;
    if (carry) v[0] ^= 0xE1;
}

NA_DEV void gf_mul_bytes(const uint8_t x[16], const uint8_t h[16], uint8_t out[16])
{
    uint8_t z[16] = {0}, v[16];
    for (int j = 0; j < 16; ++j) v[j] = h[j];
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int j = 0; j < 16; ++j) z[j] ^= v[j];
        gf_mulx(v);
    }
    for (int j = 0; j < 16; ++j) out[j] = z[j];
}

#ifndef NA_NO_SETUP_KERNELS
/* One workgroup per state: round keys, H, and the H^1..H^4 tables. */
__global__ __launch_bounds__(256) void gcm_prepare(const uint8_t *__restrict__ raw_keys,
                                                   AesCtx *__restrict__ ctx, uint32_t n_states)
{
    __shared__ uint32_t te[256], sb[256], rk[60];
    __shared__ uint8_t hp[GCM_LANES + 1][16];       /* H^1..H^4, H^8, bytes */
    __shared__ uint8_t V[GCM_LANES + 1][128][16];   /* x^i * H^m */
    const uint32_t st = blockIdx.x;
    if (st >= n_states) return;
    const int t = threadIdx.x;
    te[t] = g_te0[t];
    sb[t] = g_sbox[t];
    __syncthreads();
    if (t == 0) {
        const uint8_t *k = raw_keys + (size_t)st * 32;
        for (int i = 0; i < 8; ++i)
            rk[i] = ((uint32_t)k[4 * i] << 24) | ((uint32_t)k[4 * i + 1] << 16) |
                    ((uint32_t)k[4 * i + 2] << 8) | k[4 * i + 3];
        uint32_t rcon = 1;
        for (int i = 8; i < 60; ++i) {
            uint32_t tmp = rk[i - 1];
            if (i % 8 == 0) {
                tmp = (tmp << 8) | (tmp >> 24); /* RotWord */
                tmp = (sb[tmp >> 24] << 24) | (sb[(tmp >> 16) & 255] << 16) |
                      (sb[(tmp >> 8) & 255] << 8) | sb[tmp & 255];
                tmp ^= rcon << 24;
                rcon = xtime8(rcon);
            } else if (i % 8 == 4) {
                tmp = (sb[tmp >> 24] << 24) | (sb[(tmp >> 16) & 255] << 16) |
                      (sb[(tmp >> 8) & 255] << 8) | sb[tmp & 255];
            }
            rk[i] = rk[i - 8] ^ tmp;
        }
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        aes256_block(rk, te, sb, s0, s1, s2, s3);
        const uint32_t hw[4] = {s0, s1, s2, s3};
        for (int i = 0; i < 16; ++i) hp[0][i] = (uint8_t)(hw[i >> 2] >> (24 - 8 * (i & 3)));
        for (int m = 1; m < GCM_LANES; ++m) gf_mul_bytes(hp[m - 1], hp[0], hp[m]);
        gf_mul_bytes(hp[GCM_LANES - 1], hp[GCM_LANES - 1], hp[GCM_LANES]); /* H^8 */
    }
    __syncthreads();
    if (t < GCM_LANES + 1) {
        uint8_t v[16];
        for (int j = 0; j < 16; ++j) v[j] = hp[t][j];
        for (int i = 0; i < 128; ++i) {
            for (int j = 0; j < 16; ++j) V[t][i][j] = v[j];
            gf_mulx(v);
        }
    }
    __syncthreads();
    AesCtx *c = ctx + st;
    if (t < 60) c->rk[t] = rk[t];
    if (t < 4) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) w |= (uint32_t)hp[0][4 * t + j] << (8 * j);
        c->h[t] = w;
    }
    if (t < 4 * (GCM_LANES + 1)) { /* H^1..H^4, H^8, natural domain */
        const int m = t >> 2, q = t & 3;
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) w |= (uint32_t)hp[m][4 * q + j] << (8 * j);
        if (m < GCM_LANES) c->hn[m][q] = gh_nat(w);
        else c->hn8[q] = gh_nat(w);
    }
    for (int e = t; e < (GCM_LANES + 1) * GHASH_TAB_ENTRIES; e += 256) {
        const int m = e / GHASH_TAB_ENTRIES, p = (e / 16) % 32, val = e % 16;
        uint8_t acc[16] = {0};
        for (int bit = 0; bit < 4; ++bit)
            if ((val >> (3 - bit)) & 1)
                for (int j = 0; j < 16; ++j) acc[j] ^= V[m][4 * p + bit][j];
        uint32_t *dst = m < GCM_LANES ? c->tab[m][p * 16 + val] : c->tab8[p * 16 + val];
        for (int w = 0; w < 4; ++w)
            dst[w] = (uint32_t)acc[4 * w] | ((uint32_t)acc[4 * w + 1] << 8) |
                     ((uint32_t)acc[4 * w + 2] << 16) | ((uint32_t)acc[4 * w + 3] << 24);
    }
}
#endif

/* ---------------------------------------------------------------- records */

struct GcmView {
    const uint8_t *src;
    uint8_t *dst;
    const uint8_t *ad;
    const AesCtx *ctx;
    uint64_t nonce;
    uint32_t len, ad_len;
};

/* Returns (seal) true; (open) whether the tag verified. */
template <bool OPEN, bool CT>
NA_DEV bool gcm_record(const GcmView &rv, int l, const uint32_t *te, const uint32_t *sb)
{
    constexpr int K = GCM_LANES;
    const AesCtx *ctx = rv.ctx;
    const uint32_t *rk = ctx->rk;
    const uint32_t A = (rv.ad_len + 15) / 16, M = (rv.len + 15) / 16;
    const uint32_t n = A + M + 1;
    const uint32_t c0 = ((uint32_t)l + n) % K;
    const uint4 *tabH4 = (const uint4 *)ctx->tab[K - 1];
    uint32_t h4n[4] = {0, 0, 0, 0};
    if constexpr (CT) {
#pragma unroll
        for (int w = 0; w < 4; ++w) h4n[w] = ctx->hn[K - 1][w];
    }
    uint32_t acc[4] = {0, 0, 0, 0};
    for (uint32_t i = c0; i < n; i += K) {
        if (i != c0) {
            if constexpr (CT) gh_mul_ct(acc, h4n);
            else gh_mul(acc, tabH4);
        }
        uint32_t x[4];
        if (i < A) {
            const uint32_t rem = rv.ad_len - 16 * i;
            load16(rv.ad + 16 * i, rem >= 16 ? 16u : rem, x);
        } else if (i < A + M) {
            const uint32_t d = i - A;
            const uint32_t rem = rv.len - 16 * d;
            const uint32_t nb = rem >= 16 ? 16u : rem;
            load16(rv.src + 16 * d, nb, x);
            if (!OPEN) {
                uint32_t ks[4];
                aes_ctr_block(rk, te, sb, rv.nonce, 2 + d, ks);
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const int rb = (int)nb - 4 * w;
                    const uint32_t m = rb >= 4 ? 0xffffffffu : (rb <= 0 ? 0u : ((1u << (8 * rb)) - 1u));
                    x[w] = (x[w] ^ ks[w]) & m;
                }
                store16(rv.dst + 16 * d, nb, x);
            }
        } else {
            const uint64_t ab = (uint64_t)rv.ad_len * 8, cb = (uint64_t)rv.len * 8;
            x[0] = __builtin_bswap32((uint32_t)(ab >> 32)); x[1] = __builtin_bswap32((uint32_t)ab);
            x[2] = __builtin_bswap32((uint32_t)(cb >> 32)); x[3] = __builtin_bswap32((uint32_t)cb);
        }
        if constexpr (CT) gh_to_nat(x);
        acc[0] ^= x[0]; acc[1] ^= x[1]; acc[2] ^= x[2]; acc[3] ^= x[3];
    }
    /* scale by H^(K-l) (lane l's last block has exponent K-l) */
    gh_scale<CT>(acc, ctx, K - 1 - l);
#pragma unroll
    for (int off = 1; off < K; off <<= 1)
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[w] ^= (uint32_t)__shfl_xor((int)acc[w], off, 64);
    if constexpr (CT) gh_to_nat(acc); /* back to the GCM domain */
    /* tag = E_K(J0) xor S: every lane of the group computes it (one AES) */
    uint32_t ej[4];
    aes_ctr_block(rk, te, sb, rv.nonce, 1u, ej);
    uint32_t tag[4] = {acc[0] ^ ej[0], acc[1] ^ ej[1], acc[2] ^ ej[2], acc[3] ^ ej[3]};
    if (!OPEN) {
        if (l == K - 1) store16(rv.dst + rv.len, 16, tag);
        return true;
    }
    uint32_t got[4];
    load16(rv.src + rv.len, 16, got);
    const uint32_t diff = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
    if (diff) return false; /* cipher-aesgcm.c:184-186: nothing decrypted */
    for (uint32_t d = (c0 + K - (A % K)) % K; d < M; d += K) {
        const uint32_t rem = rv.len - 16 * d;
        const uint32_t nb = rem >= 16 ? 16u : rem;
        uint32_t x[4], ks[4];
        load16(rv.src + 16 * d, nb, x);
        aes_ctr_block(rk, te, sb, rv.nonce, 2 + d, ks);
#pragma unroll
        for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
        store16(rv.dst + 16 * d, nb, x);
    }
    return true;
}

NA_DEV void load_aes_tables(uint32_t *te, uint32_t *sb)
{
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        te[i] = g_te0[i];
        sb[i] = g_sbox[i];
    }
    __syncthreads();
}

template <bool OPEN, bool CT>
__global__ __launch_bounds__(256) void gcm_uniform(UniformArgs a)
{
    __shared__ uint32_t te[256], sb[256];
    load_aes_tables(te, sb);
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / GCM_LANES;
    if (rec >= a.n_records) return;
    const int l = (int)(gtid % GCM_LANES);
    const uint32_t st = rec / a.rps;
    GcmView rv;
    rv.src = a.in + (size_t)rec * a.in_stride;
    rv.dst = a.out + (size_t)rec * a.out_stride;
    rv.ad = a.ad ? a.ad + (size_t)rec * a.ad_stride : nullptr;
    rv.ctx = (const AesCtx *)a.keys + st;
    rv.nonce = a.nonce_base[st] + (uint64_t)(rec - st * a.rps);
    rv.len = a.len;
    rv.ad_len = a.ad_len;
    const bool ok = gcm_record<OPEN, CT>(rv, l, te, sb); /* open: verifies first */
    if (OPEN && l == GCM_LANES - 1 && a.status) a.status[rec] = ok ? 0 : 1;
    if (!ok && !a.vf) scrub_rejected(rv.dst, rv.src, rv.len, (uint32_t)l, GCM_LANES);
}

template <bool OPEN, bool CT>
__global__ __launch_bounds__(256) void gcm_ragged(RaggedArgs a)
{
    __shared__ uint32_t te[256], sb[256];
    __shared__ uint32_t order[256 / GCM_LANES];
    load_aes_tables(te, sb);
    const uint32_t rec = window_rec<256 / GCM_LANES>(a.recs, a.n_records,
                                                     blockIdx.x * (256u / GCM_LANES),
                                                     threadIdx.x / GCM_LANES, order);
    if (rec >= a.n_records) return;
    const int l = (int)(threadIdx.x % GCM_LANES);
    const RecDesc d = a.recs[rec];
    if (reject_len(a, rec, d.len, l == GCM_LANES - 1)) return;
    GcmView rv;
    rv.src = a.in + d.in_off;
    rv.dst = a.out + d.out_off;
    rv.ad = a.ad ? a.ad + d.ad_off : nullptr;
    rv.ctx = (const AesCtx *)((uintptr_t)a.keys + d.ctx_off);
    rv.nonce = d.nonce;
    rv.len = d.len;
    rv.ad_len = d.ad_len;
    const bool ok = gcm_record<OPEN, CT>(rv, l, te, sb);
    if (l == GCM_LANES - 1 && a.status) a.status[rec] = ok ? 0 : 1;
    if (!ok && !a.vf) scrub_rejected(rv.dst, rv.src, rv.len, (uint32_t)l, GCM_LANES);
}

/* ---------------------------- staged (uniform FAST, one state per workgroup)
 *
 * For uniform batches whose 256 records per workgroup share one CipherState
 * (recs_per_state a multiple of 256) and FAST layouts.  1024-thread
 * workgroups (one per CU, 4 waves per SIMD) hold in LDS:
 *  - the four AES T-tables, each replicated 32x so that lane c (mod 32) of a
 *    ds_read_b32 lane group always hits bank c: conflict-free lookups (the
 *    b32 reads bank on (a/4) mod 32, MI355X_MICROARCH.md §LDS).  Row i of a
 *    table is 128 B (32 copies of Te_t[i]); Te0|Te1 rows interleave in the
 *    first 64 KB (row stride 256 B), Te2|Te3 in the second.  The lookup
 *    address (t>=2)<<16 | byte<<8 | (t&1)<<7 | 4c is one v_perm_b32 of the
 *    state word and a per-lane template word;
 *  - the state's round keys and its multiply-by-H^4 GHASH table (16 entries
 *    x 16 B per nibble position: a 16-lane b128 group is conflict-free).
 * The per-block work then touches no global memory but the record bytes.
 */

struct GcmLds {
    uint32_t te[2][256][64]; /* [Te0|Te1 or Te2|Te3][row][32 + 32 copies] */
    uint4 h4[GHASH_TAB_ENTRIES];
    uint32_t rk[60];
};

NA_DEV void gcm_lds_fill(GcmLds &L, const AesCtx *ctx)
{
    const int t = threadIdx.x;
    /* 2 regions x 256 rows x 64 words = 32768 words: 8 uint4 per thread */
    for (int q = t; q < 2 * 256 * 16; q += GCM_WG) {
        const int reg = q >> 12, row = (q >> 4) & 255, quad = q & 15;
        const int tab = 2 * reg + (quad >> 3); /* words 0-31: Te(2reg), 32-63: Te(2reg+1) */
        const uint32_t v = rotr(g_te0[row], 8 * tab);
        ((uint4 *)&L.te[reg][row][0])[quad] = make_uint4(v, v, v, v);
    }
    const uint4 *src = (const uint4 *)ctx->tab[GCM_LANES - 1];
    for (int i = t; i < GHASH_TAB_ENTRIES; i += GCM_WG) L.h4[i] = src[i];
    if (t < 60) L.rk[t] = ctx->rk[t];
    __syncthreads();
}

/* te: the LDS base of the replicated Te0|Te1, Te2|Te3 regions (GcmLds::te) */
template <int TAB, int K>
NA_DEV uint32_t te_lookup(const uint8_t *te, uint32_t s, uint32_t lane_tpl)
{
    /* perm: out byte0 = tpl byte0 (4c) or byte1 (128 + 4c) for Te1/Te3,
       byte1 = s byte K, byte2 = tpl byte2 (1) for Te2/Te3 else 0, byte3 = 0 */
    constexpr uint32_t sel = (0x0cu << 24) | ((TAB >= 2 ? 2u : 0x0cu) << 16) | ((4u + K) << 8) |
                             (TAB & 1 ? 1u : 0u);
    const uint32_t addr = __builtin_amdgcn_perm(s, lane_tpl, sel);
    return *(const uint32_t *)(te + addr);
}

template <typename RK>
NA_DEV void aes256_lds(const uint8_t *L, RK rk, uint32_t tpl, uint32_t &s0,
                       uint32_t &s1, uint32_t &s2, uint32_t &s3)
{
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        /* Te0[a>>24] ^ Te1[(b>>16)&255] ^ Te2[(c>>8)&255] ^ Te3[d&255] ^ rk */
#define NA_COL(a, b, c, d, k)                                                        \
    xor3(xor3(te_lookup<0, 3>(L, a, tpl), te_lookup<1, 2>(L, b, tpl),                   \
              te_lookup<2, 1>(L, c, tpl)),                                             \
         te_lookup<3, 0>(L, d, tpl), rk[k])
        const uint32_t t0 = NA_COL(s0, s1, s2, s3, 4 * r);
        const uint32_t t1 = NA_COL(s1, s2, s3, s0, 4 * r + 1);
        const uint32_t t2 = NA_COL(s2, s3, s0, s1, 4 * r + 2);
        const uint32_t t3 = NA_COL(s3, s0, s1, s2, 4 * r + 3);
#undef NA_COL
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    /* last round: S-box bytes out of the T-tables (Te0 = [2s,s,s,3s] MSB first,
       Te1 = [3s,2s,s,s], Te2 = [s,3s,2s,s], Te3 = [s,s,3s,2s]) */
#define NA_SB4(a, b, c, d)                                                          \
    ((te_lookup<2, 3>(L, a, tpl) & 0xff000000u) | (te_lookup<3, 2>(L, b, tpl) & 0x00ff0000u) | \
     (te_lookup<0, 1>(L, c, tpl) & 0x0000ff00u) | (te_lookup<1, 0>(L, d, tpl) & 0x000000ffu))
    const uint32_t o0 = NA_SB4(s0, s1, s2, s3), o1 = NA_SB4(s1, s2, s3, s0);
    const uint32_t o2 = NA_SB4(s2, s3, s0, s1), o3 = NA_SB4(s3, s0, s1, s2);
#undef NA_SB4
    s0 = o0 ^ rk[56]; s1 = o1 ^ rk[57]; s2 = o2 ^ rk[58]; s3 = o3 ^ rk[59];
}

template <typename RK>
NA_DEV void aes_ctr_lds(const uint8_t *te, RK rk, uint32_t tpl, uint32_t n_hi,
                        uint32_t n_lo, uint32_t ctr, uint32_t ks[4])
{
    uint32_t s0 = 0, s1 = n_hi, s2 = n_lo, s3 = ctr;
    aes256_lds(te, rk, tpl, s0, s1, s2, s3);
    ks[0] = __builtin_bswap32(s0); ks[1] = __builtin_bswap32(s1);
    ks[2] = __builtin_bswap32(s2); ks[3] = __builtin_bswap32(s3);
}

/* Counter-mode caching.  Within one record the CTR input blocks
   0^32 || BE64(n) || BE32(ctr) differ only in ctr, and ctr <= 4097 (a record
   is at most 65519 bytes, the 16-bit counter rule of cipher-aesgcm.c:105-112)
   so only the two low bytes of state word 3 vary.  After the first round two
   of the four columns are constant and the other two each have one varying
   lookup; in the second round 8 of the 16 lookups read those constant
   columns.  AesPre holds the constant parts, computed once per record:
   22 of a block's 240 table lookups are then done once per record instead
   of once per block. */
struct AesPre {
    uint32_t c0, c1;         /* round 1, columns 0 and 1 without their ctr lookup */
    uint32_t d0, d1, d2, d3; /* round 2, each column's two constant lookups + key */
};

template <typename RK>
NA_DEV AesPre aes_pre_lds(const uint8_t *L, RK rk, uint32_t tpl, uint32_t n_hi,
                          uint32_t n_lo)
{
    const uint32_t s0 = rk[0], s1 = n_hi ^ rk[1], s2 = n_lo ^ rk[2], s3 = rk[3];
    AesPre p;
    p.c0 = xor3(te_lookup<0, 3>(L, s0, tpl), te_lookup<1, 2>(L, s1, tpl),
                te_lookup<2, 1>(L, s2, tpl)) ^ rk[4];
    p.c1 = xor3(te_lookup<0, 3>(L, s1, tpl), te_lookup<1, 2>(L, s2, tpl),
                te_lookup<3, 0>(L, s0, tpl)) ^ rk[5];
    /* s3's bytes 2 and 3 are rk[3]'s: ctr < 2^16 */
    const uint32_t t2 = xor3(xor3(te_lookup<0, 3>(L, s2, tpl), te_lookup<1, 2>(L, s3, tpl),
                                  te_lookup<2, 1>(L, s0, tpl)), te_lookup<3, 0>(L, s1, tpl), rk[6]);
    const uint32_t t3 = xor3(xor3(te_lookup<0, 3>(L, s3, tpl), te_lookup<1, 2>(L, s0, tpl),
                                  te_lookup<2, 1>(L, s1, tpl)), te_lookup<3, 0>(L, s2, tpl), rk[7]);
    p.d0 = xor3(te_lookup<2, 1>(L, t2, tpl), te_lookup<3, 0>(L, t3, tpl), rk[8]);
    p.d1 = xor3(te_lookup<1, 2>(L, t2, tpl), te_lookup<2, 1>(L, t3, tpl), rk[9]);
    p.d2 = xor3(te_lookup<0, 3>(L, t2, tpl), te_lookup<1, 2>(L, t3, tpl), rk[10]);
    p.d3 = xor3(te_lookup<0, 3>(L, t3, tpl), te_lookup<3, 0>(L, t2, tpl), rk[11]);
    return p;
}

/* E_K(0^32 || BE64(n) || BE32(ctr)) from the record's AesPre (ctr < 2^16),
   as little-endian memory words; equals aes_ctr_lds. */
template <typename RK>
NA_DEV void aes_ctr_pre(const uint8_t *L, RK rk, uint32_t tpl, const AesPre &p,
                        uint32_t ctr, uint32_t ks[4])
{
    const uint32_t s3 = ctr ^ rk[3];
    const uint32_t t0 = p.c0 ^ te_lookup<3, 0>(L, s3, tpl);
    const uint32_t t1 = p.c1 ^ te_lookup<2, 1>(L, s3, tpl);
    uint32_t s0 = xor3(p.d0, te_lookup<0, 3>(L, t0, tpl), te_lookup<1, 2>(L, t1, tpl));
    uint32_t s1 = xor3(p.d1, te_lookup<0, 3>(L, t1, tpl), te_lookup<3, 0>(L, t0, tpl));
    uint32_t s2 = xor3(p.d2, te_lookup<2, 1>(L, t0, tpl), te_lookup<3, 0>(L, t1, tpl));
    uint32_t s3b = xor3(p.d3, te_lookup<1, 2>(L, t0, tpl), te_lookup<2, 1>(L, t1, tpl));
#pragma unroll
    for (int r = 3; r < 14; ++r) {
#define NA_COL(a, b, c, d, k)                                                        \
    xor3(xor3(te_lookup<0, 3>(L, a, tpl), te_lookup<1, 2>(L, b, tpl),                   \
              te_lookup<2, 1>(L, c, tpl)),                                             \
         te_lookup<3, 0>(L, d, tpl), rk[k])
        const uint32_t u0 = NA_COL(s0, s1, s2, s3b, 4 * r);
        const uint32_t u1 = NA_COL(s1, s2, s3b, s0, 4 * r + 1);
        const uint32_t u2 = NA_COL(s2, s3b, s0, s1, 4 * r + 2);
        const uint32_t u3 = NA_COL(s3b, s0, s1, s2, 4 * r + 3);
#undef NA_COL
        s0 = u0; s1 = u1; s2 = u2; s3b = u3;
    }
#define NA_SB4(a, b, c, d)                                                          \
    ((te_lookup<2, 3>(L, a, tpl) & 0xff000000u) | (te_lookup<3, 2>(L, b, tpl) & 0x00ff0000u) | \
     (te_lookup<0, 1>(L, c, tpl) & 0x0000ff00u) | (te_lookup<1, 0>(L, d, tpl) & 0x000000ffu))
    const uint32_t o0 = NA_SB4(s0, s1, s2, s3b), o1 = NA_SB4(s1, s2, s3b, s0);
    const uint32_t o2 = NA_SB4(s2, s3b, s0, s1), o3 = NA_SB4(s3b, s0, s1, s2);
#undef NA_SB4
    ks[0] = __builtin_bswap32(o0 ^ rk[56]); ks[1] = __builtin_bswap32(o1 ^ rk[57]);
    ks[2] = __builtin_bswap32(o2 ^ rk[58]); ks[3] = __builtin_bswap32(o3 ^ rk[59]);
}

/* byte mask of the first nb (0..16) bytes of a 16-B block, word w */
NA_DEV uint32_t blk_mask(uint32_t nb, int w)
{
    const int rb = (int)nb - 4 * w;
    return rb >= 4 ? 0xffffffffu : (rb <= 0 ? 0u : ((1u << (8 * rb)) - 1u));
}

/* CTR over one lane's data blocks d = d0, d0 + K, ... < M of a record, src to
   dst: the decrypt pass of a VERIFY_FIRST open, after the tag verified. */
template <bool FAST = true, typename RK = const uint32_t *>
NA_DEV void gcm_ctr_lane(const uint8_t *TE, RK rk, uint32_t tpl, const AesPre &pre,
                         const uint8_t *src, uint8_t *dst, uint32_t len, uint32_t d0, uint32_t M,
                         uint32_t K)
{
#pragma unroll 1
    for (uint32_t d = d0; d < M; d += K) {
        const uint32_t nb = min(len - 16 * d, 16u);
        uint32_t x[4], ks[4];
        if (FAST) {
            const uint4 v = *(const uint4 *)(src + 16 * d);
            x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
        } else {
            load16(src + 16 * d, nb, x);
        }
        aes_ctr_pre(TE, rk, tpl, pre, 2 + d, ks);
#pragma unroll
        for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
        if (FAST && nb == 16) *(uint4 *)(dst + 16 * d) = make_uint4(x[0], x[1], x[2], x[3]);
        else store16(dst + 16 * d, nb, x);
    }
}

/* This thread's record of block blk (records [blk * 256, blk * 256 + 256))
   of a uniform staged job, with the T-tables at TE and the state's
   multiply-by-H^4 table and round keys (h4_lds, rk) in LDS. */
template <bool OPEN, bool CT, typename RK>
NA_DEV void gcm_staged_rec(const UniformArgs &a, const uint8_t *TE, const uint4 *h4_lds,
                           RK rk, uint32_t blk)
{
    constexpr int K = GCM_LANES;
    const uint32_t rec0 = blk * (uint32_t)GCM_WG_RECS;
    const uint32_t st = rec0 / a.rps; /* one state per workgroup (host-checked) */
    const AesCtx *ctx = (const AesCtx *)a.keys + st;
    const uint32_t rec = rec0 + threadIdx.x / K;
    if (rec >= a.n_records) return;
    const uint32_t lane = threadIdx.x & 63;
    /* lookup template: byte0 = 4c (Te0/Te2 copy c = lane mod 32), byte1 =
       128 + 4c (Te1/Te3), byte2 = 1 (the Te2|Te3 region at 64 KB) */
    const uint32_t tpl = (1u << 16) | ((128u + 4u * (lane & 31)) << 8) | (4u * (lane & 31));
    const int l = (int)(threadIdx.x % K);
    const uint64_t nonce = a.nonce_base[st] + (uint64_t)(rec - st * a.rps);
    const uint32_t n_hi = (uint32_t)(nonce >> 32), n_lo = (uint32_t)nonce;
    const uint8_t *src = a.in + (size_t)rec * a.in_stride;
    uint8_t *dst = a.out + (size_t)rec * a.out_stride;
    const uint32_t len = a.len, ad_len = a.ad_len;
    const uint32_t A = (ad_len + 15) / 16, M = (len + 15) / 16;
    const uint32_t n = A + M + 1;
    const uint32_t c0 = ((uint32_t)l + n) % K;

    /* GHASH (and, sealing, CTR) over this lane's blocks i = c0, c0+K, ... */
    uint32_t h4n[4] = {0, 0, 0, 0};
    if constexpr (CT) {
#pragma unroll
        for (int w = 0; w < 4; ++w) h4n[w] = ctx->hn[K - 1][w];
    }
    uint32_t acc[4] = {0, 0, 0, 0};
    const AesPre pre = aes_pre_lds(TE, rk, tpl, n_hi, n_lo);
#pragma unroll 1
    for (uint32_t i = c0; i < n; i += K) {
        if (i != c0) gh_step<CT>(acc, h4_lds, h4n);
        uint32_t x[4];
        if (i >= A && i < A + M) {
            const uint32_t d = i - A;
            const uint4 v = *(const uint4 *)(src + 16 * d); /* FAST: readable */
            x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
            const uint32_t nb = min(len - 16 * d, 16u);
            /* CTR for both directions in this one pass: the ciphertext is read
               once (open: GHASH over the block as read, plaintext out now,
               repaired below if the tag fails).  VERIFY_FIRST opens only
               authenticate here and decrypt after the verdict. */
            if (!OPEN || !a.vf) {
                uint32_t ks[4], y[4];
                aes_ctr_pre(TE, rk, tpl, pre, 2 + d, ks);
#pragma unroll
                for (int w = 0; w < 4; ++w) y[w] = x[w] ^ ks[w];
                if (nb == 16) *(uint4 *)(dst + 16 * d) = make_uint4(y[0], y[1], y[2], y[3]);
                else store16(dst + 16 * d, nb, y);
                if (!OPEN) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) x[w] = y[w];
                }
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) x[w] &= blk_mask(nb, w);
        } else if (i < A) {
            const uint32_t rem = ad_len - 16 * i;
            load16(a.ad + (size_t)rec * a.ad_stride + 16 * i, rem >= 16 ? 16u : rem, x);
        } else {
            const uint64_t ab = (uint64_t)ad_len * 8, cb = (uint64_t)len * 8;
            x[0] = __builtin_bswap32((uint32_t)(ab >> 32)); x[1] = __builtin_bswap32((uint32_t)ab);
            x[2] = __builtin_bswap32((uint32_t)(cb >> 32)); x[3] = __builtin_bswap32((uint32_t)cb);
        }
        if constexpr (CT) gh_to_nat(x);
        acc[0] ^= x[0]; acc[1] ^= x[1]; acc[2] ^= x[2]; acc[3] ^= x[3];
    }
    /* scale by H^(K-l) from the context's tables (once per lane) */
    gh_scale<CT>(acc, ctx, K - 1 - l);
#pragma unroll
    for (int off = 1; off < K; off <<= 1)
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[w] ^= (uint32_t)__shfl_xor((int)acc[w], off, 64);
    if constexpr (CT) gh_to_nat(acc);
    uint32_t ej[4];
    aes_ctr_pre(TE, rk, tpl, pre, 1u, ej);
    const uint32_t tag[4] = {acc[0] ^ ej[0], acc[1] ^ ej[1], acc[2] ^ ej[2], acc[3] ^ ej[3]};
    if (!OPEN) {
        if (l == K - 1) {
            if ((len & 15) == 0) *(uint4 *)(dst + len) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
            else if ((len & 7) == 0) {
                *(uint2 *)(dst + len) = make_uint2(tag[0], tag[1]);
                *(uint2 *)(dst + len + 8) = make_uint2(tag[2], tag[3]);
            } else store16(dst + len, 16, tag);
        }
        return;
    }
    uint32_t got[4];
    load16(src + len, 16, got);
    const bool ok = ((tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3])) == 0;
    if (l == K - 1 && a.status) a.status[rec] = ok ? 0 : 1;
    if (a.vf) { /* verified: decrypt now; rejected: nothing was written */
        if (ok) gcm_ctr_lane(TE, rk, tpl, pre, src, dst, len, (c0 + K - (A % K)) % K, M, K);
        return;
    }
    if (ok) return;
    /* MAC failure (taken only for a forged or damaged record): the reference
       verifies before decrypting and leaves the buffer untouched
       (cipher-aesgcm.c:184-186).  In place, XOR the lane's blocks with their
       key stream once more — the ciphertext as given comes back; out of place,
       zero the plaintext written (scrub_rejected's contract). */
    if (dst != src) {
        scrub_rejected(dst, src, len, (uint32_t)l, K);
        return;
    }
    for (uint32_t d = (c0 + K - (A % K)) % K; d < M; d += K) {
        const uint4 v = *(const uint4 *)(dst + 16 * d);
        uint32_t x[4] = {v.x, v.y, v.z, v.w}, ks[4];
        aes_ctr_pre(TE, rk, tpl, pre, 2 + d, ks);
#pragma unroll
        for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
        const uint32_t nb = min(len - 16 * d, 16u);
        if (nb == 16) *(uint4 *)(dst + 16 * d) = make_uint4(x[0], x[1], x[2], x[3]);
        else store16(dst + 16 * d, nb, x);
    }
}

/* One 1024-thread workgroup of a uniform staged job. */
template <bool OPEN, bool CT>
NA_DEV void gcm_staged_wg(const UniformArgs &a, GcmLds &L, uint32_t blk)
{
    const uint32_t st = blk * (uint32_t)GCM_WG_RECS / a.rps;
    gcm_lds_fill(L, (const AesCtx *)a.keys + st);
    gcm_staged_rec<OPEN, CT>(a, (const uint8_t *)&L.te[0][0][0], L.h4, L.rk, blk);
}

template <bool OPEN, bool CT>
__global__ __launch_bounds__(GCM_WG) void gcm_staged(UniformArgs a)
{
    __shared__ GcmLds L;
    gcm_staged_wg<OPEN, CT>(a, L, blockIdx.x);
}

/* Duplex: one launch sealing uniform job s and opening job o (the
   ChaChaPoly duplex of chachapoly.hip), workgroups alternating between the
   two while both have some left.  A uniform C3-sized job is 256 workgroups,
   one per CU, each holding its CU until its slowest wave ends; in one launch
   the second job's workgroups fill the CUs the first job's leave. */
template <bool CT>
__global__ __launch_bounds__(GCM_WG) void gcm_duplex_staged(UniformArgs s, UniformArgs o,
                                                             uint32_t s_blocks, uint32_t o_blocks)
{
    __shared__ GcmLds L;
    const uint32_t n = min(s_blocks, o_blocks);
    uint32_t b = blockIdx.x;
    bool open;
    if (b < 2 * n) {
        open = b & 1;
        b >>= 1;
    } else {
        open = o_blocks > s_blocks;
        b -= n;
    }
    if (open) gcm_staged_wg<true, CT>(o, L, b);
    else gcm_staged_wg<false, CT>(s, L, b);
}

/* Fused duplex: workgroup b seals block b of job s, then opens block b of
   job o, on ONE fill of the LDS T-tables (a second slot holds the open
   job's state: H^4 table and round keys).  Each wave goes on to its open
   record as soon as its seal record is done, so a CU's SIMDs stay busy
   through the first half's uneven finish and the workgroup drains once, not
   twice.  Results are those of the separate kernels (same per-record code). */
/* Round keys through the scalar cache.  Where a wave's records share one
   state its 60 round-key words are wave-uniform: read with s_load from the
   context in global memory they cost no LDS cycle, where the LDS copy costs
   15 ds_read_b128 per block (≈10 % of the kernel's LDS cycles).  The
   compiler reloads them per block (48 of 60 words: six s_load_dwordx8) and
   a scalar load's wait is lgkmcnt(0), which also drains the LDS lookups in
   flight: measured (profiles/r05/rk_scalar_ab.txt) the ragged seal gains
   3.5 % (0.787 -> 0.760 ms at C5), the verify-first ragged open loses 14 %
   and C3's fused duplex 1.5 %, so only the ragged seal takes it. */
typedef const __attribute__((address_space(4))) uint32_t *RkS;

/* the wave-uniform address p as a constant-address-space pointer */
NA_DEV RkS rk_scalar(const uint32_t *p)
{
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return (RkS)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

struct GcmLds2 {
    uint32_t te[2][256][64];
    uint4 h4[2][GHASH_TAB_ENTRIES];
    uint32_t rk[2][60];
};

NA_DEV void gcm_key_fill(uint4 *h4, uint32_t *rk, const AesCtx *ctx)
{
    const uint4 *src = (const uint4 *)ctx->tab[GCM_LANES - 1];
    for (int i = threadIdx.x; i < GHASH_TAB_ENTRIES; i += GCM_WG) h4[i] = src[i];
    if (threadIdx.x < 60) rk[threadIdx.x] = ctx->rk[threadIdx.x];
}

template <bool CT>
__global__ __launch_bounds__(GCM_WG) void gcm_duplex_fused(UniformArgs s, UniformArgs o,
                                                            uint32_t s_blocks, uint32_t o_blocks)
{
    __shared__ GcmLds2 L;
    const uint32_t b = blockIdx.x;
    const int t = threadIdx.x;
    for (int q = t; q < 2 * 256 * 16; q += GCM_WG) {
        const int reg = q >> 12, row = (q >> 4) & 255, quad = q & 15;
        const int tab = 2 * reg + (quad >> 3);
        const uint32_t v = rotr(g_te0[row], 8 * tab);
        ((uint4 *)&L.te[reg][row][0])[quad] = make_uint4(v, v, v, v);
    }
    if (b < s_blocks) gcm_key_fill(L.h4[0], L.rk[0], (const AesCtx *)s.keys + b * (uint32_t)GCM_WG_RECS / s.rps);
    if (b < o_blocks) gcm_key_fill(L.h4[1], L.rk[1], (const AesCtx *)o.keys + b * (uint32_t)GCM_WG_RECS / o.rps);
    __syncthreads();
    const uint8_t *TE = (const uint8_t *)&L.te[0][0][0];
    if (b < s_blocks) gcm_staged_rec<false, CT>(s, TE, L.h4[0], L.rk[0], b);
    if (b < o_blocks) gcm_staged_rec<true, CT>(o, TE, L.h4[1], L.rk[1], b);
}


/* ------------------------------ staged ragged (any mix of states / lengths)
 *
 * 1024-thread workgroups over windows of 256 descriptors, with the same
 * replicated LDS T-tables as gcm_staged.  A ragged window may mix states, so
 * the GHASH Horner table and the round keys of up to two states are staged
 * in LDS slots (the states of the window's first and last records: a window
 * that spans a run boundary of per-state records holds exactly these two);
 * a record of any other state reads its own context from global memory.
 * Records are taken in length order inside the window (window_rec) so the
 * 16 records of a wave have near-equal lengths.
 */
template <int NREC>
struct GcmLdsR {
    uint32_t te[2][256][64];
    uint4 h4[2][GHASH_TAB_ENTRIES];
    uint32_t rk[2][60];
    uint32_t order[NREC];
};

/* One record, 4 lanes (l = 0..3): gcm_staged's GHASH/CTR core with the
   record's tables passed in; FAST as in chachapoly.hip (16-B aligned record,
   input readable to roundup16). */
template <bool OPEN, bool FAST, bool CT, int KL = GCM_LANES, typename RK = const uint32_t *>
NA_DEV bool gcm_record_staged(const GcmView &rv, int l, const uint8_t *TE, uint32_t tpl,
                              RK rk, const uint4 *h4, bool vf)
{
    /* KL lanes per record (4, or 8 with the H^8 Horner table): the Horner
       step is H^KL, h4 its multiply table */
    constexpr int K = KL;
    static_assert(K == 4 || K == 8, "lanes per AES-GCM record");
    uint32_t h4n[4] = {0, 0, 0, 0};
    if constexpr (CT) {
#pragma unroll
        for (int w = 0; w < 4; ++w) h4n[w] = K == 8 ? rv.ctx->hn8[w] : rv.ctx->hn[K - 1][w];
    }
    const uint32_t n_hi = (uint32_t)(rv.nonce >> 32), n_lo = (uint32_t)rv.nonce;
    const uint32_t len = rv.len, ad_len = rv.ad_len;
    const uint32_t A = (ad_len + 15) / 16, M = (len + 15) / 16;
    const uint32_t n = A + M + 1;
    const uint32_t c0 = ((uint32_t)l + n) % K;
    uint32_t acc[4] = {0, 0, 0, 0};
    const AesPre pre = aes_pre_lds(TE, rk, tpl, n_hi, n_lo);
#pragma unroll 1
    for (uint32_t i = c0; i < n; i += K) {
        if (i != c0) gh_step<CT>(acc, h4, h4n);
        uint32_t x[4];
        if (i >= A && i < A + M) {
            const uint32_t d = i - A;
            const uint32_t nb = min(len - 16 * d, 16u);
            if (FAST) {
                const uint4 v = *(const uint4 *)(rv.src + 16 * d);
                x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
            } else {
                load16(rv.src + 16 * d, nb, x);
            }
            /* one pass for both directions (gcm_staged): open decrypts as it
               authenticates and repairs on a MAC failure; VERIFY_FIRST opens
               decrypt after the verdict */
            if (!OPEN || !vf) {
                uint32_t ks[4], y[4];
                aes_ctr_pre(TE, rk, tpl, pre, 2 + d, ks);
#pragma unroll
                for (int w = 0; w < 4; ++w) y[w] = x[w] ^ ks[w];
                if (FAST && nb == 16) *(uint4 *)(rv.dst + 16 * d) = make_uint4(y[0], y[1], y[2], y[3]);
                else store16(rv.dst + 16 * d, nb, y);
                if (!OPEN) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) x[w] = y[w];
                }
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) x[w] &= blk_mask(nb, w);
        } else if (i < A) {
            const uint32_t rem = ad_len - 16 * i;
            load16(rv.ad + 16 * i, rem >= 16 ? 16u : rem, x);
        } else {
            const uint64_t ab = (uint64_t)ad_len * 8, cb = (uint64_t)len * 8;
            x[0] = __builtin_bswap32((uint32_t)(ab >> 32)); x[1] = __builtin_bswap32((uint32_t)ab);
            x[2] = __builtin_bswap32((uint32_t)(cb >> 32)); x[3] = __builtin_bswap32((uint32_t)cb);
        }
        if constexpr (CT) gh_to_nat(x);
        acc[0] ^= x[0]; acc[1] ^= x[1]; acc[2] ^= x[2]; acc[3] ^= x[3];
    }
    gh_scale<CT, K>(acc, rv.ctx, K - 1 - l);
#pragma unroll
    for (int off = 1; off < K; off <<= 1)
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[w] ^= (uint32_t)__shfl_xor((int)acc[w], off, 64);
    if constexpr (CT) gh_to_nat(acc);
    uint32_t ej[4];
    aes_ctr_pre(TE, rk, tpl, pre, 1u, ej);
    const uint32_t tag[4] = {acc[0] ^ ej[0], acc[1] ^ ej[1], acc[2] ^ ej[2], acc[3] ^ ej[3]};
    if (!OPEN) {
        if (l == K - 1) store16(rv.dst + len, 16, tag);
        return true;
    }
    uint32_t got[4];
    load16(rv.src + len, 16, got);
    const bool ok = ((tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3])) == 0;
    if (vf) {
        if (ok) gcm_ctr_lane<FAST>(TE, rk, tpl, pre, rv.src, rv.dst, len, (c0 + K - (A % K)) % K, M, K);
        return ok;
    }
    if (ok) return true;
    /* MAC failure: in place, the lane's blocks XORed with their key stream
       once more give back the ciphertext as given (the reference leaves the
       buffer untouched, cipher-aesgcm.c:184-186); out of place the caller's
       scrub_rejected zeroes the plaintext written */
    if (rv.dst == rv.src) {
        for (uint32_t d = (c0 + K - (A % K)) % K; d < M; d += K) {
            const uint32_t nb = min(len - 16 * d, 16u);
            uint32_t x[4], ks[4];
            if (FAST) {
                const uint4 v = *(const uint4 *)(rv.dst + 16 * d);
                x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
            } else {
                load16(rv.dst + 16 * d, nb, x);
            }
            aes_ctr_pre(TE, rk, tpl, pre, 2 + d, ks);
#pragma unroll
            for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
            if (FAST && nb == 16) *(uint4 *)(rv.dst + 16 * d) = make_uint4(x[0], x[1], x[2], x[3]);
            else store16(rv.dst + 16 * d, nb, x);
        }
    }
    return false;
}

/* the cold path: a record whose state has no LDS slot.  Inlined: as an
   out-of-line call its frame and caller-saved registers cost the slot path
   scratch traffic (open 176 -> 104 B/lane, seal 64 -> 0) and C5's AES
   kernels 2-5 % (profiles/r01_aes_inline_ab.jsonl). */
template <int KL>
NA_DEV const uint4 *horner_tab(const AesCtx *ctx)
{
    return (const uint4 *)(KL == 8 ? ctx->tab8 : ctx->tab[GCM_LANES - 1]);
}

template <bool OPEN, bool FAST, bool CT, int KL>
__device__ __forceinline__ bool gcm_record_global(const GcmView &rv, int l,
                                                  const uint8_t *TE, uint32_t tpl, bool vf)
{
    return gcm_record_staged<OPEN, FAST, CT, KL>(rv, l, TE, tpl, rv.ctx->rk, horner_tab<KL>(rv.ctx),
                                                 vf);
}

/* WG threads per workgroup (1024, or 256 for batches too small to give
   every CU a 1024-thread workgroup); WG / KL record groups of KL lanes (4,
   or 8 with the H^8 Horner table), each running R records of the window's
   R * WG / KL one after another (snake_rank).  The T-tables hold the CU's
   LDS, so a workgroup owns its CU until its longest wave ends: with R = 1 a
   window of mixed lengths leaves most waves idle while the one holding the
   longest records finishes; R = 2 pairs long with short records so every
   wave carries about the window's mean (KL = 8 keeps that at 256 records
   per window). */
template <bool OPEN, bool FAST, int WG, bool CT, int R = 1, int KL = GCM_LANES>
__global__ __launch_bounds__(WG) void gcm_ragged_staged(RaggedArgs a)
{
    constexpr int K = KL, NG = WG / KL, NREC = NG * R;
    __shared__ GcmLdsR<NREC> L;
    const uint8_t *TE = (const uint8_t *)&L.te[0][0][0];
    const uint32_t base = blockIdx.x * (uint32_t)NREC;
    const uint32_t last = min(base + (uint32_t)NREC, a.n_records) - 1;
    const uint64_t slot_off[2] = {a.recs[base].ctx_off, a.recs[last].ctx_off};
    /* T-tables (as gcm_lds_fill) and the two slots' tables */
    for (int q = threadIdx.x; q < 2 * 256 * 16; q += WG) {
        const int reg = q >> 12, row = (q >> 4) & 255, quad = q & 15;
        const int tab = 2 * reg + (quad >> 3);
        const uint32_t v = rotr(g_te0[row], 8 * tab);
        ((uint4 *)&L.te[reg][row][0])[quad] = make_uint4(v, v, v, v);
    }
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
        const AesCtx *ctx = (const AesCtx *)(a.keys + slot_off[sl]);
        const uint4 *src = horner_tab<KL>(ctx);
        if (!CT)
            for (int i = threadIdx.x; i < GHASH_TAB_ENTRIES; i += WG) L.h4[sl][i] = src[i];
        if (threadIdx.x < 60) L.rk[sl][threadIdx.x] = ctx->rk[threadIdx.x];
    }
    const uint32_t g = threadIdx.x / K;
    if constexpr (R > 1) { /* sort the whole window; groups take ranks by snake_rank */
        window_rec<NREC>(a.recs, a.n_records, base, 0, L.order);
    }
    const int l = (int)(threadIdx.x % K);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t tpl = (1u << 16) | ((128u + 4u * (lane & 31)) << 8) | (4u * (lane & 31));
#pragma unroll 1
    for (int p = 0; p < R; ++p) {
        uint32_t rec;
        if constexpr (R == 1) {
            rec = window_rec<NREC>(a.recs, a.n_records, base, g, L.order);
        } else {
            const uint32_t key = L.order[snake_rank<NG>(g, p)];
            rec = key != 0xFFFFFFFFu ? base + (key & (NREC <= 256 ? 0xFFu : 0x1FFu)) : 0xFFFFFFFFu;
        }
        if (rec >= a.n_records) continue;
        const RecDesc d = a.recs[rec];
        if (reject_len(a, rec, d.len, l == K - 1)) continue;
        GcmView rv;
        rv.src = a.in + d.in_off;
        rv.dst = a.out + d.out_off;
        rv.ad = a.ad ? a.ad + d.ad_off : nullptr;
        rv.ctx = (const AesCtx *)(a.keys + d.ctx_off);
        rv.nonce = d.nonce;
        rv.len = d.len;
        rv.ad_len = d.ad_len;
        bool ok = false; /* every path below sets it */
        const int sl = d.ctx_off == slot_off[0] ? 0 : (d.ctx_off == slot_off[1] ? 1 : -1);
        const bool vf = OPEN && a.vf;
        bool done = false;
        if constexpr (!OPEN) { /* seals only: measured slower in the opens and in C3's fused duplex */
            const int s0 = __builtin_amdgcn_readfirstlane(sl);
            if (s0 >= 0 && __all(sl == s0)) { /* the wave's records share an LDS slot */
                ok = gcm_record_staged<OPEN, FAST, CT, KL>(
                    rv, l, TE, tpl, rk_scalar(((const AesCtx *)(a.keys + slot_off[s0]))->rk), L.h4[s0], vf);
                done = true;
            }
        }
        if (done) {
        } else if (sl >= 0)
            ok = gcm_record_staged<OPEN, FAST, CT, KL>(rv, l, TE, tpl, L.rk[sl], L.h4[sl], vf);
        else /* a third state in the window: its own context, from global memory */
            ok = gcm_record_global<OPEN, FAST, CT, KL>(rv, l, TE, tpl, vf);
        if (l == K - 1 && a.status) a.status[rec] = ok ? 0 : 1;
        if (!ok && !vf) scrub_rejected(rv.dst, rv.src, rv.len, (uint32_t)l, K);
    }
}

/* GHASH input block i of a record: AD blocks, CT blocks (zero-padded), the
   lengths block BE64(8|AD|) || BE64(8|CT|) (cipher-aesgcm.c:135-154) */
NA_DEV void gh_input_block(const uint8_t *ad, uint32_t ad_len, const uint8_t *ct, uint32_t len, uint32_t A,
                           uint32_t M, uint32_t i, uint32_t x[4])
{
    if (i < A) {
        const uint32_t rem = ad_len - 16 * i;
        load16(ad + 16 * i, rem >= 16 ? 16u : rem, x);
    } else if (i < A + M) {
        const uint32_t b = i - A, rem = len - 16 * b;
        load16(ct + 16 * b, rem >= 16 ? 16u : rem, x);
    } else {
        const uint64_t ab = (uint64_t)ad_len * 8, cb = (uint64_t)len * 8;
        x[0] = __builtin_bswap32((uint32_t)(ab >> 32)); x[1] = __builtin_bswap32((uint32_t)ab);
        x[2] = __builtin_bswap32((uint32_t)(cb >> 32)); x[3] = __builtin_bswap32((uint32_t)cb);
    }
}

/* ------------------------------------ row-collaborative GHASH multiply
 *
 * A 16-lane DPP row multiplies one GHASH value by a table T, each lane
 * holding ONE byte of the value: lane p looks up the two nibble positions of
 * byte p (2p: high nibble, 2p+1: low) in the 4-bit positional table T, and
 * the 16 partial products (128 bits each) are reduce-scattered so that lane
 * p ends with byte p of the product — exactly what its next lookups index.
 * Partners: p ^ 8 (row_ror 8: words 0-1 vs 2-3), 7 - p within the half
 * (row_half_mirror: differs in bit 2, keeps the word), p ^ 2 and p ^ 1
 * (quad_perm: the 16-bit half, the byte); the four partner sets together
 * cover all 16 lanes.  Two lookups, 5 DPP moves and ~20 VALU per multiply
 * instead of one lane's 32 lookups: the latency form of gh_mul_lds for the
 * single records of gcm_wide_record (the resident worker's AES-GCM calls). */
template <int CTRL>
NA_DEV uint32_t dpp_mov(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

NA_DEV uint32_t gh_mul_row_byte(uint32_t yb, const uint4 *tab, uint32_t p)
{
    const uint4 e = tab[(2 * p) * 16 + (yb >> 4)];
    const uint4 f = tab[(2 * p + 1) * 16 + (yb & 15u)];
    const bool hi = p & 8, b2 = p & 4;
    /* lanes p < 8 keep words 0-1, p >= 8 words 2-3; each sends the partner's */
    const uint32_t k0 = hi ? e.z ^ f.z : e.x ^ f.x, k1 = hi ? e.w ^ f.w : e.y ^ f.y;
    const uint32_t s0 = hi ? e.x ^ f.x : e.z ^ f.z, s1 = hi ? e.y ^ f.y : e.w ^ f.w;
    const uint32_t a0 = k0 ^ dpp_mov<0x128>(s0), a1 = k1 ^ dpp_mov<0x128>(s1); /* row_ror 8 */
    const uint32_t w = (b2 ? a1 : a0) ^ dpp_mov<0x141>(b2 ? a0 : a1);          /* row_half_mirror */
    const uint32_t v = w ^ dpp_mov<0x4E>(w);                                   /* quad_perm [2,3,0,1] */
    const uint32_t h = (p & 2) ? v >> 16 : v & 0xffffu;
    const uint32_t u = h ^ dpp_mov<0xB1>(h);                                   /* quad_perm [1,0,3,2] */
    return (p & 1) ? (u >> 8) & 255u : u & 255u;
}

/* byte p of GHASH input block i (gh_input_block's bytes, memory order) */
NA_DEV uint32_t gh_input_byte(const uint8_t *ad, uint32_t ad_len, const uint8_t *ct, uint32_t len, uint32_t A,
                              uint32_t M, uint32_t i, uint32_t p)
{
    if (i < A) return 16 * i + p < ad_len ? ad[16 * i + p] : 0u;
    if (i < A + M) {
        const uint32_t o = 16 * (i - A) + p;
        return o < len ? ct[o] : 0u;
    }
    const uint64_t bits = p < 8 ? (uint64_t)ad_len * 8 : (uint64_t)len * 8;
    return (uint32_t)(bits >> (8 * (7 - (p & 7)))) & 255u;
}

/* ------------------------------------------ wide (small batches, latency)
 *
 * One record per 256-thread workgroup, for batches of at most 512 records
 * (the single-call path of noise_cipherstate_*, short wire buffers), and the
 * resident worker's AES-GCM records.  Latency first: counter block v + 1 is
 * "virtual block" v, v = 0 being E_K(J0) (the tag mask, cipher-aesgcm.c:
 * 99-125) and v >= 1 data block v - 1, so E_K(J0) comes out of the same
 * SIMT pass as the CTR blocks instead of after GHASH.  GHASH is gcm_record's
 * K-lane Horner (H^K steps, scale by H^(K-l), XOR-reduce; K = 8 with the
 * H^8 table) run by lanes 0..K-1 of wave 0, the table in LDS.
 *   Seal: CTR (and E_K(J0)), then GHASH over the CT just written.
 *   Open: the waves GHASH leaves free compute E_K(J0) and the first key
 *   stream blocks meanwhile; the tag is checked first and the keystream
 *   applied only when it verified (cipher-aesgcm.c:184-186): no plaintext
 *   byte of a rejected record is ever written.
 * GHASH (table form, round 4): chain l of the K Horner chains runs on DPP
 * row l (16 lanes, one byte of the value each, gh_mul_row_byte), so a
 * Horner step is two lookups per lane and a 5-move reduce-scatter instead
 * of 32 lookups on one lane; waves 0-1 hold the 8 rows, waves 2-3 run the
 * open's early key stream.  The CT form keeps
 * one lane per chain (gh_mul_ct has no table to spread).
 */
/* One record on a 256-thread workgroup (the whole workgroup calls it):
   te/sb/hk are the LDS tables (hk: the record's H^K multiply table when not
   CT), wl five LDS words (verdict, E_K(J0)).  Returns (open) whether the tag
   verified; writes status when given; a rejected record's output is left
   alone here (the caller scrubs).  Shared by gcm_wide and the resident
   worker (worker.hip); dbg, when given, takes thread 0's s_memtime stamps. */
template <bool OPEN, bool CT, int K = 8>
NA_DEV bool gcm_wide_record(const uint8_t *src, uint8_t *dst, const uint8_t *ad, uint32_t ad_len,
                            uint32_t len, uint64_t nonce, const AesCtx *ctx, const uint32_t *te,
                            const uint32_t *sb, const uint4 *hk, uint32_t *wl, uint8_t *status,
                            uint32_t *dbg = nullptr)
{
    static_assert(K == 4 || K == 8, "GHASH lanes: 4 (H^4) or 8 (H^8)");
#define NA_GSTAMP(k) do { if (dbg && threadIdx.x == 0) dbg[k] = (uint32_t)__builtin_amdgcn_s_memtime(); } while (0)
    /* threads running GHASH: K lanes (CT) or K rows of 16 (tables); the
       others compute the open's first EARLY virtual blocks meanwhile */
    constexpr uint32_t GH = CT ? 64u : 16u * K;
    constexpr uint32_t EARLY = 256u - GH;
    const uint32_t t = threadIdx.x, M = (len + 15) / 16;
    const uint32_t *rk = ctx->rk;
    uint32_t ks[4] = {0, 0, 0, 0};
    bool early = false;
    if (!OPEN) {
        for (uint32_t v = t; v <= M; v += 256) {
            aes_ctr_block(rk, te, sb, nonce, v + 1, ks);
            if (v == 0) {
                wl[1] = ks[0]; wl[2] = ks[1]; wl[3] = ks[2]; wl[4] = ks[3];
            } else {
                const uint32_t b = v - 1, nb = len - 16 * b >= 16 ? 16u : len - 16 * b;
                uint32_t x[4];
                load16(src + 16 * b, nb, x);
#pragma unroll
                for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
                store16(dst + 16 * b, nb, x);
            }
        }
    } else if (t >= GH) {
        const uint32_t v = t - GH;
        early = v <= M && v < EARLY;
        if (dbg && t == GH) dbg[6] = (uint32_t)__builtin_amdgcn_s_memtime();
        if (early) aes_ctr_block(rk, te, sb, nonce, v + 1, ks);
        if (dbg && t == GH) dbg[7] = (uint32_t)__builtin_amdgcn_s_memtime();
        if (v == 0) { wl[1] = ks[0]; wl[2] = ks[1]; wl[3] = ks[2]; wl[4] = ks[3]; }
    }
    if (!OPEN) __syncthreads(); /* the GHASH lanes read this CT back (same CU) */
    NA_GSTAMP(0);
    uint32_t acc[4] = {0, 0, 0, 0};
    const uint8_t *ct = OPEN ? src : dst;
    const uint32_t A = (ad_len + 15) / 16, n = A + M + 1;
    if constexpr (CT) {
        if (t < (uint32_t)K) {
            const int l = (int)t;
            const uint32_t c0 = ((uint32_t)l + n) % K;
            uint32_t hkn[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) hkn[w] = K == 8 ? ctx->hn8[w] : ctx->hn[K - 1][w];
            for (uint32_t i = c0; i < n; i += K) {
                if (i != c0) gh_mul_ct(acc, hkn);
                uint32_t x[4];
                gh_input_block(ad, ad_len, ct, len, A, M, i, x);
                gh_to_nat(x);
                acc[0] ^= x[0]; acc[1] ^= x[1]; acc[2] ^= x[2]; acc[3] ^= x[3];
            }
            NA_GSTAMP(1);
            gh_scale<true, K>(acc, ctx, K - 1 - l);
#pragma unroll
            for (int off = 1; off < K; off <<= 1)
#pragma unroll
                for (int w = 0; w < 4; ++w) acc[w] ^= (uint32_t)__shfl_xor((int)acc[w], off, 64);
            gh_to_nat(acc);
            NA_GSTAMP(2);
        }
    } else {
        if (t < GH) {
            const uint32_t l = t >> 4, p = t & 15; /* chain l on row l, byte p on lane p */
            const uint32_t c0 = (l + n) % K;
            uint32_t yb = 0;
            for (uint32_t i = c0; i < n; i += K) {
                const uint32_t xb = gh_input_byte(ad, ad_len, ct, len, A, M, i, p);
                if (i != c0) yb = gh_mul_row_byte(yb, hk, p);
                yb ^= xb;
            }
            NA_GSTAMP(1);
            /* scale by H^(K - l): H^K itself (hk), else H^4 first when
               K - l > 4, then H^(m+1) */
            uint32_t m = K - 1 - l;
            if (m == (uint32_t)K - 1) {
                yb = gh_mul_row_byte(yb, hk, p);
            } else {
                if (m >= (uint32_t)GCM_LANES) {
                    yb = gh_mul_row_byte(yb, (const uint4 *)ctx->tab[GCM_LANES - 1], p);
                    m -= GCM_LANES;
                }
                yb = gh_mul_row_byte(yb, (const uint4 *)ctx->tab[m], p);
            }
            ((uint8_t *)(wl + 8 + 4 * l))[p] = (uint8_t)yb;
        }
        __syncthreads();
        if (t == 0 || t == (uint32_t)K - 1) { /* the rows' sum: open checks on thread 0, seal stores on K-1 */
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t v = 0;
#pragma unroll
                for (int l = 0; l < K; ++l) v ^= wl[8 + 4 * l + w];
                acc[w] = v;
            }
        }
        NA_GSTAMP(2);
    }
    if (OPEN) __syncthreads(); /* E_K(J0) from the early waves */
    NA_GSTAMP(3);
    if (!OPEN) {
        if (t == (uint32_t)K - 1) {
            const uint32_t tag[4] = {acc[0] ^ wl[1], acc[1] ^ wl[2], acc[2] ^ wl[3], acc[3] ^ wl[4]};
            store16(dst + len, 16, tag);
            if (status) *status = 0;
        }
        return true;
    }
    if (t == 0) {
        uint32_t got[4];
        load16(src + len, 16, got);
        const bool ok = ((acc[0] ^ wl[1] ^ got[0]) | (acc[1] ^ wl[2] ^ got[1]) | (acc[2] ^ wl[3] ^ got[2]) |
                         (acc[3] ^ wl[4] ^ got[3])) == 0;
        wl[0] = ok;
        if (status) *status = ok ? 0 : 1;
    }
    __syncthreads();
    NA_GSTAMP(4);
    if (!wl[0]) return false; /* nothing decrypted */
    if (early && t > GH) { /* keystream block t - GH - 1, computed beside GHASH */
        const uint32_t b = t - GH - 1, nb = len - 16 * b >= 16 ? 16u : len - 16 * b;
        uint32_t x[4];
        load16(src + 16 * b, nb, x);
#pragma unroll
        for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
        store16(dst + 16 * b, nb, x);
    }
    for (uint32_t b = EARLY - 1 + t; b < M; b += 256) {
        const uint32_t nb = len - 16 * b >= 16 ? 16u : len - 16 * b;
        uint32_t x[4];
        load16(src + 16 * b, nb, x);
        aes_ctr_block(rk, te, sb, nonce, 2 + b, ks);
#pragma unroll
        for (int w = 0; w < 4; ++w) x[w] ^= ks[w];
        store16(dst + 16 * b, nb, x);
    }
    NA_GSTAMP(5);
#undef NA_GSTAMP
    return true;
}

template <bool OPEN, bool CT>
__global__ __launch_bounds__(256) void gcm_wide(RaggedArgs a)
{
    __shared__ uint32_t te[256], sb[256];
    __shared__ uint4 h8[GHASH_TAB_ENTRIES];
    __shared__ uint32_t wl[40]; /* verdict, E_K(J0), the GHASH rows' sums */
    const uint32_t rec = blockIdx.x, t = threadIdx.x;
    const RecDesc d = a.recs[rec];
    if (reject_len(a, rec, d.len, t == 0)) return; /* uniform over the workgroup */
    const AesCtx *ctx = (const AesCtx *)(a.keys + d.ctx_off);
    const uint8_t *src = a.in + d.in_off;
    uint8_t *dst = a.out + d.out_off;
    for (uint32_t i = t; i < 256; i += 256) {
        te[i] = g_te0[i];
        sb[i] = g_sbox[i];
    }
    if (!CT)
        for (uint32_t i = t; i < (uint32_t)GHASH_TAB_ENTRIES; i += 256)
            h8[i] = ((const uint4 *)ctx->tab8)[i];
    __syncthreads();
    const bool ok = gcm_wide_record<OPEN, CT>(src, dst, a.ad + d.ad_off, d.ad_len, d.len, d.nonce, ctx,
                                              te, sb, h8, wl, a.status ? a.status + rec : nullptr);
    if (OPEN && !ok && !a.vf) scrub_rejected(dst, src, d.len, t, 256);
}

} // namespace na

