/*
 * noise_oracle.c — CPU restatement of noise-c's transport AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY (see noise_oracle.h).  Written from the published
 * algorithms (RFC 8439 ChaCha20/Poly1305, FIPS-197 AES, NIST SP 800-38D GCM)
 * following the reference's composition line by line; every function cites
 * the reference file:line it restates.  Deliberately simple and scalar: it is
 * the checker, never the thing measured or shipped.
 */
#include "noise_oracle.h"
#include <string.h>

/* ------------------------------------------------------------------ utils */

static uint32_t ld32le(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}
static uint64_t ld64le(const uint8_t *p)
{
    return (uint64_t)ld32le(p) | ((uint64_t)ld32le(p + 4) << 32);
}
static void st32le(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static void st64le(uint8_t *p, uint64_t v)
{
    st32le(p, (uint32_t)v); st32le(p + 4, (uint32_t)(v >> 32));
}
static void st64be(uint8_t *p, uint64_t v)
{
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (56 - 8 * i));
}
static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* constant-time compare, util.c:188-200 noise_is_equal */
static int ct_equal(const uint8_t *a, const uint8_t *b, size_t n)
{
    uint8_t d = 0;
    for (size_t i = 0; i < n; ++i) d |= (uint8_t)(a[i] ^ b[i]);
    return d == 0;
}

/* ---------------------------------------------------------------- ChaCha20
 * State layout of chacha.c:74-133: words 0-3 "expand 32-byte k", 4-11 key
 * (LE), 12-13 64-bit block counter, 14-15 64-bit IV.  20 rounds
 * (chacha.c:62-72 quarterRound, :149-204 encrypt loop). */
#define QR(a, b, c, d)                 \
    a += b; d ^= a; d = rotl32(d, 16); \
    c += d; b ^= c; b = rotl32(b, 12); \
    a += b; d ^= a; d = rotl32(d, 8);  \
    c += d; b ^= c; b = rotl32(b, 7)

void oracle_chacha20_block(const uint8_t key[32], uint64_t counter,
                           uint64_t iv, uint8_t out[64])
{
    uint32_t in[16], x[16];
    in[0] = 0x61707865; in[1] = 0x3320646e; in[2] = 0x79622d32; in[3] = 0x6b206574;
    for (int i = 0; i < 8; ++i) in[4 + i] = ld32le(key + 4 * i);
    in[12] = (uint32_t)counter; in[13] = (uint32_t)(counter >> 32);
    in[14] = (uint32_t)iv;      in[15] = (uint32_t)(iv >> 32);
    memcpy(x, in, sizeof(x));
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]);  QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);  QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) st32le(out + 4 * i, x[i] + in[i]);
}

/* ---------------------------------------------------------------- Poly1305
 * Radix-2^64 evaluation (h in three words) of the same polynomial that
 * poly1305-donna-64.h:101-151 evaluates with 44-bit limbs.  r is clamped as
 * in poly1305-donna-64.h:80-86; the final h + s mod 2^128 as in :154-223. */
typedef unsigned __int128 u128;

typedef struct {
    uint64_t r0, r1, h0, h1, h2, s0, s1;
    uint8_t buf[16];
    size_t fill;
} poly_t;

static void poly_init(poly_t *st, const uint8_t key[32])
{
    st->r0 = ld64le(key) & 0x0ffffffc0fffffffULL;
    st->r1 = ld64le(key + 8) & 0x0ffffffc0ffffffcULL;
    st->s0 = ld64le(key + 16);
    st->s1 = ld64le(key + 24);
    st->h0 = st->h1 = st->h2 = 0;
    st->fill = 0;
}

/* h = (h + m + hibit*2^128) * r mod 2^130-5, partially reduced. */
static void poly_block(poly_t *st, const uint8_t m[16], uint64_t hibit)
{
    u128 t;
    uint64_t h0, h1, h2, r0 = st->r0, r1 = st->r1;
    t = (u128)st->h0 + ld64le(m);
    h0 = (uint64_t)t;
    t = (u128)st->h1 + ld64le(m + 8) + (uint64_t)(t >> 64);
    h1 = (uint64_t)t;
    h2 = st->h2 + (uint64_t)(t >> 64) + hibit;
    /* h2 <= 7, so the products below fit in 128 bits. r1 is a multiple of
       4, so r1 * 2^128 = (r1/4) * 2^130 == 5*(r1/4) mod p. */
    uint64_t sr1 = r1 + (r1 >> 2); /* 5*r1/4 */
    u128 d0 = (u128)h0 * r0 + (u128)h1 * sr1;
    u128 d1 = (u128)h0 * r1 + (u128)h1 * r0 + (u128)h2 * sr1;
    uint64_t d2 = h2 * r0;
    /* fold: value = d0 + d1*2^64 + d2*2^128 */
    uint64_t c0 = (uint64_t)d0;
    d1 += (uint64_t)(d0 >> 64);
    uint64_t c1 = (uint64_t)d1;
    uint64_t c2 = d2 + (uint64_t)(d1 >> 64);
    /* reduce bits >= 130: c2 = top; keep low 2 bits, add 5 * (c2 >> 2) */
    uint64_t hi = c2 >> 2;
    c2 &= 3;
    t = (u128)c0 + hi * 5;
    h0 = (uint64_t)t;
    t = (u128)c1 + (uint64_t)(t >> 64);
    h1 = (uint64_t)t;
    h2 = c2 + (uint64_t)(t >> 64);
    st->h0 = h0; st->h1 = h1; st->h2 = h2;
}

/* poly1305_update semantics (poly1305-donna.c:26-61): buffer partial blocks */
static void poly_update(poly_t *st, const uint8_t *m, size_t len)
{
    while (len > 0) {
        size_t take = 16 - st->fill;
        if (take > len) take = len;
        memcpy(st->buf + st->fill, m, take);
        st->fill += take; m += take; len -= take;
        if (st->fill == 16) { poly_block(st, st->buf, 1); st->fill = 0; }
    }
}

static void poly_finish(poly_t *st, uint8_t tag[16])
{
    if (st->fill) { /* poly1305-donna-64.h:162-169: 0x01 then zeros, no hibit */
        st->buf[st->fill] = 1;
        memset(st->buf + st->fill + 1, 0, 16 - st->fill - 1);
        poly_block(st, st->buf, 0);
    }
    /* full reduction: compute h - p and select */
    uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2;
    /* carry h2 overflow bits (h2 < 8 here) */
    u128 t = (u128)h0 + 5;
    uint64_t g0 = (uint64_t)t;
    t = (u128)h1 + (uint64_t)(t >> 64);
    uint64_t g1 = (uint64_t)t;
    uint64_t g2 = h2 + (uint64_t)(t >> 64);
    if (g2 >> 2) { h0 = g0; h1 = g1; } /* h >= p: use h - p = h + 5 - 2^130 */
    t = (u128)h0 + st->s0;
    h0 = (uint64_t)t;
    h1 = h1 + st->s1 + (uint64_t)(t >> 64);
    st64le(tag, h0);
    st64le(tag + 8, h1);
}

void oracle_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len,
                     uint8_t tag[16])
{
    poly_t st;
    poly_init(&st, key);
    poly_update(&st, msg, len);
    poly_finish(&st, tag);
}

/* ----------------------------------------------------------------- AES-256
 * Byte-oriented FIPS-197 cipher.  Same function as the reference's T-table
 * rijndaelKeySetupEnc (rijndael-alg-fst.c:728-807, Nk = 8) and
 * rijndaelEncrypt (:854-1033, Nr = 14). */
static uint8_t g_sbox[256];
static int g_sbox_ready = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b)
{
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

static void sbox_init(void)
{
    if (g_sbox_ready) return;
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x) for (int y = 1; y < 256; ++y)
            if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv, v = inv;
        for (int i = 0; i < 4; ++i) { v = (uint8_t)((v << 1) | (v >> 7)); s ^= v; }
        g_sbox[x] = (uint8_t)(s ^ 0x63);
    }
    g_sbox_ready = 1;
}

static void aes256_expand(const uint8_t key[32], uint8_t rk[240])
{
    sbox_init();
    memcpy(rk, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            uint8_t u = t[0];
            t[0] = (uint8_t)(g_sbox[t[1]] ^ rcon); t[1] = g_sbox[t[2]];
            t[2] = g_sbox[t[3]]; t[3] = g_sbox[u];
            rcon = gf_mul(rcon, 2);
        } else if (i % 8 == 4) {
            for (int j = 0; j < 4; ++j) t[j] = g_sbox[t[j]];
        }
        for (int j = 0; j < 4; ++j) rk[4 * i + j] = (uint8_t)(rk[4 * (i - 8) + j] ^ t[j]);
    }
}

static void aes256_encrypt_rk(const uint8_t rk[240], const uint8_t in[16],
                              uint8_t out[16])
{
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int round = 1; round <= 14; ++round) {
        for (int i = 0; i < 16; ++i) s[i] = g_sbox[s[i]];
        /* ShiftRows: byte (row r, col c) at index 4c + r */
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) t[4 * c + r] = s[4 * ((c + r) % 4) + r];
        if (round != 14) {
            for (int c = 0; c < 4; ++c) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = (uint8_t)(gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3);
                s[4 * c + 1] = (uint8_t)(a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3);
                s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3));
                s[4 * c + 3] = (uint8_t)(gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2));
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

void oracle_aes256_encrypt_block(const uint8_t key[32], const uint8_t in[16],
                                 uint8_t out[16])
{
    uint8_t rk[240];
    aes256_expand(key, rk);
    aes256_encrypt_rk(rk, in, out);
}

/* ------------------------------------------------------------------ GHASH
 * SP 800-38D Algorithm 1, bit-serial, R = 0xE1 || 0^120 — the function
 * ghash.c:78-108 (GF128_mul) computes. */
void oracle_gf128_mul(const uint8_t x[16], const uint8_t h[16], uint8_t y[16])
{
    uint8_t z[16] = {0}, v[16];
    memcpy(v, h, 16);
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int j = 0; j < 16; ++j) z[j] ^= v[j];
        int lsb = v[15] & 1;
        for (int j = 15; j > 0; --j) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xE1;
    }
    memcpy(y, z, 16);
}

typedef struct { uint8_t h[16], y[16], buf[16]; size_t fill; } ghash_t;

static void gh_block(ghash_t *g, const uint8_t b[16])
{
    uint8_t t[16];
    for (int i = 0; i < 16; ++i) t[i] = (uint8_t)(g->y[i] ^ b[i]);
    oracle_gf128_mul(t, g->h, g->y);
}
/* ghash_update (ghash.c:188-206) and ghash_pad (ghash.c:216-224) */
static void gh_update(ghash_t *g, const uint8_t *m, size_t len)
{
    while (len > 0) {
        size_t take = 16 - g->fill;
        if (take > len) take = len;
        memcpy(g->buf + g->fill, m, take);
        g->fill += take; m += take; len -= take;
        if (g->fill == 16) { gh_block(g, g->buf); g->fill = 0; }
    }
}
static void gh_pad(ghash_t *g)
{
    if (g->fill) {
        memset(g->buf + g->fill, 0, 16 - g->fill);
        gh_block(g, g->buf);
        g->fill = 0;
    }
}

/* ------------------------------------------------------------------ AEADs */

/* cipher-chachapoly.c:62-73 setup, :81-105 pad/lengths, :107-143 enc/dec */
static void chachapoly_tag(const uint8_t key[32], uint64_t n,
                           const uint8_t *ad, size_t ad_len,
                           const uint8_t *ct, size_t len, uint8_t tag[16])
{
    static const uint8_t zeros[16] = {0};
    uint8_t block[64], lens[16];
    poly_t st;
    oracle_chacha20_block(key, 0, n, block); /* counter 0 -> Poly key */
    poly_init(&st, block);
    if (ad_len) {
        poly_update(&st, ad, ad_len);
        if (ad_len % 16) poly_update(&st, zeros, 16 - ad_len % 16);
    }
    poly_update(&st, ct, len);
    if (len % 16) poly_update(&st, zeros, 16 - len % 16);
    st64le(lens, (uint64_t)ad_len);
    st64le(lens + 8, (uint64_t)len);
    poly_update(&st, lens, 16);
    poly_finish(&st, tag);
}

static void chacha_xor(const uint8_t key[32], uint64_t n, uint8_t *data, size_t len)
{
    uint8_t ks[64];
    for (size_t off = 0, blk = 1; off < len; off += 64, ++blk) {
        oracle_chacha20_block(key, blk, n, ks); /* data counter starts at 1 */
        size_t take = len - off < 64 ? len - off : 64;
        for (size_t i = 0; i < take; ++i) data[off + i] ^= ks[i];
    }
}

/* cipher-aesgcm.c:38-50 init_key (H = E(0)), :70-90 setup_iv
   (J0 = 0^32 || BE64(n) || 0x00000001), :99-125 CTR from J0+1,
   :135-154 finalize (bit lengths, BE), :156-188 enc/dec. */
static void aesgcm_j0(uint64_t n, uint8_t j0[16])
{
    memset(j0, 0, 16);
    st64be(j0 + 4, n);
    j0[15] = 1;
}

static void aesgcm_tag(const uint8_t rk[240], uint64_t n,
                       const uint8_t *ad, size_t ad_len,
                       const uint8_t *ct, size_t len, uint8_t tag[16])
{
    ghash_t g;
    uint8_t zero[16] = {0}, j0[16], ej0[16], lens[16];
    memset(&g, 0, sizeof(g));
    aes256_encrypt_rk(rk, zero, g.h);
    aesgcm_j0(n, j0);
    aes256_encrypt_rk(rk, j0, ej0);
    if (ad_len) { gh_update(&g, ad, ad_len); gh_pad(&g); }
    gh_update(&g, ct, len);
    gh_pad(&g);
    st64be(lens, (uint64_t)ad_len * 8);
    st64be(lens + 8, (uint64_t)len * 8);
    gh_update(&g, lens, 16);
    for (int i = 0; i < 16; ++i) tag[i] = (uint8_t)(ej0[i] ^ g.y[i]);
}

static void aesgcm_ctr(const uint8_t rk[240], uint64_t n, uint8_t *data, size_t len)
{
    uint8_t ctr[16], ks[16];
    aesgcm_j0(n, ctr);
    uint32_t c = 1;
    for (size_t off = 0; off < len; off += 16) {
        ++c; /* the reference bumps only the low 16 bits (:105-112); equal
                for every legal length (<= 4097 blocks) */
        ctr[12] = (uint8_t)(c >> 24); ctr[13] = (uint8_t)(c >> 16);
        ctr[14] = (uint8_t)(c >> 8);  ctr[15] = (uint8_t)c;
        aes256_encrypt_rk(rk, ctr, ks);
        size_t take = len - off < 16 ? len - off : 16;
        for (size_t i = 0; i < take; ++i) data[off + i] ^= ks[i];
    }
}

int oracle_aead_encrypt(int cipher, const uint8_t key[32], uint64_t n,
                        const uint8_t *ad, size_t ad_len,
                        uint8_t *data, size_t len)
{
    if (cipher == ORACLE_CHACHAPOLY) {
        chacha_xor(key, n, data, len);
        chachapoly_tag(key, n, ad, ad_len, data, len, data + len);
        return 0;
    }
    if (cipher == ORACLE_AESGCM) {
        uint8_t rk[240];
        aes256_expand(key, rk);
        aesgcm_ctr(rk, n, data, len);
        aesgcm_tag(rk, n, ad, ad_len, data, len, data + len);
        return 0;
    }
    return -1;
}

int oracle_aead_decrypt(int cipher, const uint8_t key[32], uint64_t n,
                        const uint8_t *ad, size_t ad_len,
                        uint8_t *data, size_t len)
{
    uint8_t tag[16];
    if (cipher == ORACLE_CHACHAPOLY) {
        chachapoly_tag(key, n, ad, ad_len, data, len, tag);
        if (!ct_equal(tag, data + len, 16)) return ORACLE_MAC_FAILURE;
        chacha_xor(key, n, data, len);
        return 0;
    }
    if (cipher == ORACLE_AESGCM) {
        uint8_t rk[240];
        aes256_expand(key, rk);
        aesgcm_tag(rk, n, ad, ad_len, data, len, tag);
        if (!ct_equal(tag, data + len, 16)) return ORACLE_MAC_FAILURE;
        aesgcm_ctr(rk, n, data, len);
        return 0;
    }
    return -1;
}

/* ------------------------------------------------------------- batch glue */

void oracle_seal_uniform(int cipher, const uint8_t *keys,
                         const uint64_t *nonce_base, uint32_t recs_per_state,
                         const uint8_t *in, size_t in_stride,
                         uint8_t *out, size_t out_stride,
                         uint32_t len, uint32_t count)
{
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t s = i / recs_per_state;
        uint8_t *o = out + (size_t)i * out_stride;
        memmove(o, in + (size_t)i * in_stride, len);
        oracle_aead_encrypt(cipher, keys + 32 * (size_t)s,
                            nonce_base[s] + (i % recs_per_state), 0, 0, o, len);
    }
}

/* oracle_seal_uniform with associated data: record i's AD at ad + i * ad_stride */
void oracle_seal_uniform_ad(int cipher, const uint8_t *keys,
                            const uint64_t *nonce_base, uint32_t recs_per_state,
                            const uint8_t *in, size_t in_stride,
                            uint8_t *out, size_t out_stride,
                            uint32_t len, uint32_t count,
                            const uint8_t *ad, size_t ad_stride, uint32_t ad_len)
{
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t s = i / recs_per_state;
        uint8_t *o = out + (size_t)i * out_stride;
        memmove(o, in + (size_t)i * in_stride, len);
        oracle_aead_encrypt(cipher, keys + 32 * (size_t)s,
                            nonce_base[s] + (i % recs_per_state),
                            ad_len ? ad + (size_t)i * ad_stride : 0, ad_len, o, len);
    }
}

/* A ragged batch (the 48-byte NoiseAeadRecord descriptors of
   include/noise_aead_hip.h): record i sealed from in + in_off to
   out + out_off (ct || tag) with the key key_idx[i] of keys and its own
   nonce and AD; records longer than 65519 bytes are skipped, as the device
   kernels refuse them. */
void oracle_seal_ragged(int cipher, const uint8_t *keys, const uint32_t *key_idx,
                        const uint8_t *recs, uint32_t count,
                        const uint8_t *in, uint8_t *out, const uint8_t *ad)
{
    for (uint32_t i = 0; i < count; ++i) {
        const uint8_t *d = recs + 48 * (size_t)i;
        uint64_t in_off, out_off, nonce, ad_off;
        uint32_t len, ad_len;
        memcpy(&in_off, d, 8);
        memcpy(&out_off, d + 8, 8);
        memcpy(&nonce, d + 16, 8);
        memcpy(&ad_off, d + 32, 8);
        memcpy(&len, d + 40, 4);
        memcpy(&ad_len, d + 44, 4);
        if (len > 65535 - 16) continue;
        uint8_t *o = out + out_off;
        memmove(o, in + in_off, len);
        oracle_aead_encrypt(cipher, keys + 32 * (size_t)key_idx[i], nonce,
                            ad_len ? ad + ad_off : 0, ad_len, o, len);
    }
}

void oracle_open_uniform(int cipher, const uint8_t *keys,
                         const uint64_t *nonce_base, uint32_t recs_per_state,
                         const uint8_t *in, size_t in_stride,
                         uint8_t *out, size_t out_stride,
                         uint32_t len, uint32_t count, uint8_t *status)
{
    uint8_t tmp[65536 + 16];
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t s = i / recs_per_state;
        memcpy(tmp, in + (size_t)i * in_stride, (size_t)len + 16);
        int rc = oracle_aead_decrypt(cipher, keys + 32 * (size_t)s,
                                     nonce_base[s] + (i % recs_per_state), 0, 0,
                                     tmp, len);
        status[i] = rc ? 1 : 0;
        if (!rc) memcpy(out + (size_t)i * out_stride, tmp, len);
    }
}

/* SplitMix64 finalizer of x + golden gamma */
uint64_t oracle_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void oracle_fill_splitmix(uint64_t seed, uint64_t word0, uint8_t *out, size_t nbytes)
{
    size_t w = 0;
    for (; (w + 1) * 8 <= nbytes; ++w) st64le(out + 8 * w, oracle_splitmix64(seed + word0 + w));
    if (w * 8 < nbytes) {
        uint8_t tmp[8];
        st64le(tmp, oracle_splitmix64(seed + word0 + w));
        memcpy(out + 8 * w, tmp, nbytes - 8 * w);
    }
}

/* ---------------------------------------------------------------- RandState
 * randstate.c:230-375 restated over a snapshot (see noise_oracle.h). */
#define ORACLE_PADDING_ZERO 0x4701 /* constants.h:123 NOISE_PADDING_ZERO */

static void rand_block(const OracleRand *s, uint8_t out[64])
{
    uint8_t k[32];
    for (int i = 0; i < 8; ++i) st32le(k + 4 * i, s->key[i]);
    oracle_chacha20_block(k, s->counter, s->iv, out);
}

/* randstate.c:230-247: 40 key-stream bytes at the current position become
   the new key and IV, counter 0 */
static void rand_rekey(OracleRand *s)
{
    uint8_t b[64];
    rand_block(s, b);
    for (int i = 0; i < 8; ++i) s->key[i] = ld32le(b + 4 * i);
    s->iv = (uint64_t)ld32le(b + 32) | ((uint64_t)ld32le(b + 36) << 32);
    s->counter = 0;
    memset(b, 0, sizeof b);
}

int oracle_rand_pad(OracleRand *s, uint8_t *payload, size_t orig_len, size_t padded_len, int mode)
{
    if (!payload) return 0x450B;
    if (!s) {
        if (padded_len > orig_len) memset(payload + orig_len, 0, padded_len - orig_len);
        return 0x450B;
    }
    if (padded_len <= orig_len) return 0;
    const size_t len = padded_len - orig_len;
    uint8_t *out = payload + orig_len;
    if (mode == ORACLE_PADDING_ZERO) {
        memset(out, 0, len);
        return 0;
    }
    /* every 64-byte chunk, the partial last one too, spends 64 of `left` */
    const size_t chunks = (len + 63) / 64;
    if (s->left < len || s->left < 64 * chunks) return 0x450C;
    unsigned blocks = 0;
    for (size_t c = 0; c < chunks; ++c) {
        s->left -= 64;
        if (blocks++ >= 16) { /* NOISE_RAND_REKEY_COUNT */
            rand_rekey(s);
            blocks = 0;
        }
        uint8_t b[64];
        rand_block(s, b);
        ++s->counter;
        const size_t n = len - 64 * c < 64 ? len - 64 * c : 64;
        memcpy(out + 64 * c, b, n);
    }
    rand_rekey(s);
    return 0;
}
