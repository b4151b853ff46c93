/*
 * noise_oracle_hash.c — CPU restatement of noise-c's four hash functions and
 * its HMAC/HKDF (TEST INFRASTRUCTURE ONLY: the checker for the device key
 * fan-out of csrc/kdf.hip, never linked into the product).
 *
 *   SHA-256      FIPS 180-4; the reference's src/crypto/sha2/sha256.c
 *   SHA-512      FIPS 180-4; src/crypto/sha2/sha512.c
 *   BLAKE2s-256  RFC 7693, unkeyed; src/crypto/blake2/blake2s.c
 *   BLAKE2b-512  RFC 7693, unkeyed; src/crypto/blake2/blake2b.c
 *   HMAC         src/protocol/hashstate.c:407-448 (noise_hashstate_hmac:
 *                key hashed when longer than the block, zero-padded,
 *                ipad 0x36 / opad 0x5c)
 *   HKDF         src/protocol/hashstate.c:476-516 (noise_hashstate_hkdf:
 *                temp = HMAC(key, data); out1 = HMAC(temp, 0x01);
 *                out2 = HMAC(temp, out1 || 0x02); outputs truncated)
 *
 * Pinned by the FIPS/RFC example vectors and by golden HKDF vectors the
 * reference library produced (tests/golden/hkdf.json, gen_hkdf.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define H_BLAKE2S 0x4801 /* constants.h:43-46 */
#define H_BLAKE2B 0x4802
#define H_SHA256 0x4803
#define H_SHA512 0x4804

static uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static uint32_t ld32be(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
static uint64_t ld64be(const uint8_t *p) { return (uint64_t)ld32be(p) << 32 | ld32be(p + 4); }
static uint32_t ld32le(const uint8_t *p) { return (uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]; }
static uint64_t ld64le(const uint8_t *p) { return (uint64_t)ld32le(p + 4) << 32 | ld32le(p); }

/* ---------------------------------------------------------------- SHA-256 */

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static void sha256_block(uint32_t h[8], const uint8_t *p)
{
    uint32_t w[64], a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 16; ++i) w[i] = ld32be(p + 4 * i);
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = k + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

/* ---------------------------------------------------------------- SHA-512 */

static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static void sha512_block(uint64_t h[8], const uint8_t *p)
{
    uint64_t w[80], a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 16; ++i) w[i] = ld64be(p + 8 * i);
    for (int i = 16; i < 80; ++i) {
        uint64_t s0 = rotr64(w[i - 15], 1) ^ rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = rotr64(w[i - 2], 19) ^ rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    for (int i = 0; i < 80; ++i) {
        uint64_t t1 = k + (rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
        uint64_t t2 = (rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

/* ---------------------------------------------------------------- BLAKE2 */

static const uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
static const uint32_t IV32[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                                 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
static const uint64_t IV64[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

static void blake2s_compress(uint32_t h[8], const uint8_t *p, uint64_t t, int last)
{
    uint32_t m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = ld32le(p + 4 * i);
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = IV32[i]; }
    v[12] ^= (uint32_t)t; v[13] ^= (uint32_t)(t >> 32);
    if (last) v[14] = ~v[14];
#define G32(a, b, c, d, x, y)                                  \
    v[a] += v[b] + x; v[d] = rotr32(v[d] ^ v[a], 16);          \
    v[c] += v[d]; v[b] = rotr32(v[b] ^ v[c], 12);              \
    v[a] += v[b] + y; v[d] = rotr32(v[d] ^ v[a], 8);           \
    v[c] += v[d]; v[b] = rotr32(v[b] ^ v[c], 7)
    for (int r = 0; r < 10; ++r) {
        const uint8_t *s = SIGMA[r];
        G32(0, 4, 8, 12, m[s[0]], m[s[1]]); G32(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G32(2, 6, 10, 14, m[s[4]], m[s[5]]); G32(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G32(0, 5, 10, 15, m[s[8]], m[s[9]]); G32(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G32(2, 7, 8, 13, m[s[12]], m[s[13]]); G32(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef G32
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

static void blake2b_compress(uint64_t h[8], const uint8_t *p, uint64_t t, int last)
{
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; ++i) m[i] = ld64le(p + 8 * i);
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = IV64[i]; }
    v[12] ^= t; /* t < 2^64 here: the high counter word stays 0 */
    if (last) v[14] = ~v[14];
#define G64(a, b, c, d, x, y)                                  \
    v[a] += v[b] + x; v[d] = rotr64(v[d] ^ v[a], 32);          \
    v[c] += v[d]; v[b] = rotr64(v[b] ^ v[c], 24);              \
    v[a] += v[b] + y; v[d] = rotr64(v[d] ^ v[a], 16);          \
    v[c] += v[d]; v[b] = rotr64(v[b] ^ v[c], 63)
    for (int r = 0; r < 12; ++r) {
        const uint8_t *s = SIGMA[r];
        G64(0, 4, 8, 12, m[s[0]], m[s[1]]); G64(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G64(2, 6, 10, 14, m[s[4]], m[s[5]]); G64(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G64(0, 5, 10, 15, m[s[8]], m[s[9]]); G64(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G64(2, 7, 8, 13, m[s[12]], m[s[13]]); G64(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef G64
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

/* ------------------------------------------------ one-shot over 2 pieces */

typedef struct {
    int id;
    size_t hash_len, block_len;
} HashInfo;

static int hash_info(int id, HashInfo *hi)
{
    hi->id = id;
    switch (id) {
    case H_SHA256: case H_BLAKE2S: hi->hash_len = 32; hi->block_len = 64; return 0;
    case H_SHA512: case H_BLAKE2B: hi->hash_len = 64; hi->block_len = 128; return 0;
    }
    return -1;
}

/* hash(a || b) */
static void hash2(const HashInfo *hi, const uint8_t *a, size_t an, const uint8_t *b, size_t bn,
                  uint8_t *out)
{
    size_t n = an + bn;
    uint8_t *msg = (uint8_t *)malloc(n + 2 * hi->block_len + 1);
    if (!msg) abort();
    memcpy(msg, a, an);
    if (bn) memcpy(msg + an, b, bn);
    const size_t B = hi->block_len;
    if (hi->id == H_SHA256 || hi->id == H_SHA512) {
        size_t lenfield = hi->id == H_SHA256 ? 8 : 16;
        size_t total = ((n + 1 + lenfield + B - 1) / B) * B;
        memset(msg + n, 0, total - n);
        msg[n] = 0x80;
        uint64_t bits = (uint64_t)n * 8;
        for (int i = 0; i < 8; ++i) msg[total - 1 - i] = (uint8_t)(bits >> (8 * i));
        if (hi->id == H_SHA256) {
            uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                             0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
            for (size_t o = 0; o < total; o += B) sha256_block(h, msg + o);
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
        } else {
            uint64_t h[8];
            memcpy(h, IV64, sizeof(h)); /* SHA-512 IV = BLAKE2b IV */
            for (size_t o = 0; o < total; o += B) sha512_block(h, msg + o);
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
        }
        free(msg);
        return;
    }
    /* BLAKE2: every full block but the last compressed with the running
       byte count; the last (possibly partial or empty) one zero-padded */
    size_t nblocks = n ? (n + B - 1) / B : 1;
    memset(msg + n, 0, nblocks * B - n);
    if (hi->id == H_BLAKE2S) {
        uint32_t h[8];
        memcpy(h, IV32, sizeof(h));
        h[0] ^= 0x01010000u ^ 32u;
        for (size_t i = 0; i < nblocks; ++i)
            blake2s_compress(h, msg + i * B, i + 1 < nblocks ? (i + 1) * B : n, i + 1 == nblocks);
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
    } else {
        uint64_t h[8];
        memcpy(h, IV64, sizeof(h));
        h[0] ^= 0x01010000ULL ^ 64u;
        for (size_t i = 0; i < nblocks; ++i)
            blake2b_compress(h, msg + i * B, i + 1 < nblocks ? (i + 1) * B : n, i + 1 == nblocks);
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (8 * j));
    }
    free(msg);
}

int oracle_hash(int id, const uint8_t *data, size_t len, uint8_t *out)
{
    HashInfo hi;
    if (hash_info(id, &hi)) return -1;
    hash2(&hi, data, len, NULL, 0, out);
    return (int)hi.hash_len;
}

/* hashstate.c:407-448 */
static void hmac(const HashInfo *hi, const uint8_t *key, size_t key_len, const uint8_t *data,
                 size_t data_len, uint8_t *out)
{
    uint8_t kb[128], inner[64];
    const size_t B = hi->block_len;
    memset(kb, 0, sizeof(kb));
    if (key_len <= B) memcpy(kb, key, key_len);
    else hash2(hi, key, key_len, NULL, 0, kb);
    for (size_t i = 0; i < B; ++i) kb[i] ^= 0x36;
    hash2(hi, kb, B, data, data_len, inner);
    for (size_t i = 0; i < B; ++i) kb[i] ^= 0x36 ^ 0x5c;
    hash2(hi, kb, B, inner, hi->hash_len, out);
}

/* hashstate.c:476-516 */
int oracle_hkdf(int id, const uint8_t *key, size_t key_len, const uint8_t *data, size_t data_len,
                uint8_t *out1, size_t out1_len, uint8_t *out2, size_t out2_len)
{
    HashInfo hi;
    if (hash_info(id, &hi) || out1_len > hi.hash_len || out2_len > hi.hash_len ||
        key_len > 512 || data_len > 512)
        return -1;
    uint8_t tk[64], t[65];
    hmac(&hi, key, key_len, data, data_len, tk);
    t[0] = 0x01;
    hmac(&hi, tk, hi.hash_len, t, 1, t);
    memcpy(out1, t, out1_len);
    t[hi.hash_len] = 0x02;
    hmac(&hi, tk, hi.hash_len, t, hi.hash_len + 1, t);
    memcpy(out2, t, out2_len);
    return 0;
}
