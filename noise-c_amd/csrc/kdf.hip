/*
 * kdf.hip — session key fan-out on the GPU.
 *
 * A server that completes many handshakes holds one chaining key ck per
 * session; noise_symmetricstate_split (symmetricstate.c:514-573) turns each
 * into the two transport keys with HKDF(ck, "") (hashstate.c:476-516) and
 * noise_symmetricstate_mix_key does HKDF(ck, ikm) during the handshake.
 * hkdf_batch runs that for a whole batch of sessions, one lane per session,
 * for the four Noise hashes (constants.h:43-46):
 *   SHA-256 / SHA-512 (FIPS 180-4; src/crypto/sha2), BLAKE2s / BLAKE2b
 *   (RFC 7693, unkeyed; src/crypto/blake2), HMAC as noise_hashstate_hmac
 *   (hashstate.c:407-448: the key hashed when longer than a block,
 *   zero-padded, ipad 0x36 / opad 0x5c).
 * Its outputs are the raw keys noise_aead_dev_prepare turns into key
 * contexts, so a batch of finished handshakes becomes a batch of transport
 * CipherStates without leaving the device.
 *
 * This is scalar per-lane work (a split is 6 compressions), not a hot loop;
 * it is written for clarity and checked byte for byte against the oracle
 * and the reference's own HKDF outputs (tests/golden/hkdf.json).
 */
#pragma once
#include "aead_device.h"

namespace na {

constexpr int H_BLAKE2S = 0x4801, H_BLAKE2B = 0x4802, H_SHA256 = 0x4803, H_SHA512 = 0x4804;
constexpr uint32_t KDF_MAX_IN = 256; /* key_len, data_len limits of the device HKDF */

__constant__ uint32_t c_k256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__constant__ uint64_t c_k512[80] = {
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

/* BLAKE2 message schedule (RFC 7693 §2.7); rows 10, 11 repeat 0, 1 for BLAKE2b */
__constant__ uint8_t c_sigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

/* SHA-512's initial value is BLAKE2b's IV; SHA-256's is BLAKE2s's */
__constant__ uint64_t c_iv64[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                   0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                   0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
__constant__ uint32_t c_iv32[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                                   0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};

NA_DEV uint32_t rr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
NA_DEV uint64_t rr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

NA_DEV uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
NA_DEV uint32_t le32(const uint8_t *p) { return (uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]; }

NA_DEV void sha256_compress(uint32_t h[8], const uint8_t *p)
{
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = be32(p + 4 * i);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t x = w[(i + 1) & 15], y = w[(i + 14) & 15];
            wi = w[i & 15] + (rr32(x, 7) ^ rr32(x, 18) ^ (x >> 3)) + w[(i + 9) & 15] +
                 (rr32(y, 17) ^ rr32(y, 19) ^ (y >> 10));
            w[i & 15] = wi;
        }
        const uint32_t t1 = k + (rr32(e, 6) ^ rr32(e, 11) ^ rr32(e, 25)) + ((e & f) ^ (~e & g)) + c_k256[i] + wi;
        const uint32_t t2 = (rr32(a, 2) ^ rr32(a, 13) ^ rr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

NA_DEV void sha512_compress(uint64_t h[8], const uint8_t *p)
{
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = (uint64_t)be32(p + 8 * i) << 32 | be32(p + 8 * i + 4);
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
    for (int i = 0; i < 80; ++i) {
        uint64_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint64_t x = w[(i + 1) & 15], y = w[(i + 14) & 15];
            wi = w[i & 15] + (rr64(x, 1) ^ rr64(x, 8) ^ (x >> 7)) + w[(i + 9) & 15] +
                 (rr64(y, 19) ^ rr64(y, 61) ^ (y >> 6));
            w[i & 15] = wi;
        }
        const uint64_t t1 = k + (rr64(e, 14) ^ rr64(e, 18) ^ rr64(e, 41)) + ((e & f) ^ (~e & g)) + c_k512[i] + wi;
        const uint64_t t2 = (rr64(a, 28) ^ rr64(a, 34) ^ rr64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

NA_DEV void blake2s_compress(uint32_t h[8], const uint8_t *p, uint32_t t, bool last)
{
    uint32_t m[16], v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = le32(p + 4 * i);
#pragma unroll
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = c_iv32[i]; }
    v[12] ^= t; /* messages here are far below 2^32 bytes */
    if (last) v[14] = ~v[14];
#define NA_G32(a, b, c, d, x, y)                                 \
    v[a] += v[b] + (x); v[d] = rr32(v[d] ^ v[a], 16);            \
    v[c] += v[d]; v[b] = rr32(v[b] ^ v[c], 12);                  \
    v[a] += v[b] + (y); v[d] = rr32(v[d] ^ v[a], 8);             \
    v[c] += v[d]; v[b] = rr32(v[b] ^ v[c], 7)
    for (int r = 0; r < 10; ++r) {
        const uint8_t *s = c_sigma[r];
        NA_G32(0, 4, 8, 12, m[s[0]], m[s[1]]); NA_G32(1, 5, 9, 13, m[s[2]], m[s[3]]);
        NA_G32(2, 6, 10, 14, m[s[4]], m[s[5]]); NA_G32(3, 7, 11, 15, m[s[6]], m[s[7]]);
        NA_G32(0, 5, 10, 15, m[s[8]], m[s[9]]); NA_G32(1, 6, 11, 12, m[s[10]], m[s[11]]);
        NA_G32(2, 7, 8, 13, m[s[12]], m[s[13]]); NA_G32(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef NA_G32
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

NA_DEV void blake2b_compress(uint64_t h[8], const uint8_t *p, uint64_t t, bool last)
{
    uint64_t m[16], v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = (uint64_t)le32(p + 8 * i + 4) << 32 | le32(p + 8 * i);
#pragma unroll
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = c_iv64[i]; }
    v[12] ^= t;
    if (last) v[14] = ~v[14];
#define NA_G64(a, b, c, d, x, y)                                 \
    v[a] += v[b] + (x); v[d] = rr64(v[d] ^ v[a], 32);            \
    v[c] += v[d]; v[b] = rr64(v[b] ^ v[c], 24);                  \
    v[a] += v[b] + (y); v[d] = rr64(v[d] ^ v[a], 16);            \
    v[c] += v[d]; v[b] = rr64(v[b] ^ v[c], 63)
    for (int r = 0; r < 12; ++r) {
        const uint8_t *s = c_sigma[r];
        NA_G64(0, 4, 8, 12, m[s[0]], m[s[1]]); NA_G64(1, 5, 9, 13, m[s[2]], m[s[3]]);
        NA_G64(2, 6, 10, 14, m[s[4]], m[s[5]]); NA_G64(3, 7, 11, 15, m[s[6]], m[s[7]]);
        NA_G64(0, 5, 10, 15, m[s[8]], m[s[9]]); NA_G64(1, 6, 11, 12, m[s[10]], m[s[11]]);
        NA_G64(2, 7, 8, 13, m[s[12]], m[s[13]]); NA_G64(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef NA_G64
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

/* Incremental hash of one lane: update() in pieces, final() once.  BLAKE2
   keeps the last block back until final (it must carry the last-block flag
   even when full); SHA-2 compresses full blocks as they fill. */
struct Hasher {
    int id;
    uint32_t blen, hlen, fill;
    uint64_t total;
    uint8_t buf[128];
    uint32_t h32[8];
    uint64_t h64[8];

    NA_DEV void init(int hid)
    {
        id = hid;
        const bool big = hid == H_SHA512 || hid == H_BLAKE2B;
        blen = big ? 128 : 64;
        hlen = big ? 64 : 32;
        fill = 0;
        total = 0;
        for (int i = 0; i < 8; ++i) {
            h32[i] = c_iv32[i];
            h64[i] = c_iv64[i];
        }
        if (hid == H_BLAKE2S) h32[0] ^= 0x01010000u ^ 32u;
        if (hid == H_BLAKE2B) h64[0] ^= 0x01010000ull ^ 64u;
        if (hid == H_SHA256) { /* same words as c_iv32 */ }
    }
    NA_DEV void compress(bool last)
    {
        switch (id) {
        case H_SHA256: sha256_compress(h32, buf); break;
        case H_SHA512: sha512_compress(h64, buf); break;
        case H_BLAKE2S: blake2s_compress(h32, buf, (uint32_t)total, last); break;
        default: blake2b_compress(h64, buf, total, last); break;
        }
    }
    NA_DEV void update(const uint8_t *p, uint32_t n)
    {
        const bool blake = id == H_BLAKE2S || id == H_BLAKE2B;
        for (uint32_t i = 0; i < n; ++i) {
            if (fill == blen) { /* a full block and more input: not the last */
                compress(false);
                fill = 0;
            }
            buf[fill++] = p[i];
            ++total;
            if (!blake && fill == blen) {
                compress(false);
                fill = 0;
            }
        }
    }
    NA_DEV void final(uint8_t *out)
    {
        if (id == H_BLAKE2S || id == H_BLAKE2B) {
            for (uint32_t i = fill; i < blen; ++i) buf[i] = 0;
            compress(true);
            for (uint32_t i = 0; i < hlen; ++i)
                out[i] = id == H_BLAKE2S ? (uint8_t)(h32[i / 4] >> (8 * (i % 4)))
                                         : (uint8_t)(h64[i / 8] >> (8 * (i % 8)));
            return;
        }
        const uint64_t bits = total * 8;
        const uint32_t lenfield = id == H_SHA256 ? 8 : 16;
        buf[fill++] = 0x80;
        if (fill > blen - lenfield) {
            for (uint32_t i = fill; i < blen; ++i) buf[i] = 0;
            compress(false);
            fill = 0;
        }
        for (uint32_t i = fill; i < blen; ++i) buf[i] = 0;
        for (int i = 0; i < 8; ++i) buf[blen - 1 - i] = (uint8_t)(bits >> (8 * i));
        compress(false);
        for (uint32_t i = 0; i < hlen; ++i)
            out[i] = id == H_SHA256 ? (uint8_t)(h32[i / 4] >> (24 - 8 * (i % 4)))
                                    : (uint8_t)(h64[i / 8] >> (56 - 8 * (i % 8)));
    }
};

/* noise_hashstate_hmac (hashstate.c:407-448), two data pieces */
NA_DEV void kdf_hmac(int hid, const uint8_t *key, uint32_t key_len, const uint8_t *d1, uint32_t n1,
                     const uint8_t *d2, uint32_t n2, uint8_t *out)
{
    Hasher H;
    H.init(hid);
    uint8_t kb[128], inner[64];
    for (int i = 0; i < 128; ++i) kb[i] = 0;
    if (key_len <= H.blen) {
        for (uint32_t i = 0; i < key_len; ++i) kb[i] = key[i];
    } else {
        H.update(key, key_len);
        H.final(kb);
        H.init(hid);
    }
    for (uint32_t i = 0; i < H.blen; ++i) kb[i] ^= 0x36;
    H.update(kb, H.blen);
    H.update(d1, n1);
    if (n2) H.update(d2, n2);
    H.final(inner);
    for (uint32_t i = 0; i < H.blen; ++i) kb[i] ^= 0x36 ^ 0x5c;
    H.init(hid);
    H.update(kb, H.blen);
    H.update(inner, H.hlen);
    H.final(out);
}

struct KdfArgs {
    int hash_id;
    const uint8_t *keys;
    const uint8_t *data;
    uint8_t *out1, *out2;
    uint32_t key_len, data_len, out1_len, out2_len, n;
};

/* noise_hashstate_hkdf (hashstate.c:476-516), one lane per session */
__global__ __launch_bounds__(64) void hkdf_batch(KdfArgs a)
{
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t *key = a.keys + (size_t)i * a.key_len;
    const uint8_t *data = a.data ? a.data + (size_t)i * a.data_len : nullptr;
    uint8_t tk[64], t[65];
    const uint32_t hl = (a.hash_id == H_SHA512 || a.hash_id == H_BLAKE2B) ? 64 : 32;
    kdf_hmac(a.hash_id, key, a.key_len, data, a.data_len, nullptr, 0, tk);
    const uint8_t one = 0x01, two = 0x02;
    kdf_hmac(a.hash_id, tk, hl, &one, 1, nullptr, 0, t);
    for (uint32_t j = 0; j < a.out1_len; ++j) a.out1[(size_t)i * a.out1_len + j] = t[j];
    kdf_hmac(a.hash_id, tk, hl, t, hl, &two, 1, t);
    for (uint32_t j = 0; j < a.out2_len; ++j) a.out2[(size_t)i * a.out2_len + j] = t[j];
    for (int j = 0; j < 64; ++j) tk[j] = 0; /* hashstate.c:512-513 cleans its temporaries */
}

/* ------------------------------------------------ handshake-payload MixHash
 *
 * noise_symmetricstate_{encrypt,decrypt}_and_hash (symmetricstate.c
 * :352-445) for a batch of SymmetricStates: after (before, for decrypt) the
 * AEAD of record i under AD = h_i, h_i = HASH(h_i || ciphertext_i || tag_i)
 * (noise_symmetricstate_mix_hash, :244-258).  One lane per record. */
struct MixHashArgs {
    int hash_id;
    uint32_t hlen, n;
    const uint8_t *h_in;
    uint8_t *h_out;
    const uint8_t *base;   /* the job's `out` (encrypt) or `in` (decrypt) */
    const RecDesc *recs;
    int use_out_off;
};

__global__ __launch_bounds__(64) void mix_hash_batch(MixHashArgs a)
{
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= a.n) return;
    const RecDesc d = a.recs[i];
    Hasher H;
    H.init(a.hash_id);
    uint8_t h[64];
    for (uint32_t j = 0; j < a.hlen; ++j) h[j] = a.h_in[(size_t)i * a.hlen + j];
    H.update(h, a.hlen);
    H.update(a.base + (a.use_out_off ? d.out_off : d.in_off), d.len + 16);
    H.final(h);
    for (uint32_t j = 0; j < a.hlen; ++j) a.h_out[(size_t)i * a.hlen + j] = h[j];
}

/* decrypt_and_hash keeps the new hash only when the tag verified (:436-443) */
__global__ __launch_bounds__(256) void commit_hash(uint8_t *h, const uint8_t *h_new,
                                                   const uint8_t *status, uint32_t hlen, uint32_t n)
{
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= (uint64_t)n * hlen) return;
    if (status[t / hlen] == 0) h[t] = h_new[t];
}

} // namespace na
