/*
 * chachapoly.hip — ChaCha20-Poly1305 ("ChaChaPoly") transport AEAD for gfx950.
 *
 * Replaces, for batches of records, the per-record CPU path
 *   noise_cipherstate_{en,de}crypt_with_ad   (src/protocol/cipherstate.c:293-410)
 *   -> noise_chachapoly_{encrypt,decrypt}   (src/backend/ref/cipher-chachapoly.c:107-143)
 *   -> chacha_encrypt_bytes / poly1305_*    (src/crypto/chacha/chacha.c:141-310,
 *                                            src/crypto/donna/poly1305-donna*.c)
 * bit for bit: IV = LE64(n), counter 0 -> Poly1305 key, data counters 1..;
 * Poly input = AD || pad16 || CT || pad16 || LE64(|AD|) || LE64(|CT|).
 *
 * Work decomposition (one "group" of K lanes per record, K | 64):
 *   The record's ChaCha blocks are numbered v = 0 (Poly key) .. J (J = ceil(len/64)
 *   data "units" of 64 B).  Blocks are dealt round-robin to the K lanes, aligned so
 *   that the LAST block lands on lane K-1 (slot t = v + o, lane t % K, step t / K,
 *   o = leading empty slots).  The ChaCha counter of block v is v itself.
 *   Each lane Horner-evaluates Poly1305 over the 16-B blocks of its own units:
 *   inside a unit the multiplier is r, between two of its units r^(4K-3) (the
 *   4(K-1) blocks of the other lanes sit in between).  The lane holding unit 0
 *   first absorbs the AD blocks; lane K-1 finally absorbs the length block.
 *   Lane k < K-1 then scales by r^(4(K-1-k)+q-2) (q = Poly blocks in the last
 *   unit), lane K-1 by r, and the group sums its K partial values: the result
 *   is exactly sum_i b_i r^(n-i) mod 2^130-5, the donna Horner value.
 *
 * Decrypt verifies first (Poly over the ciphertext), then decrypts; a record
 * whose tag fails writes nothing (cipher-chachapoly.c:139-141).  The ciphertext
 * is read twice; the second read is served by L2.
 */
#include "aead_device.h"
#include "aead_kernels.h"

namespace na {

template <int K>
struct GroupCtx {
    uint32_t rec;      /* record index */
    int k;             /* lane within group */
    uint32_t J, steps, o, q;
};

template <int K>
NA_DEV GroupCtx<K> group_ctx(uint32_t rec, int k, uint32_t len)
{
    GroupCtx<K> g;
    g.rec = rec; g.k = k;
    g.J = (len + 63) / 64;
    const uint32_t nblk = g.J + 1;
    g.steps = (nblk + K - 1) / K;
    g.o = g.steps * K - nblk;
    const uint32_t tail = g.J ? len - 64 * (g.J - 1) : 0;
    g.q = (tail + 15) / 16;
    return g;
}

/* Poly key from key-stream block 0, broadcast from lane `src` of the group. */
NA_DEV void poly_key_bcast(const uint32_t x[16], int src_lane, Fe &r, uint32_t s[4])
{
    uint32_t kw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) kw[i] = (uint32_t)__shfl((int)x[i], src_lane, 64);
    r = fe_clamp_r(kw[0], kw[1], kw[2], kw[3]);
    s[0] = kw[4]; s[1] = kw[5]; s[2] = kw[6]; s[3] = kw[7];
}

/* Powers the lane needs: the inter-unit jump r^(4K-3) and the final scale. */
template <int K>
NA_DEV void poly_powers(const Fe &r, int k, uint32_t q, Mul &mjump, Mul &mfinal)
{
    const Mul mr = mk_mul(r);
    if constexpr (K == 1) {
        mjump = mr;
        mfinal = mr;
        return;
    } else {
        const Fe r2 = fe_mul(r, mr);
        const Mul m2 = mk_mul(r2);
        const Fe r4 = fe_mul(r2, m2);
        const Mul m4 = mk_mul(r4);
        /* Q = r^(q+2), q in 1..4 */
        const Fe qa = (q >= 3) ? r4 : r2;
        const Mul qb = (q & 1) ? mr : m2;
        Fe Q = fe_mul(qa, qb);
        if (q == 2) Q = r4;
        Fe jump;
        Fe fin = Q;
        const int d = K - 2 - k; /* (r^4)^d scales lane k < K-1 */
        if constexpr (K == 2) {
            jump = fe_mul(r4, mr); /* r^5 */
        } else {
            const Fe r8 = fe_mul(r4, m4);
            const Mul m8 = mk_mul(r8);
            if constexpr (K == 4) {
                jump = fe_mul(fe_mul(r8, m4), mr); /* r^13 */
                const Fe one = Fe{1, 0, 0, 0, 0};
                const Fe sc = d == 2 ? r8 : (d == 1 ? r4 : one);
                fin = fe_mul(Q, sc);
            } else { /* K == 8 */
                const Fe r16 = fe_mul(r8, m8);
                const Mul m16 = mk_mul(r16);
                jump = fe_mul(fe_mul(fe_mul(r16, m8), m4), mr); /* r^29 */
                const Fe one = Fe{1, 0, 0, 0, 0};
                Fe sc = (d & 1) ? r4 : one;
                sc = fe_mul(sc, (d & 2) ? m8 : mk_mul(one));
                sc = fe_mul(sc, (d & 4) ? m16 : mk_mul(one));
                fin = fe_mul(Q, sc);
            }
        }
        mjump = mk_mul(jump);
        mfinal = (k == K - 1) ? mr : mk_mul(fin);
    }
}

/* Horner over AD (lane holding unit 0 only): acc = acc*r + block, padded. */
NA_DEV void poly_ad(Fe &acc, const Mul &mr, const uint8_t *ad, uint32_t ad_len)
{
    for (uint32_t off = 0; off < ad_len; off += 16) {
        uint32_t w[4];
        const uint32_t n = ad_len - off;
        load16(ad + off, n >= 16 ? 16u : n, w);
        acc = fe_mul(acc, mr);
        fe_add_block(acc, w[0], w[1], w[2], w[3]);
    }
}

/* Horner over one 64-B unit of ciphertext (nb Poly blocks, 1..4). */
NA_DEV void poly_unit(Fe &acc, const Mul &mjump, const Mul &mr, const uint32_t c[16], uint32_t nb)
{
    acc = fe_mul(acc, mjump);
    fe_add_block(acc, c[0], c[1], c[2], c[3]);
#pragma unroll
    for (uint32_t b = 1; b < 4; ++b) {
        if (b < nb) {
            acc = fe_mul(acc, mr);
            fe_add_block(acc, c[4 * b], c[4 * b + 1], c[4 * b + 2], c[4 * b + 3]);
        }
    }
}

/* Close the group's Poly1305: length block, scale, group sum, + s. */
template <int K>
NA_DEV void poly_close(Fe acc, int k, const Mul &mr, const Mul &mfinal, uint64_t ad_len,
                       uint64_t len, const uint32_t s[4], uint32_t tag[4])
{
    if (k == K - 1) {
        acc = fe_mul(acc, mr);
        fe_add_block(acc, (uint32_t)ad_len, (uint32_t)(ad_len >> 32), (uint32_t)len,
                     (uint32_t)(len >> 32));
    }
    acc = fe_mul(acc, mfinal);
    acc = fe_group_sum<K>(acc);
    fe_finish(acc, s, tag);
}

/* One record as seen by its group of K lanes. */
struct RecView {
    const uint8_t *src;
    uint8_t *dst;
    const uint8_t *ad;
    const uint8_t *key;   /* 32-B raw key */
    uint64_t nonce;
    uint32_t len, ad_len;
};

NA_DEV void load_key(const uint8_t *kp8, uint32_t key[8])
{
    const uint4 *kp = (const uint4 *)kp8;
    uint4 k0 = kp[0], k1 = kp[1];
    key[0] = k0.x; key[1] = k0.y; key[2] = k0.z; key[3] = k0.w;
    key[4] = k1.x; key[5] = k1.y; key[6] = k1.z; key[7] = k1.w;
}

/* ------------------------------------------------------------- encrypt */

template <int K>
NA_DEV void seal_record(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint64_t nonce = rv.nonce;
    const uint32_t len = rv.len;
    const GroupCtx<K> g = group_ctx<K>(0, k, len);
    const int lane = (int)(threadIdx.x & 63);
    const int gbase = lane & ~(K - 1);

    Fe acc = fe_zero(), r;
    Mul mr, mjump, mfinal;
    uint32_t s[4];
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
        uint32_t x[16];
        chacha20_block(key, (uint32_t)v, 0u, (uint32_t)nonce, (uint32_t)(nonce >> 32), x);
        if (m == 0) {
            poly_key_bcast(x, gbase + (int)g.o, r, s);
            mr = mk_mul(r);
            poly_powers<K>(r, k, g.q, mjump, mfinal);
            /* unit 0 (block 1) sits in lane (o+1) % K; with no units, lane K-1 */
            const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
            if (k == k0 && rv.ad_len) poly_ad(acc, mr, rv.ad, rv.ad_len);
        }
        if (v >= 1) {
            const uint32_t j = (uint32_t)v - 1;
            const uint32_t nbytes = (j + 1 < g.J) ? 64u : len - 64 * j;
            uint32_t w[16];
            load_unit(rv.src + 64 * j, nbytes, w);
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] ^= x[i];
            mask_unit(w, nbytes);
            store_unit(rv.dst + 64 * j, nbytes, w);
            /* A lane's first unit follows the AD directly (exponent gap 1) or
               starts from acc = 0, where any multiplier works: use r. */
            const bool first = (m == 0) || (m == 1 && k <= (int)g.o);
            poly_unit(acc, first ? mr : mjump, mr, w, (nbytes + 15) / 16);
        }
    }
    uint32_t tag[4];
    poly_close<K>(acc, k, mr, mfinal, rv.ad_len, len, s, tag);
    if (k == K - 1) store16(rv.dst + len, 16, tag);
}

/* ------------------------------------------------------------- decrypt */

/* Returns true when the tag verified (identical on every lane of the group). */
template <int K>
NA_DEV bool open_record(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint64_t nonce = rv.nonce;
    const uint32_t len = rv.len;
    const GroupCtx<K> g = group_ctx<K>(0, k, len);
    const int lane = (int)(threadIdx.x & 63);
    const int gbase = lane & ~(K - 1);

    /* step-0 key stream: block 0 on lane o (Poly key), data on the others —
       kept in registers for the decrypt phase */
    const int v0 = k - (int)g.o;
    uint32_t x0[16];
    chacha20_block(key, (uint32_t)v0, 0u, (uint32_t)nonce, (uint32_t)(nonce >> 32), x0);
    Fe r;
    uint32_t s[4];
    poly_key_bcast(x0, gbase + (int)g.o, r, s);
    const Mul mr = mk_mul(r);
    Mul mjump, mfinal;
    poly_powers<K>(r, k, g.q, mjump, mfinal);
    Fe acc = fe_zero();
    const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
    if (k == k0 && rv.ad_len) poly_ad(acc, mr, rv.ad, rv.ad_len);

    /* phase 1: authenticate the ciphertext */
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
        if (v >= 1) {
            const uint32_t j = (uint32_t)v - 1;
            const uint32_t nbytes = (j + 1 < g.J) ? 64u : len - 64 * j;
            uint32_t w[16];
            load_unit(rv.src + 64 * j, nbytes, w);
            const bool first = (m == 0) || (m == 1 && k <= (int)g.o);
            poly_unit(acc, first ? mr : mjump, mr, w, (nbytes + 15) / 16);
        }
    }
    uint32_t tag[4], got[4];
    poly_close<K>(acc, k, mr, mfinal, rv.ad_len, len, s, tag);
    load16(rv.src + len, 16, got);
    const uint32_t diff = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
    if (diff != 0) return false; /* noise_is_equal, util.c:188-200: nothing written */

    /* phase 2: decrypt (the ciphertext re-read is served by L2) */
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
        if (v >= 1) {
            uint32_t x[16];
            if (m == 0) {
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] = x0[i];
            } else {
                chacha20_block(key, (uint32_t)v, 0u, (uint32_t)nonce, (uint32_t)(nonce >> 32), x);
            }
            const uint32_t j = (uint32_t)v - 1;
            const uint32_t nbytes = (j + 1 < g.J) ? 64u : len - 64 * j;
            uint32_t w[16];
            load_unit(rv.src + 64 * j, nbytes, w);
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] ^= x[i];
            store_unit(rv.dst + 64 * j, nbytes, w);
        }
    }
    return true;
}

/* ------------------------------------------------------------- kernels */

NA_DEV RecView uniform_view(const UniformArgs &a, uint32_t rec)
{
    const uint32_t st = rec / a.rps;
    RecView rv;
    rv.src = a.in + (size_t)rec * a.in_stride;
    rv.dst = a.out + (size_t)rec * a.out_stride;
    rv.ad = a.ad ? a.ad + (size_t)rec * a.ad_stride : nullptr;
    rv.key = a.keys + (size_t)st * 32;
    rv.nonce = a.nonce_base[st] + (uint64_t)(rec - st * a.rps);
    rv.len = a.len;
    rv.ad_len = a.ad_len;
    return rv;
}

NA_DEV RecView ragged_view(const RaggedArgs &a, uint32_t rec)
{
    const RecDesc d = a.recs[rec];
    RecView rv;
    rv.src = a.in + d.in_off;
    rv.dst = a.out + d.out_off;
    rv.ad = a.ad ? a.ad + d.ad_off : nullptr;
    rv.key = (const uint8_t *)((uintptr_t)a.keys + d.ctx_off);
    rv.nonce = d.nonce;
    rv.len = d.len;
    rv.ad_len = d.ad_len;
    return rv;
}

template <int K>
__global__ __launch_bounds__(256) void chachapoly_seal_uniform(UniformArgs a)
{
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / K;
    if (rec >= a.n_records) return; /* whole groups leave together (K | 64) */
    seal_record<K>(uniform_view(a, rec), (int)(gtid % K));
}

template <int K>
__global__ __launch_bounds__(256) void chachapoly_open_uniform(UniformArgs a)
{
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / K;
    if (rec >= a.n_records) return;
    const int k = (int)(gtid % K);
    const bool ok = open_record<K>(uniform_view(a, rec), k);
    if (k == K - 1 && a.status) a.status[rec] = ok ? 0 : 1;
}

template <int K>
__global__ __launch_bounds__(256) void chachapoly_seal_ragged(RaggedArgs a)
{
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / K;
    if (rec >= a.n_records) return;
    seal_record<K>(ragged_view(a, rec), (int)(gtid % K));
}

template <int K>
__global__ __launch_bounds__(256) void chachapoly_open_ragged(RaggedArgs a)
{
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / K;
    if (rec >= a.n_records) return;
    const int k = (int)(gtid % K);
    const bool ok = open_record<K>(ragged_view(a, rec), k);
    if (k == K - 1 && a.status) a.status[rec] = ok ? 0 : 1;
}

} // namespace na
