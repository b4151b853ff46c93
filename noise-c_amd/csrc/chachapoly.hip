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
 * A record's ChaCha blocks are v = 0 (the Poly1305 key block) .. J, J =
 * ceil(len/64); block v >= 1 is data "unit" v-1 (64 bytes, the last one
 * partial).  The ChaCha counter of block v is v itself.  A group of K lanes
 * (K | 64) owns one record; two decompositions:
 *
 *  contiguous (K = 1, 2): block v goes to lane v / P, P = ceil((J+1)/K).
 *    Each lane's Poly1305 run is a plain Horner chain with the clamped r, in
 *    radix 2^32 (p32_block, 20 v_mad_u64_u32 per 16 B).  Lane 0 absorbs the
 *    AD first, the lane with the last unit absorbs the length block; with
 *    K = 2 lane 0's value is scaled by r^A (A = Poly blocks after its run).
 *
 *  interleaved (K = 4, 8): blocks are dealt round-robin, end-aligned so the
 *    last block lands on lane K-1 (slot t = v + o, lane t % K, step t / K).
 *    Each lane runs Horner in radix 2^26: multiplier r inside a unit,
 *    r^(4K-3) between two of its units; the lane with unit 0 absorbs the AD,
 *    lane K-1 the length block; lane k < K-1 is scaled by r^(4(K-1-k)+q-2)
 *    (q = Poly blocks of the last unit), lane K-1 by r, then the group sums.
 *  Both give exactly sum_i b_i r^(n-i) mod 2^130-5, the donna Horner value.
 *
 * Memory: a lane loads the unit of its NEXT step before running the ChaCha
 * block of the current one.  FAST layouts (16-B aligned record slots whose
 * input may be read up to roundup64(len)) use straight-line dwordx4 traffic
 * in the loop; only the record's last unit and the tag take an exact-size
 * path, after the loop.  The generic path accepts any alignment.
 *
 * Decrypt comes in two forms.  The verify-first opens (open_il, open_ct,
 * the one-lane AUTH + DEC passes: the default since round 6) verify first,
 * then decrypt; a record whose tag fails writes nothing
 * (cipher-chachapoly.c:139-141) and the second ciphertext read is served by
 * L2 / MALL.  The one-pass opens (open_il_1p, open_il_staged, solo_pass
 * OPEN1: the opt-in NOISE_AEAD_FLAG_ONE_PASS of the FAST layouts) decrypt as
 * they authenticate and undo the plaintext of a rejected record before the
 * kernel ends (restored in place, zeroed out of place).
 */
#include "aead_device.h"
#include "aead_kernels.h"

namespace na {

typedef __attribute__((address_space(3))) void lds_void;

/* One record as seen by its group of lanes. */
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

/* ------------------------------------------------------------ record I/O */

/* Unit j of a record: FAST = four dwordx4 (bytes past len are garbage and
   are masked by the caller); generic = exact bytes, zero-filled. */
template <bool FAST>
NA_DEV void unit_in(const uint8_t *rec, uint32_t j, uint32_t len, uint32_t w[16])
{
    if constexpr (FAST) {
        const uint4 *q = (const uint4 *)(rec + 64 * j);
        const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
        w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
        w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w;
        w[12] = d.x; w[13] = d.y; w[14] = d.z; w[15] = d.w;
    } else {
        const uint32_t nb = len - 64 * j;
        load_unit(rec + 64 * j, nb >= 64 ? 64u : nb, w);
    }
}

/* Prefetch of unit j when `ok`.  FAST loads unconditionally (unit 0 when not
   ok: FAST slots are readable up to roundup64(max(len,1))), so no branch
   join forces hipcc to wait for the data right after issuing the loads. */
template <bool FAST>
NA_DEV void unit_prefetch(const uint8_t *rec, bool ok, uint32_t j, uint32_t len, uint32_t w[16])
{
    if constexpr (FAST) {
        unit_in<true>(rec, ok ? j : 0u, len, w);
    } else {
        if (ok) unit_in<false>(rec, j, len, w);
    }
}

template <bool FAST>
NA_DEV void unit_out_full(uint8_t *p, const uint32_t w[16])
{
    if constexpr (FAST) {
        uint4 *q = (uint4 *)p;
        q[0] = make_uint4(w[0], w[1], w[2], w[3]);
        q[1] = make_uint4(w[4], w[5], w[6], w[7]);
        q[2] = make_uint4(w[8], w[9], w[10], w[11]);
        q[3] = make_uint4(w[12], w[13], w[14], w[15]);
    } else {
        store_unit(p, 64, w);
    }
}

/* the 16-B chunk c (0..3, runtime) of a unit, without dynamic indexing */
NA_DEV void pick_chunk(const uint32_t w[16], uint32_t c, uint32_t o[4])
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
        o[i] = c == 0 ? w[i] : (c == 1 ? w[4 + i] : (c == 2 ? w[8 + i] : w[12 + i]));
}

/* Exact-size store of the last unit's bytes [64(J-1), len), then (seal) the
   tag at len.  FAST: aligned chunks as dwordx4, the partial chunk merged with
   the tag into 8-B stores when len % 8 == 0. */
template <bool FAST, bool TAG>
NA_DEV void tail_out(uint8_t *rec, uint32_t J, uint32_t len, const uint32_t w[16],
                     const uint32_t tag[4])
{
    if constexpr (FAST) {
        uint32_t rem = 0, part[4] = {0, 0, 0, 0};
        if (J >= 1) {
            const uint32_t base = 64 * (J - 1), nb = len - base;
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c)
                if (16 * c + 16 <= nb)
                    *(uint4 *)(rec + base + 16 * c) =
                        make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
            rem = nb & 15;
            if (rem) pick_chunk(w, nb >> 4, part);
        }
        const uint32_t pstart = len - rem;
        if (rem == 8) {
            *(uint2 *)(rec + pstart) = make_uint2(part[0], part[1]);
            if (TAG) {
                *(uint2 *)(rec + len) = make_uint2(tag[0], tag[1]);
                *(uint2 *)(rec + len + 8) = make_uint2(tag[2], tag[3]);
            }
        } else {
            if (rem) store16(rec + pstart, rem, part);
            if (TAG) store16(rec + len, 16, tag);
        }
    } else {
        if (J >= 1) store_unit(rec + 64 * (J - 1), len - 64 * (J - 1), w);
        if (TAG) store16(rec + len, 16, tag);
    }
}

template <bool FAST>
NA_DEV void tag_in(const uint8_t *rec, uint32_t len, uint32_t t[4])
{
    if constexpr (FAST) {
        if ((len & 15) == 0) {
            const uint4 v = *(const uint4 *)(rec + len);
            t[0] = v.x; t[1] = v.y; t[2] = v.z; t[3] = v.w;
            return;
        }
        if ((len & 7) == 0) {
            const uint2 a = *(const uint2 *)(rec + len), b = *(const uint2 *)(rec + len + 8);
            t[0] = a.x; t[1] = a.y; t[2] = b.x; t[3] = b.y;
            return;
        }
    }
    load16(rec + len, 16, t);
}

NA_DEV bool tag_equal(const uint32_t a[4], const uint32_t b[4])
{
    /* constant-time, as noise_is_equal (src/protocol/util.c:188-200) */
    return ((a[0] ^ b[0]) | (a[1] ^ b[1]) | (a[2] ^ b[2]) | (a[3] ^ b[3])) == 0;
}

/* ------------------------------------------------- interleaved (K = 4, 8) */

template <int K>
struct GroupCtx {
    uint32_t J, steps, o, q;
};

template <int K>
NA_DEV GroupCtx<K> group_ctx(uint32_t len)
{
    GroupCtx<K> g;
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

/* r^e for 1 <= e < 2^9, square-and-multiply (the wide groups' powers). */
NA_DEV Fe fe_pow(Fe b, uint32_t e)
{
    Fe acc = Fe{1, 0, 0, 0, 0};
    for (;;) {
        if (e & 1) acc = fe_mul(acc, mk_mul(b));
        e >>= 1;
        if (!e) break;
        b = fe_mul(b, mk_mul(b));
    }
    return acc;
}

/* The inter-unit jump r^(4K-3) and the final scale of lane k. */
template <int K>
NA_DEV void poly_powers(const Fe &r, int k, uint32_t q, Mul &mjump, Mul &mfinal)
{
    const Mul mr = mk_mul(r);
    if constexpr (K >= 16) {
        /* wide groups (small batches of long records): lane k < K-1 is
           scaled by r^(4(K-1-k)+q-2), as below, by direct powers */
        mjump = mk_mul(fe_pow(r, 4 * K - 3));
        mfinal = (k == K - 1) ? mr : mk_mul(fe_pow(r, 4u * (uint32_t)(K - 1 - k) + q - 2));
        return;
    }
    const Fe r2 = fe_mul(r, mr);
    const Mul m2 = mk_mul(r2);
    const Fe r4 = fe_mul(r2, m2);
    const Mul m4 = mk_mul(r4);
    /* Q = r^(q+2), q in 1..4 */
    const Fe qa = (q >= 3) ? r4 : r2;
    const Mul qb = (q & 1) ? mr : m2;
    Fe Q = fe_mul(qa, qb);
    if (q == 2) Q = r4;
    const Fe r8 = fe_mul(r4, m4);
    const Mul m8 = mk_mul(r8);
    const Fe one = Fe{1, 0, 0, 0, 0};
    const int d = K - 2 - k; /* lane k < K-1 is scaled by (r^4)^d * Q */
    Fe jump, fin;
    if constexpr (K == 4) {
        jump = fe_mul(fe_mul(r8, m4), mr); /* r^13 */
        fin = fe_mul(Q, d == 2 ? r8 : (d == 1 ? r4 : one));
    } else { /* K == 8 */
        const Fe r16 = fe_mul(r8, m8);
        const Mul m16 = mk_mul(r16);
        jump = fe_mul(fe_mul(fe_mul(r16, m8), m4), mr); /* r^29 */
        Fe sc = (d & 1) ? r4 : one;
        sc = fe_mul(sc, (d & 2) ? m8 : mk_mul(one));
        sc = fe_mul(sc, (d & 4) ? m16 : mk_mul(one));
        fin = fe_mul(Q, sc);
    }
    mjump = mk_mul(jump);
    mfinal = (k == K - 1) ? mr : mk_mul(fin);
}

/* Horner over AD (radix 2^26): acc = acc*r + block, zero-padded. */
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

/* Horner over one unit of ciphertext (nb Poly blocks, 1..4). */
NA_DEV void poly_unit(Fe &acc, const Mul &mfirst, const Mul &mr, const uint32_t c[16], uint32_t nb)
{
    acc = fe_mul(acc, mfirst);
    fe_add_block(acc, c[0], c[1], c[2], c[3]);
#pragma unroll
    for (uint32_t b = 1; b < 4; ++b) {
        if (b < nb) {
            acc = fe_mul(acc, mr);
            fe_add_block(acc, c[4 * b], c[4 * b + 1], c[4 * b + 2], c[4 * b + 3]);
        }
    }
}

/* Length block on lane K-1, scale, group sum, + s. */
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

/* Wide groups (K >= 16) whose record fits one step (each lane holds at most
   one unit, the single-record and small-batch case): no r^(4K-3) jump and
   no per-lane power of r.  Lane k < K-1 holds a full unit at position
   p = K-2-k from the right (h_p: Horner over its blocks, the AD first on the
   unit-0 lane), lane K-1 the last unit and the length block.  With R = r^4,
     S = sum_p h_p R^p   (a right-aligned tree over the lanes: level L adds
                          lane k-L's value times R^L into lane k),
     poly = S r^(q+2) + h_last r,
   q+2 = the blocks after lane K-2's last block plus the final r.  log2(K)
   multiplies deep instead of ~2 log2(4K) squarings and multiplies per lane
   (fe_pow), for the latency of one record on one wave.  Every lane of the
   group gets the tag. */
template <int K>
NA_DEV void poly_tree_close(Fe acc, int k, const Fe &r, const Mul &mr, uint32_t J, uint32_t q,
                            uint64_t ad_len, uint64_t len, const uint32_t s[4], uint32_t tag[4])
{
    const int lane = (int)(threadIdx.x & 63), gbase = lane & ~(K - 1);
    if (k == K - 1) {
        acc = fe_mul(acc, mr);
        fe_add_block(acc, (uint32_t)ad_len, (uint32_t)(ad_len >> 32), (uint32_t)len,
                     (uint32_t)(len >> 32));
    }
    const Fe r2 = fe_mul(r, mr);
    const Mul m2 = mk_mul(r2);
    const Fe r4 = fe_mul(r2, m2);
    const Mul m4 = mk_mul(r4);
    Fe v = (k == K - 1) ? fe_zero() : acc;
    const int p = K - 2 - k;
    const uint32_t full = J ? J - 1 : 0; /* lanes holding a full unit */
    Mul mR = m4;
#pragma unroll
    for (int L = 1; L < K - 1; L <<= 1) {
        if (!__any((uint32_t)L < full)) break; /* no group has a level this wide */
        Fe w;
        const int src = lane - L;
        w.l0 = (uint32_t)__shfl((int)v.l0, src, 64);
        w.l1 = (uint32_t)__shfl((int)v.l1, src, 64);
        w.l2 = (uint32_t)__shfl((int)v.l2, src, 64);
        w.l3 = (uint32_t)__shfl((int)v.l3, src, 64);
        w.l4 = (uint32_t)__shfl((int)v.l4, src, 64);
        const Fe t = fe_mul(w, mR);
        if (p >= 0 && (p & (2 * L - 1)) == 0 && k - L >= 0) v = fe_carry(fe_add(v, t));
        if (2 * L < K - 1) mR = mk_mul(fe_mul(mul_fe(mR), mR)); /* R^(2L) */
    }
    /* lane K-1: S from lane K-2, then S r^(q+2) + h_last r */
    Fe S;
    const int from = gbase + K - 2;
    S.l0 = (uint32_t)__shfl((int)v.l0, from, 64);
    S.l1 = (uint32_t)__shfl((int)v.l1, from, 64);
    S.l2 = (uint32_t)__shfl((int)v.l2, from, 64);
    S.l3 = (uint32_t)__shfl((int)v.l3, from, 64);
    S.l4 = (uint32_t)__shfl((int)v.l4, from, 64);
    /* r^(q+2), q = 1..4: r^3, r^4, r^5, r^6 (any value when there is no full unit) */
    const Fe rq = (q <= 2) ? ((q == 2) ? r4 : fe_mul(r2, mr)) : fe_mul(r4, (q == 3) ? mr : m2);
    Fe T = fe_add(fe_mul(acc, mr), fe_mul(S, mk_mul(rq)));
    uint32_t t4[4];
    fe_finish(T, s, t4);
    const int last = gbase + K - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) tag[i] = (uint32_t)__shfl((int)t4[i], last, 64);
}

/* The key stream of lane slot v of a staged step.  Slots before block 0
   (v < 0: the end alignment's padding, 1 of 24 at 1400 B, 3 of 20 at 1024 B)
   carry no block, and their lanes run the step switched off instead of
   computing a block no one reads.  The issue slots are the same; what it
   saves is energy, and the chip holds its clock by energy under this load
   (MI355X_MICROARCH.md, DVFS give-back): C4 +1.1 %, perf +0.9 % in three
   interleaved rounds (profiles/r02/mask_idle_ab.jsonl).  RUNS (the staged
   kernels: four waves per SIMD) issues the block in runs with priority
   toggles (aead_device.h chacha20_block_runs, round 6); the windowed
   kernels, whose small batches often hold under one wave per SIMD, keep
   hipcc's schedule.  early (a one-generation launch, UniformArgs.balance,
   in the first half of the wave's steps): toggles 3 / 1, the progress
   balance of solo_blocks2 — the standalone C2 seal 55.5-60.1 -> 54.1-55.3
   us per launch in four interleaved rounds (profiles/r06/staged_early_ab/). */
template <bool RUNS = false>
NA_DEV void slot_block(const uint32_t key[8], const ChaPre &pre, int v, uint32_t n_lo,
                       uint32_t n_hi, uint32_t x[16], bool early = false)
{
    if (v < 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = 0;
        return;
    }
    if constexpr (RUNS) {
        if (early) chacha20_block_runs<3, 1, 1>(key, pre, (uint32_t)v, n_lo, n_hi, x);
        else chacha20_block_runs<2, 0, 0>(key, pre, (uint32_t)v, n_lo, n_hi, x);
    } else {
        chacha20_block_pre(key, pre, (uint32_t)v, n_lo, n_hi, x);
    }
}

template <int K, bool FAST>
NA_DEV void seal_il(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint32_t n_lo = (uint32_t)rv.nonce, n_hi = (uint32_t)(rv.nonce >> 32);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = rv.len;
    const GroupCtx<K> g = group_ctx<K>(len);
    const int gbase = (int)(threadIdx.x & 63) & ~(K - 1);
    const bool tree = K >= 16 && g.steps == 1; /* poly_tree_close */

    Fe acc = fe_zero(), r;
    Mul mr, mjump, mfinal;
    uint32_t s[4], wn[16], wc[16], x[16];
    bool seen = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) wn[i] = 0;
    {
        const int v = k - (int)g.o;
        unit_prefetch<FAST>(rv.src, v >= 1, (uint32_t)v - 1, len, wn);
    }
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        const int vn = v + K; /* the unit of the next step, loaded now */
        unit_prefetch<FAST>(rv.src, m + 1 < g.steps && vn >= 1, (uint32_t)vn - 1, len, wn);
        slot_block(key, pre, v, n_lo, n_hi, x);
        if (m == 0) {
            poly_key_bcast(x, gbase + (int)g.o, r, s);
            mr = mk_mul(r);
            if (!tree) poly_powers<K>(r, k, g.q, mjump, mfinal);
            /* unit 0 (block 1) sits in lane (o+1) % K; with no units, lane K-1 */
            const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
            if (k == k0 && rv.ad_len) poly_ad(acc, mr, rv.ad, rv.ad_len);
        }
        if (v >= 1 && (uint32_t)v < g.J) { /* a full unit */
            uint32_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
            unit_out_full<FAST>(rv.dst + 64 * (v - 1), w);
            /* a lane's first unit follows the AD directly (gap 1) or starts
               from acc = 0, where any multiplier works: use r */
            poly_unit(acc, seen ? mjump : mr, mr, w, 4);
            seen = true;
        }
    }
    /* the last unit (block J) is lane K-1's last step */
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
    if (k == K - 1 && g.J >= 1) {
        const uint32_t nb = len - 64 * (g.J - 1);
        mask_unit(w, nb);
        poly_unit(acc, seen ? mjump : mr, mr, w, (nb + 15) / 16);
    }
    uint32_t tag[4];
    if (tree) poly_tree_close<K>(acc, k, r, mr, g.J, g.q, rv.ad_len, len, s, tag);
    else poly_close<K>(acc, k, mr, mfinal, rv.ad_len, len, s, tag);
    if (k == K - 1) tail_out<FAST, true>(rv.dst, g.J, len, w, tag);
}

/* Open in one pass (FAST layouts): seal_il's loop with Poly1305 over the
   ciphertext as read, each unit decrypted and stored as it goes, so the
   ciphertext is read once.  The verdict comes after the plaintext is written:
   on a MAC failure in place the lane XORs its units with their key stream
   once more — the buffer reads as given, as after the reference's verify-
   then-decrypt (cipher-chachapoly.c:125-143) — and out of place the caller's
   scrub_rejected zeroes the output. */
template <int K>
NA_DEV bool open_il_1p(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint32_t n_lo = (uint32_t)rv.nonce, n_hi = (uint32_t)(rv.nonce >> 32);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = rv.len;
    const GroupCtx<K> g = group_ctx<K>(len);
    const int gbase = (int)(threadIdx.x & 63) & ~(K - 1);
    const bool tree = K >= 16 && g.steps == 1; /* poly_tree_close */
    const uint32_t tail = g.J ? len - 64 * (g.J - 1) : 0; /* bytes of unit J-1 */

    Fe acc = fe_zero(), r;
    Mul mr, mjump, mfinal;
    uint32_t s[4], wn[16], wc[16], x[16];
    bool seen = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) wn[i] = 0;
    {
        const int v = k - (int)g.o;
        unit_prefetch<true>(rv.src, v >= 1, (uint32_t)v - 1, len, wn);
    }
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        const int vn = v + K;
        unit_prefetch<true>(rv.src, m + 1 < g.steps && vn >= 1, (uint32_t)vn - 1, len, wn);
        slot_block(key, pre, v, n_lo, n_hi, x);
        if (m == 0) {
            poly_key_bcast(x, gbase + (int)g.o, r, s);
            mr = mk_mul(r);
            if (!tree) poly_powers<K>(r, k, g.q, mjump, mfinal);
            const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
            if (k == k0 && rv.ad_len) poly_ad(acc, mr, rv.ad, rv.ad_len);
        }
        if (v >= 1 && (uint32_t)v < g.J) { /* a full unit */
            poly_unit(acc, seen ? mjump : mr, mr, wc, 4);
            seen = true;
            uint32_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
            unit_out_full<true>(rv.dst + 64 * (v - 1), w);
        }
    }
    /* the last unit (block J) is lane K-1's last step */
    if (k == K - 1 && g.J >= 1) {
        uint32_t c[16], w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            c[i] = wc[i];
            w[i] = wc[i] ^ x[i];
        }
        mask_unit(c, tail);
        poly_unit(acc, seen ? mjump : mr, mr, c, (tail + 15) / 16);
        tail_out<true, false>(rv.dst, g.J, len, w, nullptr);
    }
    uint32_t tag[4], got[4];
    if (tree) poly_tree_close<K>(acc, k, r, mr, g.J, g.q, rv.ad_len, len, s, tag);
    else poly_close<K>(acc, k, mr, mfinal, rv.ad_len, len, s, tag);
    tag_in<true>(rv.src, len, got); /* the tag bytes are never written */
    const bool ok = tag_equal(tag, got);
    if (ok || rv.dst != rv.src) return ok;
    /* repair in place: plaintext XOR key stream = the ciphertext as given */
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
        if (v < 1) continue;
        slot_block(key, pre, v, n_lo, n_hi, x);
        uint32_t w[16];
        unit_in<true>(rv.dst, (uint32_t)v - 1, len, w);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        if ((uint32_t)v < g.J) unit_out_full<true>(rv.dst + 64 * (v - 1), w);
        else tail_out<true, false>(rv.dst, g.J, len, w, nullptr);
    }
    return false;
}

template <int K, bool FAST>
NA_DEV bool open_il(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint32_t n_lo = (uint32_t)rv.nonce, n_hi = (uint32_t)(rv.nonce >> 32);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = rv.len;
    const GroupCtx<K> g = group_ctx<K>(len);
    const int gbase = (int)(threadIdx.x & 63) & ~(K - 1);
    const bool tree = K >= 16 && g.steps == 1; /* poly_tree_close */

    /* step-0 key stream: block 0 on lane o, data on the others (kept) */
    const int v0 = k - (int)g.o;
    uint32_t x0[16];
    chacha20_block_pre(key, pre, (uint32_t)v0, n_lo, n_hi, x0);
    Fe r;
    uint32_t s[4];
    poly_key_bcast(x0, gbase + (int)g.o, r, s);
    const Mul mr = mk_mul(r);
    Mul mjump, mfinal;
    if (!tree) poly_powers<K>(r, k, g.q, mjump, mfinal);
    Fe acc = fe_zero();
    const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
    if (k == k0 && rv.ad_len) poly_ad(acc, mr, rv.ad, rv.ad_len);

    /* phase 1: authenticate the ciphertext */
    uint32_t wn[16], wc[16];
    bool seen = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) wn[i] = 0;
    unit_prefetch<FAST>(rv.src, v0 >= 1, (uint32_t)v0 - 1, len, wn);
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        const int vn = v + K;
        unit_prefetch<FAST>(rv.src, m + 1 < g.steps && vn >= 1, (uint32_t)vn - 1, len, wn);
        if (v >= 1) {
            const uint32_t j = (uint32_t)v - 1;
            uint32_t nb = 4;
            if (j + 1 == g.J) {
                const uint32_t bytes = len - 64 * j;
                mask_unit(wc, bytes);
                nb = (bytes + 15) / 16;
            }
            poly_unit(acc, seen ? mjump : mr, mr, wc, nb);
            seen = true;
        }
    }
    uint32_t tag[4], got[4];
    if (tree) poly_tree_close<K>(acc, k, r, mr, g.J, g.q, rv.ad_len, len, s, tag);
    else poly_close<K>(acc, k, mr, mfinal, rv.ad_len, len, s, tag);
    tag_in<FAST>(rv.src, len, got);
    if (!tag_equal(tag, got)) return false; /* identical verdict on the group */

    /* phase 2: decrypt (the ciphertext re-read is served by L2) */
#pragma unroll
    for (int i = 0; i < 16; ++i) wn[i] = 0;
    unit_prefetch<FAST>(rv.src, v0 >= 1, (uint32_t)v0 - 1, len, wn);
    uint32_t x[16];
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int v = (int)(m * K + (uint32_t)k) - (int)g.o;
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        const int vn = v + K;
        unit_prefetch<FAST>(rv.src, m + 1 < g.steps && vn >= 1, (uint32_t)vn - 1, len, wn);
        if (m == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = x0[i];
        } else {
            chacha20_block_pre(key, pre, (uint32_t)v, n_lo, n_hi, x);
        }
        if (v >= 1 && (uint32_t)v < g.J) {
            uint32_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
            unit_out_full<FAST>(rv.dst + 64 * (v - 1), w);
        }
    }
    if (k == K - 1 && g.J >= 1) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
        tail_out<FAST, false>(rv.dst, g.J, len, w, nullptr);
    }
    return true;
}

/* --------------------------- interleaved, LDS-staged (uniform FAST batches)
 *
 * Same decomposition as seal_il/open_il, but the wave's global traffic is
 * re-shaped through a 4 KB LDS tile.  At every step lane L of the wave owns
 * one unit (unit j0 + L%K of record rec0 + L/K).  Coalesced wave-instruction
 * i (0..3), lane l moves chunk c = l%4 of the unit owned by L = 16i + l/4, so
 * one instruction covers the 256-B (K=4) or 512-B (K=8) contiguous runs of
 * whole records: full 128-B lines instead of 64 scattered 16-B pieces.  The
 * tile slot of (L, c) is L*4 + (c ^ ((L>>2)&3)) (uint4 units): the XOR makes
 * both the owner-side and the coalesced-side ds_*_b128 bank-conflict-free.
 * Every lane of the wave takes part in every exchange (no early exit); lanes
 * past the batch end are clamped onto the last record and store nothing.
 */

NA_DEV RecView uniform_view(const UniformArgs &a, uint32_t rec);

NA_DEV uint32_t tile_slot(uint32_t L, uint32_t c) { return L * 4 + (c ^ ((L >> 2) & 3)); }

NA_DEV void tile_get_unit(const uint4 *t, uint32_t L, uint32_t w[16])
{
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) {
        const uint4 v = t[tile_slot(L, c)];
        w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
    }
}

/* four coalesced 16-B pieces, held by value (an array here gets demoted to
   scratch by hipcc once it is live across the ChaCha block) */
struct Quad { uint4 a, b, c, d; };

NA_DEV void tile_put_coalesced(uint4 *t, uint32_t lane, const Quad &P)
{
    const uint32_t q = lane >> 2, c = lane & 3;
    t[tile_slot(q, c)] = P.a;
    t[tile_slot(16u + q, c)] = P.b;
    t[tile_slot(32u + q, c)] = P.c;
    t[tile_slot(48u + q, c)] = P.d;
}

NA_DEV void tile_put_unit(uint4 *t, uint32_t L, const uint32_t w[16])
{
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c)
        t[tile_slot(L, c)] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
}

/* The wave's coalesced view: for instruction i, this lane serves owner
   L = 16i + lane/4 — record rq + i*16/K, unit offset kk = L%K (the same for
   all four i since K | 16), chunk lane%4.  Addresses are rebuilt from the
   kernel arguments at each use instead of being held in 16 VGPRs. */
template <int K>
struct WaveIO {
    uint32_t rq;   /* record of instruction 0 (unclamped) */
    uint32_t c16;  /* byte offset of this lane's chunk (register-staged) */
    uint32_t d16;  /* byte offset of the chunk this lane DMAs (see wave_dma) */
    int kk;
};

template <int K>
NA_DEV WaveIO<K> wave_io(uint32_t rec0, uint32_t lane)
{
    WaveIO<K> io;
    io.rq = rec0 + (lane >> 2) / K;
    io.c16 = 16u * (lane & 3);
    io.d16 = 16u * ((lane ^ (lane >> 4)) & 3);
    io.kk = (int)((lane >> 2) % K);
    return io;
}

template <int K>
NA_DEV uint32_t wave_rec(const WaveIO<K> &io, int i) { return io.rq + (uint32_t)i * (16 / K); }

/* Coalesced loads of the step with unit base j0 (owner unit j0 + kk, clamped
   to unit 0 below the record start, records clamped to the batch end). */
template <int K>
NA_DEV Quad wave_load(const UniformArgs &a, const WaveIO<K> &io, int j0)
{
    const int u = j0 + io.kk;
    const uint32_t off = io.c16 + 64u * (uint32_t)(u > 0 ? u : 0);
    const uint32_t last = a.n_records - 1;
    Quad P;
    P.a = *(const uint4 *)(a.in + (size_t)min(wave_rec(io, 0), last) * a.in_stride + off);
    P.b = *(const uint4 *)(a.in + (size_t)min(wave_rec(io, 1), last) * a.in_stride + off);
    P.c = *(const uint4 *)(a.in + (size_t)min(wave_rec(io, 2), last) * a.in_stride + off);
    P.d = *(const uint4 *)(a.in + (size_t)min(wave_rec(io, 3), last) * a.in_stride + off);
    return P;
}

/* The same step as wave_load, but straight into the tile by LDS-DMA
   (global_load_lds_dwordx4: no VGPRs, no ds_write).  The DMA fills the tile
   lane-linearly (slot 64i + lane), so the tile_slot swizzle moves to the
   source: slot 64i + l holds owner L = 16i + l/4, chunk (l ^ l>>4) & 3. */
template <int K>
NA_DEV void wave_dma(const UniformArgs &a, const WaveIO<K> &io, int j0, uint4 *t)
{
    const int u = j0 + io.kk;
    const uint32_t off = io.d16 + 64u * (uint32_t)(u > 0 ? u : 0);
    const uint32_t last = a.n_records - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds(
            (const void *)(a.in + (size_t)min(wave_rec(io, i), last) * a.in_stride + off),
            (lds_void *)(t + 64 * i), 16, 0, 0);
}

/* One LDS-DMA instruction (global_load_lds_dwordx4: lane l's 16 bytes land
   at LDS address lds + 16 l), written as inline asm so that hipcc does not
   see an LDS write: it would otherwise wait for the youngest such DMA before
   every later LDS access of the wave (tile reads AND writes), i.e. for the
   next step's DMA right after issuing it.  The one-lane kernels place their
   own s_waitcnt vmcnt(0) instead (solo_wait).  m0 carries the LDS address:
   m0 is reserved to the compiler (a clobber of it is not honoured), so the
   statement saves and restores it (cdna_hip_programming.md, LDS-DMA
   recipe) — the segmented kernels fault without that. */
NA_DEV void dma16_asm(const void *g, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

/* The staged kernels' coalesced step DMA (wave_dma) issued as inline asm
   (dma16_asm): hipcc does not see these LDS writes, so it does not wait for
   the youngest of them before every tile read; the caller waits itself
   (s_waitcnt vmcnt: four instructions per step). */
template <int K>
NA_DEV void wave_dma_asm(const UniformArgs &a, const WaveIO<K> &io, int j0, uint4 *t)
{
    const int u = j0 + io.kk;
    const uint32_t off = io.d16 + 64u * (uint32_t)(u > 0 ? u : 0);
    const uint32_t last = a.n_records - 1;
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)t);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        dma16_asm((const void *)(a.in + (size_t)min(wave_rec(io, i), last) * a.in_stride + off),
                  base + 1024u * (uint32_t)i);
}

/* A 16-B record store of the staged kernels: non-temporal (streaming), so
   the written lines need not displace the ciphertext lines the next step of
   an open still reads.  Round 4: the 4-lane kernels' standalone C2 seal+open
   +1.0-1.9 % in three interleaved rounds, C5 unchanged
   (profiles/r04/nt_store_ab.jsonl). */
typedef uint32_t na_u32x4 __attribute__((ext_vector_type(4)));
NA_DEV void rec_store16(uint8_t *p, const uint4 &q)
{
    na_u32x4 v = {q.x, q.y, q.z, q.w};
    __builtin_nontemporal_store(v, (na_u32x4 *)p);
}

/* Coalesced stores of the step's full units (unit <= last_full) from the
   tile; okm bit i gates instruction i (open: the owner's verdict). */
template <int K>
NA_DEV void wave_store(const UniformArgs &a, const WaveIO<K> &io, int j0, int last_full,
                       const uint4 *t, uint32_t lane, uint32_t okm)
{
    const int u = j0 + io.kk;
    if (u < 0 || u > last_full) return;
    const uint32_t off = io.c16 + 64u * (uint32_t)u;
    uint4 q[4]; /* all tile reads first: one LDS wait, not one per store (solo_store) */
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = t[tile_slot(16u * i + (lane >> 2), lane & 3)];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t r = wave_rec(io, i);
        if (r < a.n_records && ((okm >> i) & 1)) rec_store16(a.out + (size_t)r * a.out_stride + off, q[i]);
    }
}

/* FAST exact-size store of a record's last unit: nb (1..64) bytes at p
   (16-B aligned). */
NA_DEV void last_unit_out(uint8_t *p, uint32_t nb, const uint32_t w[16])
{
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c)
        if (16 * c + 16 <= nb)
            *(uint4 *)(p + 16 * c) = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    const uint32_t rem = nb & 15;
    if (rem) {
        uint32_t part[4];
        pick_chunk(w, nb >> 4, part);
        uint8_t *q = p + (nb & ~15u);
        if (rem == 8) *(uint2 *)q = make_uint2(part[0], part[1]);
        else store16(q, rem, part);
    }
}

/* FAST tag store at p = record + len (p is 16-B aligned iff len % 16 == 0). */
NA_DEV void tag_out(uint8_t *p, uint32_t len, const uint32_t t[4])
{
    if ((len & 15) == 0) {
        *(uint4 *)p = make_uint4(t[0], t[1], t[2], t[3]);
    } else if ((len & 7) == 0) {
        *(uint2 *)p = make_uint2(t[0], t[1]);
        *(uint2 *)(p + 8) = make_uint2(t[2], t[3]);
    } else {
        store16(p, 16, t);
    }
}

/* Per-lane scratch the staged seal kernel parks outside its loop: lane k's
   final Poly1305 scale (an Fe), written at step 0 and read after the loop so
   it is not held in 5 VGPRs across the ChaCha blocks. */
struct FinSlot { uint32_t l[5][64]; };

NA_DEV void fin_put(FinSlot *f, uint32_t lane, const Mul &m)
{
    f->l[0][lane] = m.r0; f->l[1][lane] = m.r1; f->l[2][lane] = m.r2;
    f->l[3][lane] = m.r3; f->l[4][lane] = m.r4;
}

NA_DEV Mul fin_get(const FinSlot *f, uint32_t lane)
{
    return mk_mul(Fe{f->l[0][lane], f->l[1][lane], f->l[2][lane], f->l[3][lane], f->l[4][lane]});
}

/* Record pointers of the uniform batch, rebuilt at each use (a handful of
   VALU) instead of being held in 64-bit VGPR pairs across the loop. */
NA_DEV const uint8_t *u_src(const UniformArgs &a, uint32_t rc) { return a.in + (size_t)rc * a.in_stride; }
NA_DEV uint8_t *u_dst(const UniformArgs &a, uint32_t rc) { return a.out + (size_t)rc * a.out_stride; }
NA_DEV const uint8_t *u_ad(const UniformArgs &a, uint32_t rc) { return a.ad + (size_t)rc * a.ad_stride; }

/* Key and nonce of record rc.  UKEY: the host guarantees that all records of
   a wave share one CipherState (recs_per_state a multiple of 64/K), so the
   key is wave-uniform and lives in SGPRs — 8 VGPRs the loop keeps free. */
template <bool UKEY>
NA_DEV void u_key_nonce(const UniformArgs &a, uint32_t rec0, uint32_t rc, uint32_t key[8],
                        uint32_t &n_lo, uint32_t &n_hi)
{
    uint64_t n;
    if constexpr (UKEY) {
        const uint32_t st = __builtin_amdgcn_readfirstlane(rec0) / a.rps;
        load_key(a.keys + (size_t)st * 32, key);
#pragma unroll
        for (int i = 0; i < 8; ++i) key[i] = __builtin_amdgcn_readfirstlane(key[i]);
        n = a.nonce_base[st] + (uint64_t)(rc - st * a.rps);
    } else {
        const uint32_t st = rc / a.rps;
        load_key(a.keys + (size_t)st * 32, key);
        n = a.nonce_base[st] + (uint64_t)(rc - st * a.rps);
    }
    n_lo = (uint32_t)n;
    n_hi = (uint32_t)(n >> 32);
}

/* wave_job: the wave's 64/K consecutive records start at wave_job * (64/K) */
template <int K, bool UKEY>
NA_DEV void seal_il_staged(const UniformArgs &a, uint4 *tiles, FinSlot *fin, uint32_t wave_job)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rec0 = wave_job * (64 / K);
    const uint32_t rec_raw = rec0 + lane / K;
    const bool live = rec_raw < a.n_records;
    const uint32_t rc = live ? rec_raw : a.n_records - 1;
    const int k = (int)(lane % K);
    uint32_t key[8], n_lo, n_hi;
    u_key_nonce<UKEY>(a, rec0, rc, key, n_lo, n_hi);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = a.len;
    const GroupCtx<K> g = group_ctx<K>(len); /* wave-uniform (uniform batch) */
    const int gbase = (int)lane & ~(K - 1);
    const WaveIO<K> io = wave_io<K>(rec0, lane);
    const int last_full = (int)g.J - 2; /* unit J-1 is stored by its owner */

    Fe acc = fe_zero();
    Mul mr, mjump;
    uint32_t s[4];
    bool seen = false;
    wave_dma_asm<K>(a, io, -(int)g.o - 1, tiles);
    for (uint32_t m = 0; m < g.steps; ++m) {
        if (a.balance) prio_by_progress(m, g.steps);
        const int j0 = (int)(m * K) - (int)g.o - 1;
        const int v = j0 + 1 + k;
        uint4 *cur = tiles + 256 * (m & 1), *nxt = tiles + 256 * ((m + 1) & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* last step's reads and writes of nxt are done */
        __builtin_amdgcn_wave_barrier();
        /* next step's bytes go into the other tile while this one computes */
        if (m + 1 < g.steps) wave_dma_asm<K>(a, io, j0 + K, nxt);
        uint32_t x[16];
        slot_block<true>(key, pre, v, n_lo, n_hi, x, a.balance && 2 * m < g.steps);
        if (m == 0) {
            Fe r;
            poly_key_bcast(x, gbase + (int)g.o, r, s);
            mr = mk_mul(r);
            Mul mfinal;
            poly_powers<K>(r, k, g.q, mjump, mfinal);
            fin_put(fin, lane, mfinal);
            const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
            if (k == k0 && a.ad_len) poly_ad(acc, mr, u_ad(a, rc), a.ad_len);
        }
        __builtin_amdgcn_wave_barrier();
        /* this step's DMA (a step old) landed; the next step's may still fly */
        if (m + 1 < g.steps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t w[16];
        tile_get_unit(cur, lane, w);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        if (v >= 1 && (uint32_t)v <= g.J) {
            /* one Poly path for full units and the last (lane K-1's last
               step), so a wave never runs both */
            uint32_t nb = 4;
            if ((uint32_t)v == g.J) {
                const uint32_t bytes = len - 64 * (g.J - 1);
                if (live) last_unit_out(u_dst(a, rc) + 64 * (g.J - 1), bytes, w);
                mask_unit(w, bytes);
                nb = (bytes + 15) / 16;
            }
            poly_unit(acc, seen ? mjump : mr, mr, w, nb);
            seen = true;
        }
        tile_put_unit(cur, lane, w);
        __builtin_amdgcn_wave_barrier();
        wave_store<K>(a, io, j0, last_full, cur, lane, 0xfu);
    }
    uint32_t tag[4];
    poly_close<K>(acc, k, mr, fin_get(fin, lane), a.ad_len, len, s, tag);
    if (k == K - 1 && live) tag_out(u_dst(a, rc) + len, len, tag);
}

/* Open, single pass (the structure of seal_il_staged): each step's
   ciphertext unit goes through Poly1305 and, XORed with its key stream, out
   as plaintext, so the ciphertext is read once.  The verdict comes after the
   plaintext is written; a wave holding a rejected record then runs a repair
   pass (taken only on MAC failure): in place it re-encrypts that record's
   plaintext back into the ciphertext it was given — the buffer reads as
   untouched, as after the reference's verify-then-decrypt
   (cipher-chachapoly.c:140-150) — and out of place it zeroes the record's
   output (scrub_rejected's contract). */
template <int K, bool UKEY>
NA_DEV void open_il_staged(const UniformArgs &a, uint4 *tiles, FinSlot *fin, uint32_t wave_job)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rec0 = wave_job * (64 / K);
    const uint32_t rec_raw = rec0 + lane / K;
    const bool live = rec_raw < a.n_records;
    const uint32_t rc = live ? rec_raw : a.n_records - 1;
    const int k = (int)(lane % K);
    uint32_t key[8], n_lo, n_hi;
    u_key_nonce<UKEY>(a, rec0, rc, key, n_lo, n_hi);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = a.len;
    const GroupCtx<K> g = group_ctx<K>(len);
    const int gbase = (int)lane & ~(K - 1);
    const WaveIO<K> io = wave_io<K>(rec0, lane);
    const int last_full = (int)g.J - 2;
    const uint32_t tail = g.J ? len - 64 * (g.J - 1) : 0; /* bytes of unit J-1 */

    Fe acc = fe_zero();
    Mul mr, mjump;
    uint32_t s[4];
    bool seen = false;
    wave_dma_asm<K>(a, io, -(int)g.o - 1, tiles);
    for (uint32_t m = 0; m < g.steps; ++m) {
        if (a.balance) prio_by_progress(m, g.steps);
        const int j0 = (int)(m * K) - (int)g.o - 1;
        const int v = j0 + 1 + k;
        uint4 *cur = tiles + 256 * (m & 1), *nxt = tiles + 256 * ((m + 1) & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* last step's reads and writes of nxt are done */
        __builtin_amdgcn_wave_barrier();
        if (m + 1 < g.steps) wave_dma_asm<K>(a, io, j0 + K, nxt);
        uint32_t x[16];
        slot_block<true>(key, pre, v, n_lo, n_hi, x, a.balance && 2 * m < g.steps);
        if (m == 0) {
            Fe r;
            poly_key_bcast(x, gbase + (int)g.o, r, s);
            mr = mk_mul(r);
            Mul mfinal;
            poly_powers<K>(r, k, g.q, mjump, mfinal);
            fin_put(fin, lane, mfinal);
            const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
            if (k == k0 && a.ad_len) poly_ad(acc, mr, u_ad(a, rc), a.ad_len);
        }
        __builtin_amdgcn_wave_barrier();
        /* this step's DMA (a step old) landed; the next step's may still fly */
        if (m + 1 < g.steps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t w[16];
        tile_get_unit(cur, lane, w);
        if (v >= 1 && (uint32_t)v <= g.J) {
            uint32_t nb = 4;
            if ((uint32_t)v == g.J) { /* bytes past len are never stored */
                mask_unit(w, tail);
                nb = (tail + 15) / 16;
            }
            poly_unit(acc, seen ? mjump : mr, mr, w, nb);
            seen = true;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        if (v >= 1 && (uint32_t)v == g.J && live) last_unit_out(u_dst(a, rc) + 64 * (g.J - 1), tail, w);
        tile_put_unit(cur, lane, w);
        __builtin_amdgcn_wave_barrier();
        wave_store<K>(a, io, j0, last_full, cur, lane, 0xfu);
    }
    uint32_t tag[4], got[4];
    poly_close<K>(acc, k, mr, fin_get(fin, lane), a.ad_len, len, s, tag);
    tag_in<true>(u_src(a, rc), len, got); /* the tag bytes are never written */
    const bool ok = tag_equal(tag, got);
    if (k == K - 1 && live && a.status) a.status[rec_raw] = ok ? 0 : 1;
    const bool bad = live && !ok;
    if (__ballot(bad) == 0) return; /* wave-uniform: the common case */

    /* repair pass: bit i of badm = the owner coalesced instruction i serves */
    uint32_t badm = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        badm |= (__shfl((int)bad, (int)(16u * i + (lane >> 2)), 64) != 0 ? 1u : 0u) << i;
    const bool inplace = a.in == a.out && a.in_stride == a.out_stride;
    __threadfence(); /* this wave's plaintext stores, visible to its reads below */
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int j0 = (int)(m * K) - (int)g.o - 1;
        const int v = j0 + 1 + k;
        uint32_t w[16];
        __builtin_amdgcn_wave_barrier();
        if (inplace) {
            wave_dma<K>(a, io, j0, tiles);
            uint32_t x[16];
            chacha20_block_pre(key, pre, (uint32_t)v, n_lo, n_hi, x);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            tile_get_unit(tiles, lane, w);
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = 0;
        }
        if (v >= 1 && (uint32_t)v == g.J && bad) last_unit_out(u_dst(a, rc) + 64 * (g.J - 1), tail, w);
        __builtin_amdgcn_wave_barrier();
        tile_put_unit(tiles, lane, w);
        __builtin_amdgcn_wave_barrier();
        wave_store<K>(a, io, j0, last_full, tiles, lane, badm);
    }
}

/* ---------------- one lane per record, LDS-staged (uniform FAST batches)
 *
 * Round 4.  Every lane owns a whole record: its ChaCha blocks 0..J in order
 * and ONE Poly1305 Horner chain over the record's blocks with the clamped r
 * itself, so every Poly block is a radix-2^32 p32_block (20 v_mad_u64_u32, no
 * limb split) and there is no r^(4K-3) jump, no per-lane power of r and no
 * group sum — the per-record work of the 4-lane kernels (powers, group sum,
 * tag) is paid once per 64 records instead of once per 16.  Per 1400-B
 * record: 23 ChaCha blocks (no end-alignment slot) + 89 p32 blocks.
 *
 * A step moves two units (128 B, one whole line of the 128-B record slots)
 * of all 64 records of the wave through an 8 KB LDS tile, double-buffered:
 * LDS-DMA instruction i (0..7) fills slots 64i..64i+63 with the 128-B runs
 * of records 8i..8i+7, so every instruction covers eight whole lines, and
 * the stores leave the same way.  Owner L's chunk c (0..7) sits in slot
 * 8L + (c ^ (L & 7)): the XOR makes the owner-side ds_*_b128 (lanes 8 apart
 * in the same chunk) bank-conflict-free.  16 KB of LDS per wave caps a CU at
 * 8 waves (two per SIMD), which is all a VALU-bound wave needs: one wave
 * issues the ChaCha stream at ~4.15 cycles per instruction on its own
 * (DESIGN §5), and the 64 Ki records of C2 are 1024 waves per job.
 */
constexpr uint32_t SOLO_TILE = 512; /* uint4 slots per tile: 64 owners x 8 chunks */

NA_DEV void p32_ad(P32 &acc, const R32 &r, const uint8_t *ad, uint32_t ad_len);
NA_DEV void p32_unit(P32 &acc, const R32 &r, const uint32_t c[16], uint32_t nb);

NA_DEV uint32_t solo_slot(uint32_t L, uint32_t c) { return L * 8 + (c ^ (L & 7)); }

/* chunk this lane moves in a coalesced instruction (slot 64i + lane holds
   owner 8i + lane/8, chunk (lane ^ lane/8) & 7) */
NA_DEV uint32_t solo_chunk(uint32_t lane) { return (lane ^ (lane >> 3)) & 7; }

/* every vector-memory operation of the wave done (the DMA into the tile
   about to be read, issued a step earlier, and the stores issued with it) */
NA_DEV void solo_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

/* all but the youngest 8 (one step's DMA) done: the AUTH pass keeps two
   steps in flight */
NA_DEV void solo_wait_step_old() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }

/* DMA of step m (units 2m, 2m+1) of the wave's records into tile t.  Chunks
   at or past lim (= 64 J, the end of the record's last unit) re-read the
   step's first unit instead: FAST slots are only readable up to
   roundup64(len). */
NA_DEV void solo_dma(const UniformArgs &a, uint32_t rec0, uint32_t lane, uint32_t m,
                     uint32_t lim, uint4 *t)
{
    const uint32_t c = solo_chunk(lane);
    uint32_t off = 128u * m + 16u * c;
    if (off >= lim) off -= 64u;
    const uint32_t last = a.n_records - 1;
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)t);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        dma16_asm((const void *)(a.in + (size_t)min(rec0 + 8u * i + (lane >> 3), last) * a.in_stride + off),
                  base + 1024u * (uint32_t)i);
}

/* coalesced stores of step m's chunks below full_lim (the full units before
   the record's last one; the owner stores that one exactly); okm bit i gates
   instruction i */
NA_DEV void solo_store(const UniformArgs &a, uint32_t rec0, uint32_t lane, uint32_t m,
                       uint32_t full_lim, const uint4 *t, uint32_t okm)
{
    const uint32_t off = 128u * m + 16u * solo_chunk(lane);
    if (off + 16u > full_lim) return;
    /* The eight tile reads first and one wait for them: with a read inside
       each conditional store hipcc waited on every read in turn (eight LDS
       round trips per step).  The explicit wait also orders the reads before
       the caller's next LDS-DMA into this tile (dma16_asm: hipcc does not
       see that write). */
    uint4 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = t[64 * i + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t r = rec0 + 8u * i + (lane >> 3);
        /* non-temporal (rec_store16): the one-lane kernels' store pattern
           (8 x 128 B per instruction) alone runs at 4.9 vs 3.8 TB/s, and C4 /
           perf gain 1-3 % (tools/microbench/solo_dma.hip,
           profiles/r04/nt_store_ab.jsonl) */
        if (r < a.n_records && ((okm >> i) & 1)) rec_store16(a.out + (size_t)r * a.out_stride + off, q[i]);
    }
}

NA_DEV void solo_get(const uint4 *t, uint32_t L, uint32_t u, uint32_t w[16])
{
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) {
        const uint4 v = t[solo_slot(L, 4 * u + c)];
        w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
    }
}

NA_DEV void solo_put(uint4 *t, uint32_t L, uint32_t u, const uint32_t w[16])
{
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c)
        t[solo_slot(L, 4 * u + c)] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
}

/* Poly key block 0: r (clamped, radix 2^32), s; AD absorbed. */
NA_DEV void solo_poly_key(const uint32_t key[8], const ChaPre &pre, uint32_t n_lo, uint32_t n_hi,
                          const uint8_t *ad, uint32_t ad_len, R32 &r, uint32_t s[4], P32 &h)
{
    uint32_t x[16];
    chacha20_block_pre(key, pre, 0u, n_lo, n_hi, x);
    r = r32_from_key(x[0], x[1], x[2], x[3]);
    s[0] = x[4]; s[1] = x[5]; s[2] = x[6]; s[3] = x[7];
    h = p32_zero();
    if (ad_len) p32_ad(h, r, ad, ad_len);
}

NA_DEV void solo_tag(P32 h, const R32 &r, uint32_t ad_len, uint32_t len, const uint32_t s[4],
                     uint32_t tag[4])
{
    p32_block(h, r, ad_len, 0u, len, 0u);
    fe_finish(p32_to_fe(h), s, tag);
}

/* Per-lane view of a wave's 64 records in the one-lane kernels. */
struct SoloRec {
    uint32_t lane, rec0, rec_raw, rc, len, J, S, lim, full_lim, tail;
    bool live;
};

NA_DEV SoloRec solo_rec(const UniformArgs &a, uint32_t wave_job)
{
    SoloRec q;
    q.lane = threadIdx.x & 63;
    q.rec0 = wave_job * 64u;
    q.rec_raw = q.rec0 + q.lane;
    q.live = q.rec_raw < a.n_records;
    q.rc = q.live ? q.rec_raw : a.n_records - 1;
    q.len = a.len;
    q.J = (q.len + 63) / 64;
    q.S = (q.J + 1) / 2;
    q.lim = 64u * q.J;
    q.full_lim = q.J ? 64u * (q.J - 1) : 0u; /* the full units before the last */
    q.tail = q.len - q.full_lim;             /* bytes of unit J-1 */
    return q;
}

/* The one pass over a wave's records (seal: plaintext -> CT; open: CT ->
   plaintext, Poly1305 over the CT as read), leaving the Horner value in h.
   Order inside step m, chosen so that every wait for memory is for work
   issued a whole step earlier:
     wait   -- DMA(m), issued during step m-1, and the stores of step m-2
     read   -- step m's two units, tile m&1 -> registers
     store  -- step m-1's output, still in the other tile, leaves
     DMA    -- step m+1's units into that other tile
     compute-- two ChaCha blocks, Poly1305, output into tile m&1
   (hipcc waits before an LDS read for the youngest LDS-DMA; reading the tile
   after issuing the next DMA, as the 4-lane kernels do, made every step wait
   for the DMA it had just issued and serialised the stores behind it.) */
/* The key stream of a one-lane step: blocks c0 and c0 + 1 of the lane's
   record in lock step, issued in runs, rotate runs at s_setprio 2 and fast
   runs at 0 (aead_device.h chacha20_2block_runs; round 6).  Measured
   against hipcc's schedule of two chacha20_block_pre calls, interleaved on
   one box (profiles/r06/runs_ab/): C2 duplex +4 %, C4 +10 %, perf +8 %,
   C5 +5 %; toggles 3 / 1 measured the same, runs without the toggles
   nothing.  A standalone one-lane launch of < 2 waves per SIMD lost 11 %
   with it (a lone wave has no partner to fill the slots a rotate run
   leaves), so those keep hipcc's schedule (RUNS = false).
   early (a launch of one generation, UniformArgs.balance, in the first half
   of the wave's steps): the toggles one level up, 3 / 1 — the progress
   balance of prio_by_progress, which the toggles override, in two levels:
   C2 duplex 1497-1530 -> 1555-1612 GiB/s in three interleaved rounds, while
   with it at C4 (16 generations) 1736-1741 -> 1716-1726, hence the
   one-generation condition (profiles/r06/prio_ab/). */
template <bool RUNS>
NA_DEV void solo_blocks2(const uint32_t key[8], const ChaPre &pre, uint32_t c0, uint32_t n_lo, uint32_t n_hi,
                         uint32_t (&x0)[16], uint32_t (&x1)[16], bool early = false)
{
    if constexpr (RUNS) {
        if (early) chacha20_2block_runs<3, 1, 1>(key, pre, c0, c0 + 1, n_lo, n_hi, x0, x1);
        else chacha20_2block_runs<2, 0, 0>(key, pre, c0, c0 + 1, n_lo, n_hi, x0, x1);
    } else {
        chacha20_block_pre(key, pre, c0, n_lo, n_hi, x0);
        chacha20_block_pre(key, pre, c0 + 1, n_lo, n_hi, x1);
    }
}

/* solo_pass modes: SEAL and OPEN1 (the opt-in one-pass open,
   NOISE_AEAD_FLAG_ONE_PASS) as above; the verify-first open (the default)
   runs solo_auth and then solo_dec_rev (below). */
enum SoloMode { SOLO_SEAL, SOLO_OPEN1 };

template <int MODE, bool RUNS>
NA_DEV void solo_pass(const UniformArgs &a, const SoloRec &q, uint4 *tiles, const uint32_t key[8],
                      const ChaPre &pre, uint32_t n_lo, uint32_t n_hi, const R32 &r, P32 &h)
{
    constexpr uint32_t okm = 0xffu;
    for (uint32_t m = 0; m < q.S; ++m) {
        uint4 *cur = tiles + SOLO_TILE * (m & 1), *nxt = tiles + SOLO_TILE * ((m + 1) & 1);
        uint32_t wu[2][16];
        solo_wait();
        solo_get(cur, q.lane, 0, wu[0]);
        solo_get(cur, q.lane, 1, wu[1]);
        if (m >= 1) solo_store(a, q.rec0, q.lane, m - 1, q.full_lim, nxt, okm);
        __builtin_amdgcn_wave_barrier();
        if (m + 1 < q.S) solo_dma(a, q.rec0, q.lane, m + 1, q.lim, nxt);
        /* Two waves share a SIMD and the older one takes the issue slots:
           without this the pair ran nearly one after the other and the
           second finished alone, at one wave's issue rate.  A wave that is
           ahead lowers its priority (aead_device.h): C2 +5-8 %, C4 +0.5 %
           (profiles/r04/solo_prio_ab.jsonl). */
        prio_by_progress(m, q.S);
        uint32_t xs[2][16];
        if constexpr (RUNS) solo_blocks2<true>(key, pre, 2 * m + 1, n_lo, n_hi, xs[0], xs[1], a.balance && 2 * m < q.S);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t j = 2 * m + u; /* unit, ChaCha block j + 1 */
            if (j < q.J) {
                uint32_t x[16], w[16];
                if constexpr (RUNS) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] = xs[u][i];
                } else {
                    chacha20_block_pre(key, pre, j + 1, n_lo, n_hi, x);
                }
                uint32_t nb = 4;
                if constexpr (MODE == SOLO_OPEN1) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = wu[u][i];
                    if (j == q.J - 1) { /* bytes past len are never stored */
                        mask_unit(w, q.tail);
                        nb = (q.tail + 15) / 16;
                    }
                    p32_unit(h, r, w, nb);
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] ^= x[i];
                    if (j == q.J - 1 && q.live) last_unit_out(u_dst(a, q.rc) + q.full_lim, q.tail, w);
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = wu[u][i] ^ x[i];
                    if (j == q.J - 1) {
                        if (q.live) last_unit_out(u_dst(a, q.rc) + q.full_lim, q.tail, w);
                        mask_unit(w, q.tail);
                        nb = (q.tail + 15) / 16;
                    }
                    p32_unit(h, r, w, nb);
                }
                solo_put(cur, q.lane, u, w);
            }
        }
    }
    if (q.S) {
        __builtin_amdgcn_wave_barrier();
        solo_store(a, q.rec0, q.lane, q.S - 1, q.full_lim, tiles + SOLO_TILE * ((q.S - 1) & 1), okm);
    }
}

template <bool UKEY, bool RUNS>
NA_DEV void seal_solo_staged(const UniformArgs &a, uint4 *tiles, uint32_t wave_job)
{
    const SoloRec q = solo_rec(a, wave_job);
    uint32_t key[8], n_lo, n_hi;
    u_key_nonce<UKEY>(a, q.rec0, q.rc, key, n_lo, n_hi);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    if (q.S) solo_dma(a, q.rec0, q.lane, 0, q.lim, tiles);
    R32 r;
    uint32_t s[4];
    P32 h;
    solo_poly_key(key, pre, n_lo, n_hi, a.ad_len ? u_ad(a, q.rc) : nullptr, a.ad_len, r, s, h);
    solo_pass<SOLO_SEAL, RUNS>(a, q, tiles, key, pre, n_lo, n_hi, r, h);
    uint32_t tag[4];
    solo_tag(h, r, a.ad_len, q.len, s, tag);
    if (q.live) tag_out(u_dst(a, q.rc) + q.len, q.len, tag);
}

/* The verify-first open's AUTH pass: Poly1305 over the ciphertext only,
   nothing stored, so both tiles serve as a two-deep queue — a step's units
   are read into registers and the tile takes the DMA two steps ahead
   (DMA(0) was issued by the caller).  At top priority: it takes the issue
   slots it needs as its loads land while the SIMD's other wave computes
   (tools/microbench/timeline_solo.hip, steady state: 133 -> 125 us per C2
   duplex launch; at the default priority the seal wave beside it starved
   it). */
NA_DEV void solo_auth(const UniformArgs &a, const SoloRec &q, uint4 *tiles, const R32 &r, P32 &h)
{
    if (q.S > 1) solo_dma(a, q.rec0, q.lane, 1, q.lim, tiles + SOLO_TILE);
    for (uint32_t m = 0; m < q.S; ++m) {
        uint4 *cur = tiles + SOLO_TILE * (m & 1);
        uint32_t wu[2][16];
        if (m + 1 < q.S) solo_wait_step_old();
        else solo_wait();
        solo_get(cur, q.lane, 0, wu[0]);
        solo_get(cur, q.lane, 1, wu[1]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the tile is read before the DMA refills it */
        __builtin_amdgcn_wave_barrier();
        if (m + 2 < q.S) solo_dma(a, q.rec0, q.lane, m + 2, q.lim, cur);
                __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t j = 2 * m + u;
            if (j < q.J) {
                uint32_t nb = 4;
                if (j == q.J - 1) {
                    mask_unit(wu[u], q.tail);
                    nb = (q.tail + 15) / 16;
                }
                p32_unit(h, r, wu[u], nb);
            }
        }
    }
}

/* The verify-first open's DEC pass from the last step back to the first:
   key-stream blocks are independent of each other, and the AUTH pass leaves
   steps S-1 and S-2 in the two tiles (it refills a tile with step m+2 only
   while m+2 < S), so those two are decrypted without reading them again and
   the pass starts without a DMA wait.  Per step: the wait, the read of step
   m, the store of step m+1's output from the other tile (gated by okm, the
   owners' verdicts per coalesced instruction), the DMA of step m-1 into it,
   the key stream into this tile.  Round 5 measured it against the forward
   order: C2 verify-first 1396-1431 -> 1460-1468 GiB/s, three interleaved
   rounds (profiles/r05/dec_rev_ab.txt; the forward pass is NA_DEC_REV=0 at
   the ab-arms-r5 revision, tools/ab/README.md); the last steps read by the
   AUTH pass are also the likeliest still in L2. */
template <bool RUNS>
NA_DEV void solo_dec_rev(const UniformArgs &a, const SoloRec &q, uint4 *tiles, const uint32_t key[8],
                         const ChaPre &pre, uint32_t n_lo, uint32_t n_hi, uint32_t okm, bool ok)
{
    for (uint32_t k = 0; k < q.S; ++k) {
        const uint32_t m = q.S - 1 - k;
        uint4 *cur = tiles + SOLO_TILE * (m & 1), *nxt = tiles + SOLO_TILE * ((m + 1) & 1);
        uint32_t wu[2][16];
        solo_wait();
        solo_get(cur, q.lane, 0, wu[0]);
        solo_get(cur, q.lane, 1, wu[1]);
        if (k >= 1) solo_store(a, q.rec0, q.lane, m + 1, q.full_lim, nxt, okm);
        __builtin_amdgcn_wave_barrier();
        if (k >= 1 && m >= 1) solo_dma(a, q.rec0, q.lane, m - 1, q.lim, nxt); /* k = 0: step S-2 is there */
        prio_by_progress(k, q.S);
        uint32_t xs[2][16];
        if constexpr (RUNS) solo_blocks2<true>(key, pre, 2 * m + 1, n_lo, n_hi, xs[0], xs[1], a.balance && 2 * k < q.S);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t j = 2 * m + u;
            if (j < q.J) {
                uint32_t x[16], w[16];
                if constexpr (RUNS) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] = xs[u][i];
                } else {
                    chacha20_block_pre(key, pre, j + 1, n_lo, n_hi, x);
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = wu[u][i] ^ x[i];
                if (j == q.J - 1 && q.live && ok) last_unit_out(u_dst(a, q.rc) + q.full_lim, q.tail, w);
                solo_put(cur, q.lane, u, w);
            }
        }
    }
    if (q.S) {
        __builtin_amdgcn_wave_barrier();
        solo_store(a, q.rec0, q.lane, 0, q.full_lim, tiles, okm);
    }
}


/* Open.  Verify-first (a.vf: the default, the reference's order,
   cipher-chachapoly.c:135-141): an AUTH pass over the wave's records, the
   verdicts, then a DEC pass writing only verified records — a rejected
   record's output is never written.  One pass (NOISE_AEAD_FLAG_ONE_PASS):
   Poly1305 over each ciphertext unit as it arrives, then the plaintext out;
   a wave holding a rejected record repairs it after the verdict exactly as
   open_il_staged does (in place: XOR with the key stream once more; out of
   place: zeroed).  The DEC pass reads the ciphertext
   again, mostly from L2 / MALL (a wave's 64 records are ~90 KB). */
template <bool UKEY, bool RUNS>
NA_DEV void open_solo_staged(const UniformArgs &a, uint4 *tiles, uint32_t wave_job)
{
    const SoloRec q = solo_rec(a, wave_job);
    const uint32_t lane = q.lane, rec0 = q.rec0, rec_raw = q.rec_raw, rc = q.rc, len = q.len;
    const uint32_t J = q.J, S = q.S, lim = q.lim, full_lim = q.full_lim, tail = q.tail;
    const bool live = q.live;
    uint32_t key[8], n_lo, n_hi;
    u_key_nonce<UKEY>(a, rec0, rc, key, n_lo, n_hi);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    if (S) solo_dma(a, rec0, lane, 0, lim, tiles);
    R32 r;
    uint32_t s[4];
    P32 h;
    solo_poly_key(key, pre, n_lo, n_hi, a.ad_len ? u_ad(a, rc) : nullptr, a.ad_len, r, s, h);
    if (a.vf) solo_auth(a, q, tiles, r, h);
    else solo_pass<SOLO_OPEN1, RUNS>(a, q, tiles, key, pre, n_lo, n_hi, r, h);
    uint32_t tag[4], got[4];
    solo_tag(h, r, a.ad_len, len, s, tag);
    tag_in<true>(u_src(a, rc), len, got); /* the tag bytes are never written */
    const bool ok = tag_equal(tag, got);
    if (live && a.status) a.status[rec_raw] = ok ? 0 : 1;
#ifndef NA_SOLO_AUTH_HOOK
#define NA_SOLO_AUTH_HOOK() /* tools/microbench/timeline_solo.hip stamps the AUTH pass's end here */
#endif
    NA_SOLO_AUTH_HOOK();
    if (a.vf) {
        if (__ballot(live && ok) == 0) return;
        uint32_t okm = 0; /* bit i: the owner coalesced instruction i serves verified */
#pragma unroll
        for (int i = 0; i < 8; ++i)
            okm |= (__shfl((int)ok, (int)(8u * i + (lane >> 3)), 64) != 0 ? 1u : 0u) << i;
        __builtin_amdgcn_wave_barrier(); /* the AUTH pass's tile reads are done */
        solo_dec_rev<RUNS>(a, q, tiles, key, pre, n_lo, n_hi, okm, ok);
        return;
    }
    const bool bad = live && !ok;
    if (__ballot(bad) == 0) return; /* wave-uniform: the common case */

    /* repair pass: bit i of badm = the owner coalesced instruction i serves */
    uint32_t badm = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        badm |= (__shfl((int)bad, (int)(8u * i + (lane >> 3)), 64) != 0 ? 1u : 0u) << i;
    const bool inplace = a.in == a.out && a.in_stride == a.out_stride;
    __threadfence(); /* this wave's plaintext stores, visible to its reads below */
    for (uint32_t m = 0; m < S; ++m) {
        __builtin_amdgcn_wave_barrier();
        if (inplace) solo_dma(a, rec0, lane, m, lim, tiles);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t j = 2 * m + u;
            if (j < J) {
                uint32_t w[16];
                if (inplace) {
                    uint32_t x[16];
                    chacha20_block_pre(key, pre, j + 1, n_lo, n_hi, x);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_wave_barrier();
                    solo_get(tiles, lane, u, w);
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] ^= x[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = 0;
                }
                if (j == J - 1 && bad) last_unit_out(u_dst(a, rc) + full_lim, tail, w);
                __builtin_amdgcn_wave_barrier();
                solo_put(tiles, lane, u, w);
            }
        }
        __builtin_amdgcn_wave_barrier();
        solo_store(a, rec0, lane, m, full_lim, tiles, badm);
    }
}

/* ------------------------------------------------- contiguous (K = 1, 2) */

NA_DEV void p32_ad(P32 &acc, const R32 &r, const uint8_t *ad, uint32_t ad_len)
{
    for (uint32_t off = 0; off < ad_len; off += 16) {
        uint32_t w[4];
        const uint32_t n = ad_len - off;
        load16(ad + off, n >= 16 ? 16u : n, w);
        p32_block(acc, r, w[0], w[1], w[2], w[3]);
    }
}

NA_DEV void p32_unit(P32 &acc, const R32 &r, const uint32_t c[16], uint32_t nb)
{
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b)
        if (b < nb) p32_block(acc, r, c[4 * b], c[4 * b + 1], c[4 * b + 2], c[4 * b + 3]);
}

struct CtPlan {
    uint32_t J, nblk, P, v0, v1, M;
    bool holds_last;
};

template <int G>
NA_DEV CtPlan ct_plan(uint32_t len, int k)
{
    CtPlan p;
    p.J = (len + 63) / 64;
    p.nblk = p.J + 1;
    p.P = (p.nblk + G - 1) / G;
    p.v0 = (uint32_t)k * p.P;
    p.v1 = min(p.v0 + p.P, p.nblk);
    p.M = (len + 15) / 16;
    p.holds_last = p.v0 < p.nblk && p.v1 == p.nblk;
    return p;
}

/* Length block on the last lane; with G = 2 lane 0 scaled by r^A; + s. */
template <int G>
NA_DEV void ct_close(P32 acc, const CtPlan &p, int k, const R32 &r, const Fe &r26,
                     uint64_t ad_len, uint64_t len, const uint32_t s[4], uint32_t tag[4])
{
    if (p.holds_last)
        p32_block(acc, r, (uint32_t)ad_len, (uint32_t)(ad_len >> 32), (uint32_t)len,
                  (uint32_t)(len >> 32));
    Fe a = p32_to_fe(acc);
    if constexpr (G == 2) {
        /* Poly blocks after lane 0's run: lane 1's units + the length block */
        const uint32_t A = p.nblk > p.P ? p.M - 4 * (p.P - 1) + 1 : 0u;
        const Fe rA = fe_pow_uniform(r26, A);
        if (k == 0) a = fe_mul(a, mk_mul(rA));
        a = fe_group_sum<2>(a);
    }
    fe_finish(a, s, tag);
}

template <int G>
NA_DEV void key_words_bcast(const uint32_t x[16], int gbase, uint32_t kw[8])
{
#pragma unroll
    for (int i = 0; i < 8; ++i) kw[i] = G == 1 ? x[i] : (uint32_t)__shfl((int)x[i], gbase, 64);
}

template <int G, bool FAST>
NA_DEV void seal_ct(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint32_t n_lo = (uint32_t)rv.nonce, n_hi = (uint32_t)(rv.nonce >> 32);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = rv.len;
    const CtPlan p = ct_plan<G>(len, k);
    const int gbase = (int)(threadIdx.x & 63) & ~(G - 1);

    uint32_t wn[16], wc[16], x[16], wt[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) wn[i] = wt[i] = 0;
    unit_prefetch<FAST>(rv.src, p.v0 >= 1 && p.v0 < p.v1, p.v0 - 1, len, wn);
    P32 acc = p32_zero();
    R32 r;
    Fe r26;
    uint32_t s[4];
    for (uint32_t m = 0; m < p.P; ++m) {
        const uint32_t v = p.v0 + m;
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        unit_prefetch<FAST>(rv.src, v + 1 < p.v1, v, len, wn); /* unit of block v+1 */
        chacha20_block_pre(key, pre, v, n_lo, n_hi, x);
        if (m == 0) {
            uint32_t kw[8];
            key_words_bcast<G>(x, gbase, kw);
            r = r32_from_key(kw[0], kw[1], kw[2], kw[3]);
            r26 = fe_clamp_r(kw[0], kw[1], kw[2], kw[3]);
            s[0] = kw[4]; s[1] = kw[5]; s[2] = kw[6]; s[3] = kw[7];
            if (k == 0 && rv.ad_len) p32_ad(acc, r, rv.ad, rv.ad_len);
        }
        if (v >= 1 && v < p.v1) {
            uint32_t w[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
            if (v < p.J) {
                unit_out_full<FAST>(rv.dst + 64 * (v - 1), w);
                p32_unit(acc, r, w, 4);
            } else { /* the last unit */
                const uint32_t nb = len - 64 * (v - 1);
                mask_unit(w, nb);
                p32_unit(acc, r, w, (nb + 15) / 16);
#pragma unroll
                for (int i = 0; i < 16; ++i) wt[i] = w[i];
            }
        }
    }
    uint32_t tag[4];
    ct_close<G>(acc, p, k, r, r26, rv.ad_len, len, s, tag);
    if (p.holds_last) tail_out<FAST, true>(rv.dst, p.J, len, wt, tag);
}

template <int G, bool FAST>
NA_DEV bool open_ct(const RecView &rv, int k)
{
    uint32_t key[8];
    load_key(rv.key, key);
    const uint32_t n_lo = (uint32_t)rv.nonce, n_hi = (uint32_t)(rv.nonce >> 32);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = rv.len;
    const CtPlan p = ct_plan<G>(len, k);
    const int gbase = (int)(threadIdx.x & 63) & ~(G - 1);

    uint32_t x0[16];
    chacha20_block_pre(key, pre, p.v0, n_lo, n_hi, x0);
    uint32_t kw[8];
    key_words_bcast<G>(x0, gbase, kw);
    const R32 r = r32_from_key(kw[0], kw[1], kw[2], kw[3]);
    const Fe r26 = fe_clamp_r(kw[0], kw[1], kw[2], kw[3]);
    const uint32_t s[4] = {kw[4], kw[5], kw[6], kw[7]};
    P32 acc = p32_zero();
    if (k == 0 && rv.ad_len) p32_ad(acc, r, rv.ad, rv.ad_len);

    /* phase 1: authenticate (one unit ahead) */
    const uint32_t u0 = p.v0 >= 1 ? p.v0 : 1u; /* first block with data */
    uint32_t wn[16], wc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) wn[i] = 0;
    unit_prefetch<FAST>(rv.src, u0 < p.v1, u0 - 1, len, wn);
    for (uint32_t v = u0; v < p.v1; ++v) {
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        unit_prefetch<FAST>(rv.src, v + 1 < p.v1, v, len, wn);
        uint32_t nb = 4;
        if (v == p.J) {
            const uint32_t bytes = len - 64 * (v - 1);
            mask_unit(wc, bytes);
            nb = (bytes + 15) / 16;
        }
        p32_unit(acc, r, wc, nb);
    }
    uint32_t tag[4], got[4];
    ct_close<G>(acc, p, k, r, r26, rv.ad_len, len, s, tag);
    tag_in<FAST>(rv.src, len, got);
    if (!tag_equal(tag, got)) return false;

    /* phase 2: decrypt; the ciphertext re-read is served by L2 */
    unit_prefetch<FAST>(rv.src, u0 < p.v1, u0 - 1, len, wn);
    for (uint32_t v = u0; v < p.v1; ++v) {
#pragma unroll
        for (int i = 0; i < 16; ++i) wc[i] = wn[i];
        unit_prefetch<FAST>(rv.src, v + 1 < p.v1, v, len, wn);
        uint32_t x[16];
        if (v == p.v0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = x0[i];
        } else {
            chacha20_block_pre(key, pre, v, n_lo, n_hi, x);
        }
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = wc[i] ^ x[i];
        if (v < p.J) unit_out_full<FAST>(rv.dst + 64 * (v - 1), w);
        else tail_out<FAST, false>(rv.dst, p.J, len, w, nullptr);
    }
    return true;
}

/* ------------------------------------------------------------- kernels */

/* 4 waves per SIMD: one C2-sized batch (64 Ki records, 4 lanes each) is then
   exactly one resident round of the 1024 SIMDs */
#define NA_UNIFORM_OCC __attribute__((amdgpu_waves_per_eu(4)))

/* lanes per record: 1 or 2 -> contiguous runs, 4 .. 64 -> interleaved units */
template <int K, bool FAST>
NA_DEV void seal_any(const RecView &rv, int k)
{
    if constexpr (K <= 2) seal_ct<K, FAST>(rv, k);
    else seal_il<K, FAST>(rv, k);
}

template <int K, bool FAST>
NA_DEV bool open_any(const RecView &rv, int k)
{
    if constexpr (K <= 2) return open_ct<K, FAST>(rv, k);
    else return open_il<K, FAST>(rv, k);
}

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

/* the grid-wide wave index of this thread's wave in workgroup b */
NA_DEV uint32_t wave_of(uint32_t b) { return (b * 256u + threadIdx.x) >> 6; }

/* LDS-staged uniform FAST batches, K = 4 or 8 lanes per record */
/* Verify-first open with K lanes per record (round 6): the reference's order
   (cipher-chachapoly.c:135-141) at the staged kernels' four waves per SIMD,
   for standalone opens (the one-lane verify-first open holds one wave per
   SIMD at 64 Ki records).
     AUTH: Poly1305 over the ciphertext only, the two tiles a two-step DMA
           queue (inline-asm DMA, explicit waits), at top priority;
     DEC:  verified waves only — the one-pass loop's key stream and XOR, the
           stores gated per owner by the verdicts (okm), step 0's key stream
           kept from the AUTH pass (its blocks gave r and s).
   A rejected record's output is never written. */
template <int K, bool UKEY>
NA_DEV void open_il_staged_vf(const UniformArgs &a, uint4 *tiles, FinSlot *fin, uint32_t wave_job)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rec0 = wave_job * (64 / K);
    const uint32_t rec_raw = rec0 + lane / K;
    const bool live = rec_raw < a.n_records;
    const uint32_t rc = live ? rec_raw : a.n_records - 1;
    const int k = (int)(lane % K);
    uint32_t key[8], n_lo, n_hi;
    u_key_nonce<UKEY>(a, rec0, rc, key, n_lo, n_hi);
    ChaPre pre;
    chacha_pre(key, n_lo, n_hi, pre);
    const uint32_t len = a.len;
    const GroupCtx<K> g = group_ctx<K>(len);
    const int gbase = (int)lane & ~(K - 1);
    const WaveIO<K> io = wave_io<K>(rec0, lane);
    const int last_full = (int)g.J - 2;
    const uint32_t tail = g.J ? len - 64 * (g.J - 1) : 0; /* bytes of unit J-1 */

    /* AUTH */
    wave_dma_asm<K>(a, io, -(int)g.o - 1, tiles);
    if (g.steps > 1) wave_dma_asm<K>(a, io, K - (int)g.o - 1, tiles + 256);
    Fe acc = fe_zero();
    Mul mr, mjump;
    uint32_t s[4];
    uint32_t x0[16]; /* step 0's blocks: the key block on one lane, data key stream on the others */
    slot_block<true>(key, pre, k - (int)g.o, n_lo, n_hi, x0, a.balance != 0);
    {
        Fe r;
        poly_key_bcast(x0, gbase + (int)g.o, r, s);
        mr = mk_mul(r);
        Mul mfinal;
        poly_powers<K>(r, k, g.q, mjump, mfinal);
        fin_put(fin, lane, mfinal);
        const int k0 = g.J ? (int)((g.o + 1) % K) : K - 1;
        if (k == k0 && a.ad_len) poly_ad(acc, mr, u_ad(a, rc), a.ad_len);
    }
    bool seen = false;
    for (uint32_t m = 0; m < g.steps; ++m) {
        const int j0 = (int)(m * K) - (int)g.o - 1;
        const int v = j0 + 1 + k;
        uint4 *cur = tiles + 256 * (m & 1);
        if (m + 1 < g.steps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); /* this step's four, not the next's */
        else solo_wait();
        uint32_t w[16];
        tile_get_unit(cur, lane, w);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* the tile is read before the DMA refills it */
        __builtin_amdgcn_wave_barrier();
        if (m + 2 < g.steps) wave_dma_asm<K>(a, io, j0 + 2 * K, cur);
        __builtin_amdgcn_s_setprio(3);
        if (v >= 1 && (uint32_t)v <= g.J) {
            uint32_t nb = 4;
            if ((uint32_t)v == g.J) {
                mask_unit(w, tail);
                nb = (tail + 15) / 16;
            }
            poly_unit(acc, seen ? mjump : mr, mr, w, nb);
            seen = true;
        }
    }
    __builtin_amdgcn_s_setprio(0);
    uint32_t tag[4], got[4];
    poly_close<K>(acc, k, mr, fin_get(fin, lane), a.ad_len, len, s, tag);
    tag_in<true>(u_src(a, rc), len, got); /* the tag bytes are never written */
    const bool ok = tag_equal(tag, got);
    if (k == K - 1 && live && a.status) a.status[rec_raw] = ok ? 0 : 1;
    if (__ballot(live && ok) == 0) return;

    /* DEC: bit i of okm = the owner coalesced instruction i serves is verified */
    uint32_t okm = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        okm |= (__shfl((int)ok, (int)(16u * i + (lane >> 2)), 64) != 0 ? 1u : 0u) << i;
    __builtin_amdgcn_wave_barrier(); /* the AUTH pass's tile reads are done */
    wave_dma_asm<K>(a, io, -(int)g.o - 1, tiles);
    for (uint32_t m = 0; m < g.steps; ++m) {
        if (a.balance) prio_by_progress(m, g.steps);
        const int j0 = (int)(m * K) - (int)g.o - 1;
        const int v = j0 + 1 + k;
        uint4 *cur = tiles + 256 * (m & 1), *nxt = tiles + 256 * ((m + 1) & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* last step's reads and writes of nxt are done */
        __builtin_amdgcn_wave_barrier();
        if (m + 1 < g.steps) wave_dma_asm<K>(a, io, j0 + K, nxt);
        uint32_t x[16];
        if (m == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = x0[i];
        } else {
            slot_block<true>(key, pre, v, n_lo, n_hi, x, a.balance && 2 * m < g.steps);
        }
        __builtin_amdgcn_wave_barrier();
        /* this step's DMA (a step old) landed; the next step's may still fly */
        if (m + 1 < g.steps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t w[16];
        tile_get_unit(cur, lane, w);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        if (v >= 1 && (uint32_t)v == g.J && live && ok) last_unit_out(u_dst(a, rc) + 64 * (g.J - 1), tail, w);
        tile_put_unit(cur, lane, w);
        __builtin_amdgcn_wave_barrier();
        wave_store<K>(a, io, j0, last_full, cur, lane, okm);
    }
}

template <int K, bool UKEY>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void chachapoly_seal_staged(UniformArgs a)
{
    __shared__ uint4 tiles[4][512]; /* two 4 KB tiles per wave */
    __shared__ FinSlot fin[4];
    seal_il_staged<K, UKEY>(a, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], wave_of(blockIdx.x));
}

template <int K, bool UKEY>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void chachapoly_open_staged(UniformArgs a)
{
    __shared__ uint4 tiles[4][512];
    __shared__ FinSlot fin[4];
    open_il_staged<K, UKEY>(a, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], wave_of(blockIdx.x));
}

/* verify-first (open_il_staged_vf) */
template <int K, bool UKEY>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void chachapoly_open_staged_vf(UniformArgs a)
{
    __shared__ uint4 tiles[4][512];
    __shared__ FinSlot fin[4];
    open_il_staged_vf<K, UKEY>(a, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], wave_of(blockIdx.x));
}

/* Duplex: one launch over two independent uniform jobs — seal job `s` and
   open job `o` (an echo server's two directions, or a pipeline sealing batch
   b while opening batch b-2).  Workgroups alternate between the two while
   both have some left (so every XCD and CU gets both kinds), then the longer
   job's remainder follows.  Each workgroup runs exactly the code of the
   separate seal/open kernels on its own job, so results are identical; one
   launch instead of two removes a kernel boundary (≈5 µs of idle GPU at C2)
   and lets one job's waves backfill the other's tail. */
template <int K, bool UKEY>
__global__ __launch_bounds__(256) NA_UNIFORM_OCC void chachapoly_duplex_staged(
    UniformArgs s, UniformArgs o, uint32_t s_blocks, uint32_t o_blocks)
{
    __shared__ uint4 tiles[4][512];
    __shared__ FinSlot fin[4];
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
    if (open) open_il_staged<K, UKEY>(o, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], wave_of(b));
    else seal_il_staged<K, UKEY>(s, tiles[threadIdx.x >> 6], &fin[threadIdx.x >> 6], wave_of(b));
}


/* One lane per record (seal_solo_staged): two waves per SIMD, 16 KB of LDS
   each; 256 records per workgroup. */
#define NA_SOLO_OCC __attribute__((amdgpu_waves_per_eu(2)))

/* RUNS: the key stream in runs (solo_blocks2) — for launches of at least
   two waves per SIMD (launch_chacha.hip picks) */
template <bool UKEY, bool RUNS>
__global__ __launch_bounds__(256) NA_SOLO_OCC void chachapoly_seal_solo(UniformArgs a)
{
    __shared__ uint4 tiles[4][2 * SOLO_TILE];
    seal_solo_staged<UKEY, RUNS>(a, tiles[threadIdx.x >> 6], wave_of(blockIdx.x));
}

template <bool UKEY, bool RUNS>
__global__ __launch_bounds__(256) NA_SOLO_OCC void chachapoly_open_solo(UniformArgs a)
{
    __shared__ uint4 tiles[4][2 * SOLO_TILE];
    open_solo_staged<UKEY, RUNS>(a, tiles[threadIdx.x >> 6], wave_of(blockIdx.x));
}

/* chachapoly_duplex_staged's two-job launch over the one-lane kernels */
template <bool UKEY>
/* chunk C > 0: the paired blocks go in runs of C, seal and open runs
   alternating (C = the CU count: the dispatcher hands each CU one block of
   the seal run and one of the open run, so a SIMD's two waves are one seal
   and one open); C = 0: blocks alternate one by one (then block b and
   block b + #CUs, which share a CU, are the same kind). */
__global__ __launch_bounds__(256) NA_SOLO_OCC void chachapoly_duplex_solo(
    UniformArgs s, UniformArgs o, uint32_t s_blocks, uint32_t o_blocks, uint32_t C)
{
    __shared__ uint4 tiles[4][2 * SOLO_TILE];
    const uint32_t n = min(s_blocks, o_blocks);
    const uint32_t full = C ? n / C * C : 0; /* pairs placed in whole runs */
    uint32_t b = blockIdx.x;
    bool open;
    if (b < 2 * full) {
        const uint32_t run = b / C;
        open = run & 1;
        b = (run >> 1) * C + b % C;
    } else if (b < 2 * n) {
        b -= 2 * full;
        open = b & 1;
        b = full + (b >> 1);
    } else {
        open = o_blocks > s_blocks;
        b -= n;
    }
    if (open) open_solo_staged<UKEY, true>(o, tiles[threadIdx.x >> 6], wave_of(b));
    else seal_solo_staged<UKEY, true>(s, tiles[threadIdx.x >> 6], wave_of(b));
}

template <int K, bool FAST>
__global__ __launch_bounds__(256) void chachapoly_seal_uniform(UniformArgs a)
{
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / K;
    if (rec >= a.n_records) return; /* whole groups leave together (K | 64) */
    seal_any<K, FAST>(uniform_view(a, rec), (int)(gtid % K));
}

template <int K, bool FAST>
__global__ __launch_bounds__(256) void chachapoly_open_uniform(UniformArgs a)
{
    const uint32_t gtid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t rec = gtid / K;
    if (rec >= a.n_records) return;
    const int k = (int)(gtid % K);
    const RecView rv = uniform_view(a, rec);
    const bool ok = open_any<K, FAST>(rv, k); /* verifies first, then decrypts */
    if (k == K - 1 && a.status) a.status[rec] = ok ? 0 : 1;
    if (!ok && !a.vf) scrub_rejected(rv.dst, rv.src, rv.len, (uint32_t)k, K);
}

/* Ragged batches: the workgroup's 256/K records are taken in length order
   (window_rec), so the records sharing a wave have near-equal lengths.
   Open: VF (NOISE_AEAD_FLAG_VERIFY_FIRST) takes the two-pass open_any —
   authenticate, then decrypt only a verified record, nothing written for a
   rejected one (cipher-chachapoly.c:135-141) — instead of the one-pass
   open_il_1p, whose plaintext exists before the verdict. */
template <int K, bool FAST>
__global__ __launch_bounds__(256) void chachapoly_seal_ragged(RaggedArgs a)
{
    __shared__ uint32_t order[256 / K];
    const uint32_t rec = window_rec<256 / K>(a.recs, a.n_records, blockIdx.x * (256u / K),
                                             threadIdx.x / K, order);
    if (rec >= a.n_records) return;
    const RecView rv = ragged_view(a, rec);
    if (reject_len(a, rec, rv.len, threadIdx.x % K == K - 1)) return;
    seal_any<K, FAST>(rv, (int)(threadIdx.x % K));
    if (threadIdx.x % K == K - 1 && a.status) a.status[rec] = 0;
}

template <int K, bool FAST, bool VF = false>
__global__ __launch_bounds__(256) void chachapoly_open_ragged(RaggedArgs a)
{
    __shared__ uint32_t order[256 / K];
    const uint32_t rec = window_rec<256 / K>(a.recs, a.n_records, blockIdx.x * (256u / K),
                                             threadIdx.x / K, order);
    if (rec >= a.n_records) return;
    const int k = (int)(threadIdx.x % K);
    const RecView rv = ragged_view(a, rec);
    if (reject_len(a, rec, rv.len, k == K - 1)) return;
    bool ok;
    if constexpr (FAST && K >= 4 && !VF) {
        ok = open_il_1p<K>(rv, k); /* one pass: the ciphertext is read once */
    } else {
        ok = open_any<K, FAST>(rv, k);
    }
    if (k == K - 1 && a.status) a.status[rec] = ok ? 0 : 1;
    if (!ok && !a.vf) scrub_rejected(rv.dst, rv.src, rv.len, (uint32_t)k, K);
}

} // namespace na
