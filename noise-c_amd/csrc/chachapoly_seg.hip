/*
 * chachapoly_seg.hip — segmented one-lane ChaChaPoly (round 5).
 *
 * The one-lane kernels (chachapoly.hip seal_solo_staged) give every record
 * one lane: one radix-2^32 Poly1305 chain with the clamped r, the per-record
 * work paid once per 64 records, LDS-DMA tiles read a whole step after they
 * were issued.  Two shapes do not fit them:
 *   - a standalone launch of 64 Ki records is one wave per SIMD, where the
 *     issue rate is ~20 % below that of two waves;
 *   - a ragged batch (C5: 64 B - 16 KiB) would make a wave as slow as its
 *     longest record and the batch as slow as its longest wave.
 * Here a record of B = J + 1 ChaCha blocks (block 0 = the Poly1305 key, block
 * v >= 1 = data unit v - 1, cipher-chachapoly.c:62-73,107-123) is cut into K
 * contiguous SEGMENTS (K a power of two, the record's lanes K-aligned in the
 * wave): lane k runs blocks [k c, min((k+1) c, B)), c = 2 ceil(ceil(B/K)/2),
 * two blocks per step exactly as the one-lane kernels do, with its own
 * Horner chain h_k over its units' Poly1305 blocks.  The record's lanes then
 * combine
 *     acc = sum_k h_k r^(e_k),   e_k = Poly blocks after segment k,
 * (each lane raises r to its e_k by square-and-multiply; the group sums with
 * xor-shuffles), and the first lane absorbs the length block and finishes:
 * exactly the donna Horner value sum_i b_i r^(n-i+1) of poly1305-donna-64.h
 * :101-151 (the same algebra as the K = 2 contiguous kernels of
 * chachapoly.hip).  The key block is part of lane 0's first step; the other
 * lanes take r from it by a shuffle after that step's ChaCha.
 *
 * Uniform jobs take K = 2 (64 Ki <= n < 128 Ki standalone records: two waves
 * per SIMD); ragged FAST jobs take K from each record's length (SEG_TARGET
 * blocks per lane at most, K <= SEG_KMAX) through a PLAN: records bucketed by
 * J (counting sort, longest first), each record's lanes placed K-aligned, so
 * every wave's lanes run near-equal numbers of blocks; persistent waves take
 * the plan's 64-lane jobs from a ticket counter in that order (longest first:
 * the short jobs fill the tail).
 *
 * Coalesced I/O as in the one-lane kernels: per step each lane's two units
 * land in a 16 KB double-buffered LDS tile by LDS-DMA, eight 128-B owner runs
 * per instruction; the owners' segment bases, limits and verdicts are
 * gathered once per job (SegIOU / SegIOL).
 */

namespace na {

/* NA_SEG_DEBUG (A/B variant builds only, `make variant DEFS=-DNA_SEG_DEBUG`):
   every global access of these kernels is checked against two address
   ranges set by noise_aead_debug_seg_arena (the caller's buffers) and the
   launcher (the plan scratch); an access outside both is skipped and logged
   instead of faulting. */
#ifdef NA_SEG_DEBUG
__device__ uint64_t g_seg_arena[4];
__device__ uint64_t g_seg_viol[64];
__device__ uint32_t g_seg_nviol;
NA_DEV bool seg_ok(const void *p, uint32_t n, uint32_t kind, uint32_t info)
{
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const bool ok = (a >= g_seg_arena[0] && a + n <= g_seg_arena[1]) || (a >= g_seg_arena[2] && a + n <= g_seg_arena[3]);
    if (!ok) {
        const uint32_t i = atomicAdd(&g_seg_nviol, 1u);
        if (i < 32) {
            g_seg_viol[2 * i] = a;
            g_seg_viol[2 * i + 1] = ((uint64_t)kind << 56) | ((uint64_t)n << 40) | info;
        }
    }
    return ok;
}
#define SEG_OK(p, n, kind, info) seg_ok((const void *)(p), (n), (kind), (info))
#else
#define SEG_OK(p, n, kind, info) true
#endif

/* NA_SEG_TL (A/B variant builds only): per-wave cycle accounting of the
   persistent ragged kernel (s_memtime, wave-uniform): [0] the wave's life,
   [1] job set-up (ticket, plan entry, descriptor, key, owner table), [2]
   the first step's wait for its DMA, [3] the other steps' waits, [4] the
   passes, [5] combine + tag, [6] the end-of-job store drain, [7] jobs.  Each
   wave writes its row of g_seg_tlw at exit (last launch wins);
   noise_aead_debug_seg_tl sums them. */
#ifdef NA_SEG_TL
__device__ unsigned long long g_seg_tlw[4096][8];
struct SegTL {
    uint64_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    NA_DEV static uint64_t now() { return __builtin_amdgcn_s_memtime(); }
    NA_DEV void add(int k, uint64_t v) { c[k] += v; }
    NA_DEV void flush()
    {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 8; ++k) g_seg_tlw[blockIdx.x * 4 + (threadIdx.x >> 6)][k] = c[k];
    }
};
#else
struct SegTL {
    NA_DEV static uint64_t now() { return 0; }
    NA_DEV void add(int, uint64_t) {}
    NA_DEV void flush() {}
};
#endif

/* Blocks per lane a ragged record aims at (K = the smallest power of two with
   ceil(B/K) <= SEG_TARGET, at most SEG_KMAX; 24/32/48/64 measured, 32 the
   fastest, profiles/r05/) */
constexpr uint32_t SEG_TARGET = 32;
constexpr uint32_t SEG_KMAX = 16;
constexpr uint32_t SEG_BUCKETS = 1025; /* J = 0 .. 1024 (65519-byte records) */

NA_DEV uint32_t seg_k_of(uint32_t J)
{
    const uint32_t B = J + 1;
    uint32_t K = 1;
    while (K < SEG_KMAX && (B + K - 1) / K > SEG_TARGET) K <<= 1;
    return K;
}

/* One lane's segment. */
struct SegLane {
    const uint8_t *src, *ad;
    uint8_t *dst;
    uint32_t len, ad_len, J, tail;
    uint32_t b0, nb;   /* ChaCha blocks [b0, b0 + nb) */
    uint32_t k, K;     /* segment k of the record's K (lanes K-aligned) */
    uint32_t rec;      /* index for status */
    uint32_t n_lo, n_hi;
    bool live;
};

NA_DEV void seg_blocks(SegLane &q)
{
    q.J = (q.len + 63) / 64;
    q.tail = q.J ? q.len - 64 * (q.J - 1) : 0;
    const uint32_t B = q.J + 1;
    const uint32_t per = (B + q.K - 1) / q.K;
    const uint32_t c = (per + 1) & ~1u;
    q.b0 = q.k * c;
    q.nb = B > q.b0 ? min(c, B - q.b0) : 0u;
    if (!q.live) q.nb = 0;
}

/* Poly1305 blocks of the record after this lane's segment (0: it holds the
   last unit, or nothing) */
NA_DEV uint32_t seg_suffix(const SegLane &q)
{
    if (!q.live || q.nb == 0 || q.J == 0) return 0;
    const uint32_t end = q.b0 + q.nb - 1; /* exclusive end unit */
    if (end >= q.J) return 0;
    return 4 * (q.J - 1 - end) + (q.tail + 15) / 16;
}

/* The owners' I/O geometry.  Coalesced instruction i serves owner lane
   o = 8i + lane/8 (chunk solo_chunk(lane) of its step run); offsets are
   relative to the owner's base = record + 64 (b0 - 1): [lo, hi) readable
   (lo = 64 when the segment starts with the key block, whose 64 B are no
   data), stores below slim (the full units before the record's last one,
   which its owner writes exactly).  Two policies with one interface:
     SegIOU — a uniform K = 2 job: the owners' records are rec0 + 4i + lane/16,
              segment (lane/8) & 1, so every address is arithmetic;
     SegIOL — a ragged job: the owners' bases and limits in a per-wave LDS
              table written once per job (SegOwner), read per instruction
              (ds_read broadcasts), so no register holds eight owners. */
struct SegOwner {
    uint64_t in, out;
    uint32_t hi;   /* readable end; 0: no blocks */
    uint32_t sl;   /* slim | lo << 31 */
};

NA_DEV SegOwner seg_geom(const SegLane &q)
{
    SegOwner o;
    o.in = (uint64_t)(uintptr_t)q.src + 64ull * q.b0 - 64ull;
    o.out = (uint64_t)(uintptr_t)q.dst + 64ull * q.b0 - 64ull;
    o.hi = 0;
    o.sl = 0;
    if (!q.live || q.nb == 0) return o;
    const uint32_t lo = q.b0 == 0 ? 64u : 0u;
    uint32_t end = q.b0 + q.nb - 1; /* exclusive end unit */
    if (end > q.J) end = q.J;
    uint32_t hi = 64u * (end + 1 - q.b0);
    if (hi < lo + 64) hi = lo + 64; /* a record of 0 bytes: its 64 readable bytes */
    const int32_t send = min((int32_t)(q.b0 + q.nb) - 1, (int32_t)q.J - 1);
    const int32_t slim = max(64 * (send - (int32_t)q.b0 + 1), 0);
    o.hi = hi;
    o.sl = (uint32_t)slim | (lo ? 0x80000000u : 0u);
    return o;
}

NA_DEV uint32_t seg_dma_off(uint32_t m, uint32_t c, uint32_t hi, uint32_t sl)
{
    uint32_t off = 128u * m + 16u * c;
    if ((sl >> 31) && off < 64u) off += 64u;
    if (off >= hi) off = hi - 64u + (off & 63u);
    return off;
}

NA_DEV bool seg_store_ok(uint32_t off, uint32_t sl)
{
    return !((sl >> 31) && off < 64u) && off + 16u <= (sl & 0x7fffffffu);
}

/* rec_store16 to an address held as an integer, as a global (not flat)
   store: a flat store also counts in lgkmcnt, so every later LDS wait would
   wait for it too */
typedef __attribute__((address_space(1))) na_u32x4 seg_gvec;
NA_DEV void seg_store16(uint64_t a, const uint4 &q)
{
    const na_u32x4 v = {q.x, q.y, q.z, q.w};
    __builtin_nontemporal_store(v, (seg_gvec *)(uintptr_t)a);
}

struct SegIOL {
    SegOwner *tab; /* this wave's 64 owners (LDS) */
    /* wave-uniform: the smallest readable end and store limit over the
       owners with blocks.  A step m >= 1 with 128 (m + 1) below them is
       interior for every owner: no clamp, no limit test per instruction
       (≈100 of a step's ≈2300 VALU, the owner-geometry arithmetic) */
    uint32_t min_hi, min_sl;
    NA_DEV void init(const SegLane &q, uint32_t lane)
    {
        const SegOwner g = seg_geom(q);
        tab[lane] = g;
        uint32_t h = g.hi ? g.hi : 0xffffffffu, sl = g.hi ? (g.sl & 0x7fffffffu) : 0xffffffffu;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            h = min(h, (uint32_t)__shfl_xor((int)h, off, 64));
            sl = min(sl, (uint32_t)__shfl_xor((int)sl, off, 64));
        }
        min_hi = __builtin_amdgcn_readfirstlane(h);
        min_sl = __builtin_amdgcn_readfirstlane(sl);
        __builtin_amdgcn_wave_barrier();
    }
    NA_DEV void dma(uint32_t lane, uint32_t m, uint4 *t) const
    {
        const uint32_t c = solo_chunk(lane);
        const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)t);
        if (m >= 1 && 128u * m + 128u <= min_hi) { /* interior step (wave-uniform) */
            const uint32_t off = 128u * m + 16u * c;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const SegOwner &o = tab[8 * i + (lane >> 3)];
                const uint64_t ga = o.in + off;
                if (o.hi && SEG_OK(ga, 16, 1, m << 16 | lane << 8 | i)) dma16_asm((const void *)(uintptr_t)ga, base + 1024u * (uint32_t)i);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const SegOwner &o = tab[8 * i + (lane >> 3)];
            const uint32_t hi = o.hi;
            const uint64_t ga = o.in + seg_dma_off(m, c, hi, o.sl);
            if (hi && SEG_OK(ga, 16, 1, m << 16 | lane << 8 | i)) dma16_asm((const void *)(uintptr_t)ga, base + 1024u * (uint32_t)i);
        }
    }
    NA_DEV void store(uint32_t lane, uint32_t m, const uint4 *t, uint32_t okm) const
    {
        /* the tile values and owner entries first, one wait, then the stores
           (a read and its wait inside each store's branch serialised them) */
        const uint32_t off = 128u * m + 16u * solo_chunk(lane);
        const bool interior = m >= 1 && 128u * m + 128u <= min_sl; /* wave-uniform */
        uint4 v[8];
        uint64_t dst[8];
        uint32_t ok = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const SegOwner &o = tab[8 * i + (lane >> 3)];
            v[i] = t[64 * i + lane];
            dst[i] = o.out + off;
            ok |= (o.hi && (interior || seg_store_ok(off, o.sl)) ? 1u : 0u) << i;
        }
        ok &= okm;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (((ok >> i) & 1) && SEG_OK(dst[i], 16, 2, m << 16 | lane << 8 | i)) seg_store16(dst[i], v[i]);
    }
};

struct SegIOU {
    const uint8_t *in; /* the wave's first record (wave-uniform) */
    uint8_t *out;
    uint64_t in_stride, out_stride;
    int64_t lin, lout; /* this lane's owner: (lane/16) strides + 64 (b0 - 1) */
    uint32_t hi, sl;   /* its geometry (every record has the same length) */
    uint32_t livem;    /* bit i: owner record rec0 + 4i + lane/16 exists */
    bool full;         /* wave-uniform: all 32 records of the wave exist */
    NA_DEV void init(const UniformArgs &a, uint32_t rec0, const SegLane &q, uint32_t lane)
    {
        in = a.in + (size_t)rec0 * a.in_stride;
        out = a.out + (size_t)rec0 * a.out_stride;
        in_stride = a.in_stride;
        out_stride = a.out_stride;
        /* lane/8's owner is segment (lane/8) & 1 of record 4i + lane/16: its
           geometry is that of lane 0 or 1 (record 0's two segments) */
        const int src_lane = (lane >> 3) & 1;
        SegLane g = q;
        g.b0 = (uint32_t)__shfl((int)q.b0, src_lane, 64);
        g.nb = (uint32_t)__shfl((int)q.nb, src_lane, 64);
        g.live = true;
        const SegOwner o = seg_geom(g);
        hi = o.hi;
        sl = o.sl;
        lin = (int64_t)(lane >> 4) * (int64_t)a.in_stride + 64ll * g.b0 - 64ll;
        lout = (int64_t)(lane >> 4) * (int64_t)a.out_stride + 64ll * g.b0 - 64ll;
        livem = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) livem |= (rec0 + 4u * i + (lane >> 4) < a.n_records ? 1u : 0u) << i;
        full = rec0 + 32u <= a.n_records;
    }
    NA_DEV void dma(uint32_t lane, uint32_t m, uint4 *t) const
    {
        const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void *)t);
        const uint32_t off = seg_dma_off(m, solo_chunk(lane), hi, sl);
        if (full) { /* wave-uniform: no per-instruction predicate */
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (hi) dma16_asm(in + (size_t)(4 * i) * in_stride + lin + off, base + 1024u * (uint32_t)i);
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (((livem >> i) & 1) && hi)
                dma16_asm(in + (size_t)(4 * i) * in_stride + lin + off, base + 1024u * (uint32_t)i);
    }
    NA_DEV void store(uint32_t lane, uint32_t m, const uint4 *t, uint32_t okm) const
    {
        const uint32_t off = 128u * m + 16u * solo_chunk(lane);
        if (!hi || !seg_store_ok(off, sl)) return;
        uint4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = t[64 * i + lane]; /* all reads, one wait */
        if (full && okm == 0xffu) { /* wave-uniform: every owner stores */
#pragma unroll
            for (int i = 0; i < 8; ++i) rec_store16(out + (size_t)(4 * i) * out_stride + lout + off, v[i]);
            return;
        }
        const uint32_t ok = livem & okm;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if ((ok >> i) & 1) rec_store16(out + (size_t)(4 * i) * out_stride + lout + off, v[i]);
    }
};

/* last_unit_out with the partial chunk picked by masks: pick_chunk's select
   chain was folded into a dynamic index here, which put the whole unit in
   scratch memory */
NA_DEV void seg_last_out(uint8_t *p, uint32_t nb, const uint32_t w[16])
{
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c)
        if (16 * c + 16 <= nb)
            *(uint4 *)(p + 16 * c) = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    const uint32_t rem = nb & 15;
    if (rem) {
        const uint32_t q = nb >> 4;
        uint32_t part[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t v = 0;
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c) v |= w[4 * c + i] & (0u - (uint32_t)(q == c));
            part[i] = v;
        }
        uint8_t *d = p + (nb & ~15u);
        if (rem == 8) *(uint2 *)d = make_uint2(part[0], part[1]);
        else store16(d, rem, part);
    }
}

/* the lane holding segment 0 of this lane's record */
NA_DEV int seg_leader(const SegLane &q, uint32_t lane) { return (int)(lane - q.k); }

NA_DEV uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return v;
}

enum SegMode { SEG_SEAL, SEG_OPEN1, SEG_DEC };

/* The key block's r (first four words) from the record's leader, as R32, and
   the Fe r the combine uses */
NA_DEV void seg_bcast_r(const SegLane &q, uint32_t lane, const uint32_t kw[4], R32 &r, uint32_t rw[4])
{
    const int ld = seg_leader(q, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) rw[i] = (uint32_t)__shfl((int)kw[i], ld, 64);
    r = r32_from_key(rw[0], rw[1], rw[2], rw[3]);
}

/* Data unit j of this lane, in solo_pass's order and registers: w holds the
   tile's unit on entry and leaves with what the tile takes (SEAL: CT;
   OPEN1 / DEC: plaintext; past len the bytes are never stored).  SEAL /
   OPEN1 chain the unit's Poly1305 blocks (the CT, zero past len) unless
   DEFER: then w leaves as that Poly input and the caller chains it and
   (OPEN1) XORs x itself — step 0, before r has arrived. */
template <int MODE, bool DEFER = false>
NA_DEV void seg_data(const SegLane &q, uint32_t j, uint32_t w[16], const uint32_t x[16], const R32 &r,
                     P32 &h, bool ok, uint32_t &nbp)
{
    const bool last = j == q.J - 1;
    nbp = last ? (q.tail + 15) / 16 : 4u;
    if constexpr (MODE == SEG_OPEN1) {
        if (last) mask_unit(w, q.tail);
        if constexpr (DEFER) return;
        p32_unit(h, r, w, nbp);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        if (last && SEG_OK(q.dst + 64 * j, q.tail, 3, j)) seg_last_out(q.dst + 64 * j, q.tail, w);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= x[i];
        if (last) {
            if ((MODE == SEG_SEAL || ok) && SEG_OK(q.dst + 64 * j, q.tail, 3, j)) seg_last_out(q.dst + 64 * j, q.tail, w);
            if (MODE == SEG_SEAL) mask_unit(w, q.tail);
        }
        if constexpr (MODE == SEG_SEAL && !DEFER) p32_unit(h, r, w, nbp);
    }
}

/* Step m of a pass (the order of solo_pass: wait for the DMA a step old,
   read the tile, store the previous step from the other tile, issue the
   next DMA, compute).  FIRST (SEAL / OPEN1 step 0): the leader's first
   block is the key block — slot 0's block is computed and its unit XORed /
   kept, r reaches every lane from its record's leader, the leader absorbs
   the AD, then slot 0's Poly1305 and slot 1.  Step 0 is peeled out of the
   loop: inside it, its branch doubled the loop's register allocation (256
   VGPRs and spills against 158). */
template <int MODE, bool PRIO, bool FIRST, class IO>
NA_DEV void seg_step(const SegLane &q, const IO &io, uint32_t lane, uint32_t m, uint32_t S, uint4 *tiles,
                     const uint32_t key[8], const ChaPre &pre, R32 &r, uint32_t rw[4], uint32_t s[4],
                     P32 &h, uint32_t okm, bool ok, SegTL &tl)
{
    uint4 *cur = tiles + SOLO_TILE * (m & 1), *nxt = tiles + SOLO_TILE * ((m + 1) & 1);
    uint32_t wu[2][16];
    const uint64_t tw = SegTL::now();
    solo_wait();
    tl.add(FIRST ? 2 : 3, SegTL::now() - tw);
    solo_get(cur, lane, 0, wu[0]);
    solo_get(cur, lane, 1, wu[1]);
    if (!FIRST && m >= 1) io.store(lane, m - 1, nxt, okm);
    __builtin_amdgcn_wave_barrier();
    if (m + 1 < S) io.dma(lane, m + 1, nxt);
    if (PRIO) prio_by_progress(m, S);
    if constexpr (FIRST) {
        uint32_t x[16], kw[4] = {0, 0, 0, 0}, nb0 = 0;
        const bool d0 = q.nb > 0 && q.b0 != 0; /* slot 0 holds data */
        if (q.nb > 0) {
            chacha20_block_pre(key, pre, q.b0, q.n_lo, q.n_hi, x);
            if (q.b0 == 0) {
                kw[0] = x[0]; kw[1] = x[1]; kw[2] = x[2]; kw[3] = x[3];
                s[0] = x[4]; s[1] = x[5]; s[2] = x[6]; s[3] = x[7];
            } else {
                seg_data<MODE, true>(q, q.b0 - 1, wu[0], x, r, h, ok, nb0);
            }
        }
        seg_bcast_r(q, lane, kw, r, rw);
        if (q.b0 == 0 && q.live && q.ad_len && SEG_OK(q.ad, q.ad_len, 4, 0)) p32_ad(h, r, q.ad, q.ad_len);
        if (d0) {
            p32_unit(h, r, wu[0], nb0);
            if (MODE == SEG_OPEN1) {
                const uint32_t j = q.b0 - 1;
#pragma unroll
                for (int i = 0; i < 16; ++i) wu[0][i] ^= x[i];
                if (j == q.J - 1 && SEG_OK(q.dst + 64 * j, q.tail, 3, j)) seg_last_out(q.dst + 64 * j, q.tail, wu[0]);
            }
            solo_put(cur, lane, 0, wu[0]);
        }
        if (q.nb > 1) {
            uint32_t x1[16], nbp;
            chacha20_block_pre(key, pre, q.b0 + 1, q.n_lo, q.n_hi, x1);
            seg_data<MODE>(q, q.b0, wu[1], x1, r, h, ok, nbp);
            solo_put(cur, lane, 1, wu[1]);
        }
    } else {
        /* both blocks in lock step, issued in runs (chachapoly.hip
           solo_blocks2: the persistent and the K = 2 kernels hold two waves
           per SIMD) */
        uint32_t xs[2][16];
        if (2 * m < q.nb && (MODE != SEG_DEC || ok))
            solo_blocks2<true>(key, pre, q.b0 + 2 * m, q.n_lo, q.n_hi, xs[0], xs[1]);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t blk = q.b0 + 2 * m + u;
            if (2 * m + u < q.nb && blk != 0 && (MODE != SEG_DEC || ok)) {
                uint32_t x[16], nbp;
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] = xs[u][i];
                seg_data<MODE>(q, blk - 1, wu[u], x, r, h, ok, nbp);
                solo_put(cur, lane, u, wu[u]);
            }
        }
    }
}

/* One pass over the wave's segments, two blocks per step.  DEC
   (verify-first, r known): key stream only; block 0 skipped. */
template <int MODE, bool PRIO, class IO>
NA_DEV void seg_pass(const SegLane &q, const IO &io, uint32_t lane, uint32_t S, uint4 *tiles,
                     const uint32_t key[8], const ChaPre &pre, R32 &r, uint32_t rw[4], uint32_t s[4],
                     P32 &h, uint32_t okm, bool ok, SegTL &tl)
{
    const uint64_t t0 = SegTL::now();
    uint32_t m0 = 0;
    if (MODE != SEG_DEC && S) {
        seg_step<MODE, PRIO, true>(q, io, lane, 0u, S, tiles, key, pre, r, rw, s, h, okm, ok, tl);
        m0 = 1;
    }
    for (uint32_t m = m0; m < S; ++m)
        seg_step<MODE, PRIO, false>(q, io, lane, m, S, tiles, key, pre, r, rw, s, h, okm, ok, tl);
    if (S) {
        __builtin_amdgcn_wave_barrier();
        io.store(lane, S - 1, tiles + SOLO_TILE * ((S - 1) & 1), okm);
    }
    tl.add(4, SegTL::now() - t0);
}

/* The verify-first AUTH pass: r from the leader's key block first, then
   Poly1305 over the segment's units only (no key stream, nothing stored),
   two steps of DMA in flight at top priority as solo_auth. */
template <class IO>
NA_DEV void seg_auth(const SegLane &q, const IO &io, uint32_t lane, uint32_t S, uint4 *tiles,
                     const uint32_t key[8], const ChaPre &pre, R32 &r, uint32_t rw[4], uint32_t s[4],
                     P32 &h)
{
    if (S > 1) io.dma(lane, 1, tiles + SOLO_TILE);
    uint32_t kw[4] = {0, 0, 0, 0};
    if (q.live && q.b0 == 0) {
        uint32_t x[16];
        chacha20_block_pre(key, pre, 0u, q.n_lo, q.n_hi, x);
        kw[0] = x[0]; kw[1] = x[1]; kw[2] = x[2]; kw[3] = x[3];
        s[0] = x[4]; s[1] = x[5]; s[2] = x[6]; s[3] = x[7];
    }
    seg_bcast_r(q, lane, kw, r, rw);
    if (q.b0 == 0 && q.live && q.ad_len && SEG_OK(q.ad, q.ad_len, 4, 0)) p32_ad(h, r, q.ad, q.ad_len);
    for (uint32_t m = 0; m < S; ++m) {
        uint4 *cur = tiles + SOLO_TILE * (m & 1);
        uint32_t wu[2][16];
        if (m + 1 < S) solo_wait_step_old();
        else solo_wait();
        solo_get(cur, lane, 0, wu[0]);
        solo_get(cur, lane, 1, wu[1]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (m + 2 < S) io.dma(lane, m + 2, cur);
        __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t blk = q.b0 + 2 * m + u;
            if (2 * m + u < q.nb && blk != 0) {
                const uint32_t j = blk - 1;
                uint32_t nbp = 4;
                if (j == q.J - 1) {
                    mask_unit(wu[u], q.tail);
                    nbp = (q.tail + 15) / 16;
                }
                p32_unit(h, r, wu[u], nbp);
            }
        }
    }
    __builtin_amdgcn_s_setprio(0);
}

/* The record's Poly1305 accumulator from its lanes' chains (valid on the
   leader): each lane scales h_k by r^(e_k), the group sums. */
NA_DEV Fe seg_combine(const SegLane &q, const uint32_t rw[4], const P32 &h, uint32_t kmax)
{
    Fe v = p32_to_fe(h);
    if (kmax <= 1) return v;
    const uint32_t e = seg_suffix(q);
    const uint32_t emax = wave_max(e);
    if (emax) {
        const Fe rf = fe_clamp_r(rw[0], rw[1], rw[2], rw[3]);
        const Mul mr = mk_mul(rf);
        Fe p = Fe{1, 0, 0, 0, 0};
        for (int bit = 31 - __builtin_clz(emax); bit >= 0; --bit) {
            p = fe_mul(p, mk_mul(p));
            const Fe t = fe_mul(p, mr);
            if ((e >> bit) & 1u) p = t;
        }
        const Fe sv = fe_mul(v, mk_mul(p));
        if (e) v = sv;
    }
    /* sum over the record's K lanes (K-aligned groups: partners stay inside) */
    for (uint32_t off = 1; off < kmax; off <<= 1) { /* kmax wave-uniform */
        v = fe_carry(v);
        Fe o;
        o.l0 = (uint32_t)__shfl_xor((int)v.l0, (int)off, 64);
        o.l1 = (uint32_t)__shfl_xor((int)v.l1, (int)off, 64);
        o.l2 = (uint32_t)__shfl_xor((int)v.l2, (int)off, 64);
        o.l3 = (uint32_t)__shfl_xor((int)v.l3, (int)off, 64);
        o.l4 = (uint32_t)__shfl_xor((int)v.l4, (int)off, 64);
        if (off < q.K) v = fe_add(v, o);
    }
    return v;
}

/* tag from the accumulator (leader): the length block, then finish */
NA_DEV void seg_tag(Fe acc, const SegLane &q, const uint32_t rw[4], const uint32_t s[4], uint32_t tag[4])
{
    acc = fe_carry(acc);
    fe_add_block(acc, q.ad_len, 0u, q.len, 0u);
    acc = fe_mul(acc, mk_mul(fe_clamp_r(rw[0], rw[1], rw[2], rw[3])));
    fe_finish(acc, s, tag);
}

/* bit i: owner 8i + lane/8 has flag set */
NA_DEV uint32_t seg_owner_mask(bool f, uint32_t lane)
{
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) m |= (__shfl((int)f, (int)(8u * i + (lane >> 3)), 64) != 0 ? 1u : 0u) << i;
    return m;
}

/* A one-pass open's repair of rejected records' segments (in place: the
   plaintext XORed with the key stream again; out of place: zeroed), over
   the same coalesced stores, gated by badm.  `inplace` is per lane (a
   ragged batch may mix in-place and out-of-place records), but lane l's DMA
   chunk belongs to owner 8i + l/8, not to lane l's record: the DMA runs on
   every lane whenever any lane of the wave is in place (an out-of-place
   owner's chunks are read and not used), so each in-place owner's tile is
   filled whatever its neighbours are. */
template <class IO>
NA_DEV void seg_repair(const SegLane &q, const IO &io, uint32_t lane, uint32_t S, uint4 *tiles,
                       const uint32_t key[8], const ChaPre &pre, bool bad, uint32_t badm, bool inplace)
{
    const bool any_inplace = __ballot(inplace) != 0; /* wave-uniform */
    __threadfence(); /* this wave's plaintext stores, visible to its reads below */
    for (uint32_t m = 0; m < S; ++m) {
        __builtin_amdgcn_wave_barrier();
        if (any_inplace) {
            /* the DMA reads the output (in place: the same bytes) */
            io.dma(lane, m, tiles);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t blk = q.b0 + 2 * m + u;
            if (2 * m + u < q.nb && blk != 0) {
                uint32_t w[16];
                if (inplace) {
                    uint32_t x[16];
                    chacha20_block_pre(key, pre, blk, q.n_lo, q.n_hi, x);
                    solo_get(tiles, lane, u, w);
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] ^= x[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = 0;
                }
                if (blk - 1 == q.J - 1 && bad) seg_last_out(q.dst + 64 * (blk - 1), q.tail, w);
                __builtin_amdgcn_wave_barrier();
                solo_put(tiles, lane, u, w);
            }
        }
        __builtin_amdgcn_wave_barrier();
        io.store(lane, m, tiles, badm);
    }
}

/* A wave's job: every lane's segment q (key, nonce, pointers filled, blocks
   from seg_blocks) through seal or open; io initialised.  vf: verify-first
   open. */
struct SegNoHook {
    NA_DEV void operator()() const {}
};

template <bool OPEN, bool PRIO, class IO, class HOOK = SegNoHook>
NA_DEV void seg_job(const SegLane &q, const uint32_t key[8], const IO &io, uint32_t lane, uint4 *tiles,
                    uint8_t *status, bool vf, bool inplace, SegTL &tl, const HOOK &after_pass = HOOK())
{
    const uint32_t S = wave_max((q.nb + 1) / 2);
    const uint32_t kmax = wave_max(q.K);
    ChaPre pre;
    chacha_pre(key, q.n_lo, q.n_hi, pre);
    R32 r;
    uint32_t rw[4] = {0, 0, 0, 0}, s[4] = {0, 0, 0, 0};
    P32 h = p32_zero();
    if (S) io.dma(lane, 0, tiles);
    if (!OPEN) {
        seg_pass<SEG_SEAL, PRIO>(q, io, lane, S, tiles, key, pre, r, rw, s, h, 0xffu, true, tl);
        after_pass();
        const uint64_t tc = SegTL::now();
        const Fe acc = seg_combine(q, rw, h, kmax);
        if (q.live && q.k == 0) {
            uint32_t tag[4];
            seg_tag(acc, q, rw, s, tag);
            if (SEG_OK(q.dst + q.len, 16, 5, q.rec)) tag_out(q.dst + q.len, q.len, tag);
            if (status && SEG_OK(status + q.rec, 1, 6, q.rec)) status[q.rec] = 0;
        }
        tl.add(5, SegTL::now() - tc);
        return;
    }
    if (vf) seg_auth(q, io, lane, S, tiles, key, pre, r, rw, s, h);
    else seg_pass<SEG_OPEN1, PRIO>(q, io, lane, S, tiles, key, pre, r, rw, s, h, 0xffu, true, tl);
    after_pass();
    const Fe acc = seg_combine(q, rw, h, kmax);
    bool okl = false;
    if (q.live && q.k == 0) {
        uint32_t tag[4], got[4];
        seg_tag(acc, q, rw, s, tag);
        got[0] = got[1] = got[2] = got[3] = 0;
        if (SEG_OK(q.src + q.len, 16, 7, q.rec)) tag_in<true>(q.src, q.len, got); /* the tag bytes are never written */
        okl = tag_equal(tag, got);
        if (status && SEG_OK(status + q.rec, 1, 6, q.rec)) status[q.rec] = okl ? 0 : 1;
    }
    const bool ok = __shfl((int)okl, seg_leader(q, lane), 64) != 0;
    if (vf) {
        if (__ballot(q.live && ok && q.nb > 0) == 0) return;
        const uint32_t okm = seg_owner_mask(ok, lane);
        __builtin_amdgcn_wave_barrier(); /* the AUTH pass's tile reads are done */
        if (S) io.dma(lane, 0, tiles);
        seg_pass<SEG_DEC, PRIO>(q, io, lane, S, tiles, key, pre, r, rw, s, h, okm, ok, tl);
        return;
    }
    const bool bad = q.live && !ok;
    if (__ballot(bad) == 0) return;
    seg_repair(q, io, lane, S, tiles, key, pre, bad, seg_owner_mask(bad, lane), inplace);
}

/* ---------------------------------------------------------------- uniform */

/* lane's segment of a uniform job with K lanes per record (wave job = 64/K
   records) */
template <bool UKEY>
NA_DEV SegLane seg_uniform_lane(const UniformArgs &a, uint32_t job, uint32_t K, uint32_t lane, uint32_t key[8])
{
    SegLane q;
    const uint32_t per = 64u / K;
    const uint32_t rec0 = job * per;
    const uint32_t rec = rec0 + lane / K;
    q.live = rec < a.n_records;
    const uint32_t rc = q.live ? rec : a.n_records - 1;
    q.rec = rc;
    q.k = lane % K;
    q.K = K;
    q.src = u_src(a, rc);
    q.dst = u_dst(a, rc);
    q.len = a.len;
    q.ad_len = a.ad_len;
    q.ad = a.ad_len ? u_ad(a, rc) : nullptr;
    u_key_nonce<UKEY>(a, rec0, rc, key, q.n_lo, q.n_hi);
    return q;
}

/* K = 2 segments per record, one wave per 32 records, two waves per SIMD at
   64 Ki records (the standalone seal / open of 64 Ki <= n < 128 Ki) */
template <bool OPEN, bool UKEY>
__global__ __launch_bounds__(256) NA_SOLO_OCC void chachapoly_seg2_uniform(UniformArgs a)
{
    __shared__ uint4 tiles[4][2 * SOLO_TILE];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t job = wave_of(blockIdx.x);
    uint32_t key[8];
    SegLane q = seg_uniform_lane<UKEY>(a, job, 2u, lane, key);
    seg_blocks(q);
    SegIOU io;
    io.init(a, job * 32u, q, lane);
    const bool inplace = a.in == a.out && a.in_stride == a.out_stride;
    SegTL tl;
    seg_job<OPEN, true>(q, key, io, lane, tiles[threadIdx.x >> 6], OPEN ? a.status : nullptr, a.vf != 0,
                        inplace, tl);
}

/* ----------------------------------------------------------------- ragged */

/* The plan of a ragged job (device memory, built per launch by the three
   small kernels below): records bucketed by J, longest first, each record's
   K lanes placed K-aligned; map[lane] = record << 6 | segment. */
struct SegPlanHdr {
    uint32_t ticket;      /* next job (persistent waves) */
    uint32_t total_lanes;
    uint32_t n_jobs;
    uint32_t pad_[29];    /* header: 128 B */
    uint32_t cnt[SEG_BUCKETS];
    uint32_t cur[SEG_BUCKETS];
};
constexpr size_t SEG_MAP_OFF = (sizeof(SegPlanHdr) + 255) & ~(size_t)255;
constexpr uint32_t SEG_IDLE = 0xFFFFFFFFu;

NA_DEV bool seg_rejected(uint32_t len) { return len > MAX_RECORD_LEN; }

/* 1: records per bucket (one thread per record) */
__global__ __launch_bounds__(1024) void seg_plan_count(const RecDesc *recs, uint32_t n, SegPlanHdr *p)
{
    __shared__ uint32_t c[SEG_BUCKETS];
    for (uint32_t i = threadIdx.x; i < SEG_BUCKETS; i += blockDim.x) c[i] = 0;
    __syncthreads();
    const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
    if (rec < n) {
        const uint32_t len = recs[rec].len;
        if (!seg_rejected(len)) atomicAdd(&c[(len + 63) / 64], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < SEG_BUCKETS; i += blockDim.x)
        if (c[i]) atomicAdd(&p->cnt[i], c[i]);
}

/* 2: lane offsets of the buckets, longest J first (one wave: lane t scans
   17 consecutive buckets of the descending order) */
__global__ __launch_bounds__(64) void seg_plan_scan(SegPlanHdr *p)
{
    constexpr uint32_t PER = (SEG_BUCKETS + 63) / 64;
    const uint32_t t = threadIdx.x;
    uint32_t lanes[PER], sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
        const uint32_t d = t * PER + i;           /* descending position */
        const uint32_t J = SEG_BUCKETS - 1 - d;   /* bucket */
        lanes[i] = d < SEG_BUCKETS ? p->cnt[J] * seg_k_of(J) : 0u;
        sum += lanes[i];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)incl, off, 64);
        if (t >= (uint32_t)off) incl += o;
    }
    uint32_t run = incl - sum;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
        const uint32_t d = t * PER + i;
        if (d < SEG_BUCKETS) p->cur[SEG_BUCKETS - 1 - d] = run;
        run += lanes[i];
    }
    if (t == 63) {
        p->total_lanes = incl;
        p->n_jobs = (incl + 63) / 64;
        p->ticket = 0;
    }
}

/* 3: place every record's lanes (block-local ranks, one global reservation
   per bucket and block); refused lengths get status 2 */
__global__ __launch_bounds__(1024) void seg_plan_place(const RecDesc *recs, uint32_t n, SegPlanHdr *p,
                                                       uint32_t *map, uint8_t *status)
{
    __shared__ uint32_t c[SEG_BUCKETS], base[SEG_BUCKETS];
    for (uint32_t i = threadIdx.x; i < SEG_BUCKETS; i += blockDim.x) c[i] = 0;
    __syncthreads();
    const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t J = 0, rank = 0;
    bool in = false;
    if (rec < n) {
        const uint32_t len = recs[rec].len;
        if (seg_rejected(len)) {
            if (status) status[rec] = STATUS_BAD_LENGTH;
        } else {
            in = true;
            J = (len + 63) / 64;
            rank = atomicAdd(&c[J], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < SEG_BUCKETS; i += blockDim.x)
        if (c[i]) base[i] = atomicAdd(&p->cur[i], c[i] * seg_k_of(i));
    __syncthreads();
    if (in) {
        const uint32_t K = seg_k_of(J);
        const uint32_t pos = base[J] + rank * K;
        for (uint32_t k = 0; k < K; ++k)
            if (SEG_OK(map + pos + k, 4, 8, pos + k)) map[pos + k] = rec << 6 | k;
    }
}

/* The lane's segment of plan job `job` (SEG_IDLE lanes: live = false, a
   copy of the wave's first record for addresses) */
/* the plan entries of job `job` for this lane: e (SEG_IDLE past the
   plan's lanes) and the job's first lane's, e0 (always placed); a job at
   or past n_jobs reads nothing */
NA_DEV void seg_map_entries(const uint32_t *map, uint32_t total, uint32_t n_jobs, uint32_t job, uint32_t lane,
                            uint32_t &e, uint32_t &e0)
{
    const uint32_t gl = 64u * job + lane;
    e = job < n_jobs && gl < total && SEG_OK(map + gl, 4, 9, gl) ? map[gl] : SEG_IDLE;
    e0 = job < n_jobs && SEG_OK(map + 64u * job, 4, 9, job) ? map[64u * job] : 0u;
}

NA_DEV SegLane seg_ragged_lane(const RaggedArgs &a, uint32_t e, uint32_t e0, uint32_t key[8])
{
    SegLane q;
    q.live = e != SEG_IDLE;
    if (!q.live) e = e0 & ~63u;
    uint32_t rec = e >> 6;
    if (!SEG_OK(a.recs + rec, 48, 10, rec)) rec = 0;
    const RecDesc &d = a.recs[rec];
    q.rec = rec;
    q.len = d.len;
    q.ad_len = d.ad_len;
    q.src = a.in + d.in_off;
    q.dst = a.out + d.out_off;
    q.ad = d.ad_len ? a.ad + d.ad_off : nullptr;
    q.n_lo = (uint32_t)d.nonce;
    q.n_hi = (uint32_t)(d.nonce >> 32);
    q.K = q.live ? seg_k_of((q.len + 63) / 64) : 1u;
    q.k = q.live ? (e & 63u) : 0u;
    if (SEG_OK(a.keys + d.ctx_off, 32, 11, rec)) load_key(a.keys + d.ctx_off, key);
    else for (int i = 0; i < 8; ++i) key[i] = 0;
    return q;
}

/* Persistent: 2 workgroups per CU, each wave taking jobs from the ticket;
   the next job's ticket and plan entries are taken as the current job's
   data pass ends (below). */
template <bool OPEN>
__global__ __launch_bounds__(256) NA_SOLO_OCC void chachapoly_seg_ragged(RaggedArgs a, SegPlanHdr *p,
                                                                         const uint32_t *map)
{
    /* one block of LDS, the tiles first: every LDS-DMA address stays below
       64 KiB whatever the width of m0's LDS address */
    __shared__ struct {
        uint4 tiles[4][2 * SOLO_TILE];
        SegOwner owners[4][64];
    } sh;
    auto &tiles = sh.tiles;
    auto &owners = sh.owners;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t n_jobs = p->n_jobs, total = p->total_lanes;
    SegTL tl;
    const uint64_t born = SegTL::now();
    /* The next job's ticket and plan entries are taken as the current job's
       data pass ends, so their round trips overlap its combine and tag (a
       job's set-up was four dependent round trips: ticket, plan,
       descriptor, key — 8-9 % of a wave's life, tools/seg_tl.py).  Taken
       at the job's START instead, a busy wave held a reservation on the
       next (long: longest first) job while free waves went on to shorter
       ones: 10 % slower (profiles/r05/seg_prefetch_ab.txt). */
    uint32_t t = 0, e_nx = 0, e0_nx = 0;
    const auto next = [&]() {
        uint32_t tn = 0;
        if (lane == 0) tn = atomicAdd(&p->ticket, 1u);
        t = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)tn, 0, 64));
        seg_map_entries(map, total, n_jobs, t, lane, e_nx, e0_nx);
    };
    next();
    for (;;) {
        const uint64_t t0 = SegTL::now();
        if (t >= n_jobs) break; /* every wave draws one ticket past the end */
        const uint32_t e = e_nx, e0 = e0_nx;
        uint32_t key[8];
        SegLane q = seg_ragged_lane(a, e, e0, key);
        seg_blocks(q);
        SegIOL io;
        io.tab = owners[w];
        io.init(q, lane);
        const bool inplace = q.src == q.dst;
        tl.add(1, SegTL::now() - t0);
        seg_job<OPEN, false>(q, key, io, lane, tiles[w], a.status, a.vf != 0, inplace, tl, next);
        const uint64_t td = SegTL::now();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* the job's stores left before the tile is reused */
        __builtin_amdgcn_wave_barrier();
        tl.add(6, SegTL::now() - td);
        tl.add(7, 1);
    }
    tl.add(0, SegTL::now() - born);
    tl.flush();
}

} // namespace na
