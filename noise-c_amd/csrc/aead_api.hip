/*
 * aead_api.hip — the thin C-ABI layer between the plain-C host front end
 * (cipherstate.c) and the gfx950 kernels.  Device-resident entry points of
 * include/noise_aead_hip.h: plain pointers, sizes and an opaque stream; no
 * C++ or torch types cross this boundary.  HIP errors map to
 * NOISE_ERROR_SYSTEM (constants.h:137), bad arguments to
 * NOISE_ERROR_INVALID_PARAM / _INVALID_LENGTH / _UNKNOWN_ID.
 */
#include "launch.h"
#include <cstdlib>
#include <cstring>

#include "kdf.hip"
#include "pad.hip"

using namespace na;

namespace {

/* Lanes per record for ChaChaPoly: 4 (the fastest split at 64 Ki and 1 Mi
   records, profiles/r01_sweep_*), 8 when the batch is too small to give
   every SIMD four waves that way.  Batches of at most WIDE_MAX_RECORDS — the
   single-call latency path, where a long record's blocks would otherwise run
   serially on a few lanes — get wider groups, up to one wave per record, but
   no wider than the longest record needs (two ChaCha blocks per lane;
   max_len = 0 when unknown).  Larger pipelined chunks (≈ 3 K records of
   1400 B) measured faster at 8 (profiles/r01_hostpaths_ab). */
constexpr uint32_t WIDE_MAX_RECORDS = 512;

int auto_lanes(uint32_t n_records, uint32_t max_len)
{
    const uint64_t target = 256ull * 16 * 64; /* 4 waves on each of 1024 SIMDs */
    if (n_records > WIDE_MAX_RECORDS) /* throughput regime: 4, or 8 below 64 Ki */
        return (uint64_t)n_records * 4 < target ? 8 : 4;
    int k = 4;
    while (k < 64 && (uint64_t)n_records * k < target) k <<= 1;
    if (max_len) {
        const uint32_t blocks = (max_len + 63) / 64 + 1;
        int need = 4;
        while (need < 64 && (uint32_t)need * 2 < blocks) need <<= 1;
        if (k > need) k = need;
    }
    return k;
}

/* FAST layout (chachapoly.hip): 16-B aligned record slots whose input may be
   read up to roundup64(len) — and, for open, holds CT || tag. */
bool uniform_fast(const NoiseAeadUniform *j, bool open)
{
    const uint64_t a = (uint64_t)(uintptr_t)j->in | (uint64_t)(uintptr_t)j->out |
                       j->in_stride | j->out_stride;
    if (a & 15) return false;
    const uint64_t need = ((uint64_t)(j->len ? j->len : 1) + 63) & ~63ull;
    if (j->in_stride < need) return false;
    if (open && j->in_stride < (uint64_t)j->len + 16) return false;
    return true;
}


/* One lane per record (chachapoly.hip seal_solo_staged) for the duplex
   launch of two uniform FAST jobs of at least SOLO_MIN_RECORDS each: one
   Poly1305 chain per record with the clamped r, the per-record work paid
   once per 64 records, and a seal and an open wave on every SIMD; C2
   +8-17 %, C4 +13-18 % over four lanes (profiles/r04/solo_ab.jsonl,
   solo_prio_ab.jsonl).  A standalone seal or open takes one lane from
   SOLO_MIN_STANDALONE records, two waves per SIMD: C4's 1 Mi records as
   back-to-back seal and open launches 1624-1636 vs 1410-1415 GiB/s at four
   lanes, while a 64 Ki-record job alone (one wave per SIMD) runs 3 % faster
   at four lanes (1315-1321 vs 1280-1283, profiles/r04/separate_lanes_ab.jsonl);
   a verify-first open (the default) too since round 6's 4/8-lane
   verify-first staged kernel (chachapoly.hip open_il_staged_vf): 1388-1389
   vs 1236-1262 GiB/s at 64 Ki x 1400 B (profiles/r06/vf_staged_ab/).
   NOISE_AEAD_SOLO=0 keeps the 4-lane kernels everywhere (A/B runs). */
constexpr uint32_t SOLO_MIN_RECORDS = 65536;
constexpr uint32_t SOLO_MIN_STANDALONE = 2 * SOLO_MIN_RECORDS;

bool solo_enabled()
{
    static const bool on = [] {
        const char *e = getenv("NOISE_AEAD_SOLO");
        return !(e && e[0] == '0');
    }();
    return on;
}

/* The segmented kernels (chachapoly_seg.hip).  NOISE_AEAD_SEG=0 turns them
   off (the ragged path then keeps the windowed 8-lane kernels); =2 also
   makes a standalone job of SOLO_MIN_RECORDS <= n < SOLO_MIN_STANDALONE FAST
   records take two segments per record (2048 waves at 64 Ki records, two
   per SIMD).  Round 5 measured that shape slower than the four-lane staged
   kernel it would replace — C2 standalone seal 73 vs 63 us
   (profiles/r05/seg2_standalone_ab.jsonl): 7 % fewer VALU instructions than
   four lanes but 16 % more than one lane per record (the split's second
   chain, r^e, the 24th block slot), and two waves of six steps per SIMD
   issue 11 % slower than the duplex launch's seal + open pair — so the
   default keeps four lanes there.  lanes_per_record = 2 on a FAST layout
   always takes it. */
int seg_mode()
{
    static const int v = [] {
        const char *e = getenv("NOISE_AEAD_SEG");
        return e ? (e[0] == '0' ? 0 : (e[0] == '2' ? 2 : 1)) : 1;
    }();
    return v;
}

bool seg_enabled() { return seg_mode() != 0; }

int standalone_lanes(uint32_t n)
{
    if (n >= SOLO_MIN_STANDALONE) return 1;
    return seg_mode() == 2 ? 2 : 0;
}

int uniform_lanes(const NoiseAeadUniform *j, bool open, bool duplex)
{
    if (j->lanes_per_record) return (int)j->lanes_per_record;
    if (j->n_records >= SOLO_MIN_RECORDS && solo_enabled() && uniform_fast(j, open)) {
        if (duplex) return 1;
        const int k = standalone_lanes(j->n_records);
        if (k) return k;
    }
    return auto_lanes(j->n_records, 0);
}

/* Ragged FAST ChaChaPoly batches of at least SEG_RAGGED_MIN records with
   automatic lanes take the segmented one-lane kernel (a per-launch plan by
   record length, chachapoly_seg.hip); smaller ones keep the windowed 4/8-lane
   kernels and the wide groups of the latency path. */
constexpr uint32_t SEG_RAGGED_MIN = 16384;
/* The plan packs record << 6 | segment into 32 bits (chachapoly_seg.hip
   seg_plan_place) and counts lanes in 32 bits: batches of 2^26 records or
   more keep the windowed kernels. */
constexpr uint32_t SEG_RAGGED_MAX = 1u << 26;

void job_span(const NoiseAeadUniform *j, bool out, bool open, uint64_t &lo, uint64_t &hi);

/* open = the job is an open (its input holds CT || tag).  In-place jobs must
   be exactly in place (in == out, one stride): records whose input and output
   spans overlap any other way would race with their neighbours' reads (and a
   rejected record's scrub would wipe input other records still need). */
int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); } /* b > 0 */

/* Does any input record [in + i s, in + i s + rin) meet any output record
   [out + k s, out + k s + rout), i, k < n, one stride s for both?  With
   d = out - in they meet iff some m = i - k, |m| < n, has
   d - rin < m s < d + rout. */
bool strided_records_meet(uint64_t in, uint64_t out, uint64_t s, uint64_t rin, uint64_t rout, uint32_t n)
{
    if (!rin || !rout || !n) return false;
    const int64_t d = (int64_t)(out - in), st = (int64_t)s;
    const int64_t m_lo = floor_div(d - (int64_t)rin, st) + 1;  /* smallest m with m s > d - rin */
    const int64_t m_hi = -floor_div(-(d + (int64_t)rout), st) - 1; /* largest m with m s < d + rout */
    const int64_t lo = m_lo > -(int64_t)(n - 1) ? m_lo : -(int64_t)(n - 1);
    const int64_t hi = m_hi < (int64_t)(n - 1) ? m_hi : (int64_t)(n - 1);
    return lo <= hi;
}

int check_uniform(const NoiseAeadUniform *j, bool open)
{
    if (!j || !j->ctx || !j->nonce_base || !j->in || !j->out || !j->recs_per_state)
        return NOISE_ERROR_INVALID_PARAM;
    if (j->ad_len && !j->ad) return NOISE_ERROR_INVALID_PARAM;
    if (j->len > NOISE_MAX_PAYLOAD_LEN - 16) return NOISE_ERROR_INVALID_LENGTH;
    if ((uintptr_t)j->ctx & 15) return NOISE_ERROR_INVALID_PARAM;
    if (j->n_records && !(j->in == j->out && j->in_stride == j->out_stride)) {
        /* records of one stride may interleave (input and output slots
           alternating in one buffer) as long as no two of them meet; other
           layouts need disjoint spans */
        const uint64_t rin = (uint64_t)j->len + (open ? 16u : 0u), rout = (uint64_t)j->len + (open ? 0u : 16u);
        if (j->in_stride == j->out_stride && j->in_stride >= rin && j->in_stride >= rout) {
            if (strided_records_meet((uint64_t)(uintptr_t)j->in, (uint64_t)(uintptr_t)j->out, j->in_stride,
                                     rin, rout, j->n_records))
                return NOISE_ERROR_INVALID_PARAM;
        } else {
            uint64_t il, ih, ol, oh;
            job_span(j, false, open, il, ih);
            job_span(j, true, open, ol, oh);
            if (il < oh && ol < ih) return NOISE_ERROR_INVALID_PARAM;
        }
    }
    return NOISE_ERROR_NONE;
}

UniformArgs to_args(const NoiseAeadUniform *j)
{
    UniformArgs a;
    a.keys = (const uint8_t *)j->ctx;
    a.nonce_base = j->nonce_base;
    a.in = j->in;
    a.out = j->out;
    a.ad = j->ad;
    a.status = j->status;
    a.in_stride = j->in_stride;
    a.out_stride = j->out_stride;
    a.ad_stride = j->ad_stride;
    a.rps = j->recs_per_state;
    a.n_records = j->n_records;
    a.len = j->len;
    a.ad_len = j->ad_len;
    a.balance = 0;
    a.vf = 0;
    return a;
}

/* The open order of a job: verify first — the reference's order
   (cipher-chachapoly.c:135-141, cipher-aesgcm.c:172-188) — for every open
   unless a ChaChaPoly job opts into NOISE_AEAD_FLAG_ONE_PASS (round 6,
   VERDICT r5 item 1; the one-pass order was the ChaChaPoly default through
   round 5, DESIGN.md 4.1b gives the cost).  AES-GCM opens always verify
   first: there it costs nothing (C3 732 vs 726 GiB/s, the C5 AES-GCM open
   0.77 vs 0.82 ms: the GHASH-only pass, then CTR for the verified records,
   profiles/r04_round/).  VERIFY_FIRST overrides ONE_PASS. */
bool flags_vf(uint32_t flags)
{
    return (flags & NOISE_AEAD_FLAG_VERIFY_FIRST) || !(flags & NOISE_AEAD_FLAG_ONE_PASS);
}

bool open_vf(int cipher_id, uint32_t flags, bool open)
{
    return open && (flags_vf(flags) || cipher_id == NOISE_CIPHER_AESGCM);
}


/* NOISE_AEAD_FLAG_CT_GHASH, or NOISE_AEAD_CT_GHASH=1 in the environment
   (read once) for every job */
bool ct_ghash(uint32_t flags)
{
    static const bool env = [] {
        const char *e = getenv("NOISE_AEAD_CT_GHASH");
        return e && e[0] == '1';
    }();
    return (flags & NOISE_AEAD_FLAG_CT_GHASH) || env;
}

int run_uniform(int cipher_id, const NoiseAeadUniform *job, void *stream, bool open)
{
    int rc = check_uniform(job, open);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    UniformArgs a = to_args(job);
    a.vf = open_vf(cipher_id, job->flags, open);
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY) {
        const int k = uniform_lanes(job, open, false);
        const bool ukey = (k >= 4 || k == 1) && job->recs_per_state % (64u / (uint32_t)k) == 0;
        /* 4 resident waves on each of 1024 SIMDs (NA_UNIFORM_OCC): one
           generation balances its waves' progress (open: profiles/r01_prio_ab
           .jsonl; seal: neutral in round 2, +3-8 % once the key stream ran in
           runs, the early toggles of chachapoly.hip slot_block) */
        a.balance = (uint64_t)job->n_records * (uint32_t)k <= 4096ull * 64;
        return chacha_uniform(a, k, open, uniform_fast(job, open), ukey, s);
    }
    if (cipher_id == NOISE_CIPHER_AESGCM) {
        if (job->lanes_per_record && job->lanes_per_record != GCM_LANES)
            return NOISE_ERROR_INVALID_PARAM;
        rc = hip_rc(ensure_aes_tables());
        if (rc) return rc;
        /* one state per 256-record workgroup + FAST layout -> LDS-staged kernel */
        return aes_uniform(a, open, ct_ghash(job->flags),
                           uniform_fast(job, open) && job->recs_per_state % GCM_WG_RECS == 0, s);
    }
    return NOISE_ERROR_UNKNOWN_ID;
}

/* Byte span [lo, hi) a uniform job's input (or output) records occupy. */
void job_span(const NoiseAeadUniform *j, bool out, bool open, uint64_t &lo, uint64_t &hi)
{
    const uint64_t base = (uint64_t)(uintptr_t)(out ? (const void *)j->out : (const void *)j->in);
    const uint64_t stride = out ? j->out_stride : j->in_stride;
    const uint64_t rec = (uint64_t)j->len + ((out != open) ? 16u : 0u); /* CT || tag side */
    lo = base;
    hi = j->n_records ? base + (uint64_t)(j->n_records - 1) * stride + rec : base;
}

bool spans_overlap(const NoiseAeadUniform *a, bool a_out, bool a_open,
                   const NoiseAeadUniform *b, bool b_out, bool b_open)
{
    uint64_t al, ah, bl, bh;
    job_span(a, a_out, a_open, al, ah);
    job_span(b, b_out, b_open, bl, bh);
    return al < bh && bl < ah;
}

/* [lo, hi) of a job's AD (lo == hi: none) and of its status array */
void ad_span(const NoiseAeadUniform *j, uint64_t &lo, uint64_t &hi)
{
    lo = hi = (uint64_t)(uintptr_t)j->ad;
    if (j->ad_len && j->n_records) hi = lo + (uint64_t)(j->n_records - 1) * j->ad_stride + j->ad_len;
}

void status_span(const NoiseAeadUniform *j, uint64_t &lo, uint64_t &hi)
{
    lo = hi = (uint64_t)(uintptr_t)j->status;
    if (j->status) hi = lo + j->n_records;
}

bool range_hits_output(uint64_t lo, uint64_t hi, const NoiseAeadUniform *j, bool open)
{
    if (lo == hi) return false;
    uint64_t ol, oh;
    job_span(j, true, open, ol, oh);
    if (lo < oh && ol < hi) return true;
    if (open && j->status) {
        uint64_t sl, sh;
        status_span(j, sl, sh);
        if (lo < sh && sl < hi) return true;
    }
    return false;
}

int run_duplex(int cipher_id, const NoiseAeadUniform *sj, const NoiseAeadUniform *oj, void *stream)
{
    int rc = check_uniform(sj, false);
    if (!rc) rc = check_uniform(oj, true);
    if (rc) return rc;
    /* independent jobs: nothing one job writes (records, statuses) may overlap
       anything the other reads (records, AD) or writes */
    if (sj->n_records && oj->n_records) {
        uint64_t lo, hi;
        bool clash = spans_overlap(sj, true, false, oj, false, true) ||
                     spans_overlap(sj, true, false, oj, true, true) ||
                     spans_overlap(oj, true, true, sj, false, false);
        ad_span(oj, lo, hi);
        clash = clash || range_hits_output(lo, hi, sj, false);
        ad_span(sj, lo, hi);
        clash = clash || range_hits_output(lo, hi, oj, true);
        status_span(oj, lo, hi);
        clash = clash || range_hits_output(lo, hi, sj, false);
        if (oj->status) {
            uint64_t il, ih;
            job_span(sj, false, false, il, ih);
            clash = clash || (lo < ih && il < hi);
        }
        if (clash) return NOISE_ERROR_INVALID_PARAM;
    }
    /* a VERIFY_FIRST open shares a launch only with kernels that run its
       order: the one-lane ChaChaPoly open (AUTH + DEC passes) and the staged
       AES-GCM open (GHASH, verdict, then CTR) */
    const bool vf = open_vf(cipher_id, oj->flags, true);
    UniformArgs oa = to_args(oj);
    oa.vf = vf;
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY && sj->n_records && oj->n_records) {
        const int ks = uniform_lanes(sj, false, true), ko = uniform_lanes(oj, true, true);
        const bool us = (ks >= 4 || ks == 1) && sj->recs_per_state % (64u / (uint32_t)ks) == 0;
        const bool uo = (ko >= 4 || ko == 1) && oj->recs_per_state % (64u / (uint32_t)ko) == 0;
        if (ks == ko && (ks == 1 || ((ks == 4 || ks == 8) && !vf)) && us == uo && uniform_fast(sj, false) &&
            uniform_fast(oj, true)) {
            return chacha_duplex(to_args(sj), oa, ks, us, (hipStream_t)stream);
        }
    }
    if (cipher_id == NOISE_CIPHER_AESGCM && sj->n_records && oj->n_records &&
        !(sj->lanes_per_record && sj->lanes_per_record != GCM_LANES) &&
        !(oj->lanes_per_record && oj->lanes_per_record != GCM_LANES) &&
        uniform_fast(sj, false) && uniform_fast(oj, true) &&
        sj->recs_per_state % GCM_WG_RECS == 0 && oj->recs_per_state % GCM_WG_RECS == 0 &&
        ct_ghash(sj->flags) == ct_ghash(oj->flags)) {
        rc = hip_rc(ensure_aes_tables());
        if (rc) return rc;
        return aes_duplex(to_args(sj), oa, ct_ghash(sj->flags), (hipStream_t)stream);
    }
    rc = run_uniform(cipher_id, sj, stream, false);
    if (!rc) rc = run_uniform(cipher_id, oj, stream, true);
    return rc;
}

int run_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream, bool open)
{
    if (!job || !job->recs || !job->in || !job->out) return NOISE_ERROR_INVALID_PARAM;
    hipStream_t s = (hipStream_t)stream;
    RaggedArgs a;
    a.keys = (const uint8_t *)job->ctx_base;
    a.recs = (const RecDesc *)job->recs;
    a.in = job->in;
    a.out = job->out;
    a.ad = job->ad;
    a.status = job->status;
    a.n_records = job->n_records;
    a.vf = open_vf(cipher_id, job->flags, open);
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY) {
        int k = job->lanes_per_record ? (int)job->lanes_per_record : auto_lanes(job->n_records, 0);
        /* ragged records are often long (C5 mixes 64 B-16 KiB): 8 lanes up to
           128 Ki records, two generations of waves that even out the mixed
           lengths (C5's ChaCha kernels -2.5 % seal / -4 % open at 64 Ki
           records vs 4 lanes, profiles/r02/c5_lanes_ab.jsonl) */
        if (!job->lanes_per_record && k == 4 && job->n_records < 2u * 65536u) k = 8;
        if (!job->lanes_per_record && (job->flags & NOISE_AEAD_FLAG_FAST) && job->n_records >= SEG_RAGGED_MIN &&
            job->n_records < SEG_RAGGED_MAX && seg_enabled())
            return chacha_ragged_seg(a, open, s);
        return chacha_ragged(a, k, open, (job->flags & NOISE_AEAD_FLAG_FAST) != 0, s);
    }
    if (cipher_id == NOISE_CIPHER_AESGCM) {
        int rc = hip_rc(ensure_aes_tables());
        if (rc) return rc;
        /* small batch with automatic lanes: a workgroup per record (latency);
           lanes_per_record = 4 keeps the windowed 4-lane kernels */
        return aes_ragged(a, open, (job->flags & NOISE_AEAD_FLAG_FAST) != 0, ct_ghash(job->flags),
                          job->lanes_per_record == 0 && job->n_records <= WIDE_MAX_RECORDS, s);
    }
    return NOISE_ERROR_UNKNOWN_ID;
}

__global__ void splitmix_fill(uint8_t *out, uint64_t nbytes, uint64_t seed, uint64_t word0)
{
    const uint64_t nw = nbytes / 8;
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w * 8 < nbytes;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + word0 + w + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (w < nw) {
            ((uint64_t *)out)[w] = z;
        } else {
            for (uint64_t b = 0; b < nbytes - 8 * w; ++b) out[8 * w + b] = (uint8_t)(z >> (8 * b));
        }
    }
}

} // namespace

static_assert(sizeof(NoiseAeadRecord) == sizeof(RecDesc), "record descriptor layout");
static_assert(sizeof(NoiseRandSnapshot) == sizeof(RandSnap), "RandState snapshot layout");
static_assert(offsetof(NoiseAeadRecord, ctx_off) == offsetof(RecDesc, ctx_off), "layout");

extern "C" {

size_t noise_aead_dev_ctx_bytes(int cipher_id)
{
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY) return 32;
    if (cipher_id == NOISE_CIPHER_AESGCM) return sizeof(AesCtx);
    return 0;
}

int noise_aead_dev_prepare(int cipher_id, const uint8_t *d_raw_keys, uint32_t n_states,
                           void *d_ctx, void *stream)
{
    if (!d_raw_keys || !d_ctx) return NOISE_ERROR_INVALID_PARAM;
    if (n_states == 0) return NOISE_ERROR_NONE;
    hipStream_t s = (hipStream_t)stream;
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY)
        return hip_rc(hipMemcpyAsync(d_ctx, d_raw_keys, (size_t)n_states * 32,
                                     hipMemcpyDeviceToDevice, s));
    if (cipher_id == NOISE_CIPHER_AESGCM) {
        int rc = hip_rc(ensure_aes_tables());
        if (rc) return rc;
        return aes_prepare(d_raw_keys, n_states, d_ctx, s);
    }
    return NOISE_ERROR_UNKNOWN_ID;
}

int noise_aead_dev_seal_uniform(int cipher_id, const NoiseAeadUniform *job, void *stream)
{
    return run_uniform(cipher_id, job, stream, false);
}

int noise_aead_dev_open_uniform(int cipher_id, const NoiseAeadUniform *job, void *stream)
{
    return run_uniform(cipher_id, job, stream, true);
}

int noise_aead_dev_duplex_uniform(int cipher_id, const NoiseAeadUniform *seal_job,
                                  const NoiseAeadUniform *open_job, void *stream)
{
    return run_duplex(cipher_id, seal_job, open_job, stream);
}

int noise_aead_dev_seal_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream)
{
    return run_ragged(cipher_id, job, stream, false);
}

int noise_aead_dev_open_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream)
{
    return run_ragged(cipher_id, job, stream, true);
}

int noise_aead_dev_fill_splitmix(uint8_t *d_out, uint64_t nbytes, uint64_t seed,
                                 uint64_t word0, void *stream)
{
    if (!d_out) return NOISE_ERROR_INVALID_PARAM;
    if (!nbytes) return NOISE_ERROR_NONE;
    uint64_t words = (nbytes + 7) / 8;
    uint32_t blocks = (uint32_t)((words + 255) / 256);
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(splitmix_fill, dim3(blocks), dim3(256), 0, (hipStream_t)stream, d_out,
                       nbytes, seed, word0);
    return hip_rc(hipGetLastError());
}

int noise_aead_dev_hkdf(int hash_id, const uint8_t *d_keys, uint32_t key_len,
                        const uint8_t *d_data, uint32_t data_len, uint32_t n, uint8_t *d_out1,
                        uint32_t out1_len, uint8_t *d_out2, uint32_t out2_len, void *stream)
{
    uint32_t hl;
    switch (hash_id) {
    case NOISE_HASH_BLAKE2s: case NOISE_HASH_SHA256: hl = 32; break;
    case NOISE_HASH_BLAKE2b: case NOISE_HASH_SHA512: hl = 64; break;
    default: return NOISE_ERROR_UNKNOWN_ID;
    }
    if (!n) return NOISE_ERROR_NONE;
    if (!d_keys || !d_out1 || !d_out2 || (data_len && !d_data)) return NOISE_ERROR_INVALID_PARAM;
    /* hashstate.c:496-497 */
    if (out1_len > hl || out2_len > hl) return NOISE_ERROR_INVALID_LENGTH;
    if (key_len == 0 || key_len > KDF_MAX_IN || data_len > KDF_MAX_IN)
        return NOISE_ERROR_INVALID_LENGTH;
    KdfArgs a;
    a.hash_id = hash_id;
    a.keys = d_keys;
    a.data = data_len ? d_data : nullptr;
    a.out1 = d_out1;
    a.out2 = d_out2;
    a.key_len = key_len;
    a.data_len = data_len;
    a.out1_len = out1_len;
    a.out2_len = out2_len;
    a.n = n;
    hipLaunchKernelGGL(hkdf_batch, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, a);
    return hip_rc(hipGetLastError());
}

int noise_aead_dev_split(int hash_id, const uint8_t *d_ck, uint32_t n, uint8_t *d_k1,
                         uint8_t *d_k2, void *stream)
{
    const uint32_t hl = (hash_id == NOISE_HASH_BLAKE2b || hash_id == NOISE_HASH_SHA512) ? 64 : 32;
    return noise_aead_dev_hkdf(hash_id, d_ck, hl, nullptr, 0, n, d_k1, 32, d_k2, 32, stream);
}

static uint32_t hash_len_of(int hash_id)
{
    switch (hash_id) {
    case NOISE_HASH_BLAKE2s: case NOISE_HASH_SHA256: return 32;
    case NOISE_HASH_BLAKE2b: case NOISE_HASH_SHA512: return 64;
    }
    return 0;
}

static int launch_mix_hash(int hash_id, uint32_t hl, const uint8_t *h_in, uint8_t *h_out,
                           const NoiseAeadRagged *job, bool use_out, hipStream_t s)
{
    MixHashArgs m;
    m.hash_id = hash_id;
    m.hlen = hl;
    m.n = job->n_records;
    m.h_in = h_in;
    m.h_out = h_out;
    m.base = use_out ? job->out : job->in;
    m.recs = (const RecDesc *)job->recs;
    m.use_out_off = use_out;
    hipLaunchKernelGGL(mix_hash_batch, dim3((job->n_records + 63) / 64), dim3(64), 0, s, m);
    return hip_rc(hipGetLastError());
}

int noise_aead_dev_encrypt_and_hash(int cipher_id, int hash_id, uint8_t *d_h,
                                    const NoiseAeadRagged *job, void *stream)
{
    const uint32_t hl = hash_len_of(hash_id);
    if (!hl) return NOISE_ERROR_UNKNOWN_ID;
    if (!d_h || !job || job->ad != d_h) return NOISE_ERROR_INVALID_PARAM;
    if (job->n_records == 0) return NOISE_ERROR_NONE;
    int rc = run_ragged(cipher_id, job, stream, false);
    if (rc) return rc;
    return launch_mix_hash(hash_id, hl, d_h, d_h, job, true, (hipStream_t)stream);
}

int noise_aead_dev_decrypt_and_hash(int cipher_id, int hash_id, uint8_t *d_h,
                                    const NoiseAeadRagged *job, void *stream)
{
    const uint32_t hl = hash_len_of(hash_id);
    if (!hl) return NOISE_ERROR_UNKNOWN_ID;
    if (!d_h || !job || job->ad != d_h || !job->status) return NOISE_ERROR_INVALID_PARAM;
    if (job->n_records == 0) return NOISE_ERROR_NONE;
    hipStream_t s = (hipStream_t)stream;
    const size_t bytes = (size_t)job->n_records * hl;
    uint8_t *h_new = nullptr;
    /* stream-ordered pool allocation: no device synchronisation, and after
       the first call the pool hands the same memory back */
    if (hipMallocAsync((void **)&h_new, bytes, s) != hipSuccess) return NOISE_ERROR_NO_MEMORY;
    /* hash the ciphertext before the (in-place) decryption overwrites it */
    int rc = launch_mix_hash(hash_id, hl, d_h, h_new, job, false, s);
    if (!rc) rc = run_ragged(cipher_id, job, stream, true);
    if (!rc) {
        const uint64_t total = (uint64_t)job->n_records * hl;
        hipLaunchKernelGGL(commit_hash, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, d_h,
                           (const uint8_t *)h_new, (const uint8_t *)job->status, hl,
                           job->n_records);
        rc = hip_rc(hipGetLastError());
    }
    (void)hipFreeAsync(h_new, s);
    return rc;
}

int noise_aead_dev_pad(NoiseRandSnapshot *d_rand, uint8_t *d_payloads, uint64_t stride,
                       const uint32_t *d_orig_lens, uint32_t padded_len, uint32_t n,
                       int padding_mode, uint32_t *d_done, void *stream)
{
    if (!d_payloads || (n && !d_orig_lens)) return NOISE_ERROR_INVALID_PARAM;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) { /* NULL state: INVALID_PARAM on both branches (randstate.c:356-362) */
        const int rc = d_done ? hip_rc(hipMemsetAsync(d_done, 0, sizeof(uint32_t), s)) : NOISE_ERROR_NONE;
        return rc ? rc : (d_rand ? NOISE_ERROR_NONE : NOISE_ERROR_INVALID_PARAM);
    }
    if (!d_rand || padding_mode == NOISE_PADDING_ZERO) {
        /* randstate.c:356-362: without a state the padding is zeroed anyway */
        hipLaunchKernelGGL(pad_zero, dim3(n < 65535u ? n : 65535u), dim3(256), 0, s, d_payloads,
                           stride, d_orig_lens, padded_len, n, d_done);
        const int rc = hip_rc(hipGetLastError());
        return rc ? rc : (d_rand ? NOISE_ERROR_NONE : NOISE_ERROR_INVALID_PARAM);
    }
    hipLaunchKernelGGL(pad_random, dim3(1), dim3(64), 0, s, (RandSnap *)d_rand, d_payloads, stride,
                       d_orig_lens, padded_len, n, d_done);
    return hip_rc(hipGetLastError());
}

int noise_aead_dev_default_lanes(int cipher_id, uint32_t n_records)
{
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY) {
        if (n_records >= SOLO_MIN_RECORDS && solo_enabled() && standalone_lanes(n_records))
            return standalone_lanes(n_records);
        return auto_lanes(n_records, 0);
    }
    if (cipher_id == NOISE_CIPHER_AESGCM) return GCM_LANES;
    return 0;
}

int noise_aead_dev_duplex_lanes(int cipher_id, uint32_t n_records)
{
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY && n_records >= SOLO_MIN_RECORDS && solo_enabled()) return 1;
    return noise_aead_dev_default_lanes(cipher_id, n_records);
}

/* NOISE_AEAD_LANES=narrow: the host paths keep K <= 8 and the 4-lane AES
   kernels (an A/B switch for measurements). */
static bool lanes_narrow()
{
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("NOISE_AEAD_LANES");
        v = e && strcmp(e, "narrow") == 0;
    }
    return v != 0;
}

/* host_internal.h: the host paths know their records' lengths */
__attribute__((visibility("hidden"))) uint32_t na_chacha_lanes(uint32_t n_records, uint32_t max_len)
{
    if (lanes_narrow()) return (uint64_t)n_records * 4 < 256ull * 16 * 64 ? 8 : 4;
    return (uint32_t)auto_lanes(n_records, max_len ? max_len : 1);
}

__attribute__((visibility("hidden"))) uint32_t na_aes_lanes(uint32_t n_records)
{
    (void)n_records;
    return lanes_narrow() ? GCM_LANES : 0;
}

} // extern "C"
