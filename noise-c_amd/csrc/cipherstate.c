/*
 * cipherstate.c — plain-C host front end of the MI355X AEAD engine.
 *
 * Re-implements noise-c's CipherState surface (src/protocol/cipherstate.c
 * :77-555) with the same argument validation, nonce rules and error codes,
 * and provides the two cipher "plugins" noise-c's front end dispatches to
 * (src/protocol/internal.h:58-146, 655-656).  The plugins' encrypt/decrypt
 * ops run on the GPU through the thin C-ABI of aead_api.hip; this file does
 * no cryptographic arithmetic at all — it validates, assigns nonces, stages
 * bytes and launches.
 */
#define _DEFAULT_SOURCE
#include "host_internal.h"
#include "host_pool.h"

#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <time.h>

/* ---------------------------------------------------- util.c equivalents */

void na_clean(void *p, size_t n) /* util.c:170-177 noise_clean */
{
    volatile uint8_t *d = (volatile uint8_t *)p;
    while (n--) *d++ = 0;
}

static void *new_object(size_t size) /* util.c:135-142 noise_new_object */
{
    struct NoiseCipherState_s *obj = (struct NoiseCipherState_s *)calloc(1, size);
    if (obj) obj->size = size;
    return obj;
}

static void free_object(void *ptr, size_t size) /* util.c:152-158 noise_free */
{
    if (!ptr) return;
    na_clean(ptr, size);
    free(ptr);
}

/* ------------------------------------------------------ per-thread staging */

/* The batch path moves records through one pinned host area and one device
   area per thread, cut into chunks that form a pipeline:
     host threads pack chunk c+1 while chunk c crosses PCIe (copy-in stream)
     and runs on the GPU, and the host unpacks chunk c-1 as its D2H lands.
   H2D and D2H use different streams, so both PCIe directions are busy. */
static pthread_key_t g_stage_key;
static pthread_once_t g_stage_once = PTHREAD_ONCE_INIT;

static void stage_destroy(void *p)
{
    Staging *s = (Staging *)p;
    if (!s) return;
    if (s->h) (void)hipHostFree(s->h);
    if (s->d) (void)hipFree(s->d);
    for (int i = 0; i < MAX_CHUNKS; ++i) {
        if (s->ev_in[i]) (void)hipEventDestroy(s->ev_in[i]);
        if (s->ev_out[i]) (void)hipEventDestroy(s->ev_out[i]);
        if (s->ev_done[i]) (void)hipEventDestroy(s->ev_done[i]);
    }
    if (s->stream_out) (void)hipStreamDestroy(s->stream_out);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->stream_in) (void)hipStreamDestroy(s->stream_in);
    free(s);
}

static void stage_key_init(void) { pthread_key_create(&g_stage_key, stage_destroy); }

/* Staging area of at least `bytes` on the current device, or NULL. */
Staging *na_stage_get(size_t bytes)
{
    pthread_once(&g_stage_once, stage_key_init);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return NULL;
    Staging *s = (Staging *)pthread_getspecific(g_stage_key);
    if (s && s->device != dev) {
        stage_destroy(s);
        s = NULL;
        pthread_setspecific(g_stage_key, NULL);
    }
    if (!s) {
        s = (Staging *)calloc(1, sizeof(Staging));
        if (!s) return NULL;
        s->device = dev;
        int ok = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess &&
                 hipStreamCreateWithFlags(&s->stream_in, hipStreamNonBlocking) == hipSuccess &&
                 hipStreamCreateWithFlags(&s->stream_out, hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; ok && i < MAX_CHUNKS; ++i)
            ok = hipEventCreateWithFlags(&s->ev_in[i], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&s->ev_out[i], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&s->ev_done[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            stage_destroy(s);
            return NULL;
        }
        pthread_setspecific(g_stage_key, s);
    }
    if (s->cap < bytes) {
        size_t cap = s->cap ? s->cap : (size_t)1 << 20;
        while (cap < bytes) cap <<= 1;
        if (s->h) (void)hipHostFree(s->h);
        if (s->d) (void)hipFree(s->d);
        s->h = NULL;
        s->hd = NULL;
        s->d = NULL;
        s->cap = 0;
        if (hipHostMalloc((void **)&s->h, cap, hipHostMallocDefault) != hipSuccess) return NULL;
        if (hipHostGetDevicePointer((void **)&s->hd, s->h, 0) != hipSuccess) return NULL;
        if (hipMalloc((void **)&s->d, cap) != hipSuccess) return NULL;
        s->cap = cap;
    }
    return s;
}

/* --------------------------------------------------- device key contexts */

/* Key-context memory is recycled, never handed back to HIP while the
   library runs: hipFree / hipHostFree wait for every stream of the device,
   and a resident worker group (worker.hip) ends only after 2 ms without
   calls, up to its 5 s lifetime while calls keep coming — freeing one state
   used to stall for seconds beside another thread's single calls.  A
   released context is scrubbed first (device: zeroed and waited for; host
   copy: na_clean) and then kept on a free list per device, kind and size;
   the lists hold at most the peak number of live states' contexts. */
typedef struct CtxBuf {
    void *p;
    size_t bytes;
    int device, host;
    struct CtxBuf *next;
} CtxBuf;
static CtxBuf *g_ctx_free;
static pthread_mutex_t g_ctx_mu = PTHREAD_MUTEX_INITIALIZER;

static void *ctx_take(int device, int host, size_t bytes)
{
    pthread_mutex_lock(&g_ctx_mu);
    for (CtxBuf **pp = &g_ctx_free; *pp; pp = &(*pp)->next) {
        CtxBuf *b = *pp;
        if (b->device == device && b->host == host && b->bytes == bytes) {
            *pp = b->next;
            pthread_mutex_unlock(&g_ctx_mu);
            void *p = b->p;
            free(b);
            return p;
        }
    }
    pthread_mutex_unlock(&g_ctx_mu);
    return NULL;
}

/* p already scrubbed; if the list node cannot be had, the memory is freed
   (and that free may wait for the device, as before) */
static void ctx_give(void *p, int device, int host, size_t bytes)
{
    CtxBuf *b = (CtxBuf *)malloc(sizeof(CtxBuf));
    if (!b) {
        if (host) (void)hipHostFree(p);
        else (void)hipFree(p);
        return;
    }
    b->p = p;
    b->bytes = bytes;
    b->device = device;
    b->host = host;
    pthread_mutex_lock(&g_ctx_mu);
    b->next = g_ctx_free;
    g_ctx_free = b;
    pthread_mutex_unlock(&g_ctx_mu);
}

/* (worker_crypt) the pinned host copy of an AES-GCM context */
static int h_ctx_alloc(HipCipherState *st, size_t bytes)
{
    st->h_ctx = ctx_take(-1, 1, bytes);
    if (st->h_ctx) return 0;
    if (hipHostMalloc((void **)&st->h_ctx, bytes, hipHostMallocMapped | hipHostMallocCoherent |
                                                   hipHostMallocPortable) != hipSuccess) {
        st->h_ctx = NULL;
        return -1;
    }
    return 0;
}


/* Zero n bytes of device memory on `device` and wait for it, so that key
   material is gone before the allocation can be handed out again
   (util.c:152-158 zeroes every freed object).  Restores the current device. */
static void scrub_device(void *p, size_t n, int device)
{
    if (!p || !n) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    if (hipMemsetAsync(p, 0, n, NULL) == hipSuccess) (void)hipStreamSynchronize(NULL);
    if (cur != device) (void)hipSetDevice(cur);
}

/* Test hook (NOISE_AEAD_DEBUG_KEEP_FREED=1): destroy scrubs a state's device
   context but keeps the allocation, so a test can read back that it was
   zeroed.  Leaks by design; never set in production. */
static void *g_dbg_freed_ctx;
static size_t g_dbg_freed_bytes;

void *noise_aead_debug_last_freed_ctx(size_t *bytes)
{
    if (bytes) *bytes = g_dbg_freed_bytes;
    return g_dbg_freed_ctx;
}

static void release_ctx(HipCipherState *st)
{
    if (st->h_ctx) { /* the worker's pinned copy holds key material too */
        na_worker_forget_ctx(st->h_ctx); /* and so may a worker's LDS cache of it */
        const size_t hb = noise_aead_dev_ctx_bytes(st->parent.cipher_id);
        na_clean(st->h_ctx, hb);
        ctx_give(st->h_ctx, -1, 1, hb);
        st->h_ctx = NULL;
        st->h_ctx_ready = 0;
    }
    if (!st->d_ctx) return;
    const size_t bytes = noise_aead_dev_ctx_bytes(st->parent.cipher_id);
    scrub_device(st->d_ctx, bytes, st->device); /* the context holds key material */
    const char *keep = getenv("NOISE_AEAD_DEBUG_KEEP_FREED");
    if (keep && *keep == '1') {
        g_dbg_freed_ctx = st->d_ctx;
        g_dbg_freed_bytes = bytes;
    } else {
        ctx_give(st->d_ctx, st->device, 0, bytes);
    }
    st->d_ctx = NULL;
    st->ctx_ready = 0;
}

/* Build the device key context of `st` from its key (lazy: init_key has no
   error return in the plugin ABI, internal.h:95).  A context belongs to the
   device it was built on: used from another device it is scrubbed and
   rebuilt there, never passed to a kernel on the wrong device. */
int na_ensure_ctx(HipCipherState *st, Staging *sg)
{
    const int dev = sg->device;
    if (st->ctx_ready && st->d_ctx && st->device == dev) return NOISE_ERROR_NONE;
    if (st->d_ctx && st->device != dev) release_ctx(st);
    st->ctx_ready = 0;
    if (!st->d_ctx) {
        size_t bytes = noise_aead_dev_ctx_bytes(st->parent.cipher_id);
        st->d_ctx = ctx_take(dev, 0, bytes);
        if (!st->d_ctx && hipMalloc(&st->d_ctx, bytes) != hipSuccess) {
            st->d_ctx = NULL;
            return NOISE_ERROR_SYSTEM;
        }
        st->device = dev;
    }
    /* raw key through the tail of the staging area; both copies are zeroed
       again on every path out */
    uint8_t *h = sg->h + sg->cap - 32;
    uint8_t *d = sg->d + sg->cap - 32;
    memcpy(h, st->key, 32);
    int rc = NOISE_ERROR_NONE;
    if (hipMemcpyAsync(d, h, 32, hipMemcpyHostToDevice, sg->stream) != hipSuccess)
        rc = NOISE_ERROR_SYSTEM;
    if (!rc) rc = noise_aead_dev_prepare(st->parent.cipher_id, d, 1, st->d_ctx, sg->stream);
    (void)hipMemsetAsync(d, 0, 32, sg->stream);
    if (hipStreamSynchronize(sg->stream) != hipSuccess && !rc) rc = NOISE_ERROR_SYSTEM;
    na_clean(h, 32);
    if (rc) return rc;
    st->ctx_ready = 1;
    return NOISE_ERROR_NONE;
}

/* ------------------------------------------------------------ GPU runner */

typedef struct {
    HipCipherState *st;
    const uint8_t *ad;
    size_t ad_len;
    uint8_t *data;     /* record; tag at data + len */
    size_t len;        /* plaintext (seal) / ciphertext-without-tag (open) */
    uint64_t nonce;
    size_t idx;        /* caller's record index */
    int skip;          /* in: not dispatched (nonce exhausted) */
    int forge;         /* in (batch open): tried at the state's current n, as
                          the record after a MAC failure is */
    int status;        /* out: NOISE_ERROR_NONE / _MAC_FAILURE / _SYSTEM */
    int commit;        /* set by the decide step: copy the result to data */
    int defer;         /* set by the decide step: retry in a later round */
    size_t off, ad_off; /* staging offsets of the record slot and its AD */
    uint32_t desc;     /* descriptor index within its chunk */
} Job;

/* Decide, in record order, which finished jobs of [lo, hi) commit.  Called
   once per chunk, chunks in order, so every earlier record's fate is known. */
typedef void (*decide_fn)(Job *jobs, size_t lo, size_t hi, void *u);

typedef struct {
    size_t j0, j1;              /* jobs [j0, j1) */
    size_t recs_off, status_off, payload_off, end;
    uint32_t n_chacha, n_aes;
    uint32_t chacha_max_len;    /* longest ChaChaPoly record (lane choice) */
} Chunk;

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

/* A record's staging slot: 16-B aligned, readable up to roundup64(len) and
   large enough for CT || tag — the NOISE_AEAD_FLAG_FAST layout. */
static size_t slot_bytes(size_t len)
{
    size_t a = ((len ? len : 1) + 63) & ~(size_t)63, b = align16(len + 16);
    return a > b ? a : b;
}

static size_t job_bytes(const Job *j)
{
    return j->skip ? 0 : sizeof(NoiseAeadRecord) + 1 + align16(j->ad_len) + slot_bytes(j->len);
}

typedef struct {
    Job *jobs;
    uint8_t *h;
    int open;
} CopyArg;

static void pack_range(void *p, size_t lo, size_t hi)
{
    CopyArg *a = (CopyArg *)p;
    for (size_t k = lo; k < hi; ++k) {
        const Job *j = &a->jobs[k];
        if (j->skip) continue;
        if (j->ad_len) memcpy(a->h + j->ad_off, j->ad, j->ad_len);
        memcpy(a->h + j->off, j->data, j->len + (a->open ? 16 : 0));
    }
}

/* Copy committed results out.  Open: every slot the GPU wrote plaintext into
   (a verified record, committed or deferred) is zeroed right after, while its
   lines are still in cache — failed records hold only their ciphertext, so no
   second pass over the whole staging area is needed. */
static void unpack_range(void *p, size_t lo, size_t hi)
{
    CopyArg *a = (CopyArg *)p;
    for (size_t k = lo; k < hi; ++k) {
        const Job *j = &a->jobs[k];
        if (j->commit) memcpy(j->data, a->h + j->off, j->len + (a->open ? 0 : 16));
        if (a->open && !j->skip && j->status == NOISE_ERROR_NONE)
            explicit_bzero(a->h + j->off, j->len);
    }
}

static size_t copy_grain(const Chunk *c, size_t n)
{
    size_t per = (c->end - c->payload_off) / (n ? n : 1) + 1;
    size_t g = ((size_t)256 << 10) / per;
    return g ? g : 1;
}

/* Plan chunk c's staging layout starting at byte `at`; returns its end. */
static size_t plan_chunk(Job *jobs, Chunk *c, size_t at)
{
    size_t nd = 0;
    for (size_t k = c->j0; k < c->j1; ++k) nd += !jobs[k].skip;
    c->recs_off = at;
    c->status_off = align16(at + nd * sizeof(NoiseAeadRecord));
    c->payload_off = align16(c->status_off + nd);
    size_t p = c->payload_off;
    uint32_t desc = 0;
    c->n_chacha = c->n_aes = 0;
    c->chacha_max_len = 0;
    /* ChaCha20-Poly1305 descriptors first, then AES-GCM: one ragged launch each */
    for (int pass = 0; pass < 2; ++pass) {
        int want = pass == 0 ? NOISE_CIPHER_CHACHAPOLY : NOISE_CIPHER_AESGCM;
        for (size_t k = c->j0; k < c->j1; ++k) {
            Job *j = &jobs[k];
            if (j->skip || j->st->parent.cipher_id != want) continue;
            j->desc = desc++;
            j->ad_off = p;
            p += align16(j->ad_len);
            j->off = p;
            p += slot_bytes(j->len);
            if (pass == 0) {
                ++c->n_chacha;
                if (j->len > c->chacha_max_len) c->chacha_max_len = (uint32_t)j->len;
            } else {
                ++c->n_aes;
            }
        }
    }
    c->end = p;
    return (p + 63) & ~(size_t)63;
}

static void fill_descriptors(Job *jobs, const Chunk *c, uint8_t *h)
{
    NoiseAeadRecord *recs = (NoiseAeadRecord *)(h + c->recs_off);
    for (size_t k = c->j0; k < c->j1; ++k) {
        const Job *j = &jobs[k];
        if (j->skip) continue;
        NoiseAeadRecord *r = &recs[j->desc];
        r->in_off = r->out_off = j->off;
        r->nonce = j->nonce;
        r->ctx_off = (uint64_t)(uintptr_t)j->st->d_ctx;
        r->ad_off = j->ad_off;
        r->len = (uint32_t)j->len;
        r->ad_len = (uint32_t)j->ad_len;
    }
}

/* Batches of at most this many staged bytes, in one chunk, skip both DMA
   copies: the kernels read and write the pinned staging area over PCIe
   (zero-copy).  For a single small record that removes two copy-engine round
   trips from the call's latency.  NOISE_AEAD_ZERO_COPY_MAX overrides (0 = off). */
static size_t zero_copy_max(void)
{
    static size_t v = (size_t)-1;
    if (v == (size_t)-1) {
        const char *e = getenv("NOISE_AEAD_ZERO_COPY_MAX");
        v = e ? (size_t)strtoull(e, NULL, 10) : ZERO_COPY_DEFAULT;
    }
    return v;
}

/* Chunk ci: H2D on the copy-in stream, then (on the main stream, after it)
   the ragged kernels and the D2H of statuses + payload — or, zero-copy, the
   kernels alone on the staging bytes in host memory. */
static int launch_chunk(Staging *sg, const Chunk *c, int ci, int open, int zc)
{
    uint8_t *base = zc ? sg->hd : sg->d;
    if (!zc && (hipMemcpyAsync(sg->d + c->recs_off, sg->h + c->recs_off, c->end - c->recs_off,
                               hipMemcpyHostToDevice, sg->stream_in) != hipSuccess ||
                hipEventRecord(sg->ev_in[ci], sg->stream_in) != hipSuccess ||
                hipStreamWaitEvent(sg->stream, sg->ev_in[ci], 0) != hipSuccess))
        return NOISE_ERROR_SYSTEM;
    for (int k = 0; k < 2; ++k) {
        uint32_t first = k == 0 ? 0 : c->n_chacha, count = k == 0 ? c->n_chacha : c->n_aes;
        if (!count) continue;
        NoiseAeadRagged job;
        job.ctx_base = NULL;
        job.recs = (const NoiseAeadRecord *)(base + c->recs_off) + first;
        job.in = base;
        job.out = base;
        job.ad = base;
        job.status = base + c->status_off + first;
        job.n_records = count;
        job.lanes_per_record = k == 0 ? na_chacha_lanes(count, c->chacha_max_len) : na_aes_lanes(count);
        /* opens verify before they decrypt (cipher-chachapoly.c:135-141,
           cipher-aesgcm.c:172-188): the staging slot of a rejected record is
           never written */
        job.flags = NOISE_AEAD_FLAG_FAST | (open ? NOISE_AEAD_FLAG_VERIFY_FIRST : 0);
        job.reserved_ = 0;
        int cid = k == 0 ? NOISE_CIPHER_CHACHAPOLY : NOISE_CIPHER_AESGCM;
        int rc = open ? noise_aead_dev_open_ragged(cid, &job, sg->stream)
                      : noise_aead_dev_seal_ragged(cid, &job, sg->stream);
        if (rc) return rc;
    }
    if ((!zc && hipMemcpyAsync(sg->h + c->status_off, sg->d + c->status_off,
                               c->end - c->status_off, hipMemcpyDeviceToHost,
                               sg->stream) != hipSuccess) ||
        hipEventRecord(sg->ev_out[ci], sg->stream) != hipSuccess)
        return NOISE_ERROR_SYSTEM;
    /* open leaves plaintext in the device staging slots: zero them once the
       D2H has read them (stream order), so no plaintext outlives the call in
       device memory (a seal's slots end up holding only CT || tag) */
    if (open && !zc &&
        hipMemsetAsync(sg->d + c->payload_off, 0, c->end - c->payload_off, sg->stream) != hipSuccess)
        return NOISE_ERROR_SYSTEM;
    return NOISE_ERROR_NONE;
}

/* Wait for chunk ci, read its statuses, let `decide` pick the commits (seal:
   every dispatched job), copy the results out and scrub staged plaintext. */
static int finish_chunk(Staging *sg, Job *jobs, const Chunk *c, int ci, int open,
                        decide_fn decide, void *u, double *t_wait)
{
    double t0 = t_wait ? na_now_ms() : 0;
    if (hipEventSynchronize(sg->ev_out[ci]) != hipSuccess) return NOISE_ERROR_SYSTEM;
    if (t_wait) *t_wait += na_now_ms() - t0;
    for (size_t k = c->j0; k < c->j1; ++k) {
        Job *j = &jobs[k];
        j->commit = j->defer = 0;
        if (j->skip) continue;
        j->status = !open || sg->h[c->status_off + j->desc] == 0 ? NOISE_ERROR_NONE
                                                                 : NOISE_ERROR_MAC_FAILURE;
        if (!decide) j->commit = j->status == NOISE_ERROR_NONE;
    }
    if (decide) decide(jobs, c->j0, c->j1, u);
    CopyArg a = {jobs + c->j0, sg->h, open};
    /* after seal the slots hold only CT || tag (the D2H overwrote every
       staged plaintext byte); after open unpack_range zeroes the plaintext */
    host_pool_for(c->j1 - c->j0, copy_grain(c, c->j1 - c->j0), unpack_range, &a);
    return NOISE_ERROR_NONE;
}

/* NOISE_AEAD_TRACE=1: one stderr line per pipelined call with the time the
   calling thread spent packing, waiting for the GPU and unpacking. */
double na_now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

int na_trace_on(void)
{
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("NOISE_AEAD_TRACE");
        v = e && *e && *e != '0';
    }
    return v;
}

/* Run jobs (any mix of states and ciphers, record order) through the staging
   pipeline.  Fills job.status for every dispatched job and applies the
   commits `decide` selects (NULL: every verified job).  On a HIP error
   returns NOISE_ERROR_SYSTEM; then no job of a chunk that was not finished
   commits and their status is NOISE_ERROR_SYSTEM. */
static int run_jobs(Job *jobs, size_t n, int open, decide_fn decide, void *u)
{
    if (n == 0) return NOISE_ERROR_NONE;
    size_t total = 0;
    for (size_t k = 0; k < n; ++k) {
        jobs[k].status = jobs[k].skip ? NOISE_ERROR_INVALID_NONCE : NOISE_ERROR_SYSTEM;
        jobs[k].commit = jobs[k].defer = 0;
        total += job_bytes(&jobs[k]);
    }
    if (total == 0) { /* nothing to dispatch: only the decide step */
        if (decide) decide(jobs, 0, n, u);
        return NOISE_ERROR_NONE;
    }
    size_t target = total / (MAX_CHUNKS - 1) + 1;
    if (target < CHUNK_MIN) target = CHUNK_MIN;
    Chunk chunks[MAX_CHUNKS];
    int nc = 0;
    size_t at = 0, acc = 0, j0 = 0;
    for (size_t k = 0; k < n; ++k) {
        acc += job_bytes(&jobs[k]);
        if (acc >= target || k + 1 == n) {
            Chunk *c = &chunks[nc++];
            c->j0 = j0;
            c->j1 = k + 1;
            at = plan_chunk(jobs, c, at);
            j0 = k + 1;
            acc = 0;
        }
    }
    Staging *sg = na_stage_get(at + 64);
    if (!sg) return NOISE_ERROR_SYSTEM;
    int rc = NOISE_ERROR_NONE;
    for (size_t k = 0; k < n && !rc; ++k)
        if (!jobs[k].skip) rc = na_ensure_ctx(jobs[k].st, sg);

    int launched = 0, finished = 0;
    const int tr = na_trace_on();
    double t_start = tr ? na_now_ms() : 0, t_pack = 0, t_fin = 0, t_wait = 0, t0 = 0;
    for (int c = 0; c < nc && !rc; ++c) {
        const Chunk *ch = &chunks[c];
        if (tr) t0 = na_now_ms();
        fill_descriptors(jobs, ch, sg->h);
        CopyArg a = {jobs + ch->j0, sg->h, open};
        host_pool_for(ch->j1 - ch->j0, copy_grain(ch, ch->j1 - ch->j0), pack_range, &a);
        if (tr) t_pack += na_now_ms() - t0;
        /* AES-GCM's GHASH lanes read the CT serially: over PCIe that only
           pays for the smallest records (profiles/r01_latency.jsonl) */
        const size_t zmax = zero_copy_max();
        rc = launch_chunk(sg, ch, c, open,
                          nc == 1 && at <= (ch->n_aes && zmax > ZERO_COPY_AES ? ZERO_COPY_AES : zmax));
        if (rc) break;
        ++launched;
        if (c > 0) {
            if (tr) t0 = na_now_ms();
            rc = finish_chunk(sg, jobs, &chunks[c - 1], c - 1, open, decide, u, tr ? &t_wait : NULL);
            if (tr) t_fin += na_now_ms() - t0;
            if (rc) break;
            ++finished;
        }
    }
    if (!rc && finished < launched) {
        if (tr) t0 = na_now_ms();
        rc = finish_chunk(sg, jobs, &chunks[launched - 1], launched - 1, open, decide, u, tr ? &t_wait : NULL);
        if (tr) t_fin += na_now_ms() - t0;
        if (!rc) ++finished;
    }
    if (tr)
        fprintf(stderr, "noise_aead %s: %zu jobs, %d chunks, %zu B staged, %d threads: "
                "total %.3f ms, pack %.3f, finish %.3f (of which GPU wait %.3f)\n",
                open ? "open" : "seal", n, nc, at, host_pool_threads(), na_now_ms() - t_start,
                t_pack, t_fin, t_wait);
    if (rc) { /* drain, fail what did not finish, leave no plaintext behind */
        (void)hipStreamSynchronize(sg->stream_in);
        (void)hipStreamSynchronize(sg->stream);
        for (int c = finished; c < nc; ++c)
            for (size_t k = chunks[c].j0; k < chunks[c].j1; ++k) {
                jobs[k].status = NOISE_ERROR_SYSTEM;
                jobs[k].commit = jobs[k].defer = 0;
            }
        size_t from = finished < nc ? chunks[finished].recs_off : at;
        if (at > from) explicit_bzero(sg->h + from, at - from);
    }
    return rc;
}

/* -------------------------------------------------- plugin vtable entries */

static void hip_init_key(NoiseCipherState *state, const uint8_t *key)
{
    HipCipherState *st = (HipCipherState *)state;
    memcpy(st->key, key, 32);
    st->ctx_ready = 0;
    st->h_ctx_ready = 0;
}

/* A single record through the resident worker (worker.hip): no kernel launch
   per call.  ChaChaPoly passes the key itself; AES-GCM a pinned host copy of
   the state's device context, made once per key.  NOISE_ERROR_NOT_APPLICABLE:
   take the launch path. */
static int worker_crypt(HipCipherState *st, const uint8_t *ad, size_t ad_len, uint8_t *data,
                        size_t len, int open)
{
    if (!na_worker_enabled()) return NOISE_ERROR_NOT_APPLICABLE;
    const void *h = NULL;
    if (st->parent.cipher_id == NOISE_CIPHER_AESGCM) {
        if (!st->h_ctx_ready) {
            const size_t bytes = noise_aead_dev_ctx_bytes(NOISE_CIPHER_AESGCM);
            Staging *sg = na_stage_get(64);
            if (!sg || na_ensure_ctx(st, sg)) return NOISE_ERROR_NOT_APPLICABLE;
            if (!st->h_ctx && h_ctx_alloc(st, bytes)) return NOISE_ERROR_NOT_APPLICABLE;
            if (hipMemcpy(st->h_ctx, st->d_ctx, bytes, hipMemcpyDeviceToHost) != hipSuccess)
                return NOISE_ERROR_NOT_APPLICABLE;
            /* a new generation: the worker's cached copy of this address is stale */
            static uint32_t gen_counter;
            st->h_ctx_gen = __atomic_add_fetch(&gen_counter, 1, __ATOMIC_RELAXED);
            st->h_ctx_ready = 1;
        }
        h = st->h_ctx;
    }
    return na_worker_crypt(st->parent.cipher_id, st->key, h, st->h_ctx_gen, st->parent.n, ad, ad_len,
                           data, len, open);
}

static int hip_crypt(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                     uint8_t *data, size_t len, int open)
{
    const int wrc = worker_crypt((HipCipherState *)state, ad, ad_len, data, len, open);
    if (wrc != NOISE_ERROR_NOT_APPLICABLE) return wrc;
    Job j;
    j.st = (HipCipherState *)state;
    j.ad = ad;
    j.ad_len = ad_len;
    j.data = data;
    j.len = len;
    j.nonce = state->n; /* the backend reads n; the front end owns n++ */
    j.idx = 0;
    j.skip = 0;
    j.forge = 0;
    int rc = run_jobs(&j, 1, open, NULL, NULL);
    return rc ? rc : j.status;
}

static int hip_encrypt(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                       uint8_t *data, size_t len)
{
    return hip_crypt(state, ad, ad_len, data, len, 0);
}

static int hip_decrypt(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                       uint8_t *data, size_t len)
{
    return hip_crypt(state, ad, ad_len, data, len, 1);
}

static void hip_destroy(NoiseCipherState *state)
{
    release_ctx((HipCipherState *)state); /* scrubbed, then freed with the state */
}

static NoiseCipherState *hip_new(int cipher_id, NoiseCipherState *(*create)(void))
{
    HipCipherState *st = (HipCipherState *)new_object(sizeof(HipCipherState));
    if (!st) return NULL;
    st->parent.cipher_id = cipher_id;
    st->parent.key_len = 32;
    st->parent.mac_len = 16;
    st->parent.create = create;
    st->parent.init_key = hip_init_key;
    st->parent.encrypt = hip_encrypt;
    st->parent.decrypt = hip_decrypt;
    st->parent.destroy = hip_destroy;
    return &st->parent;
}

/* internal.h:655 — replaces cipher-chachapoly.c:145-158 */
NoiseCipherState *noise_chachapoly_new(void)
{
    return hip_new(NOISE_CIPHER_CHACHAPOLY, noise_chachapoly_new);
}

/* internal.h:656 — replaces the chooser in internal.c:40-56 */
NoiseCipherState *noise_aesgcm_new(void)
{
    return hip_new(NOISE_CIPHER_AESGCM, noise_aesgcm_new);
}

int na_is_ours(const NoiseCipherState *st) { return st && st->encrypt == hip_encrypt; }

/* ------------------------------------------ CipherState API (cipherstate.c) */

int noise_cipherstate_new_by_id(NoiseCipherState **state, int id)
{
    if (!state) return NOISE_ERROR_INVALID_PARAM;
    *state = 0;
    switch (id) {
    case NOISE_CIPHER_CHACHAPOLY: *state = noise_chachapoly_new(); break;
    case NOISE_CIPHER_AESGCM: *state = noise_aesgcm_new(); break;
    default: return NOISE_ERROR_UNKNOWN_ID;
    }
    return *state ? NOISE_ERROR_NONE : NOISE_ERROR_NO_MEMORY;
}

int noise_cipherstate_new_by_name(NoiseCipherState **state, const char *name)
{
    if (!state) return NOISE_ERROR_INVALID_PARAM;
    *state = 0;
    if (!name) return NOISE_ERROR_INVALID_PARAM;
    /* names.c:58-59 */
    if (!strcmp(name, "ChaChaPoly")) return noise_cipherstate_new_by_id(state, NOISE_CIPHER_CHACHAPOLY);
    if (!strcmp(name, "AESGCM")) return noise_cipherstate_new_by_id(state, NOISE_CIPHER_AESGCM);
    return NOISE_ERROR_UNKNOWN_NAME;
}

int noise_cipherstate_free(NoiseCipherState *state)
{
    if (!state) return NOISE_ERROR_INVALID_PARAM;
    if (state->destroy) (*state->destroy)(state);
    free_object(state, state->size);
    return NOISE_ERROR_NONE;
}

int noise_cipherstate_get_cipher_id(const NoiseCipherState *state)
{
    return state ? state->cipher_id : NOISE_CIPHER_NONE;
}

size_t noise_cipherstate_get_key_length(const NoiseCipherState *state)
{
    return state ? state->key_len : 0;
}

size_t noise_cipherstate_get_mac_length(const NoiseCipherState *state)
{
    return state ? state->mac_len : 0;
}

int noise_cipherstate_init_key(NoiseCipherState *state, const uint8_t *key, size_t key_len)
{
    if (!state || !key) return NOISE_ERROR_INVALID_PARAM;
    if (key_len != state->key_len) return NOISE_ERROR_INVALID_LENGTH;
    (*state->init_key)(state, key);
    state->has_key = 1;
    state->n = 0;
    return NOISE_ERROR_NONE;
}

int noise_cipherstate_has_key(const NoiseCipherState *state)
{
    return state ? state->has_key : 0;
}

/* Validation of cipherstate.c:299-322.  Returns NOISE_ERROR_NONE when the
   record must be encrypted; *passthrough set when there is no key. */
static int check_encrypt(const NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                         const NoiseBuffer *buffer, int *passthrough)
{
    *passthrough = 0;
    if (!state || (!ad && ad_len) || !buffer || !buffer->data) return NOISE_ERROR_INVALID_PARAM;
    if (buffer->size > buffer->max_size) return NOISE_ERROR_INVALID_LENGTH;
    if (!state->has_key) {
        if (buffer->size > NOISE_MAX_PAYLOAD_LEN) return NOISE_ERROR_INVALID_LENGTH;
        *passthrough = 1;
        return NOISE_ERROR_NONE;
    }
    if (ad_len > UINT32_MAX) return NOISE_ERROR_INVALID_LENGTH; /* device descriptors hold 32 bits */
    if (buffer->size > (size_t)(NOISE_MAX_PAYLOAD_LEN - state->mac_len))
        return NOISE_ERROR_INVALID_LENGTH;
    if ((buffer->max_size - buffer->size) < state->mac_len) return NOISE_ERROR_INVALID_LENGTH;
    if (state->n == NONCE_LIMIT) return NOISE_ERROR_INVALID_NONCE;
    return NOISE_ERROR_NONE;
}

/* Validation of cipherstate.c:379-397 (nonce checked by the caller). */
static int check_decrypt(const NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                         const NoiseBuffer *buffer, int *passthrough)
{
    *passthrough = 0;
    if (!state || (!ad && ad_len) || !buffer || !buffer->data) return NOISE_ERROR_INVALID_PARAM;
    if (buffer->size > buffer->max_size || buffer->size > NOISE_MAX_PAYLOAD_LEN)
        return NOISE_ERROR_INVALID_LENGTH;
    if (!state->has_key) {
        *passthrough = 1;
        return NOISE_ERROR_NONE;
    }
    if (ad_len > UINT32_MAX) return NOISE_ERROR_INVALID_LENGTH; /* device descriptors hold 32 bits */
    if (buffer->size < state->mac_len) return NOISE_ERROR_INVALID_LENGTH;
    return NOISE_ERROR_NONE;
}

int noise_cipherstate_encrypt_with_ad(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                                      NoiseBuffer *buffer)
{
    int pass, err = check_encrypt(state, ad, ad_len, buffer, &pass);
    if (err || pass) return err;
    err = (*state->encrypt)(state, ad, ad_len, buffer->data, buffer->size);
    ++(state->n); /* advanced even when the backend fails (cipherstate.c:325-326) */
    if (err != NOISE_ERROR_NONE) return err;
    buffer->size += state->mac_len;
    return NOISE_ERROR_NONE;
}

int noise_cipherstate_decrypt_with_ad(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                                      NoiseBuffer *buffer)
{
    int pass, err = check_decrypt(state, ad, ad_len, buffer, &pass);
    if (err || pass) return err;
    if (state->n == NONCE_LIMIT) return NOISE_ERROR_INVALID_NONCE;
    err = (*state->decrypt)(state, ad, ad_len, buffer->data, buffer->size - state->mac_len);
    if (err != NOISE_ERROR_NONE) return err; /* n not advanced (cipherstate.c:400-405) */
    ++(state->n);
    buffer->size -= state->mac_len;
    return NOISE_ERROR_NONE;
}

int noise_cipherstate_encrypt(NoiseCipherState *state, NoiseBuffer *buffer)
{
    return noise_cipherstate_encrypt_with_ad(state, NULL, 0, buffer);
}

int noise_cipherstate_decrypt(NoiseCipherState *state, NoiseBuffer *buffer)
{
    return noise_cipherstate_decrypt_with_ad(state, NULL, 0, buffer);
}

int noise_cipherstate_set_nonce(NoiseCipherState *state, uint64_t nonce)
{
    if (!state) return NOISE_ERROR_INVALID_PARAM;
    if (!state->has_key) return NOISE_ERROR_INVALID_STATE;
    if (state->n > nonce) return NOISE_ERROR_INVALID_NONCE;
    state->n = nonce;
    return NOISE_ERROR_NONE;
}

int noise_cipherstate_get_max_key_length(void) { return MAX_KEY_LEN; }

int noise_cipherstate_get_max_mac_length(void) { return MAX_MAC_LEN; }

/* ----------------------------------------------------------- batch API */

int noise_cipherstate_encrypt_batch(NoiseCipherState *const *states, const uint8_t *const *ads,
                                    const size_t *ad_lens, NoiseBuffer *buffers, size_t count,
                                    int *results)
{
    if ((!states || !buffers || !results) && count) return NOISE_ERROR_INVALID_PARAM;
    Job *jobs = (Job *)malloc((count ? count : 1) * sizeof(Job));
    if (!jobs) return NOISE_ERROR_NO_MEMORY;
    size_t nj = 0;
    for (size_t i = 0; i < count; ++i) {
        NoiseCipherState *st = states[i];
        const uint8_t *ad = ads ? ads[i] : NULL;
        size_t ad_len = ad_lens ? ad_lens[i] : 0;
        if (st && !na_is_ours(st)) { /* a foreign plugin object: its own backend */
            results[i] = noise_cipherstate_encrypt_with_ad(st, ad, ad_len, &buffers[i]);
            continue;
        }
        int pass;
        results[i] = check_encrypt(st, ad, ad_len, &buffers[i], &pass);
        if (results[i] || pass) continue;
        Job *j = &jobs[nj++];
        j->st = (HipCipherState *)st;
        j->ad = ad;
        j->ad_len = ad_len;
        j->data = buffers[i].data;
        j->len = buffers[i].size;
        j->nonce = st->n++; /* advanced even if the backend fails (cipherstate.c:325-326) */
        j->idx = i;
        j->skip = 0;
        j->forge = 0;
    }
    int rc = run_jobs(jobs, nj, 0, NULL, NULL);
    for (size_t k = 0; k < nj; ++k) {
        size_t i = jobs[k].idx;
        results[i] = jobs[k].status;
        if (jobs[k].status == NOISE_ERROR_NONE) buffers[i].size += 16;
    }
    free(jobs);
    return rc;
}

typedef struct {
    NoiseBuffer *buffers;
    int *results;
} OpenBatch;

/* records dispatched, at least, in the first optimistic round after a run of
   forgeries ended (noise_cipherstate_decrypt_batch) */
#define FORGE_RESUME 64

/* The sequential semantics of noise_cipherstate_decrypt_with_ad
   (cipherstate.c:373-410) applied in record order.  A MAC failure leaves the
   record and n untouched, so the next record of the state is tried at the
   same n.  Each round tests one hypothesis per state:
     optimistic (forge = 0): records at n, n+1, ... — right up to the first
       failure, which is final; the records after it rest on a wrong nonce and
       are deferred;
     forge (forge = 1 after a failure): every record at n — each failure is
       final (the sequential call would fail at n too) up to the first record
       that verifies, which commits; the records after it are deferred. */
static void open_batch_decide(Job *jobs, size_t lo, size_t hi, void *u)
{
    OpenBatch *b = (OpenBatch *)u;
    for (size_t k = lo; k < hi; ++k) {
        Job *j = &jobs[k];
        HipCipherState *st = j->st;
        j->commit = j->defer = 0;
        if (st->b_stop) {
            j->defer = 1;
            continue;
        }
        if (j->skip) { /* nonce exhausted (cipherstate.c:391-397): final */
            b->results[j->idx] = NOISE_ERROR_INVALID_NONCE;
            continue;
        }
        b->results[j->idx] = j->status;
        if (j->status == NOISE_ERROR_NONE) {
            j->commit = 1;
            ++st->parent.n;
            b->buffers[j->idx].size -= 16;
            if (j->forge) st->b_stop = st->b_hit = 1; /* the run of forgeries ended */
        } else if (!j->forge) {
            st->b_stop = st->b_hit = 1; /* a run of forgeries starts here */
        }
    }
}

/* Test hook: rounds and dispatched records of this thread's last
   noise_cipherstate_decrypt_batch call. */
static __thread uint64_t t_batch_rounds, t_batch_dispatched;

void noise_aead_debug_batch_stats(uint64_t *rounds, uint64_t *dispatched)
{
    if (rounds) *rounds = t_batch_rounds;
    if (dispatched) *dispatched = t_batch_dispatched;
}

int noise_cipherstate_decrypt_batch(NoiseCipherState *const *states, const uint8_t *const *ads,
                                    const size_t *ad_lens, NoiseBuffer *buffers, size_t count,
                                    int *results)
{
    if ((!states || !buffers || !results) && count) return NOISE_ERROR_INVALID_PARAM;
    static uint64_t epoch_counter = 0;
    t_batch_rounds = t_batch_dispatched = 0;
    const size_t cap = count ? count : 1;
    Job *jobs = (Job *)malloc(cap * sizeof(Job));
    size_t *pend = (size_t *)malloc(cap * sizeof(size_t));
    size_t *job_of = (size_t *)malloc(cap * sizeof(size_t));
    if (!jobs || !pend || !job_of) {
        free(jobs);
        free(pend);
        free(job_of);
        return NOISE_ERROR_NO_MEMORY;
    }
    /* Round 1 validates everything and dispatches every record with the
       nonce it gets if all earlier records of its state verify.  A MAC
       failure leaves n where it was, so the state's later records are
       re-run in later rounds (open_batch_decide): first as a run of
       forgeries — a window of records all at n, 1 record, then 2, 4, ...
       while they all fail — then, once one verifies, optimistically again in
       windows of twice the last forge window (at least FORGE_RESUME) that
       double while they verify.  A run of k forged records therefore costs
       O(log k) rounds and the records dispatched stay linear in the batch;
       k isolated forgeries cost O(k) rounds (each one moves the nonces of
       every later record). */
    size_t np = 0;
    for (size_t i = 0; i < count; ++i) {
        NoiseCipherState *st = states[i];
        const uint8_t *ad = ads ? ads[i] : NULL;
        size_t ad_len = ad_lens ? ad_lens[i] : 0;
        if (st && !na_is_ours(st)) {
            results[i] = noise_cipherstate_decrypt_with_ad(st, ad, ad_len, &buffers[i]);
            continue;
        }
        int pass;
        results[i] = check_decrypt(st, ad, ad_len, &buffers[i], &pass);
        if (results[i] || pass) continue;
        ((HipCipherState *)st)->b_window = 0;
        ((HipCipherState *)st)->b_forge = 0;
        pend[np++] = i;
    }
    OpenBatch ob = {buffers, results};
    int rc = NOISE_ERROR_NONE;
    while (np && !rc) {
        const uint64_t epoch = __atomic_add_fetch(&epoch_counter, 1, __ATOMIC_RELAXED);
        size_t nj = 0;
        for (size_t p = 0; p < np; ++p) {
            size_t i = pend[p];
            HipCipherState *st = (HipCipherState *)states[i];
            if (st->b_epoch != epoch) {
                st->b_epoch = epoch;
                st->b_next = st->parent.n;
                st->b_stop = st->b_hit = 0;
                st->b_sent = 0;
            }
            if (st->b_window && st->b_sent >= st->b_window) { /* beyond this round's window */
                job_of[p] = SIZE_MAX;
                continue;
            }
            ++st->b_sent;
            job_of[p] = nj;
            Job *j = &jobs[nj++];
            j->st = st;
            j->ad = ads ? ads[i] : NULL;
            j->ad_len = ad_lens ? ad_lens[i] : 0;
            j->data = buffers[i].data;
            j->len = buffers[i].size - 16;
            j->idx = i;
            /* optimistic: assumes the earlier records of the state verify;
               forge: that they fail.  An exhausted nonce stays exhausted
               (cipherstate.c:391-397) */
            j->forge = st->b_forge;
            j->nonce = st->b_forge ? st->parent.n : st->b_next;
            j->skip = j->nonce == NONCE_LIMIT;
            if (!j->skip && !st->b_forge) ++st->b_next;
        }
        ++t_batch_rounds;
        t_batch_dispatched += nj;
        rc = run_jobs(jobs, nj, 1, open_batch_decide, &ob);
        for (size_t k = 0; k < nj; ++k) { /* next round's mode and window of each state */
            HipCipherState *st = jobs[k].st;
            if (st->b_upd == epoch) continue;
            st->b_upd = epoch;
            if (!st->b_hit) { /* the hypothesis held for the whole window */
                if (st->b_window) st->b_window *= 2;
            } else if (!st->b_forge) { /* optimistic round hit a MAC failure */
                st->b_forge = 1;
                st->b_window = 1;
            } else { /* a forge round found the record that verifies */
                st->b_forge = 0;
                st->b_window = st->b_window * 2 > FORGE_RESUME ? st->b_window * 2 : FORGE_RESUME;
            }
        }
        size_t nnext = 0;
        for (size_t p = 0; p < np; ++p) {
            if (job_of[p] == SIZE_MAX) { /* held back, in record order */
                pend[nnext++] = pend[p];
                continue;
            }
            const Job *j = &jobs[job_of[p]];
            if (rc) {
                if (j->defer || j->status == NOISE_ERROR_SYSTEM) results[j->idx] = NOISE_ERROR_SYSTEM;
            } else if (j->defer) {
                pend[nnext++] = j->idx;
            }
        }
        np = nnext;
    }
    if (rc)
        for (size_t p = 0; p < np; ++p) results[pend[p]] = NOISE_ERROR_SYSTEM;
    free(jobs);
    free(pend);
    free(job_of);
    return rc;
}
