/*
 * wire.c — the Noise transport wire path: whole
 * receive / send buffers of framed records through the GPU in one pipelined
 * pass, in place.
 *
 * Wire format of noise-c's examples/echo (echo-common.c:643-688, echo_recv /
 * echo_send): a frame is a 2-byte big-endian length L followed by L bytes of
 * CT || tag.  The reference's echo server (echo-server.c:377-407) reads one
 * frame, decrypts it with its receive CipherState, re-encrypts it with its
 * send CipherState and writes it back; noise_wire_echo() does exactly that
 * for every complete frame of a buffer at once, noise_wire_open() and
 * noise_wire_seal() are its two halves.
 *
 * Pipeline per chunk of frames (Staging's three streams):
 *   stream_in : H2D of the chunk's descriptors + wire bytes
 *   stream    : the first AEAD pass (seal, or open with the status bytes)
 *               and, for seal, the D2H of the chunk
 *   stream_out: after the host has read the chunk's statuses, the verified
 *               prefix only: the echo re-seal and the D2H
 * so H2D of chunk c+1, the kernels of chunk c and the D2H of chunk c-1
 * overlap.  Buffers from noise_wire_alloc() are pinned: the copies go
 * straight from and to them; other buffers are staged through the thread's
 * pinned area by the host pool.
 */
#define _DEFAULT_SOURCE
#include "host_internal.h"
#include "host_pool.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------ pinned wire memory */

typedef struct PinnedRange {
    uint8_t *p;
    size_t n;
    struct PinnedRange *next;
} PinnedRange;

static PinnedRange *g_pinned = NULL;
static pthread_mutex_t g_pin_mu = PTHREAD_MUTEX_INITIALIZER;

void *noise_wire_alloc(size_t bytes)
{
    if (!bytes) return NULL;
    PinnedRange *r = (PinnedRange *)malloc(sizeof(PinnedRange));
    if (!r) return NULL;
    if (hipHostMalloc((void **)&r->p, bytes, hipHostMallocDefault) != hipSuccess) {
        free(r);
        return NULL;
    }
    r->n = bytes;
    pthread_mutex_lock(&g_pin_mu);
    r->next = g_pinned;
    g_pinned = r;
    pthread_mutex_unlock(&g_pin_mu);
    return r->p;
}

void noise_wire_free(void *p)
{
    if (!p) return;
    pthread_mutex_lock(&g_pin_mu);
    PinnedRange **pp = &g_pinned, *r = NULL;
    while (*pp && (*pp)->p != (uint8_t *)p) pp = &(*pp)->next;
    if (*pp) {
        r = *pp;
        *pp = r->next;
    }
    pthread_mutex_unlock(&g_pin_mu);
    if (!r) return;
    na_clean(r->p, r->n);
    (void)hipHostFree(r->p);
    free(r);
}

/* [p, p + n) inside one noise_wire_alloc() buffer */
static int is_pinned(const uint8_t *p, size_t n)
{
    int hit = 0;
    pthread_mutex_lock(&g_pin_mu);
    for (PinnedRange *r = g_pinned; r && !hit; r = r->next)
        hit = p >= r->p && n <= r->n && (size_t)(p - r->p) <= r->n - n;
    pthread_mutex_unlock(&g_pin_mu);
    return hit;
}

/* ------------------------------------------------------------- the engine */

enum { W_SEAL = 0, W_OPEN = 1, W_ECHO = 2 };

typedef struct {
    size_t off;   /* position of the 2-byte header in the wire buffer */
    uint32_t len; /* L: the header value */
} Frame;

typedef struct {
    size_t f0, f1;             /* frames [f0, f1) */
    size_t meta_off;           /* descA [n] | descB [n] | status [n] */
    size_t desc_b_off, status_off;
    size_t w0, w1;             /* wire bytes [w0, w1) */
    size_t prefix;             /* open/echo: frames of the chunk that verified, in order */
    int failed;                /* a frame of this chunk failed its MAC */
    uint32_t max_len;          /* longest frame (ChaChaPoly lane choice) */
} WChunk;

typedef struct {
    uint8_t *src, *dst;
    size_t base;
} BulkArg;

static void bulk_copy(void *p, size_t lo, size_t hi)
{
    BulkArg *a = (BulkArg *)p;
    na_copy_stream(a->dst + a->base + lo, a->src + a->base + lo, hi - lo);
}

static void bulk_scrub(void *p, size_t lo, size_t hi)
{
    BulkArg *a = (BulkArg *)p;
    explicit_bzero(a->dst + a->base + lo, hi - lo);
}

static void par_copy(uint8_t *dst, const uint8_t *src, size_t off, size_t n)
{
    BulkArg a = {(uint8_t *)src, dst, off};
    host_pool_for(n, (size_t)1 << 20, bulk_copy, &a);
}

static void fill_desc(NoiseAeadRecord *d, const Frame *f, uint64_t nonce, const HipCipherState *st)
{
    d->in_off = d->out_off = f->off + 2;
    d->nonce = nonce;
    d->ctx_off = (uint64_t)(uintptr_t)st->d_ctx;
    d->ad_off = 0;
    d->len = f->len - 16;
    d->ad_len = 0;
}

static int launch_ragged(int open, const HipCipherState *st, const uint8_t *d_base,
                         const NoiseAeadRecord *d_recs, uint8_t *d_status, size_t n,
                         uint32_t max_len, hipStream_t s)
{
    NoiseAeadRagged job;
    job.ctx_base = NULL;
    job.recs = d_recs;
    job.in = d_base;
    job.out = (uint8_t *)d_base;
    job.ad = d_base;
    job.status = d_status;
    job.n_records = (uint32_t)n;
    job.lanes_per_record = st->parent.cipher_id == NOISE_CIPHER_CHACHAPOLY
                               ? na_chacha_lanes((uint32_t)n, max_len) : na_aes_lanes((uint32_t)n);
    /* frames sit at 2-byte offsets: the any-alignment kernels; opens verify
       before they decrypt (the reference's order, cipher-chachapoly.c:135-141) */
    job.flags = open ? NOISE_AEAD_FLAG_VERIFY_FIRST : 0;
    job.reserved_ = 0;
    return open ? noise_aead_dev_open_ragged(st->parent.cipher_id, &job, s)
                : noise_aead_dev_seal_ragged(st->parent.cipher_id, &job, s);
}

/* Scan the complete frames at the start of wire and validate them in order
   as the per-frame CipherState calls would; returns the error that stops the
   scan before the end (NOISE_ERROR_NONE for a partial or absent frame). */
static int scan_frames(int mode, const HipCipherState *a, const HipCipherState *b,
                       const uint8_t *wire, size_t wire_len, Frame *fr, size_t cap, size_t *count)
{
    size_t k = 0, off = 0;
    int err = NOISE_ERROR_NONE;
    while (k < cap && off + 2 <= wire_len) {
        uint32_t L = ((uint32_t)wire[off] << 8) | wire[off + 1];
        if (off + 2 + L > wire_len) break;
        /* both the tag of seal and the MAC of open need L >= 16
           (cipherstate.c:305-318 / :379-390) */
        if (L < 16) { err = NOISE_ERROR_INVALID_LENGTH; break; }
        if (a->parent.n + k == NONCE_LIMIT ||
            (mode == W_ECHO && b->parent.n + k == NONCE_LIMIT)) {
            err = NOISE_ERROR_INVALID_NONCE;
            break;
        }
        fr[k].off = off;
        fr[k].len = L;
        off += 2 + L;
        ++k;
    }
    *count = k;
    return err;
}

static int wire_run(int mode, NoiseCipherState *sa, NoiseCipherState *sb, uint8_t *wire,
                    size_t wire_len, size_t *consumed, size_t *frames)
{
    if (consumed) *consumed = 0;
    if (frames) *frames = 0;
    if (!sa || !wire || (mode == W_ECHO && !sb)) return NOISE_ERROR_INVALID_PARAM;
    if (!na_is_ours(sa) || (sb && !na_is_ours(sb))) return NOISE_ERROR_INVALID_PARAM;
    if (!sa->has_key || (mode == W_ECHO && !sb->has_key)) return NOISE_ERROR_INVALID_STATE;
    HipCipherState *a = (HipCipherState *)sa, *b = (HipCipherState *)sb;
    if (mode == W_ECHO && a == b) return NOISE_ERROR_INVALID_PARAM;

    size_t max_frames = wire_len / 18 + 1;
    Frame *fr = (Frame *)malloc(max_frames * sizeof(Frame));
    if (!fr) return NOISE_ERROR_NO_MEMORY;
    size_t K = 0;
    int stop_err = scan_frames(mode, a, b, wire, wire_len, fr, max_frames, &K);
    if (K == 0) {
        free(fr);
        return stop_err;
    }
    const size_t wire_bytes = fr[K - 1].off + 2 + fr[K - 1].len;
    const int pinned = is_pinned(wire, wire_bytes);
    const int nd = mode == W_ECHO ? 2 : 1;

    /* chunks of about 4 MiB of frames (at most MAX_CHUNKS) */
    size_t target = wire_bytes / (MAX_CHUNKS - 1) + 1;
    if (target < ((size_t)4 << 20)) target = (size_t)4 << 20;
    WChunk ch[MAX_CHUNKS];
    int nc = 0;
    size_t meta = 0;
    for (size_t k = 0, f0 = 0; k < K; ++k) {
        size_t end = fr[k].off + 2 + fr[k].len;
        if (end - fr[f0].off >= target || k + 1 == K) {
            WChunk *c = &ch[nc++];
            c->f0 = f0;
            c->f1 = k + 1;
            c->w0 = fr[f0].off;
            c->w1 = end;
            size_t n = c->f1 - c->f0;
            c->meta_off = meta;
            c->desc_b_off = meta + n * sizeof(NoiseAeadRecord);
            c->status_off = meta + nd * n * sizeof(NoiseAeadRecord);
            meta = (c->status_off + n + 63) & ~(size_t)63;
            c->prefix = 0;
            c->failed = 0;
            c->max_len = 0;
            for (size_t f = c->f0; f < c->f1; ++f)
                if (fr[f].len > c->max_len) c->max_len = fr[f].len;
            f0 = k + 1;
        }
    }
    const size_t wire_base = meta;
    Staging *sg = na_stage_get(wire_base + wire_bytes + 64);
    int rc = sg ? NOISE_ERROR_NONE : NOISE_ERROR_SYSTEM;
    if (!rc) rc = na_ensure_ctx(a, sg);
    if (!rc && mode == W_ECHO) rc = na_ensure_ctx(b, sg);

    /* host and device images of wire[0..wire_bytes) */
    uint8_t *h_wire = rc ? NULL : pinned ? wire : sg->h + wire_base;
    uint8_t *d_wire = rc ? NULL : sg->d + wire_base;
    size_t done = 0;
    int launched = 0, gated = 0, finished = 0, stop = 0;
    const int tr = na_trace_on();
    double t_start = tr ? na_now_ms() : 0, t_issue = 0, t_gate = 0, t_fin = 0, t0 = 0;
    for (int c = 0; c <= nc + 1 && !rc; ++c) {
        if (tr) t0 = na_now_ms();
        if (c < nc && !stop) { /* ---- stage + launch chunk c */
            WChunk *k = &ch[c];
            size_t n = k->f1 - k->f0;
            if (!pinned) par_copy(h_wire, wire, k->w0, k->w1 - k->w0);
            NoiseAeadRecord *da = (NoiseAeadRecord *)(sg->h + k->meta_off);
            NoiseAeadRecord *db = (NoiseAeadRecord *)(sg->h + k->desc_b_off);
            for (size_t i = 0; i < n; ++i) {
                size_t f = k->f0 + i;
                fill_desc(&da[i], &fr[f], a->parent.n + f, a);
                if (mode == W_ECHO) fill_desc(&db[i], &fr[f], b->parent.n + f, b);
            }
            if (hipMemcpyAsync(sg->d + k->meta_off, sg->h + k->meta_off, k->status_off - k->meta_off,
                               hipMemcpyHostToDevice, sg->stream_in) != hipSuccess ||
                hipMemcpyAsync(d_wire + k->w0, h_wire + k->w0, k->w1 - k->w0,
                               hipMemcpyHostToDevice, sg->stream_in) != hipSuccess ||
                hipEventRecord(sg->ev_in[c], sg->stream_in) != hipSuccess ||
                hipStreamWaitEvent(sg->stream, sg->ev_in[c], 0) != hipSuccess) {
                rc = NOISE_ERROR_SYSTEM;
                break;
            }
            rc = launch_ragged(mode != W_SEAL, a, d_wire, (NoiseAeadRecord *)(sg->d + k->meta_off),
                               sg->d + k->status_off, n, k->max_len, sg->stream);
            if (rc) break;
            hipError_t e;
            if (mode == W_SEAL) { /* nothing to gate: the whole chunk comes back,
                                     on stream_out so it overlaps the next kernel */
                e = hipEventRecord(sg->ev_out[c], sg->stream);
                if (e == hipSuccess) e = hipStreamWaitEvent(sg->stream_out, sg->ev_out[c], 0);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(h_wire + k->w0, d_wire + k->w0, k->w1 - k->w0,
                                       hipMemcpyDeviceToHost, sg->stream_out);
                if (e == hipSuccess) e = hipEventRecord(sg->ev_done[c], sg->stream_out);
            } else {
                e = hipMemcpyAsync(sg->h + k->status_off, sg->d + k->status_off, n,
                                   hipMemcpyDeviceToHost, sg->stream);
                if (e == hipSuccess) e = hipEventRecord(sg->ev_out[c], sg->stream);
            }
            if (e != hipSuccess) {
                rc = NOISE_ERROR_SYSTEM;
                break;
            }
            ++launched;
        }
        if (tr) {
            double t = na_now_ms();
            t_issue += t - t0;
            t0 = t;
        }
        if (c >= 1 && gated < launched) { /* ---- gate chunk c-1: read statuses, release prefix */
            WChunk *k = &ch[gated];
            size_t n = k->f1 - k->f0;
            if (mode == W_SEAL) {
                k->prefix = n;
            } else {
                if (hipEventSynchronize(sg->ev_out[gated]) != hipSuccess) {
                    rc = NOISE_ERROR_SYSTEM;
                    break;
                }
                const uint8_t *st = sg->h + k->status_off;
                size_t p = 0;
                if (!stop) /* chunks after a failure release nothing */
                    while (p < n && st[p] == 0) ++p;
                k->prefix = p;
                k->failed = !stop && p < n;
                if (k->failed) stop = 1; /* later frames depend on this nonce */
                hipError_t e = hipSuccess;
                if (p) {
                    size_t pend = fr[k->f0 + p - 1].off + 2 + fr[k->f0 + p - 1].len;
                    e = hipStreamWaitEvent(sg->stream_out, sg->ev_out[gated], 0);
                    if (e == hipSuccess && mode == W_ECHO &&
                        launch_ragged(0, b, d_wire, (NoiseAeadRecord *)(sg->d + k->desc_b_off), NULL,
                                      p, k->max_len, sg->stream_out))
                        e = hipErrorLaunchFailure;
                    if (e == hipSuccess)
                        e = hipMemcpyAsync(h_wire + k->w0, d_wire + k->w0, pend - k->w0,
                                           hipMemcpyDeviceToHost, sg->stream_out);
                }
                if (e == hipSuccess) e = hipEventRecord(sg->ev_done[gated], sg->stream_out);
                if (e != hipSuccess) {
                    rc = NOISE_ERROR_SYSTEM;
                    break;
                }
            }
            ++gated;
        }
        if (tr) {
            double t = na_now_ms();
            t_gate += t - t0;
            t0 = t;
        }
        if (c >= 2 && finished < gated) { /* ---- finish chunk c-2: results into the caller's buffer */
            WChunk *k = &ch[finished];
            if (hipEventSynchronize(sg->ev_done[finished]) != hipSuccess) {
                rc = NOISE_ERROR_SYSTEM;
                break;
            }
            if (k->prefix) {
                size_t pend = fr[k->f0 + k->prefix - 1].off + 2 + fr[k->f0 + k->prefix - 1].len;
                if (!pinned) {
                    par_copy(wire, h_wire, k->w0, pend - k->w0);
                    if (mode == W_OPEN) { /* plaintext was staged: scrub it */
                        BulkArg z = {NULL, h_wire, k->w0};
                        host_pool_for(k->w1 - k->w0, (size_t)1 << 20, bulk_scrub, &z);
                    }
                }
                done += k->prefix;
            }
            ++finished;
        }
        if (tr) t_fin += na_now_ms() - t0;
        if (stop && finished == gated && gated == launched) break;
    }
    if (tr)
        fprintf(stderr, "noise_wire %s: %zu frames, %d chunks, %zu B, %s: total %.3f ms, "
                "issue %.3f, gate %.3f, finish %.3f\n",
                mode == W_SEAL ? "seal" : mode == W_OPEN ? "open" : "echo", K, nc, wire_bytes,
                pinned ? "pinned" : "staged", na_now_ms() - t_start, t_issue, t_gate, t_fin);
    if (rc && sg) { /* drain; frames of unfinished chunks are not reported */
        (void)hipStreamSynchronize(sg->stream_in);
        (void)hipStreamSynchronize(sg->stream);
        (void)hipStreamSynchronize(sg->stream_out);
        if (!pinned) explicit_bzero(sg->h + wire_base, wire_bytes);
    }
    if (d_wire && mode != W_SEAL) {
        /* the device image holds the plaintext of every frame that verified
           (echo re-seals only the released prefix): zero it once the last
           D2H has read it, as the host staging is scrubbed above */
        (void)hipStreamSynchronize(sg->stream_out);
        if (hipMemsetAsync(d_wire, 0, wire_bytes, sg->stream) == hipSuccess)
            (void)hipStreamSynchronize(sg->stream);
    }
    /* nonces: seal advances once per dispatched frame even on a backend error
       (cipherstate.c:325-326); open/echo only for frames that verified */
    if (mode == W_SEAL) {
        a->parent.n += rc ? K : done;
    } else {
        a->parent.n += done;
        if (mode == W_ECHO) b->parent.n += done;
    }
    int failed = 0;
    for (int c = 0; c < finished; ++c) failed |= ch[c].failed;
    if (frames) *frames = done;
    if (consumed) *consumed = done ? fr[done - 1].off + 2 + fr[done - 1].len : 0;
    free(fr);
    if (rc) return rc;
    if (failed) return NOISE_ERROR_MAC_FAILURE;
    return stop_err;
}

int noise_wire_seal(NoiseCipherState *state, uint8_t *wire, size_t wire_len, size_t *consumed,
                    size_t *frames)
{
    return wire_run(W_SEAL, state, NULL, wire, wire_len, consumed, frames);
}

int noise_wire_open(NoiseCipherState *state, uint8_t *wire, size_t wire_len, size_t *consumed,
                    size_t *frames)
{
    return wire_run(W_OPEN, state, NULL, wire, wire_len, consumed, frames);
}

int noise_wire_echo(NoiseCipherState *recv, NoiseCipherState *send, uint8_t *wire,
                    size_t wire_len, size_t *consumed, size_t *frames)
{
    return wire_run(W_ECHO, recv, send, wire, wire_len, consumed, frames);
}
