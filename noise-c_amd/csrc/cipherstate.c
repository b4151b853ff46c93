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
#include "noise_aead_hip.h"

#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------- the plugin object ABI */

/* Identical layout to struct NoiseCipherState_s, src/protocol/internal.h:58-146. */
struct NoiseCipherState_s {
    size_t size;
    int cipher_id;
    uint8_t has_key;
    uint8_t key_len;
    uint8_t mac_len;
    uint64_t n;
    NoiseCipherState *(*create)(void);
    void (*init_key)(NoiseCipherState *state, const uint8_t *key);
    int (*encrypt)(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                   uint8_t *data, size_t len);
    int (*decrypt)(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                   uint8_t *data, size_t len);
    void (*destroy)(NoiseCipherState *state);
};

#define MAX_KEY_LEN 32 /* cipherstate.c:53 */
#define MAX_MAC_LEN 16 /* cipherstate.c:56 */
#define NONCE_LIMIT 0xFFFFFFFFFFFFFFFFULL

/* Backend state appended by first-member embedding, as cipher-chachapoly.c
   :28-35 and cipher-aesgcm.c:28-36 do. */
typedef struct {
    struct NoiseCipherState_s parent;
    uint8_t key[32];
    void *d_ctx;       /* device key context (noise_aead_dev_ctx_bytes) */
    int device;        /* HIP device that owns d_ctx */
    int ctx_ready;     /* d_ctx matches key */
    /* scratch for the batch walker (a CipherState is single-owner) */
    uint64_t b_epoch;
    uint64_t b_next;   /* nonce the next record of this batch round will use */
    int b_failed;
} HipCipherState;

/* ---------------------------------------------------- util.c equivalents */

static void clean(void *p, size_t n) /* util.c:170-177 noise_clean */
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
    clean(ptr, size);
    free(ptr);
}

/* ------------------------------------------------------ per-thread staging */

typedef struct {
    int device;
    hipStream_t stream;
    uint8_t *h;        /* pinned host */
    uint8_t *d;        /* device */
    size_t cap;
    size_t scrub_off, scrub_len; /* last payload range (plaintext) */
} Staging;

static pthread_key_t g_stage_key;
static pthread_once_t g_stage_once = PTHREAD_ONCE_INIT;

static void stage_destroy(void *p)
{
    Staging *s = (Staging *)p;
    if (!s) return;
    if (s->h) (void)hipHostFree(s->h);
    if (s->d) (void)hipFree(s->d);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    free(s);
}

static void stage_key_init(void) { pthread_key_create(&g_stage_key, stage_destroy); }

/* Staging area of at least `bytes` on the current device, or NULL. */
static Staging *stage_get(size_t bytes)
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
        if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
            free(s);
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
        s->d = NULL;
        s->cap = 0;
        if (hipHostMalloc((void **)&s->h, cap, hipHostMallocDefault) != hipSuccess) return NULL;
        if (hipMalloc((void **)&s->d, cap) != hipSuccess) return NULL;
        s->cap = cap;
    }
    return s;
}

/* Zero the last payload staged on this thread: no plaintext left behind
   (the reference cleans its scratch the same way, cipher-chachapoly.c:72). */
static void stage_scrub(void)
{
    pthread_once(&g_stage_once, stage_key_init);
    Staging *s = (Staging *)pthread_getspecific(g_stage_key);
    if (s && s->h && s->scrub_len) clean(s->h + s->scrub_off, s->scrub_len);
    if (s) s->scrub_len = 0;
}

/* --------------------------------------------------- device key contexts */

static int is_ours(const NoiseCipherState *st);

/* Build the device key context of `st` from its key (lazy: init_key has no
   error return in the plugin ABI, internal.h:95). */
static int ensure_ctx(HipCipherState *st, Staging *sg)
{
    if (st->ctx_ready) return NOISE_ERROR_NONE;
    int dev = sg->device;
    if (st->d_ctx && st->device != dev) {
        (void)hipFree(st->d_ctx);
        st->d_ctx = NULL;
    }
    if (!st->d_ctx) {
        size_t bytes = noise_aead_dev_ctx_bytes(st->parent.cipher_id);
        if (hipMalloc(&st->d_ctx, bytes) != hipSuccess) {
            st->d_ctx = NULL;
            return NOISE_ERROR_SYSTEM;
        }
        st->device = dev;
    }
    /* raw key through the tail of the staging area */
    uint8_t *h = sg->h + sg->cap - 32;
    uint8_t *d = sg->d + sg->cap - 32;
    memcpy(h, st->key, 32);
    if (hipMemcpyAsync(d, h, 32, hipMemcpyHostToDevice, sg->stream) != hipSuccess)
        return NOISE_ERROR_SYSTEM;
    int rc = noise_aead_dev_prepare(st->parent.cipher_id, d, 1, st->d_ctx, sg->stream);
    if (rc) return rc;
    if (hipStreamSynchronize(sg->stream) != hipSuccess) return NOISE_ERROR_SYSTEM;
    clean(h, 32);
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
    int status;        /* out: NOISE_ERROR_NONE / _MAC_FAILURE / _SYSTEM */
    const uint8_t *result; /* out (open): verified plaintext in staging, valid
                              until the next run_jobs / stage_scrub */
} Job;

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

/* A record's staging slot: 16-B aligned, readable up to roundup64(len) and
   large enough for CT || tag — the NOISE_AEAD_FLAG_FAST layout. */
static size_t slot_bytes(size_t len)
{
    size_t a = ((len ? len : 1) + 63) & ~(size_t)63, b = align16(len + 16);
    return a > b ? a : b;
}

/* Run a set of jobs (any mix of states and ciphers) in one staging round
   trip: pack records into pinned memory, one H2D, one ragged kernel per
   cipher, one D2H.  Fills job.status.  Seal results are copied back at once;
   open results stay in staging (job.result) until the caller commits them
   in record order and calls stage_scrub() — a record verified under a
   speculative nonce must not touch the caller's buffer. */
static int run_jobs(Job *jobs, size_t n, int open)
{
    if (n == 0) return NOISE_ERROR_NONE;
    /* layout: [recs: n x 48][status: n][payload...] */
    size_t off = align16(n * sizeof(NoiseAeadRecord));
    const size_t status_off = off;
    off = align16(off + n);
    const size_t payload_off = off;
    for (size_t i = 0; i < n; ++i) off += align16(jobs[i].ad_len) + slot_bytes(jobs[i].len);
    const size_t total = off + 64;
    Staging *sg = stage_get(total);
    if (!sg) {
        for (size_t i = 0; i < n; ++i) jobs[i].status = NOISE_ERROR_SYSTEM;
        return NOISE_ERROR_SYSTEM;
    }
    int rc = NOISE_ERROR_NONE;
    for (size_t i = 0; i < n && !rc; ++i) rc = ensure_ctx(jobs[i].st, sg);
    if (rc) {
        for (size_t i = 0; i < n; ++i) jobs[i].status = NOISE_ERROR_SYSTEM;
        return rc;
    }

    /* ChaChaPoly records first, then AESGCM, so each cipher's descriptors
       are contiguous */
    NoiseAeadRecord *recs = (NoiseAeadRecord *)sg->h;
    size_t *order = (size_t *)malloc(n * sizeof(size_t));
    if (!order) {
        for (size_t i = 0; i < n; ++i) jobs[i].status = NOISE_ERROR_NO_MEMORY;
        return NOISE_ERROR_NO_MEMORY;
    }
    size_t n_chacha = 0, slot = 0;
    for (int pass = 0; pass < 2; ++pass) {
        int want = pass == 0 ? NOISE_CIPHER_CHACHAPOLY : NOISE_CIPHER_AESGCM;
        for (size_t i = 0; i < n; ++i)
            if (jobs[i].st->parent.cipher_id == want) order[slot++] = i;
        if (pass == 0) n_chacha = slot;
    }
    size_t p = payload_off;
    for (size_t s = 0; s < n; ++s) {
        Job *j = &jobs[order[s]];
        NoiseAeadRecord *r = &recs[s];
        r->ad_off = p;
        r->ad_len = (uint32_t)j->ad_len;
        if (j->ad_len) memcpy(sg->h + p, j->ad, j->ad_len);
        p += align16(j->ad_len);
        r->in_off = r->out_off = p;
        memcpy(sg->h + p, j->data, j->len + (open ? 16 : 0));
        p += slot_bytes(j->len);
        r->len = (uint32_t)j->len;
        r->nonce = j->nonce;
        r->ctx_off = (uint64_t)(uintptr_t)j->st->d_ctx;
    }
    hipStream_t stream = sg->stream;
    if (hipMemcpyAsync(sg->d, sg->h, p, hipMemcpyHostToDevice, stream) != hipSuccess)
        rc = NOISE_ERROR_SYSTEM;
    for (int c = 0; c < 2 && !rc; ++c) {
        size_t first = c == 0 ? 0 : n_chacha, count = c == 0 ? n_chacha : n - n_chacha;
        if (!count) continue;
        NoiseAeadRagged job;
        job.ctx_base = NULL;
        job.recs = (const NoiseAeadRecord *)(sg->d) + first;
        job.in = sg->d;
        job.out = sg->d;
        job.ad = sg->d;
        job.status = sg->d + status_off + first;
        job.n_records = (uint32_t)count;
        job.lanes_per_record = 0;
        job.flags = NOISE_AEAD_FLAG_FAST;
        job.reserved_ = 0;
        int cid = c == 0 ? NOISE_CIPHER_CHACHAPOLY : NOISE_CIPHER_AESGCM;
        rc = open ? noise_aead_dev_open_ragged(cid, &job, stream)
                  : noise_aead_dev_seal_ragged(cid, &job, stream);
    }
    if (!rc && hipMemcpyAsync(sg->h + status_off, sg->d + status_off, p - status_off,
                              hipMemcpyDeviceToHost, stream) != hipSuccess)
        rc = NOISE_ERROR_SYSTEM;
    if (!rc && hipStreamSynchronize(stream) != hipSuccess) rc = NOISE_ERROR_SYSTEM;
    for (size_t s = 0; s < n; ++s) {
        Job *j = &jobs[order[s]];
        if (rc) {
            j->status = NOISE_ERROR_SYSTEM;
            continue;
        }
        const uint8_t *res = sg->h + recs[s].in_off;
        j->result = NULL;
        if (!open) {
            memcpy(j->data, res, j->len + 16);
            j->status = NOISE_ERROR_NONE;
        } else if (sg->h[status_off + s] == 0) {
            j->result = res;
            j->status = NOISE_ERROR_NONE;
        } else {
            j->status = NOISE_ERROR_MAC_FAILURE;
        }
    }
    sg->scrub_off = payload_off;
    sg->scrub_len = p - payload_off;
    if (!open) stage_scrub();
    free(order);
    return rc;
}

/* -------------------------------------------------- plugin vtable entries */

static void hip_init_key(NoiseCipherState *state, const uint8_t *key)
{
    HipCipherState *st = (HipCipherState *)state;
    memcpy(st->key, key, 32);
    st->ctx_ready = 0;
}

static int hip_crypt(NoiseCipherState *state, const uint8_t *ad, size_t ad_len,
                     uint8_t *data, size_t len, int open)
{
    Job j;
    j.st = (HipCipherState *)state;
    j.ad = ad;
    j.ad_len = ad_len;
    j.data = data;
    j.len = len;
    j.nonce = state->n; /* the backend reads n; the front end owns n++ */
    j.status = NOISE_ERROR_SYSTEM;
    int rc = run_jobs(&j, 1, open);
    if (!rc && open && j.status == NOISE_ERROR_NONE) memcpy(data, j.result, len);
    stage_scrub();
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
    HipCipherState *st = (HipCipherState *)state;
    if (st->d_ctx) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != st->device) (void)hipSetDevice(st->device);
        (void)hipFree(st->d_ctx); /* context holds key material: freed with the state */
        if (cur != st->device) (void)hipSetDevice(cur);
        st->d_ctx = NULL;
    }
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

static int is_ours(const NoiseCipherState *st) { return st && st->encrypt == hip_encrypt; }

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
    size_t *idx = (size_t *)malloc((count ? count : 1) * sizeof(size_t));
    if (!jobs || !idx) {
        free(jobs);
        free(idx);
        return NOISE_ERROR_NO_MEMORY;
    }
    size_t nj = 0;
    for (size_t i = 0; i < count; ++i) {
        NoiseCipherState *st = states[i];
        const uint8_t *ad = ads ? ads[i] : NULL;
        size_t ad_len = ad_lens ? ad_lens[i] : 0;
        if (st && !is_ours(st)) { /* a foreign plugin object: its own backend */
            results[i] = noise_cipherstate_encrypt_with_ad(st, ad, ad_len, &buffers[i]);
            continue;
        }
        int pass;
        results[i] = check_encrypt(st, ad, ad_len, &buffers[i], &pass);
        if (results[i] || pass) continue;
        Job *j = &jobs[nj];
        j->st = (HipCipherState *)st;
        j->ad = ad;
        j->ad_len = ad_len;
        j->data = buffers[i].data;
        j->len = buffers[i].size;
        j->nonce = st->n++;
        idx[nj++] = i;
    }
    int rc = run_jobs(jobs, nj, 0);
    for (size_t k = 0; k < nj; ++k) {
        size_t i = idx[k];
        results[i] = jobs[k].status;
        if (jobs[k].status == NOISE_ERROR_NONE) buffers[i].size += 16;
    }
    free(jobs);
    free(idx);
    return rc;
}

int noise_cipherstate_decrypt_batch(NoiseCipherState *const *states, const uint8_t *const *ads,
                                    const size_t *ad_lens, NoiseBuffer *buffers, size_t count,
                                    int *results)
{
    if ((!states || !buffers || !results) && count) return NOISE_ERROR_INVALID_PARAM;
    static uint64_t epoch_counter = 0;
    Job *jobs = (Job *)malloc((count ? count : 1) * sizeof(Job));
    size_t *pend = (size_t *)malloc((count ? count : 1) * sizeof(size_t));
    size_t *idx = (size_t *)malloc((count ? count : 1) * sizeof(size_t));
    if (!jobs || !pend || !idx) {
        free(jobs);
        free(pend);
        free(idx);
        return NOISE_ERROR_NO_MEMORY;
    }
    /* Round 1 validates everything; records whose outcome depends on an
       earlier MAC failure of the same state are re-run in later rounds with
       the nonce the sequential calls would have used. */
    size_t np = 0;
    for (size_t i = 0; i < count; ++i) {
        NoiseCipherState *st = states[i];
        const uint8_t *ad = ads ? ads[i] : NULL;
        size_t ad_len = ad_lens ? ad_lens[i] : 0;
        if (st && !is_ours(st)) {
            results[i] = noise_cipherstate_decrypt_with_ad(st, ad, ad_len, &buffers[i]);
            continue;
        }
        int pass;
        results[i] = check_decrypt(st, ad, ad_len, &buffers[i], &pass);
        if (results[i] || pass) continue;
        pend[np++] = i;
    }
    int rc = NOISE_ERROR_NONE;
    while (np && !rc) {
        const uint64_t epoch = __atomic_add_fetch(&epoch_counter, 1, __ATOMIC_RELAXED);
        size_t nj = 0, nnext = 0;
        for (size_t p = 0; p < np; ++p) {
            size_t i = pend[p];
            HipCipherState *st = (HipCipherState *)states[i];
            if (st->b_epoch != epoch) {
                st->b_epoch = epoch;
                st->b_next = st->parent.n;
                st->b_failed = 0;
            }
            Job *j = &jobs[nj];
            j->st = st;
            j->ad = ads ? ads[i] : NULL;
            j->ad_len = ad_lens ? ad_lens[i] : 0;
            j->data = buffers[i].data;
            j->len = buffers[i].size - 16;
            /* assumes the earlier records of the state verify; an exhausted
               nonce stays exhausted (cipherstate.c:391-397) */
            j->nonce = st->b_next;
            if (st->b_next != NONCE_LIMIT) ++st->b_next;
            idx[nj++] = i;
        }
        /* nonce exhaustion is checked before dispatch */
        size_t keep = 0;
        for (size_t k = 0; k < nj; ++k) {
            if (jobs[k].nonce == NONCE_LIMIT) continue;
            jobs[keep] = jobs[k];
            idx[keep++] = idx[k];
        }
        rc = run_jobs(jobs, keep, 1);
        /* apply in record order */
        size_t k = 0;
        for (size_t p = 0; p < np; ++p) {
            size_t i = pend[p];
            HipCipherState *st = (HipCipherState *)states[i];
            int dispatched = (k < keep && idx[k] == i);
            if (st->b_failed) { /* depends on a failure earlier in this round */
                pend[nnext++] = i;
                if (dispatched) ++k;
                continue;
            }
            if (!dispatched) { /* nonce exhausted */
                results[i] = NOISE_ERROR_INVALID_NONCE;
                continue;
            }
            Job *j = &jobs[k++];
            results[i] = j->status;
            if (j->status == NOISE_ERROR_NONE) {
                memcpy(j->data, j->result, j->len);
                ++st->parent.n;
                buffers[i].size -= 16;
            } else {
                st->b_failed = 1;
            }
        }
        stage_scrub();
        np = nnext;
    }
    free(jobs);
    free(pend);
    free(idx);
    return rc;
}
