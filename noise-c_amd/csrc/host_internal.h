/*
 * host_internal.h — host-side internals shared by the CipherState front end
 * (cipherstate.c) and the wire-format path (wire.c).  Not part of the ABI.
 */
#ifndef NOISE_AEAD_HOST_INTERNAL_H
#define NOISE_AEAD_HOST_INTERNAL_H

#include "noise_aead_hip.h"

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#define NA_HIDDEN __attribute__((visibility("hidden")))

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
    int b_stop;        /* this round's later records rest on a wrong nonce guess */
    int b_forge;       /* round mode: 1 = every record tried at nonce n (a run of
                          forgeries), 0 = records at n, n+1, ... (all verify) */
    int b_hit;         /* forge round: a record verified; optimistic round: one failed */
    uint64_t b_upd;    /* round whose outcome last set b_window / b_forge */
    uint64_t b_window; /* records dispatched per round (0 = all) */
    uint64_t b_sent;   /* records dispatched in the current round */
    /* AES-GCM: pinned host copy of d_ctx for the resident worker (worker.hip) */
    uint8_t *h_ctx;
    int h_ctx_ready;
    uint32_t h_ctx_gen;  /* generation the copy was written at */
} HipCipherState;

#define MAX_CHUNKS 64
#define CHUNK_MIN ((size_t)4 << 20)
#define ZERO_COPY_DEFAULT ((size_t)128 << 10) /* cipherstate.c zero_copy_max */
#define ZERO_COPY_AES ((size_t)2 << 10)       /* ... with AES-GCM records in the batch */

typedef struct {
    int device;
    hipStream_t stream;    /* kernels + D2H */
    hipStream_t stream_in; /* H2D */
    hipStream_t stream_out; /* wire path: host-gated kernels + D2H */
    hipEvent_t ev_in[MAX_CHUNKS], ev_out[MAX_CHUNKS], ev_done[MAX_CHUNKS];
    uint8_t *h;        /* pinned host */
    uint8_t *hd;       /* the same pinned bytes as the device addresses them */
    uint8_t *d;        /* device */
    size_t cap;
} Staging;

/* The resident single-record worker (worker.hip): na_worker_crypt returns
   NOISE_ERROR_NOT_APPLICABLE when the record must take the launch path. */
NA_HIDDEN int na_worker_enabled(void);
NA_HIDDEN int na_worker_crypt(int cipher_id, const uint8_t *key, const void *h_ctx, uint32_t gen,
                              uint64_t nonce, const uint8_t *ad, size_t ad_len, uint8_t *data,
                              size_t len, int open);
/* a state's AES-GCM host context is being freed: workers that may cache it
   in LDS leave (and scrub it) */
NA_HIDDEN void na_worker_forget_ctx(const void *h_ctx);

NA_HIDDEN Staging *na_stage_get(size_t bytes);
NA_HIDDEN int na_ensure_ctx(HipCipherState *st, Staging *sg);
NA_HIDDEN int na_is_ours(const NoiseCipherState *st);
NA_HIDDEN void na_clean(void *p, size_t n);
/* ChaChaPoly lanes per record for n records of at most max_len bytes (aead_api.hip) */
NA_HIDDEN uint32_t na_chacha_lanes(uint32_t n_records, uint32_t max_len);
NA_HIDDEN uint32_t na_aes_lanes(uint32_t n_records); /* 0 (automatic) or 4 */
/* memcpy with non-temporal (streaming) stores: staging copies are written
   once and read back by DMA or by another pass much later, so skipping the
   read-for-ownership of every destination line halves their write traffic */
NA_HIDDEN void na_copy_stream(uint8_t *dst, const uint8_t *src, size_t n);
/* NOISE_AEAD_TRACE=1 timing lines on stderr */
NA_HIDDEN double na_now_ms(void);
NA_HIDDEN int na_trace_on(void);

#endif
