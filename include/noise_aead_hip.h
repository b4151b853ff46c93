/*
 * noise_aead_hip.h — C ABI of the MI355X (gfx950) transport AEAD engine.
 *
 * Drop-in for noise-c's CipherState path (rweather/noise-c v0.0.1):
 *
 *  1. The reference's public CipherState API, same names, signatures,
 *     validation and error codes (include/noise/protocol/cipherstate.h:34-53,
 *     src/protocol/cipherstate.c:77-555).  Link this library in place of the
 *     CipherState part of libnoiseprotocol.
 *  2. The reference's cipher plugin constructors (src/protocol/internal.h:
 *     655-656) returning objects whose first member has the exact layout of
 *     struct NoiseCipherState_s (internal.h:58-146), so the reference's own
 *     cipherstate.c / symmetricstate.c keep working against them.
 *  3. Additive batch entry points (host buffers): N records, any mix of
 *     CipherStates, one GPU pass — results identical to N sequential calls.
 *  4. Device-resident entry points: records, keys and nonces already in HBM.
 *
 * Every computation on the encrypt/decrypt path runs in the gfx950 kernels;
 * there is no CPU fallback.  Without a usable GPU the crypto entry points
 * return NOISE_ERROR_SYSTEM.
 */
#ifndef NOISE_AEAD_HIP_H
#define NOISE_AEAD_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------- reference types/constants */

#ifndef NOISE_BUFFER_H
#define NOISE_BUFFER_H
/* include/noise/protocol/buffer.h:33-48 */
typedef struct {
    uint8_t *data;
    size_t size;
    size_t max_size;
} NoiseBuffer;
#define noise_buffer_init(buffer) \
    ((buffer).data = 0, (buffer).size = 0, (buffer).max_size = 0)
#define noise_buffer_set_output(buffer, ptr, len) \
    ((buffer).data = (ptr), (buffer).size = 0, (buffer).max_size = (len))
#define noise_buffer_set_input(buffer, ptr, len) \
    ((buffer).data = (ptr), (buffer).size = (buffer).max_size = (len))
#define noise_buffer_set_inout(buffer, ptr, len, max) \
    ((buffer).data = (ptr), (buffer).size = (len), (buffer).max_size = (max))
#endif

#ifndef NOISE_CONSTANTS_H
/* include/noise/protocol/constants.h:31-38, 131-151 */
#define NOISE_ID(ch, num) ((((int)(ch)) << 8) | ((int)(num)))
#define NOISE_CIPHER_NONE 0
#define NOISE_CIPHER_CATEGORY NOISE_ID('C', 0)
#define NOISE_CIPHER_CHACHAPOLY NOISE_ID('C', 1)
#define NOISE_CIPHER_AESGCM NOISE_ID('C', 2)
#define NOISE_PADDING_ZERO NOISE_ID('G', 1) /* constants.h:123-124 */
#define NOISE_PADDING_RANDOM NOISE_ID('G', 2)
#define NOISE_HASH_BLAKE2s NOISE_ID('H', 1) /* constants.h:43-46 */
#define NOISE_HASH_BLAKE2b NOISE_ID('H', 2)
#define NOISE_HASH_SHA256 NOISE_ID('H', 3)
#define NOISE_HASH_SHA512 NOISE_ID('H', 4)
#define NOISE_ERROR_NONE 0
#define NOISE_ERROR_NO_MEMORY NOISE_ID('E', 1)
#define NOISE_ERROR_UNKNOWN_ID NOISE_ID('E', 2)
#define NOISE_ERROR_UNKNOWN_NAME NOISE_ID('E', 3)
#define NOISE_ERROR_MAC_FAILURE NOISE_ID('E', 4)
#define NOISE_ERROR_NOT_APPLICABLE NOISE_ID('E', 5)
#define NOISE_ERROR_SYSTEM NOISE_ID('E', 6)
#define NOISE_ERROR_INVALID_LENGTH NOISE_ID('E', 10)
#define NOISE_ERROR_INVALID_PARAM NOISE_ID('E', 11)
#define NOISE_ERROR_INVALID_STATE NOISE_ID('E', 12)
#define NOISE_ERROR_INVALID_NONCE NOISE_ID('E', 13)
#define NOISE_MAX_PAYLOAD_LEN 65535
#endif

/* ------------------------------------------------ 1. CipherState API
 * Each replaces the function of the same name in src/protocol/cipherstate.c.
 * Single encrypt/decrypt calls launch nothing: a resident worker workgroup
 * per calling thread (up to one per high-priority hardware queue of the
 * device, GPU_MAX_HW_QUEUES: 4 by default) serves them through a request
 * slot, ~8-12 us per record up to 1.4 KB; it leaves after 2 ms without
 * requests, when a batch launch fills the device, or when a state whose key
 * it caches is freed.  NOISE_AEAD_WORKER=0: one kernel launch per call. */

typedef struct NoiseCipherState_s NoiseCipherState;

int noise_cipherstate_new_by_id(NoiseCipherState **state, int id);        /* cipherstate.c:77-104 */
int noise_cipherstate_new_by_name(NoiseCipherState **state, const char *name); /* :122-140 */
int noise_cipherstate_free(NoiseCipherState *state);                      /* :152-165 */
int noise_cipherstate_get_cipher_id(const NoiseCipherState *state);       /* :174-177 */
size_t noise_cipherstate_get_key_length(const NoiseCipherState *state);   /* :188-191 */
size_t noise_cipherstate_get_mac_length(const NoiseCipherState *state);   /* :202-205 */
int noise_cipherstate_init_key(NoiseCipherState *state, const uint8_t *key,
                               size_t key_len);                           /* :221-235 */
int noise_cipherstate_has_key(const NoiseCipherState *state);             /* :247-250 */
int noise_cipherstate_encrypt_with_ad(NoiseCipherState *state, const uint8_t *ad,
                                      size_t ad_len, NoiseBuffer *buffer); /* :293-333 */
int noise_cipherstate_decrypt_with_ad(NoiseCipherState *state, const uint8_t *ad,
                                      size_t ad_len, NoiseBuffer *buffer); /* :373-410 */
int noise_cipherstate_encrypt(NoiseCipherState *state, NoiseBuffer *buffer); /* :452-455 */
int noise_cipherstate_decrypt(NoiseCipherState *state, NoiseBuffer *buffer); /* :494-497 */
int noise_cipherstate_set_nonce(NoiseCipherState *state, uint64_t nonce);    /* :518-535 */
int noise_cipherstate_get_max_key_length(void);                           /* :542-545 */
int noise_cipherstate_get_max_mac_length(void);                           /* :552-555 */

/* ------------------------------------------------ 2. plugin constructors
 * internal.h:655-656; objects start with struct NoiseCipherState_s
 * (internal.h:58-146) filled as cipher-chachapoly.c:145-158 /
 * cipher-aesgcm.c:190-203 do, plus a destroy hook (as the OpenSSL backend,
 * src/backend/openssl/cipher-aesgcm.c:188-204) that frees device memory. */
NoiseCipherState *noise_chachapoly_new(void);
NoiseCipherState *noise_aesgcm_new(void);

/* ------------------------------------------------ 3. batch (host buffers)
 *
 * Process count records: record i is buffers[i] under states[i] (states may
 * repeat and may mix ciphers) with associated data ads[i]/ad_lens[i] (both
 * arrays may be NULL for no AD).  results[i] receives exactly what
 *   noise_cipherstate_{en,de}crypt_with_ad(states[i], ads[i], ad_lens[i], &buffers[i])
 * would have returned had the calls been made one by one in index order, and
 * buffers, sizes and nonces end up exactly as after those calls (including
 * the no-key pass-through, nonce exhaustion and the "nonce not advanced on a
 * MAC failure" rule, cipherstate.c:321-326, 400-405).  One GPU pass in the
 * common case.  Returns NOISE_ERROR_NONE unless an argument is invalid or the
 * GPU fails (NOISE_ERROR_SYSTEM; then results[] is unspecified). */
int noise_cipherstate_encrypt_batch(NoiseCipherState *const *states,
                                    const uint8_t *const *ads, const size_t *ad_lens,
                                    NoiseBuffer *buffers, size_t count, int *results);
int noise_cipherstate_decrypt_batch(NoiseCipherState *const *states,
                                    const uint8_t *const *ads, const size_t *ad_lens,
                                    NoiseBuffer *buffers, size_t count, int *results);

/* ------------------------------------------------ 3b. transport wire buffers
 *
 * SURVEY.md §8f rank 1.  A wire buffer holds frames in the format of the
 * reference's examples/echo (echo-common.c:643-688, echo_recv/echo_send):
 * a 2-byte big-endian length L, then L bytes of CT || tag.  These calls work
 * in place on every complete frame at the start of the buffer, frame k under
 * nonce n + k of its CipherState, in one pipelined GPU pass:
 *
 *   noise_wire_seal : each frame holds L - 16 bytes of plaintext followed by
 *                     16 bytes of room; they become CT || tag.  The header is
 *                     already the final length (what echo_send writes).
 *   noise_wire_open : each frame's first L - 16 bytes become its plaintext
 *                     (the 16 tag bytes after it are left as they were).
 *   noise_wire_echo : the echo server's transport loop (echo-server.c
 *                     :377-407): every frame opened with `recv` and sealed
 *                     again with `send` (same length, so in place).
 *
 * *frames / *consumed report the frames processed and the bytes they span.
 * Processing stops, exactly as the per-frame CipherState calls would, at:
 *   - a partial frame at the end (returns NOISE_ERROR_NONE);
 *   - a frame with L < 16 (NOISE_ERROR_INVALID_LENGTH) or an exhausted
 *     nonce (NOISE_ERROR_INVALID_NONCE) — that frame is untouched;
 *   - open/echo: the first frame whose tag fails (NOISE_ERROR_MAC_FAILURE):
 *     it and every later frame are untouched and n stays at its nonce, the
 *     rule of cipherstate.c:400-405 applied frame by frame.
 * Nonces advance by the frames processed (seal: by every frame dispatched,
 * also on NOISE_ERROR_SYSTEM, as cipherstate.c:325-326).  The states must be
 * keyed (NOISE_ERROR_INVALID_STATE otherwise) and, for echo, distinct.
 *
 * Buffers from noise_wire_alloc() are pinned host memory: H2D and D2H use
 * them directly.  Any other buffer is staged through pinned memory. */
void *noise_wire_alloc(size_t bytes);
void noise_wire_free(void *wire);
int noise_wire_seal(NoiseCipherState *state, uint8_t *wire, size_t wire_len,
                    size_t *consumed, size_t *frames);
int noise_wire_open(NoiseCipherState *state, uint8_t *wire, size_t wire_len,
                    size_t *consumed, size_t *frames);
int noise_wire_echo(NoiseCipherState *recv, NoiseCipherState *send, uint8_t *wire,
                    size_t wire_len, size_t *consumed, size_t *frames);

/* ------------------------------------------------ 4. device-resident API
 *
 * All pointers below are device pointers on the current HIP device; `stream`
 * is a hipStream_t (NULL = default stream).  Calls are asynchronous.
 *
 * Key contexts: n_states contexts of noise_aead_dev_ctx_bytes(cipher) bytes
 * each, built from n_states raw 32-byte keys by noise_aead_dev_prepare
 * (ChaChaPoly: the key itself; AESGCM: round keys + GHASH tables). */
size_t noise_aead_dev_ctx_bytes(int cipher_id);
int noise_aead_dev_prepare(int cipher_id, const uint8_t *d_raw_keys, uint32_t n_states,
                           void *d_ctx, void *stream);

/* Uniform batch.  Record i (0 <= i < n_records) belongs to state
 * s = i / recs_per_state and uses nonce nonce_base[s] + i % recs_per_state.
 * seal: in + i*in_stride holds len plaintext bytes; out + i*out_stride
 *       receives CT || tag (len + 16 bytes).
 * open: in + i*in_stride holds CT || tag; status[i] = 0 (ok) or 1 (MAC
 *       failure).  A verified record's len plaintext bytes go to
 *       out + i*out_stride.  Open order:
 *         - AESGCM opens always authenticate first and write a record's
 *           output only after its tag verified — the order of the
 *           reference's ref backends (cipher-aesgcm.c:172-188): a rejected
 *           record's output is not written at all (in place: CT || tag read
 *           back as given; out of place: the output bytes keep whatever
 *           they held).  It costs nothing there.
 *         - CHACHAPOLY opens take the same order by default (round 6; the
 *           reference's cipher-chachapoly.c:135-141): authenticate, then
 *           decrypt and write only verified records.  With the opt-in
 *           NOISE_AEAD_FLAG_ONE_PASS a FAST-layout ChaChaPoly open decrypts
 *           as it authenticates (one pass over the ciphertext, DESIGN.md
 *           4.1b gives the rate difference), and a rejected record reads
 *           back in place exactly as given, out of place as ZEROED output
 *           bytes; until the kernel ends its output bytes may transiently
 *           hold unauthenticated plaintext, which the kernel undoes
 *           (restores / zeroes) before it completes.
 * Memory: input and output records must be either exactly in place
 * (in == out and in_stride == out_stride) or disjoint record by record:
 * with one stride for both sides the records may interleave (input and
 * output slots alternating in one buffer) as long as no input record
 * [in + i*stride, + len (+16 open)) meets an output record; with two
 * strides the two spans must be disjoint.  Anything else is refused with
 * NOISE_ERROR_INVALID_PARAM.
 * lanes_per_record: 0 = automatic; ChaChaPoly 1, 2, 4, 8, 16, 32 or 64 (wider
 * groups cut the latency of small batches of long records); AESGCM 4 (0 lets
 * a ragged batch of at most 512 records run one record per workgroup). */
typedef struct NoiseAeadUniform {
    const void *ctx;
    const uint64_t *nonce_base;
    const uint8_t *in;
    uint8_t *out;
    const uint8_t *ad;       /* may be NULL when ad_len == 0 */
    uint8_t *status;         /* open only; may be NULL */
    uint64_t in_stride, out_stride, ad_stride;
    uint32_t recs_per_state;
    uint32_t n_records;
    uint32_t len;            /* <= 65535 - 16 */
    uint32_t ad_len;
    uint32_t lanes_per_record;
    uint32_t flags;          /* NOISE_AEAD_FLAG_CT_GHASH, _VERIFY_FIRST, _ONE_PASS (FAST is derived) */
} NoiseAeadUniform;

int noise_aead_dev_seal_uniform(int cipher_id, const NoiseAeadUniform *job, void *stream);
int noise_aead_dev_open_uniform(int cipher_id, const NoiseAeadUniform *job, void *stream);

/* Duplex: seal_job and open_job in one launch — an echo server's two
 * directions (echo-server.c:377-407 opens what it receives and seals what it
 * sends) or a pipeline sealing one batch while opening an earlier one.  The
 * result is exactly noise_aead_dev_seal_uniform(seal_job) followed by
 * noise_aead_dev_open_uniform(open_job); the jobs must be independent:
 * nothing one job writes (its output records, the open job's statuses) may
 * overlap anything the other job reads (records, AD) or writes, else
 * NOISE_ERROR_INVALID_PARAM.  Either job may have n_records == 0.  When the
 * two jobs cannot share a kernel (unaligned layouts, different lane counts,
 * AESGCM without one state per 256 records, a VERIFY_FIRST ChaChaPoly open
 * on 4 or 8 lanes per record) the library issues the two launches on
 * `stream` instead; a verify-first open (the default) on one lane per record
 * (the default from 65 536 records) or on the staged AES-GCM kernel keeps the
 * one launch. */
int noise_aead_dev_duplex_uniform(int cipher_id, const NoiseAeadUniform *seal_job,
                                  const NoiseAeadUniform *open_job, void *stream);

/* Ragged batch: one descriptor per record.  The key context of a record is
 * at ctx_base + ctx_off (ctx_base may be NULL with absolute ctx_off). */
typedef struct NoiseAeadRecord {
    uint64_t in_off;
    uint64_t out_off;
    uint64_t nonce;
    uint64_t ctx_off;
    uint64_t ad_off;
    uint32_t len;
    uint32_t ad_len;
} NoiseAeadRecord;

typedef struct NoiseAeadRagged {
    const void *ctx_base;
    const NoiseAeadRecord *recs; /* device array of n_records descriptors */
    const uint8_t *in;
    uint8_t *out;
    const uint8_t *ad;
    uint8_t *status;
    uint32_t n_records;
    uint32_t lanes_per_record;
    uint32_t flags;              /* NOISE_AEAD_FLAG_* */
    uint32_t reserved_;
} NoiseAeadRagged;

/* A record longer than NOISE_MAX_PAYLOAD_LEN - 16 (65519) bytes is not
 * processed: nothing is written and, when status is given, status[i] = 2 —
 * for seal too (status is optional there: 0 sealed, 2 refused).
 *
 * Open: a rejected record's output is handled as for the uniform open (not
 * written at all by default; restored in place / zeroed out of place under
 * NOISE_AEAD_FLAG_ONE_PASS).  Each record's input and output ranges must
 * be identical (in + in_off == out + out_off) or disjoint from every other
 * record's ranges; the descriptors live in device memory, so this is the
 * caller's guarantee (not checked).
 *
 * The caller guarantees, for every record: in + in_off and out + out_off are
 * 16-byte aligned, and the input may be read up to roundup64(max(len, 1))
 * bytes (and holds CT || tag for open).  Enables the straight-line dwordx4 path.  The
 * uniform API derives this itself from the pointers and strides. */
#define NOISE_AEAD_FLAG_FAST 1u

/* AESGCM only: GHASH without lookup tables.  The default GHASH multiplies
 * by H through 4-bit tables indexed by the running hash (LDS copies are
 * bank-conflict-free; the per-lane final scale reads the context's tables in
 * global memory, whose cache-line footprint depends on secret data).  With
 * this flag every multiply is a carry-less 128x128 product built from integer
 * multiplies of masked operands (no secret-dependent address or branch) —
 * slower; DESIGN.md §4 gives both throughputs.  Setting the environment
 * variable NOISE_AEAD_CT_GHASH=1 before the first call turns it on for every
 * job, including the CipherState and wire paths. */
#define NOISE_AEAD_FLAG_CT_GHASH 2u

/* Open only: authenticate first, decrypt only a verified record, and write
 * nothing for a rejected one (the reference's verify-then-decrypt order,
 * cipher-chachapoly.c:135-141, cipher-aesgcm.c:172-188).  Since round 6
 * this is the order of every open whether or not the flag is set; the flag
 * stays accepted, and it overrides NOISE_AEAD_FLAG_ONE_PASS. */
#define NOISE_AEAD_FLAG_VERIFY_FIRST 4u

/* Open only, ChaChaPoly FAST layouts, opt-in: decrypt while authenticating
 * (one pass over the ciphertext) and undo a rejected record's plaintext
 * before the kernel ends — restored in place, zeroed out of place (see the
 * uniform open above).  Faster on the device API; the
 * host paths (CipherState API, batch, wire) never set it.  AESGCM opens and
 * non-FAST layouts ignore it (they always verify first). */
#define NOISE_AEAD_FLAG_ONE_PASS 8u

int noise_aead_dev_seal_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream);
int noise_aead_dev_open_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream);

/* ------------------------------------------------ 5. session key fan-out
 *
 * SURVEY.md §8f rank 2.  For n sessions at once, the HKDF of
 * noise_hashstate_hkdf (src/protocol/hashstate.c:476-516) with the session's
 * Noise hash (NOISE_HASH_BLAKE2s/BLAKE2b/SHA256/SHA512):
 *   out1[i] || out2[i] = HKDF(keys[i], data[i])   (each truncated)
 * keys[i] = d_keys + i*key_len (1..256 bytes), data[i] = d_data + i*data_len
 * (0..256 bytes; d_data may be NULL when data_len is 0), output lengths at
 * most the hash length (NOISE_ERROR_INVALID_LENGTH otherwise, as
 * hashstate.c:496-497).  noise_aead_dev_split is the key derivation of
 * noise_symmetricstate_split (symmetricstate.c:530-533): HKDF(ck, "") into
 * two 32-byte transport keys per session (ck is the hash length), ready for
 * noise_aead_dev_prepare.  Device pointers, asynchronous on `stream`. */
int noise_aead_dev_hkdf(int hash_id, const uint8_t *d_keys, uint32_t key_len,
                        const uint8_t *d_data, uint32_t data_len, uint32_t n, uint8_t *d_out1,
                        uint32_t out1_len, uint8_t *d_out2, uint32_t out2_len, void *stream);
int noise_aead_dev_split(int hash_id, const uint8_t *d_ck, uint32_t n, uint8_t *d_k1,
                         uint8_t *d_k2, void *stream);

/* Handshake-payload AEAD for a batch of SymmetricStates (SURVEY.md §8f
 * rank 3): noise_symmetricstate_encrypt_and_hash / decrypt_and_hash
 * (symmetricstate.c:352-445) on n keyed states at once.  d_h holds the n
 * handshake hashes (hash-length bytes each); the job's AD must be those
 * hashes: job->ad == d_h and record i's ad_off = i * hash_len, ad_len =
 * hash_len.  Encrypt seals record i with AD = h_i, then
 * h_i = HASH(h_i || CT_i || tag_i).  Decrypt hashes CT_i || tag_i first,
 * opens, and keeps the new h_i only where status[i] == 0 (the reference
 * leaves h unchanged on a MAC failure, :425-443); job->status is required. */
int noise_aead_dev_encrypt_and_hash(int cipher_id, int hash_id, uint8_t *d_h,
                                    const NoiseAeadRagged *job, void *stream);
int noise_aead_dev_decrypt_and_hash(int cipher_id, int hash_id, uint8_t *d_h,
                                    const NoiseAeadRagged *job, void *stream);

/* ------------------------------------------------ 6. batched padding
 *
 * SURVEY.md §8f rank 4.  n calls of noise_randstate_pad(state, payload_i,
 * orig_lens[i], padded_len, padding_mode) (randstate.c:348-375) in record
 * order, payload_i = d_payloads + i*stride, so that messages padded to one
 * length (echo-client -g, echo-client.c:400-410) go through
 * noise_aead_dev_seal_uniform.  A record with padded_len <= orig_lens[i] is
 * left alone and does not touch the generator.
 *  - NOISE_PADDING_ZERO: the padding bytes are zeroed.
 *  - NOISE_PADDING_RANDOM (and, as in the reference, any unknown mode): the
 *    bytes of noise_randstate_generate (:263-316) drawn from *d_rand, a device
 *    copy of the RandState generator (its ChaCha key, 64-bit block counter,
 *    64-bit IV and reseed budget `left`, randstate.c:47-58), advanced in place
 *    exactly as the sequential calls advance it (rekeys included).  When a
 *    call would need a reseed from OS entropy (left too small) the walk stops
 *    before that record: records from there on are untouched and *d_done
 *    (optional) = records processed — the caller reseeds and calls again.
 *  - d_rand == NULL: the padding is zeroed and NOISE_ERROR_INVALID_PARAM is
 *    returned (the reference's NULL-state rule).
 * Device pointers, asynchronous on `stream`. */
typedef struct NoiseRandSnapshot {
    uint32_t key[8];
    uint64_t counter;
    uint64_t iv;
    uint64_t left;
} NoiseRandSnapshot;

int noise_aead_dev_pad(NoiseRandSnapshot *d_rand, uint8_t *d_payloads, uint64_t stride,
                       const uint32_t *d_orig_lens, uint32_t padded_len, uint32_t n,
                       int padding_mode, uint32_t *d_done, void *stream);

/* ------------------------------------------------ error reports
 * include/noise/protocol/errors.h; src/protocol/errors.c:92-127. */
void noise_perror(const char *s, int err);
int noise_strerror(int err, char *buf, size_t size);

/* ------------------------------------------------ test / debug hooks
 * Not part of the reference surface; used by the test suite.
 * noise_aead_debug_batch_stats: GPU rounds and records dispatched by this
 *   thread's last noise_cipherstate_decrypt_batch call (a run of forged
 *   records must cost rounds, not re-dispatches of the whole batch).
 * noise_aead_debug_last_freed_ctx: with NOISE_AEAD_DEBUG_KEEP_FREED=1 in the
 *   environment, freeing a CipherState scrubs its device key context but keeps
 *   the allocation; this returns it (and its size) so a test can read back
 *   zeros.  Leaks by design; never set it in production. */
void noise_aead_debug_batch_stats(uint64_t *rounds, uint64_t *dispatched);
/* noise_aead_debug_worker_stamps: the phase times (10-ns ticks) of the
 *   resident single-record worker's last request on the current device:
 *   fence, inputs in LDS, computed, results written, released (n <= 5). */
void noise_aead_debug_worker_stamps(uint32_t *out, int n);
/* noise_aead_debug_worker_clock_mhz: the shader clock of that request's
 *   compute phase (s_memtime cycles / s_memrealtime time), 0 if none. */
double noise_aead_debug_worker_clock_mhz(void);
/* noise_aead_debug_worker_fast_stamps: shader-cycle stamps through the
 *   worker's latency-first ChaChaPoly path, or its AES-GCM record (n <= 8). */
void noise_aead_debug_worker_fast_stamps(uint32_t *out, int n);
/* noise_aead_debug_worker_placement: where the current device's worker
 *   takes requests: 0 not started, 1 pinned host memory, 2 device memory
 *   written through the BAR (large-BAR devices, NOISE_AEAD_WORKER_VRAM). */
int noise_aead_debug_worker_placement(void);
/* noise_aead_debug_worker_host_ns: the calling thread's last worker call on
 *   the host, ns from its start: packed, doorbell, done seen, returned. */
void noise_aead_debug_worker_host_ns(uint64_t *out, int n);
void *noise_aead_debug_last_freed_ctx(size_t *bytes);
/* noise_aead_debug_workers_resident: request slots (one workgroup each) of
 *   the current device whose worker group is still running (-1: no device). */
int noise_aead_debug_workers_resident(void);
/* noise_aead_debug_worker_launches: worker group kernels launched on the
 *   current device so far. */
unsigned noise_aead_debug_worker_launches(void);
/* noise_aead_debug_worker_group_launches: out[g] = launches of group g
 *   (g < 8), out[8..11] = the relaunch checks by cause (not launched,
 *   slot exiting at the call, slot exiting while waiting, no launch needed). */
void noise_aead_debug_worker_group_launches(unsigned *out, int n);
/* noise_aead_debug_worker_leave_reason / _leave_info: why slot `slot` of
 *   group `group` last left (1 stop, 2 another slot closed the group, 4 idle,
 *   8 lifetime) and its born / leave times (10-ns ticks), lifetime, launch. */
unsigned noise_aead_debug_worker_leave_reason(int group, int slot);
void noise_aead_debug_worker_leave_info(int group, int slot, unsigned *out);

/* Default lanes per record the library picks for a standalone uniform seal
 * or open of n records (noise_aead_dev_{seal,open}_uniform, lanes 0) in a
 * FAST layout: ChaChaPoly 1 from 128 Ki records (the one-lane kernels at
 * two waves per SIMD), else 4 or 8, and up to 64 for batches of at most 512
 * records (a VERIFY_FIRST open of at least 64 Ki records: 1); AES-GCM 4.
 * Other layouts and ragged batches keep the multi-lane rules. */
int noise_aead_dev_default_lanes(int cipher_id, uint32_t n_records);
/* ...and for each job of a noise_aead_dev_duplex_uniform launch: ChaChaPoly
 * jobs of at least 64 Ki records in FAST layouts (16-B aligned slots
 * readable up to roundup64(len)) take one lane per record (the LDS-staged
 * one-lane kernels, a seal and an open wave on every SIMD), else as above. */
int noise_aead_dev_duplex_lanes(int cipher_id, uint32_t n_records);

/* Deterministic synthetic bytes (bench/test input): 64-bit LE word w of the
 * output = SplitMix64(seed + word0 + w), SURVEY.md §8d. */
int noise_aead_dev_fill_splitmix(uint8_t *d_out, uint64_t nbytes, uint64_t seed,
                                 uint64_t word0, void *stream);

#ifdef __cplusplus
}
#endif
#endif
