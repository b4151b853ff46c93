/*
 * dev_stub.c — SANITIZER TEST HARNESS ONLY (make -C noise-c_amd asan).
 *
 * The noise_aead_dev_* entry points the host front end calls, computed on
 * the CPU by the repo's oracle restatement (oracle/noise_oracle.c) over the
 * stub's "device" bytes (hip_host_stub.c).  Same contracts as aead_api.hip:
 * a key context per state, ragged descriptors, open writes plaintext only
 * for a verified record and reports status 0 / 1, a record over 65519 bytes
 * is refused with status 2.  It exists so that cipherstate.c / wire.c /
 * host_pool.c run end to end under ASan/UBSan; it is never in the product
 * library, and the GPU parity of the kernels is tested elsewhere.
 */
#include "noise_aead_hip.h"
#include "noise_oracle.h"

#include <stdlib.h>
#include <string.h>

size_t noise_aead_dev_ctx_bytes(int cipher_id)
{
    return (cipher_id == NOISE_CIPHER_CHACHAPOLY || cipher_id == NOISE_CIPHER_AESGCM) ? 32 : 0;
}

int noise_aead_dev_prepare(int cipher_id, const uint8_t *d_raw_keys, uint32_t n_states,
                           void *d_ctx, void *stream)
{
    (void)stream;
    if (!noise_aead_dev_ctx_bytes(cipher_id)) return NOISE_ERROR_UNKNOWN_ID;
    if (!d_raw_keys || !d_ctx) return NOISE_ERROR_INVALID_PARAM;
    memcpy(d_ctx, d_raw_keys, (size_t)n_states * 32);
    return NOISE_ERROR_NONE;
}

static int cid(int cipher_id) { return cipher_id == NOISE_CIPHER_AESGCM ? ORACLE_AESGCM : ORACLE_CHACHAPOLY; }

static int run(int cipher_id, const NoiseAeadRagged *job, int open)
{
    if (!job || !job->recs || !job->in || !job->out) return NOISE_ERROR_INVALID_PARAM;
    if (!noise_aead_dev_ctx_bytes(cipher_id)) return NOISE_ERROR_UNKNOWN_ID;
    for (uint32_t i = 0; i < job->n_records; ++i) {
        const NoiseAeadRecord *r = &job->recs[i];
        const uint8_t *key = (const uint8_t *)job->ctx_base + r->ctx_off;
        const uint8_t *ad = r->ad_len ? job->ad + r->ad_off : NULL;
        if (r->len > 65519) {
            if (job->status) job->status[i] = 2;
            continue;
        }
        uint8_t *tmp = (uint8_t *)malloc((size_t)r->len + 16);
        if (!tmp) return NOISE_ERROR_NO_MEMORY;
        int st = 0;
        if (!open) {
            memcpy(tmp, job->in + r->in_off, r->len);
            oracle_aead_encrypt(cid(cipher_id), key, r->nonce, ad, r->ad_len, tmp, r->len);
            memcpy(job->out + r->out_off, tmp, (size_t)r->len + 16);
        } else {
            memcpy(tmp, job->in + r->in_off, (size_t)r->len + 16);
            if (oracle_aead_decrypt(cid(cipher_id), key, r->nonce, ad, r->ad_len, tmp, r->len) == 0)
                memcpy(job->out + r->out_off, tmp, r->len);
            else
                st = 1;
        }
        memset(tmp, 0, (size_t)r->len + 16);
        free(tmp);
        if (job->status) job->status[i] = (uint8_t)st;
    }
    return NOISE_ERROR_NONE;
}

int noise_aead_dev_seal_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream)
{
    (void)stream;
    return run(cipher_id, job, 0);
}

int noise_aead_dev_open_ragged(int cipher_id, const NoiseAeadRagged *job, void *stream)
{
    (void)stream;
    return run(cipher_id, job, 1);
}

uint32_t na_chacha_lanes(uint32_t n_records, uint32_t max_len)
{
    (void)n_records; (void)max_len;
    return 4;
}

uint32_t na_aes_lanes(uint32_t n_records)
{
    (void)n_records;
    return 0;
}

/* the resident worker is GPU-only: the host paths take the launch path */
int na_worker_enabled(void) { return 0; }

int na_worker_crypt(int cipher_id, const uint8_t *key, const void *h_ctx, uint32_t gen, uint64_t nonce,
                    const uint8_t *ad, size_t ad_len, uint8_t *data, size_t len, int open)
{
    (void)cipher_id; (void)key; (void)h_ctx; (void)gen; (void)nonce; (void)ad; (void)ad_len;
    (void)data; (void)len; (void)open;
    return NOISE_ERROR_NOT_APPLICABLE;
}

void na_worker_forget_ctx(const void *h_ctx) { (void)h_ctx; }

int noise_aead_debug_workers_resident(void) { return 0; }

void noise_aead_debug_worker_stamps(uint32_t *out, int n)
{
    for (int i = 0; i < n; ++i) out[i] = 0;
}

double noise_aead_debug_worker_clock_mhz(void) { return 0.0; }

int noise_aead_debug_worker_placement(void) { return 0; }

void noise_aead_debug_worker_fast_stamps(uint32_t *out, int n)
{
    for (int i = 0; i < n; ++i) out[i] = 0;
}

void noise_aead_debug_worker_host_ns(uint64_t *out, int n)
{
    for (int i = 0; i < n; ++i) out[i] = 0;
}
