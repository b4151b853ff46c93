/*
 * ref_bench.c — CPU baseline driver (TEST/BENCH INFRASTRUCTURE ONLY).
 *
 * Times noise-c's own CPU path: the public CipherState API
 * (include/noise/protocol/cipherstate.h:34-53) of the reference compiled from
 * /root/reference by oracle/Makefile (`_ref/ref_bench`), default ref backend.
 * Built with -DPORT_ORACLE it times the repo's restatement
 * (noise_oracle.c) instead (`_build/port_bench`) for boxes without _ref.
 *
 * Modes
 *   roundtrip  per thread: one encrypting and one decrypting CipherState with
 *              the same key (a send/recv pair, as in examples/echo); each
 *              record is encrypted then decrypted+verified.  Wall clock
 *              (CLOCK_MONOTONIC).  Reports GiB/s of payload processed
 *              (2 x records x len: both directions), like bench.py.
 *   perf       tests/performance/test-performance.c:140-179 perf_cipher:
 *              1024 B + 32 B AD encrypt loop, one thread, CPU-time clock,
 *              reports MiB/s.
 *   mixed      the C5 mix of SURVEY.md §8d as a roundtrip: record i has
 *              length 64 + splitmix64(0x6C656E + i) % 16321 and belongs to
 *              state i / 256; even states ChaChaPoly, odd AESGCM (CIPHER and
 *              LEN are ignored).  Thread t runs records [t*RECORDS,
 *              (t+1)*RECORDS) with a send/recv CipherState pair per cipher.
 *
 * usage: ref_bench MODE CIPHER LEN RECORDS THREADS   (CIPHER: chachapoly|aesgcm)
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifdef PORT_ORACLE
#include "noise_oracle.h"
#define CID_CHACHA ORACLE_CHACHAPOLY
#define CID_AES ORACLE_AESGCM
#else
#include <noise/protocol.h>
#define CID_CHACHA NOISE_CIPHER_CHACHAPOLY
#define CID_AES NOISE_CIPHER_AESGCM
#endif

typedef struct {
    int cipher;
    size_t len, records, ad_len;
    int ok;
    size_t first;      /* mixed: first global record index */
    double bytes;      /* mixed: payload bytes processed (one direction) */
} Work;

static uint64_t splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define MIX_MAX 16384
#define MIX_RPS 256

static void *mixed(void *arg)
{
    Work *w = (Work *)arg;
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 5 + 3);
    uint8_t *buf = (uint8_t *)malloc(MIX_MAX + 16);
    uint8_t *pt = (uint8_t *)malloc(MIX_MAX + 16);
    for (size_t i = 0; i < MIX_MAX; ++i) pt[i] = (uint8_t)(i * 131 + 7);
    w->ok = 1;
    w->bytes = 0;
#ifdef PORT_ORACLE
    uint64_t n[2] = {0, 0};
    const int cid[2] = {CID_CHACHA, CID_AES};
#else
    NoiseCipherState *enc[2], *dec[2];
    const int cid[2] = {CID_CHACHA, CID_AES};
    for (int c = 0; c < 2; ++c) {
        noise_cipherstate_new_by_id(&enc[c], cid[c]);
        noise_cipherstate_new_by_id(&dec[c], cid[c]);
        noise_cipherstate_init_key(enc[c], key, 32);
        noise_cipherstate_init_key(dec[c], key, 32);
    }
    NoiseBuffer nb;
#endif
    for (size_t r = 0; r < w->records; ++r) {
        const uint64_t i = w->first + r;
        const size_t len = 64 + (size_t)(splitmix64(0x6C656Eull + i) % 16321u);
        const int c = (int)((i / MIX_RPS) & 1);
        memcpy(buf, pt, len);
#ifdef PORT_ORACLE
        oracle_aead_encrypt(cid[c], key, n[c], NULL, 0, buf, len);
        if (oracle_aead_decrypt(cid[c], key, n[c], NULL, 0, buf, len)) w->ok = 0;
        ++n[c];
#else
        noise_buffer_set_inout(nb, buf, len, len + 16);
        if (noise_cipherstate_encrypt(enc[c], &nb)) w->ok = 0;
        if (noise_cipherstate_decrypt(dec[c], &nb)) w->ok = 0;
#endif
        if (memcmp(buf, pt, len)) w->ok = 0;
        w->bytes += (double)len;
    }
#ifndef PORT_ORACLE
    for (int c = 0; c < 2; ++c) {
        noise_cipherstate_free(enc[c]);
        noise_cipherstate_free(dec[c]);
    }
#endif
    free(buf);
    free(pt);
    return NULL;
}

static double now_mono(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double now_cpu(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *roundtrip(void *arg)
{
    Work *w = (Work *)arg;
    uint8_t key[32], ad[64];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
    for (int i = 0; i < 64; ++i) ad[i] = (uint8_t)i;
    uint8_t *buf = (uint8_t *)malloc(w->len + 16);
    uint8_t *pt = (uint8_t *)malloc(w->len + 16);
    for (size_t i = 0; i < w->len; ++i) pt[i] = (uint8_t)(i * 131 + 7);
    w->ok = 1;
#ifdef PORT_ORACLE
    uint64_t n = 0;
    for (size_t r = 0; r < w->records; ++r, ++n) {
        memcpy(buf, pt, w->len);
        oracle_aead_encrypt(w->cipher, key, n, ad, w->ad_len, buf, w->len);
        if (oracle_aead_decrypt(w->cipher, key, n, ad, w->ad_len, buf, w->len)) w->ok = 0;
    }
#else
    NoiseCipherState *enc, *dec;
    noise_cipherstate_new_by_id(&enc, w->cipher);
    noise_cipherstate_new_by_id(&dec, w->cipher);
    noise_cipherstate_init_key(enc, key, 32);
    noise_cipherstate_init_key(dec, key, 32);
    NoiseBuffer nb;
    for (size_t r = 0; r < w->records; ++r) {
        memcpy(buf, pt, w->len);
        noise_buffer_set_inout(nb, buf, w->len, w->len + 16);
        if (noise_cipherstate_encrypt_with_ad(enc, ad, w->ad_len, &nb)) w->ok = 0;
        if (noise_cipherstate_decrypt_with_ad(dec, ad, w->ad_len, &nb)) w->ok = 0;
    }
    noise_cipherstate_free(enc);
    noise_cipherstate_free(dec);
#endif
    if (memcmp(buf, pt, w->len)) w->ok = 0;
    free(buf);
    free(pt);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s roundtrip|perf|mixed chachapoly|aesgcm LEN RECORDS THREADS\n", argv[0]);
        return 2;
    }
    const char *mode = argv[1];
    int cipher = strcmp(argv[2], "aesgcm") == 0 ? CID_AES : CID_CHACHA;
    size_t len = strtoull(argv[3], 0, 10), records = strtoull(argv[4], 0, 10);
    int threads = atoi(argv[5]);
    if (threads < 1) threads = 1;

    if (!strcmp(mode, "perf")) {
        /* test-performance.c:140-179: 1024 B data + 32 B AD, encrypt only */
        Work w = {cipher, 1024, records, 32, 1};
        uint8_t key[32] = {0}, ad[32] = {0}, buf[1024 + 16];
        memset(buf, 0xAA, sizeof(buf));
        double t0 = now_cpu();
#ifdef PORT_ORACLE
        for (size_t r = 0; r < w.records; ++r)
            oracle_aead_encrypt(cipher, key, r, ad, 32, buf, 1024);
#else
        NoiseCipherState *st;
        NoiseBuffer nb;
        noise_cipherstate_new_by_id(&st, cipher);
        noise_cipherstate_init_key(st, key, 32);
        for (size_t r = 0; r < w.records; ++r) {
            noise_buffer_set_inout(nb, buf, 1024, sizeof(buf));
            noise_cipherstate_encrypt_with_ad(st, ad, 32, &nb);
        }
        noise_cipherstate_free(st);
#endif
        double dt = now_cpu() - t0;
        double mib = records * 1024.0 / (1024.0 * 1024.0);
        printf("{\"mode\":\"perf\",\"cipher\":\"%s\",\"records\":%zu,\"seconds\":%.6f,"
               "\"mib_per_s\":%.3f}\n", argv[2], records, dt, mib / dt);
        return 0;
    }

    const int is_mixed = !strcmp(mode, "mixed");
    Work *ws = (Work *)calloc((size_t)threads, sizeof(Work));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        ws[t].cipher = cipher;
        ws[t].len = len;
        ws[t].records = records;
        ws[t].ad_len = 0;
        ws[t].first = (size_t)t * records;
    }
    double t0 = now_mono();
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, is_mixed ? mixed : roundtrip, &ws[t]);
    int ok = 1;
    double moved = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        ok &= ws[t].ok;
        moved += ws[t].bytes;
    }
    double dt = now_mono() - t0;
    double bytes = is_mixed ? 2.0 * moved : 2.0 * (double)len * (double)records * threads;
    if (is_mixed) {
        printf("{\"mode\":\"mixed\",\"records_per_thread\":%zu,\"threads\":%d,\"seconds\":%.6f,"
               "\"payload_bytes\":%.0f,\"gib_per_s\":%.6f,\"ok\":%s}\n",
               records, threads, dt, bytes, bytes / dt / (1024.0 * 1024.0 * 1024.0), ok ? "true" : "false");
        return ok ? 0 : 1;
    }
    printf("{\"mode\":\"roundtrip\",\"cipher\":\"%s\",\"len\":%zu,\"records_per_thread\":%zu,"
           "\"threads\":%d,\"seconds\":%.6f,\"gib_per_s\":%.6f,\"ok\":%s}\n",
           argv[2], len, records, threads, dt, bytes / dt / (1024.0 * 1024.0 * 1024.0),
           ok ? "true" : "false");
    return ok ? 0 : 1;
}
