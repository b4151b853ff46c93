/*
 * Single-record latency of the drop-in CipherState: one
 * noise_cipherstate_encrypt then one noise_cipherstate_decrypt per message,
 * the call pattern of examples/echo (echo-client.c:414-440), timed per call.
 *
 *   latency [chachapoly|aesgcm] [bytes] [iterations]
 *
 * Prints one JSON line.  Links libnoise_aead_hip.so (tools/Makefile-free:
 * gcc -O2 -Iinclude tools/latency.c -Lnoise-c_amd/lib -lnoise_aead_hip).
 */
#include <noise_aead_hip.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv)
{
    const char *name = argc > 1 ? argv[1] : "chachapoly";
    size_t len = argc > 2 ? (size_t)atol(argv[2]) : 1024;
    int iters = argc > 3 ? atoi(argv[3]) : 5000;
    int id = strcmp(name, "aesgcm") == 0 ? NOISE_CIPHER_AESGCM : NOISE_CIPHER_CHACHAPOLY;
    NoiseCipherState *tx = NULL, *rx = NULL;
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
    if (noise_cipherstate_new_by_id(&tx, id) || noise_cipherstate_new_by_id(&rx, id)) return 1;
    if (noise_cipherstate_init_key(tx, key, 32) || noise_cipherstate_init_key(rx, key, 32)) return 1;
    uint8_t *buf = malloc(len + 16), *ref = malloc(len);
    for (size_t i = 0; i < len; ++i) ref[i] = (uint8_t)(i * 13);
    double *te = malloc(iters * sizeof(double)), *td = malloc(iters * sizeof(double));
    double ph[5] = {0, 0, 0, 0, 0}; /* resident-worker phase stamps (us), decrypt calls */
    double mhz = 0;                 /* the worker's shader clock while computing */
    double fs[8] = {0, 0, 0, 0, 0, 0, 0, 0}; /* latency-first path stamps (cycles), decrypt calls */
    double hs[4] = {0, 0, 0, 0};       /* host side of the worker call (us), decrypt calls */
    int ok = 1;
    for (int it = -50; it < iters; ++it) { /* 50 untimed warm-up messages */
        NoiseBuffer b;
        memcpy(buf, ref, len);
        noise_buffer_set_inout(b, buf, len, len + 16);
        double t0 = now_us();
        int e1 = noise_cipherstate_encrypt(tx, &b);
        double t1 = now_us();
        int e2 = noise_cipherstate_decrypt(rx, &b);
        double t2 = now_us();
        ok &= !e1 && !e2 && b.size == len && memcmp(buf, ref, len) == 0;
        if (it >= 0) {
            te[it] = t1 - t0;
            td[it] = t2 - t1;
            uint32_t st[5];
            noise_aead_debug_worker_stamps(st, 5);
            for (int i = 0; i < 5; ++i) ph[i] += st[i] * 0.01 / iters;
            mhz += noise_aead_debug_worker_clock_mhz() / iters;
            uint32_t f[8];
            noise_aead_debug_worker_fast_stamps(f, 8);
            for (int i = 0; i < 8; ++i) fs[i] += (double)f[i] / iters;
            uint64_t hn[4];
            noise_aead_debug_worker_host_ns(hn, 4);
            for (int i = 0; i < 4; ++i) hs[i] += hn[i] * 1e-3 / iters;
        }
    }
    /* the stamps of the path the decrypt calls took (cycles since the
       record's inputs were in LDS): the ChaChaPoly latency-first path, or
       gcm_wide_record; none for the other paths */
    static const char *cp_names[8] = {"chacha", "ct_in_lds", "poly_loaded", "tree", "tag", "plaintext", "-", "-"};
    static const char *gcm_names[8] = {"ctr_seal", "ghash_blocks", "ghash_reduced", "tag", "verdict",
                                       "ctr_open", "open_j0_start", "open_j0_done"};
    const char **names = id == NOISE_CIPHER_AESGCM ? gcm_names : cp_names;
    char stages[512] = "null";
    if (fs[5] > 0 || fs[3] > 0) {
        int o = snprintf(stages, sizeof stages, "{");
        for (int i = 0; i < (id == NOISE_CIPHER_AESGCM ? 8 : 6); ++i)
            o += snprintf(stages + o, sizeof stages - o, "%s\"%s\": %.0f", i ? ", " : "", names[i], fs[i]);
        snprintf(stages + o, sizeof stages - o, "}");
    }
    qsort(te, iters, sizeof(double), cmp_d);
    qsort(td, iters, sizeof(double), cmp_d);
    printf("{\"cipher\": \"%s\", \"bytes\": %zu, \"iterations\": %d, "
           "\"encrypt_us_p50\": %.2f, \"encrypt_us_p99\": %.2f, "
           "\"decrypt_us_p50\": %.2f, \"decrypt_us_p99\": %.2f, "
           "\"worker_phase_us\": {\"fence\": %.2f, \"inputs\": %.2f, \"computed\": %.2f, "
           "\"written\": %.2f, \"released\": %.2f}, \"worker_clock_mhz\": %.0f, "
           "\"stage_cycles\": %s, "
           "\"host_us\": {\"packed\": %.2f, \"doorbell\": %.2f, \"done_seen\": %.2f, \"returned\": %.2f}, "
           "\"ok\": %s}\n",
           name, len, iters, te[iters / 2], te[iters * 99 / 100], td[iters / 2],
           td[iters * 99 / 100], ph[0], ph[1], ph[2], ph[3], ph[4], mhz, stages,
           hs[0], hs[1], hs[2], hs[3], ok ? "true" : "false");
    noise_cipherstate_free(tx);
    noise_cipherstate_free(rx);
    return ok ? 0 : 1;
}
