/*
 * Single-call throughput of the drop-in CipherState across threads: each of
 * T threads owns a send/recv CipherState pair (a CipherState is single-owner
 * with no locks, src/protocol/cipherstate.c:293-410) and runs
 * noise_cipherstate_encrypt + noise_cipherstate_decrypt on its own 1400-B
 * records for a fixed wall-clock window; every record is checked to round
 * trip.  Prints one JSON line: calls/s over all threads.
 *
 *   mt_calls [chachapoly|aesgcm] [threads] [bytes] [seconds]
 *
 * gcc -O2 -pthread -Iinclude tools/mt_calls.c -Lnoise-c_amd/lib -lnoise_aead_hip
 */
#include <noise_aead_hip.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static int g_id, g_len;
static double g_secs;
static volatile int g_go;

struct Res { long calls; int ok; };

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *run(void *arg)
{
    struct Res *r = arg;
    NoiseCipherState *tx = NULL, *rx = NULL;
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 11 + (int)(size_t)arg);
    r->ok = !noise_cipherstate_new_by_id(&tx, g_id) && !noise_cipherstate_new_by_id(&rx, g_id) &&
            !noise_cipherstate_init_key(tx, key, 32) && !noise_cipherstate_init_key(rx, key, 32);
    uint8_t *buf = malloc(g_len + 16), *ref = malloc(g_len);
    for (int i = 0; i < g_len; ++i) ref[i] = (uint8_t)(i * 13 + 1);
    /* warm-up: the first calls set up the key context and the worker */
    for (int it = 0; it < 20 && r->ok; ++it) {
        NoiseBuffer b;
        memcpy(buf, ref, g_len);
        noise_buffer_set_inout(b, buf, g_len, g_len + 16);
        r->ok &= !noise_cipherstate_encrypt(tx, &b) && !noise_cipherstate_decrypt(rx, &b);
    }
    while (!__atomic_load_n(&g_go, __ATOMIC_ACQUIRE)) ;
    const double t_end = now_s() + g_secs;
    long calls = 0;
    while (r->ok && now_s() < t_end) {
        NoiseBuffer b;
        memcpy(buf, ref, g_len);
        noise_buffer_set_inout(b, buf, g_len, g_len + 16);
        r->ok &= !noise_cipherstate_encrypt(tx, &b);
        r->ok &= !noise_cipherstate_decrypt(rx, &b);
        r->ok &= b.size == (size_t)g_len && memcmp(buf, ref, g_len) == 0;
        calls += 2;
    }
    r->calls = calls;
    noise_cipherstate_free(tx);
    noise_cipherstate_free(rx);
    free(buf);
    free(ref);
    return NULL;
}

int main(int argc, char **argv)
{
    const char *name = argc > 1 ? argv[1] : "chachapoly";
    int threads = argc > 2 ? atoi(argv[2]) : 1;
    g_len = argc > 3 ? atoi(argv[3]) : 1400;
    g_secs = argc > 4 ? atof(argv[4]) : 1.0;
    g_id = strcmp(name, "aesgcm") == 0 ? NOISE_CIPHER_AESGCM : NOISE_CIPHER_CHACHAPOLY;
    pthread_t th[64];
    struct Res res[64];
    if (threads < 1 || threads > 64) return 2;
    for (int i = 0; i < threads; ++i) {
        res[i].calls = 0;
        res[i].ok = 1;
        pthread_create(&th[i], NULL, run, &res[i]);
    }
    const double t0 = now_s();
    __atomic_store_n(&g_go, 1, __ATOMIC_RELEASE);
    long calls = 0;
    int ok = 1;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        calls += res[i].calls;
        ok &= res[i].ok;
    }
    const double el = now_s() - t0;
    printf("{\"cipher\": \"%s\", \"threads\": %d, \"bytes\": %d, \"seconds\": %.3f, \"calls\": %ld, "
           "\"calls_per_s\": %.0f, \"ok\": %s}\n", name, threads, g_len, el, calls, calls / el,
           ok ? "true" : "false");
    return ok ? 0 : 1;
}
