/*
 * wire_bench.c — the end-to-end wire path timed from C (VERDICT r5 item 7;
 * DESIGN.md §8).  No Python, no ctypes: one process, steady-state keys.
 *
 * A pinned buffer (noise_wire_alloc) of N echo frames (2-byte BE length ||
 * CT || tag, examples/echo/echo-server/echo-common.c:643-688) goes through
 *   noise_wire_seal (client send) -> noise_wire_echo (server: open with its
 *   receive state, seal with its send state, echo-server.c:377-407) ->
 *   noise_wire_open (client receive)
 * and must come back as the plaintext.  Each call's wall clock
 * (CLOCK_MONOTONIC) is taken over REPS repetitions after one untimed round
 * (which builds the states' device key contexts: a per-session cost).
 *
 * Beside it, the copy floor on the same buffer: a plain hipMemcpyAsync H2D
 * of the whole frame image, a D2H, the two back to back on one stream, and
 * the two concurrently on two streams (PCIe is full duplex).  A wire call
 * moves the image in AND out, so the pair is its floor; the report gives
 * each call's fraction of the pair (serial and concurrent).
 *
 * usage: wire_bench [chachapoly|aesgcm] [RECORDS] [LEN] [REPS]
 * prints one JSON line.
 */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "noise_aead_hip.h"

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

typedef struct {
    double best, median;
} Stat;

static Stat stat_of(double *v, int n)
{
    qsort(v, (size_t)n, sizeof(double), cmp_d);
    Stat s = {v[0], v[n / 2]};
    return s;
}

#define CHECK(x)                                                                  \
    do {                                                                          \
        int rc_ = (x);                                                            \
        if (rc_) {                                                                \
            fprintf(stderr, "%s:%d %s -> %#x\n", __FILE__, __LINE__, #x, rc_);    \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main(int argc, char **argv)
{
    const int cipher = (argc > 1 && !strcmp(argv[1], "aesgcm")) ? NOISE_CIPHER_AESGCM : NOISE_CIPHER_CHACHAPOLY;
    const size_t N = argc > 2 ? (size_t)atol(argv[2]) : 65536;
    const size_t L = argc > 3 ? (size_t)atol(argv[3]) : 1400;
    const int reps = argc > 4 ? atoi(argv[4]) : 10;
    const size_t F = 2 + L + 16, bytes = N * F;
    if (L + 16 > 65535 || reps < 1 || reps > 1000) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    uint8_t *wire = (uint8_t *)noise_wire_alloc(bytes);
    uint8_t *img = (uint8_t *)malloc(bytes);
    if (!wire || !img) return 1;
    uint64_t z = 0x77697265u;
    for (size_t i = 0; i < N; ++i) {
        uint8_t *f = img + i * F;
        f[0] = (uint8_t)((L + 16) >> 8);
        f[1] = (uint8_t)((L + 16) & 0xff);
        for (size_t j = 0; j < L; ++j) {
            z = z * 6364136223846793005ull + 1442695040888963407ull;
            f[2 + j] = (uint8_t)(z >> 56);
        }
        memset(f + 2 + L, 0, 16);
    }
    uint8_t k1[32], k2[32];
    for (int i = 0; i < 32; ++i) {
        k1[i] = (uint8_t)(i * 7 + 1);
        k2[i] = (uint8_t)(i * 11 + 5);
    }
    NoiseCipherState *cs, *sr, *ss, *cr;
    CHECK(noise_cipherstate_new_by_id(&cs, cipher));
    CHECK(noise_cipherstate_new_by_id(&sr, cipher));
    CHECK(noise_cipherstate_new_by_id(&ss, cipher));
    CHECK(noise_cipherstate_new_by_id(&cr, cipher));
    CHECK(noise_cipherstate_init_key(cs, k1, 32));
    CHECK(noise_cipherstate_init_key(sr, k1, 32));
    CHECK(noise_cipherstate_init_key(ss, k2, 32));
    CHECK(noise_cipherstate_init_key(cr, k2, 32));

    double *ts = (double *)malloc(sizeof(double) * (size_t)reps);
    double *te = (double *)malloc(sizeof(double) * (size_t)reps);
    double *to = (double *)malloc(sizeof(double) * (size_t)reps);
    int ok = 1;
    for (int r = -1; r < reps; ++r) { /* r = -1: untimed (key contexts) */
        memcpy(wire, img, bytes);
        size_t used = 0, frames = 0;
        const double t0 = now();
        CHECK(noise_wire_seal(cs, wire, bytes, &used, &frames));
        const double t1 = now();
        ok &= used == bytes && frames == N;
        CHECK(noise_wire_echo(sr, ss, wire, bytes, &used, &frames));
        const double t2 = now();
        ok &= used == bytes && frames == N;
        CHECK(noise_wire_open(cr, wire, bytes, &used, &frames));
        const double t3 = now();
        ok &= used == bytes && frames == N;
        for (size_t i = 0; i < N && ok; i += 97)
            ok &= !memcmp(wire + i * F + 2, img + i * F + 2, L);
        ok &= !memcmp(wire + (N - 1) * F + 2, img + (N - 1) * F + 2, L);
        if (r >= 0) {
            ts[r] = t1 - t0;
            te[r] = t2 - t1;
            to[r] = t3 - t2;
        }
    }
    const Stat seal = stat_of(ts, reps), echo = stat_of(te, reps), open_ = stat_of(to, reps);

    /* the copy floor: the same pinned buffer to / from device memory */
    void *dbuf = NULL;
    hipStream_t s1, s2;
    if (hipMalloc(&dbuf, bytes) != hipSuccess || hipStreamCreate(&s1) != hipSuccess ||
        hipStreamCreate(&s2) != hipSuccess)
        return 1;
    double *th = (double *)malloc(sizeof(double) * (size_t)reps), *tdd = (double *)malloc(sizeof(double) * (size_t)reps);
    double *tp = (double *)malloc(sizeof(double) * (size_t)reps), *tc = (double *)malloc(sizeof(double) * (size_t)reps);
    uint8_t *wire2 = (uint8_t *)noise_wire_alloc(bytes); /* D2H target of the concurrent pair */
    if (!wire2) return 1;
    for (int r = -1; r < reps; ++r) {
        double t0 = now();
        (void)hipMemcpyAsync(dbuf, wire, bytes, hipMemcpyHostToDevice, s1);
        (void)hipStreamSynchronize(s1);
        double t1 = now();
        (void)hipMemcpyAsync(wire, dbuf, bytes, hipMemcpyDeviceToHost, s1);
        (void)hipStreamSynchronize(s1);
        double t2 = now();
        (void)hipMemcpyAsync(dbuf, wire, bytes, hipMemcpyHostToDevice, s1);
        (void)hipMemcpyAsync(wire, dbuf, bytes, hipMemcpyDeviceToHost, s1);
        (void)hipStreamSynchronize(s1);
        double t3 = now();
        (void)hipMemcpyAsync(dbuf, wire, bytes / 2, hipMemcpyHostToDevice, s1); /* disjoint halves */
        (void)hipMemcpyAsync(wire2, (uint8_t *)dbuf + bytes / 2, bytes - bytes / 2, hipMemcpyDeviceToHost, s2);
        (void)hipMemcpyAsync((uint8_t *)dbuf + bytes / 2, wire + bytes / 2, bytes - bytes / 2,
                             hipMemcpyHostToDevice, s1);
        (void)hipMemcpyAsync(wire2 + bytes / 2, dbuf, bytes / 2, hipMemcpyDeviceToHost, s2);
        (void)hipStreamSynchronize(s1);
        (void)hipStreamSynchronize(s2);
        double t4 = now();
        if (r >= 0) {
            th[r] = t1 - t0;
            tdd[r] = t2 - t1;
            tp[r] = t3 - t2;
            tc[r] = t4 - t3;
        }
    }
    const Stat h2d = stat_of(th, reps), d2h = stat_of(tdd, reps), pair = stat_of(tp, reps),
               conc = stat_of(tc, reps);
    const double gib = (double)(N * L) / (1u << 30), gb = (double)bytes / 1e9;
    printf("{\"metric\": \"GiB/s end-to-end wire AEAD from C (noise_wire_*, pinned buffer, PCIe-inclusive)\", "
           "\"cipher\": \"%s\", \"frames\": %zu, \"record_len\": %zu, \"wire_bytes\": %zu, \"reps\": %d, "
           "\"ok\": %s, "
           "\"seal_gibs\": %.3f, \"echo_gibs\": %.3f, \"open_gibs\": %.3f, "
           "\"seal_ms\": {\"best\": %.3f, \"median\": %.3f}, \"echo_ms\": {\"best\": %.3f, \"median\": %.3f}, "
           "\"open_ms\": {\"best\": %.3f, \"median\": %.3f}, "
           "\"copy\": {\"h2d_gbs\": %.2f, \"d2h_gbs\": %.2f, \"pair_serial_ms\": %.3f, \"pair_concurrent_ms\": %.3f, "
           "\"h2d_ms\": %.3f, \"d2h_ms\": %.3f}, "
           "\"frac_of_copy_pair\": {\"seal_serial\": %.3f, \"open_serial\": %.3f, \"echo_serial\": %.3f, "
           "\"seal_concurrent\": %.3f, \"open_concurrent\": %.3f, \"echo_concurrent\": %.3f}, "
           "\"timing\": \"best of reps, CLOCK_MONOTONIC around each C call; copies: hipMemcpyAsync + sync\"}\n",
           cipher == NOISE_CIPHER_AESGCM ? "aesgcm" : "chachapoly", N, L, bytes, reps, ok ? "true" : "false",
           gib / seal.best, gib / echo.best, gib / open_.best, seal.best * 1e3, seal.median * 1e3,
           echo.best * 1e3, echo.median * 1e3, open_.best * 1e3, open_.median * 1e3, gb / h2d.best,
           gb / d2h.best, pair.best * 1e3, conc.best * 1e3, h2d.best * 1e3, d2h.best * 1e3,
           pair.best / seal.best, pair.best / open_.best, pair.best / echo.best, conc.best / seal.best,
           conc.best / open_.best, conc.best / echo.best);
    noise_cipherstate_free(cs);
    noise_cipherstate_free(sr);
    noise_cipherstate_free(ss);
    noise_cipherstate_free(cr);
    noise_wire_free(wire);
    noise_wire_free(wire2);
    (void)hipFree(dbuf);
    free(img);
    return ok ? 0 : 1;
}
