/*
 * host_pool.c — persistent pthread pool used by the batch staging pipeline
 * (cipherstate.c).  One job at a time: a caller that finds the pool busy
 * runs its loop inline rather than queueing behind another thread's batch.
 */
#define _GNU_SOURCE
#include "host_pool.h"
#include "host_internal.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <emmintrin.h>

#define MAX_THREADS 64

static struct {
    pthread_once_t once;
    int nthreads;               /* including the caller */
    pthread_mutex_t busy;       /* held by the caller that owns the current job */
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    unsigned long gen;          /* job generation, bumped per job */
    pool_fn fn;
    void *arg;
    size_t n, grain;
    size_t next;                /* next unclaimed item (atomic) */
    int active;                 /* workers still inside the current job */
} P = {PTHREAD_ONCE_INIT, 1, PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER,
       PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, 0, 0, 0, 0, 0};

static void drain(pool_fn fn, void *arg, size_t n, size_t grain)
{
    for (;;) {
        size_t lo = __atomic_fetch_add(&P.next, grain, __ATOMIC_RELAXED);
        if (lo >= n) return;
        size_t hi = lo + grain < n ? lo + grain : n;
        fn(arg, lo, hi);
    }
}

static void *worker(void *unused)
{
    (void)unused;
    unsigned long seen = 0;
    for (;;) {
        pthread_mutex_lock(&P.mu);
        while (P.gen == seen) pthread_cond_wait(&P.go, &P.mu);
        seen = P.gen;
        pool_fn fn = P.fn;
        void *arg = P.arg;
        size_t n = P.n, grain = P.grain;
        pthread_mutex_unlock(&P.mu);
        drain(fn, arg, n, grain);
        pthread_mutex_lock(&P.mu);
        if (--P.active == 0) pthread_cond_signal(&P.done);
        pthread_mutex_unlock(&P.mu);
    }
    return NULL;
}

/* a forked child has no workers: run everything inline there */
static void pool_after_fork_child(void)
{
    pthread_mutex_t z = PTHREAD_MUTEX_INITIALIZER;
    pthread_cond_t c = PTHREAD_COND_INITIALIZER;
    P.busy = z;
    P.mu = z;
    P.go = c;
    P.done = c;
    P.nthreads = 1;
}

static void pool_init(void)
{
    pthread_atfork(NULL, NULL, pool_after_fork_child);
    int n = 0;
    const char *env = getenv("NOISE_AEAD_HOST_THREADS");
    if (env) n = atoi(env);
    if (n <= 0) {
        cpu_set_t set;
        n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
        if (n > 16) n = 16;
    }
    if (n > MAX_THREADS) n = MAX_THREADS;
    if (n < 1) n = 1;
    int started = 1;
    for (int i = 1; i < n; ++i) {
        pthread_t t;
        pthread_attr_t a;
        pthread_attr_init(&a);
        pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
        if (pthread_create(&t, &a, worker, NULL) == 0) ++started;
        pthread_attr_destroy(&a);
    }
    P.nthreads = started;
}

int host_pool_threads(void)
{
    pthread_once(&P.once, pool_init);
    return P.nthreads;
}

void host_pool_for(size_t n, size_t grain, pool_fn fn, void *arg)
{
    if (!n) return;
    if (!grain) grain = 1;
    pthread_once(&P.once, pool_init);
    if (P.nthreads <= 1 || n <= grain || pthread_mutex_trylock(&P.busy) != 0) {
        fn(arg, 0, n);
        return;
    }
    pthread_mutex_lock(&P.mu);
    P.fn = fn;
    P.arg = arg;
    P.n = n;
    P.grain = grain;
    __atomic_store_n(&P.next, 0, __ATOMIC_RELAXED);
    P.active = P.nthreads - 1;
    ++P.gen;
    pthread_cond_broadcast(&P.go);
    pthread_mutex_unlock(&P.mu);
    drain(fn, arg, n, grain);
    pthread_mutex_lock(&P.mu);
    while (P.active) pthread_cond_wait(&P.done, &P.mu);
    pthread_mutex_unlock(&P.mu);
    pthread_mutex_unlock(&P.busy);
}

__attribute__((visibility("hidden"))) void na_copy_stream(uint8_t *dst, const uint8_t *src,
                                                          size_t n)
{
    if (n < 256) {
        memcpy(dst, src, n);
        return;
    }
    size_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    for (; n >= 64; n -= 64, dst += 64, src += 64) {
        __m128i x0 = _mm_loadu_si128((const __m128i *)src);
        __m128i x1 = _mm_loadu_si128((const __m128i *)(src + 16));
        __m128i x2 = _mm_loadu_si128((const __m128i *)(src + 32));
        __m128i x3 = _mm_loadu_si128((const __m128i *)(src + 48));
        _mm_stream_si128((__m128i *)dst, x0);
        _mm_stream_si128((__m128i *)(dst + 16), x1);
        _mm_stream_si128((__m128i *)(dst + 32), x2);
        _mm_stream_si128((__m128i *)(dst + 48), x3);
    }
    memcpy(dst, src, n);
    _mm_sfence();
}
