/*
 * host_pool.h — a small persistent pthread pool for the host side of the
 * batch path (staging copies in and out of pinned memory, scrubbing).
 *
 * The reference has no threads (src/protocol/util.c:39-42 only uses
 * pthread_once); this pool never touches a CipherState, it only moves bytes
 * the caller's thread has already decided on, so the single-owner rule of a
 * CipherState is unchanged.
 */
#ifndef NOISE_AEAD_HOST_POOL_H
#define NOISE_AEAD_HOST_POOL_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* fn(arg, lo, hi) is called on disjoint ranges covering [0, n); the calling
   thread takes part.  Ranges are `grain` items (the last one shorter).  Runs
   inline when the pool has one thread, is busy with another caller, or n is
   at most one grain. */
typedef void (*pool_fn)(void *arg, size_t lo, size_t hi);
__attribute__((visibility("hidden"))) void host_pool_for(size_t n, size_t grain, pool_fn fn, void *arg);

/* Threads the pool uses (NOISE_AEAD_HOST_THREADS, else min(16, CPUs this
   process may run on)). */
__attribute__((visibility("hidden"))) int host_pool_threads(void);

#ifdef __cplusplus
}
#endif
#endif
