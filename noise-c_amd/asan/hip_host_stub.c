/*
 * hip_host_stub.c — SANITIZER TEST HARNESS ONLY (make -C noise-c_amd asan).
 *
 * CPU stand-ins for the HIP runtime calls the plain-C host front end makes
 * (cipherstate.c, wire.c, host_pool.c), so that host code can be built with
 * -fsanitize=address,undefined and run on a machine without a GPU, as the
 * reference's --enable-asan / --enable-ubsan builds run its C (configure.ac
 * :102-115).  "Device" and "pinned" memory are ordinary heap blocks, a copy
 * is a memcpy done when it is enqueued, so every stream and event is already
 * complete.  The product library never links this file.
 */
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

static int g_dev;

hipError_t hipGetDevice(int *d)
{
    if (!d) return hipErrorInvalidValue;
    *d = g_dev;
    return hipSuccess;
}

hipError_t hipSetDevice(int d)
{
    g_dev = d;
    return hipSuccess;
}

hipError_t hipMalloc(void **p, size_t n)
{
    if (!p) return hipErrorInvalidValue;
    *p = malloc(n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}

hipError_t hipFree(void *p)
{
    free(p);
    return hipSuccess;
}

hipError_t hipHostMalloc(void **p, size_t n, unsigned int flags)
{
    (void)flags;
    return hipMalloc(p, n);
}

hipError_t hipHostFree(void *p) { return hipFree(p); }

hipError_t hipHostGetDevicePointer(void **d, void *h, unsigned int flags)
{
    (void)flags;
    *d = h;
    return hipSuccess;
}

hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind kind, hipStream_t s)
{
    (void)kind;
    (void)s;
    if (n) memmove(dst, src, n);
    return hipSuccess;
}

hipError_t hipMemcpy(void *dst, const void *src, size_t n, hipMemcpyKind kind)
{
    return hipMemcpyAsync(dst, src, n, kind, NULL);
}

hipError_t hipMemsetAsync(void *dst, int v, size_t n, hipStream_t s)
{
    (void)s;
    if (n) memset(dst, v, n);
    return hipSuccess;
}

/* streams and events: distinct non-null handles, always complete */
static char g_handles[64];

hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int flags)
{
    (void)flags;
    *s = (hipStream_t)(void *)&g_handles[1];
    return hipSuccess;
}

hipError_t hipStreamDestroy(hipStream_t s) { (void)s; return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t s) { (void)s; return hipSuccess; }

hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int flags)
{
    (void)s; (void)e; (void)flags;
    return hipSuccess;
}

hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned flags)
{
    (void)flags;
    *e = (hipEvent_t)(void *)&g_handles[2];
    return hipSuccess;
}

hipError_t hipEventDestroy(hipEvent_t e) { (void)e; return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) { (void)e; (void)s; return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t e) { (void)e; return hipSuccess; }
