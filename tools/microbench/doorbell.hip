// Doorbell round trip: where should a resident worker poll?
//
//   doorbell [iters]
//
// One workgroup polls a request word; when it changes, it reads a 1 KiB
// payload next to it, adds it up and stores the sum and the sequence number
// into pinned host memory (system-scope vector store); the host spins on
// that word.  The host times request-written -> acknowledgement-seen.
//   host: request + payload in pinned host memory; the GPU polls over PCIe
//         (what worker.hip does today).
//   vram: request + payload in fine-grained device memory written by the
//         CPU through the BAR (only if this box maps VRAM for the CPU); the
//         GPU polls its own memory.
// Each poll loop ends after 2 s of wall clock whatever happens, so the grid
// always drains.
#include <hip/hip_runtime.h>
#include <emmintrin.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int PAYLOAD = 1024;

struct Req {
    uint32_t seq;
    uint32_t pad[63];
    uint32_t data[PAYLOAD / 4];
};

__device__ __forceinline__ uint32_t load_sys(const uint32_t *p)
{
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

__global__ __launch_bounds__(256) void pong(const Req *req, uint32_t *ack, int iters)
{
    __shared__ uint32_t s_go, part[4];
    const uint32_t t = threadIdx.x;
    const uint64_t limit = 2ull * 100000000ull; /* 2 s of the 100 MHz realtime clock */
    for (int i = 1; i <= iters; ++i) {
        if (t == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t ok = 0;
            while (__builtin_amdgcn_s_memrealtime() - t0 < limit) {
                if (load_sys(&req->seq) == (uint32_t)i) { ok = 1; break; }
            }
            s_go = ok;
        }
        __syncthreads();
        if (!s_go) return; /* every thread leaves together */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        uint32_t v = load_sys(&req->data[t]);
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((t & 63) == 0) part[t >> 6] = v;
        __syncthreads();
        if (t == 0) {
            __hip_atomic_store(&ack[1], part[0] + part[1] + part[2] + part[3], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&ack[0], (uint32_t)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
    }
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

/* can the CPU store to and load from p? */
static bool cpu_can_touch(volatile uint32_t *p)
{
    struct sigaction sa, old_segv, old_bus;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_jb, 1) == 0) {
        p[0] = 0x1234567u;
        ok = p[0] == 0x1234567u;
        p[0] = 0;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

static double now_ns()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e9 + t.tv_nsec;
}

static void run(const char *name, Req *req_host_view, const Req *req_dev_view, uint32_t *ack, int iters)
{
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    volatile uint32_t *a = ack;
    a[0] = 0;
    a[1] = 0;
    req_host_view->seq = 0;
    _mm_sfence();
    hipLaunchKernelGGL(pong, dim3(1), dim3(256), 0, s, req_dev_view, ack, iters);
    std::vector<double> rt(iters), wr(iters);
    uint32_t payload[PAYLOAD / 4];
    bool ok = true;
    for (int i = 1; i <= iters; ++i) {
        for (int k = 0; k < PAYLOAD / 4; ++k) payload[k] = (uint32_t)(i * 2654435761u + k);
        const double t0 = now_ns();
        memcpy((void *)req_host_view->data, payload, PAYLOAD);
        _mm_sfence();
        __atomic_store_n(&req_host_view->seq, (uint32_t)i, __ATOMIC_RELEASE);
        _mm_sfence();
        const double t1 = now_ns();
        const double limit = t0 + 2e9;
        while (__atomic_load_n(&a[0], __ATOMIC_ACQUIRE) != (uint32_t)i)
            if (now_ns() > limit) { ok = false; break; }
        const double t2 = now_ns();
        if (!ok) break;
        uint32_t sum = 0;
        for (int k = 0; k < PAYLOAD / 4; ++k) sum += payload[k];
        ok &= a[1] == sum;
        rt[i - 1] = t2 - t0;
        wr[i - 1] = t1 - t0;
    }
    CHECK(hipStreamSynchronize(s));
    CHECK(hipStreamDestroy(s));
    if (!ok) {
        printf("{\"doorbell\": \"%s\", \"ok\": false}\n", name);
        return;
    }
    std::sort(rt.begin(), rt.end());
    std::sort(wr.begin(), wr.end());
    printf("{\"doorbell\": \"%s\", \"payload\": %d, \"iters\": %d, \"round_trip_us_p50\": %.2f, "
           "\"round_trip_us_p99\": %.2f, \"host_write_us_p50\": %.3f, \"ok\": true}\n",
           name, PAYLOAD, iters, rt[iters / 2] * 1e-3, rt[iters * 99 / 100] * 1e-3, wr[iters / 2] * 1e-3);
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 5000;
    uint32_t *ack;
    CHECK(hipHostMalloc((void **)&ack, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    Req *hreq;
    CHECK(hipHostMalloc((void **)&hreq, sizeof(Req), hipHostMallocMapped | hipHostMallocCoherent));
    memset(hreq, 0, sizeof(Req));
    run("host", hreq, hreq, ack, iters);
    run("host", hreq, hreq, ack, iters);
    const struct { const char *name; unsigned flags; } kinds[] = {
        {"vram_finegrained", hipDeviceMallocFinegrained}, {"vram_uncached", hipDeviceMallocUncached}};
    for (auto k : kinds) {
        Req *dreq = nullptr;
        if (hipExtMallocWithFlags((void **)&dreq, sizeof(Req), k.flags) != hipSuccess) {
            printf("{\"doorbell\": \"%s\", \"alloc\": false}\n", k.name);
            continue;
        }
        CHECK(hipMemset(dreq, 0, sizeof(Req)));
        CHECK(hipDeviceSynchronize());
        if (!cpu_can_touch(&dreq->seq)) {
            printf("{\"doorbell\": \"%s\", \"cpu_access\": false}\n", k.name);
            CHECK(hipFree(dreq));
            continue;
        }
        run(k.name, dreq, dreq, ack, iters);
        run(k.name, dreq, dreq, ack, iters);
        CHECK(hipFree(dreq));
    }
    CHECK(hipHostFree(hreq));
    CHECK(hipHostFree(ack));
    return 0;
}
