/*
 * launch_aes.hip — launchers of the AES-GCM kernels (aesgcm.hip): the
 * per-device table build, key preparation, and the choice of kernel and
 * launch shape for uniform, duplex and ragged jobs.  Called by the C-ABI
 * layer (aead_api.hip) through launch.h.
 */
#include "launch.h"
#include "aesgcm.hip"
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace na {
namespace {

constexpr int kMaxDevices = 64;
std::mutex g_tab_mu[kMaxDevices];
bool g_tab_ready[kMaxDevices];

} // namespace

/* S-box / T-table are generated on each device once (aesgcm.hip), on a
   private stream — never the caller's, which may be capturing a graph —
   and waited for.  Only success is remembered: after a failure the next AES
   call on that device tries again. */
hipError_t ensure_aes_tables()
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    if (__atomic_load_n(&g_tab_ready[dev], __ATOMIC_ACQUIRE)) return hipSuccess;
    std::lock_guard<std::mutex> lk(g_tab_mu[dev]);
    if (g_tab_ready[dev]) return hipSuccess;
    hipStream_t s = nullptr;
    e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(aes_tables_init, dim3(1), dim3(256), 0, s);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    if (e == hipSuccess) __atomic_store_n(&g_tab_ready[dev], true, __ATOMIC_RELEASE);
    return e;
}

namespace {

template <typename Args>
using KernelFn = void (*)(Args);

template <bool CT, int WG, int R, int KL = GCM_LANES>
KernelFn<RaggedArgs> gcm_ragged_pick(bool open, bool fast)
{
    return open ? (fast ? gcm_ragged_staged<true, true, WG, CT, R, KL>
                        : gcm_ragged_staged<true, false, WG, CT, R, KL>)
                : (fast ? gcm_ragged_staged<false, true, WG, CT, R, KL>
                        : gcm_ragged_staged<false, false, WG, CT, R, KL>);
}

/* Ragged AES-GCM launch shape: threads per workgroup, records per group
   and lanes per record (gcm_ragged_staged).  A workgroup owns its CU (the
   LDS T-tables), so its time is its longest wave's; pairing a long with a
   short record per group (R = 2) evens the waves out: +21 % records per
   CU-second on C5's 64 B-16 KiB mix (profiles/r02/c5_gcm_shape_ab.jsonl).
   From 131072 records on every CU gets a 512-record window of 4-lane groups;
   from 65536 on, 256-record windows of 8-lane groups (KL = 8, H^8 Horner)
   keep all CUs busy with the same pairing (4-lane pairs there would idle
   half the CUs: 1.55 vs 0.94 ms); smaller batches take 256-thread
   workgroups over 64-record windows.  NOISE_AEAD_GCM_SHAPE=w1024r1 |
   w1024r2 | w1024r2k8 forces a shape (A/B runs). */
struct GcmShape { int wg, r, kl; };

GcmShape gcm_ragged_shape(uint32_t n)
{
    static const int forced = [] {
        const char *e = getenv("NOISE_AEAD_GCM_SHAPE");
        if (!e) return 0;
        if (!strcmp(e, "w1024r1")) return 1;
        if (!strcmp(e, "w1024r2")) return 2;
        if (!strcmp(e, "w1024r2k8")) return 3;
        return 0;
    }();
    if (forced == 1) return {1024, 1, 4};
    if (forced == 2) return {1024, 2, 4};
    if (forced == 3) return {1024, 2, 8};
    if (n >= 256u * 2 * GCM_WG_RECS) return {1024, 2, 4};
    if (n >= 256u * GCM_WG_RECS) return {1024, 2, 8};
    return {256, 1, 4};
}

template <bool CT>
KernelFn<RaggedArgs> gcm_ragged_fn(bool open, bool fast, GcmShape sh)
{
    if (sh.kl == 8) return gcm_ragged_pick<CT, 1024, 2, 8>(open, fast);
    if (sh.wg == 1024 && sh.r == 2) return gcm_ragged_pick<CT, 1024, 2>(open, fast);
    if (sh.wg == 1024) return gcm_ragged_pick<CT, 1024, 1>(open, fast);
    return gcm_ragged_pick<CT, 256, 1>(open, fast);
}

} // namespace

int aes_prepare(const uint8_t *raw_keys, uint32_t n_states, void *ctx, hipStream_t s)
{
    hipLaunchKernelGGL(gcm_prepare, dim3(n_states), dim3(256), 0, s, raw_keys, (AesCtx *)ctx, n_states);
    return hip_rc(hipGetLastError());
}


int aes_uniform(const UniformArgs &a, bool open, bool ct, bool staged, hipStream_t s)
{
    if (a.n_records == 0) return NOISE_ERROR_NONE;
    if (staged) { /* one state per 256-record workgroup + FAST layout */
        const uint32_t blocks = (a.n_records + GCM_WG_RECS - 1) / GCM_WG_RECS;
        worker_park_for_batch(blocks);
        hipLaunchKernelGGL(ct ? (open ? gcm_staged<true, true> : gcm_staged<false, true>)
                              : (open ? gcm_staged<true, false> : gcm_staged<false, false>),
                           dim3(blocks), dim3(GCM_WG), 0, s, a);
        return hip_rc(hipGetLastError());
    }
    const uint32_t blocks = (uint32_t)(((uint64_t)a.n_records * GCM_LANES + 255) / 256);
    worker_park_for_batch(blocks);
    hipLaunchKernelGGL(ct ? (open ? gcm_uniform<true, true> : gcm_uniform<false, true>)
                          : (open ? gcm_uniform<true, false> : gcm_uniform<false, false>),
                       dim3(blocks), dim3(256), 0, s, a);
    return hip_rc(hipGetLastError());
}

/* The fused duplex kernel (one LDS fill, seal then open per workgroup) by
   default: C3 +0.7-0.9 % in three interleaved rounds
   (profiles/r03/gcm_fused_ab.jsonl); NOISE_AEAD_GCM_DUPLEX=staged selects
   gcm_duplex_staged (A/B runs). */
static bool gcm_duplex_fused_on()
{
    static const bool v = [] {
        const char *e = getenv("NOISE_AEAD_GCM_DUPLEX");
        return !(e && !strcmp(e, "staged"));
    }();
    return v;
}

int aes_duplex(const UniformArgs &a, const UniformArgs &b, bool ct, hipStream_t s)
{
    const uint32_t sb = (a.n_records + GCM_WG_RECS - 1) / GCM_WG_RECS;
    const uint32_t ob = (b.n_records + GCM_WG_RECS - 1) / GCM_WG_RECS;
    worker_park_for_batch(sb > ob ? sb : ob);
    if (gcm_duplex_fused_on()) {
        hipLaunchKernelGGL(ct ? gcm_duplex_fused<true> : gcm_duplex_fused<false>,
                           dim3(sb > ob ? sb : ob), dim3(GCM_WG), 0, s, a, b, sb, ob);
        return hip_rc(hipGetLastError());
    }
    hipLaunchKernelGGL(ct ? gcm_duplex_staged<true> : gcm_duplex_staged<false>, dim3(sb + ob),
                       dim3(GCM_WG), 0, s, a, b, sb, ob);
    return hip_rc(hipGetLastError());
}

int aes_ragged(const RaggedArgs &a, bool open, bool fast, bool ct, bool wide, hipStream_t s)
{
    if (a.n_records == 0) return NOISE_ERROR_NONE;
    if (wide) { /* small batch: a workgroup per record (latency, not throughput) */
        hipLaunchKernelGGL(ct ? (open ? gcm_wide<true, true> : gcm_wide<false, true>)
                              : (open ? gcm_wide<true, false> : gcm_wide<false, false>),
                           dim3(a.n_records), dim3(256), 0, s, a);
        return hip_rc(hipGetLastError());
    }
    /* LDS-staged kernel: 1024-thread workgroups over 256-record windows; a
       batch too small to give every CU one of those uses 256-thread
       workgroups over 64-record windows instead (4x the workgroups) */
    const GcmShape sh = gcm_ragged_shape(a.n_records);
    const uint32_t per = (uint32_t)(sh.wg / sh.kl * sh.r); /* records per window */
    const uint32_t blocks = (a.n_records + per - 1) / per;
    KernelFn<RaggedArgs> fn = ct ? gcm_ragged_fn<true>(open, fast, sh) : gcm_ragged_fn<false>(open, fast, sh);
    worker_park_for_batch(blocks);
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(sh.wg), 0, s, a);
    return hip_rc(hipGetLastError());
}

} // namespace na
