/*
 * launch_chacha.hip — launchers of the ChaChaPoly kernels (chachapoly.hip):
 * picks the instantiation for the lane count, layout, key sharing and open
 * order of a job and launches it.  Called by the C-ABI layer (aead_api.hip)
 * through launch.h.
 */
#include "launch.h"
#include "chachapoly.hip"
#include "chachapoly_seg.hip"
#include <atomic>
#include <cstdlib>
#include <cstring>

namespace na {
namespace {

template <typename Args>
using KernelFn = void (*)(Args);

template <typename Args>
int launch(KernelFn<Args> fn, uint32_t n_records, int lanes, const Args &a, hipStream_t s)
{
    if (n_records == 0) return NOISE_ERROR_NONE;
    const uint64_t threads = (uint64_t)n_records * lanes;
    const uint32_t blocks = (uint32_t)((threads + 255) / 256);
    worker_park_for_batch(blocks);
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, s, a);
    return hip_rc(hipGetLastError());
}

template <int K>
KernelFn<UniformArgs> chacha_staged_fn(bool open, bool ukey)
{
    if (ukey) return open ? chachapoly_open_staged<K, true> : chachapoly_seal_staged<K, true>;
    return open ? chachapoly_open_staged<K, false> : chachapoly_seal_staged<K, false>;
}

/* vf: a VERIFY_FIRST open takes an AUTH + DEC kernel — the one-lane
   open_solo_staged, the 4/8-lane open_il_staged_vf (FAST layouts) or the
   two-pass chachapoly_open_uniform — never the one-pass staged kernels */
template <bool FAST>
KernelFn<UniformArgs> chacha_uniform_fn_t(int k, bool open, bool ukey, bool vf, bool runs)
{
    switch (k) {
    case 1:
        /* one lane per record, LDS-staged (seal_solo_staged); runs: the key
           stream issued in runs once the launch holds two waves per SIMD */
        if (FAST) {
            if (runs) {
                if (ukey) return open ? chachapoly_open_solo<true, true> : chachapoly_seal_solo<true, true>;
                return open ? chachapoly_open_solo<false, true> : chachapoly_seal_solo<false, true>;
            }
            if (ukey) return open ? chachapoly_open_solo<true, false> : chachapoly_seal_solo<true, false>;
            return open ? chachapoly_open_solo<false, false> : chachapoly_seal_solo<false, false>;
        }
        return open ? chachapoly_open_uniform<1, FAST> : chachapoly_seal_uniform<1, FAST>;
    case 2: return open ? chachapoly_open_uniform<2, FAST> : chachapoly_seal_uniform<2, FAST>;
    case 4:
        if (FAST && open && vf) return ukey ? chachapoly_open_staged_vf<4, true> : chachapoly_open_staged_vf<4, false>;
        if (FAST) return chacha_staged_fn<4>(open, ukey);
        return open ? chachapoly_open_uniform<4, FAST> : chachapoly_seal_uniform<4, FAST>;
    case 8:
        if (FAST && open && vf) return ukey ? chachapoly_open_staged_vf<8, true> : chachapoly_open_staged_vf<8, false>;
        if (FAST) return chacha_staged_fn<8>(open, ukey);
        return open ? chachapoly_open_uniform<8, FAST> : chachapoly_seal_uniform<8, FAST>;
    case 16: return open ? chachapoly_open_uniform<16, FAST> : chachapoly_seal_uniform<16, FAST>;
    case 32: return open ? chachapoly_open_uniform<32, FAST> : chachapoly_seal_uniform<32, FAST>;
    case 64: return open ? chachapoly_open_uniform<64, FAST> : chachapoly_seal_uniform<64, FAST>;
    }
    return nullptr;
}

/* ukey: every wave's 64/k records share one state (see u_key_nonce) */
KernelFn<UniformArgs> chacha_uniform_fn(int k, bool open, bool fast, bool ukey, bool vf, bool runs)
{
    return fast ? chacha_uniform_fn_t<true>(k, open, ukey, vf, runs)
                : chacha_uniform_fn_t<false>(k, open, ukey, vf, runs);
}

/* VF: the FAST opens' two-pass (verify-first) instantiation; the generic
   layouts' opens are two-pass already */
template <bool FAST, bool VF>
KernelFn<RaggedArgs> chacha_ragged_fn_t(int k, bool open)
{
    switch (k) {
    case 1: return open ? chachapoly_open_ragged<1, FAST> : chachapoly_seal_ragged<1, FAST>;
    case 2: return open ? chachapoly_open_ragged<2, FAST> : chachapoly_seal_ragged<2, FAST>;
    case 4: return open ? chachapoly_open_ragged<4, FAST, VF> : chachapoly_seal_ragged<4, FAST>;
    case 8: return open ? chachapoly_open_ragged<8, FAST, VF> : chachapoly_seal_ragged<8, FAST>;
    case 16: return open ? chachapoly_open_ragged<16, FAST, VF> : chachapoly_seal_ragged<16, FAST>;
    case 32: return open ? chachapoly_open_ragged<32, FAST, VF> : chachapoly_seal_ragged<32, FAST>;
    case 64: return open ? chachapoly_open_ragged<64, FAST, VF> : chachapoly_seal_ragged<64, FAST>;
    }
    return nullptr;
}

KernelFn<RaggedArgs> chacha_ragged_fn(int k, bool open, bool fast, bool vf)
{
    if (!fast) return chacha_ragged_fn_t<false, false>(k, open);
    return vf ? chacha_ragged_fn_t<true, true>(k, open) : chacha_ragged_fn_t<true, false>(k, open);
}

/* Resident workgroups of a kernel on this device (CUs x occupancy). */
template <typename F>
uint32_t resident_blocks(F fn)
{
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 256, 0) != hipSuccess || per < 1)
        return 0;
    return (uint32_t)(cus * per);
}


} // namespace

/* the current device's CU count, cached per device (0: unknown) */
static uint32_t duplex_run_chunk_cus()
{
    constexpr int MAX_DEV = 64;
    static std::atomic<uint32_t> cache[MAX_DEV];
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return 0;
    uint32_t v = cache[dev].load(std::memory_order_relaxed);
    if (!v && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
        v = (uint32_t)cus;
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

int chacha_uniform(const UniformArgs &a, int k, bool open, bool fast, bool ukey, hipStream_t s)
{
    if (k == 2 && fast) {
        /* two segments per record, LDS-staged (chachapoly_seg.hip) */
        const bool uk = a.rps % 32 == 0;
        KernelFn<UniformArgs> fn = open ? (uk ? chachapoly_seg2_uniform<true, true> : chachapoly_seg2_uniform<true, false>)
                                        : (uk ? chachapoly_seg2_uniform<false, true> : chachapoly_seg2_uniform<false, false>);
        return launch(fn, a.n_records, 2, a, s);
    }
    /* one lane per record: runs once the launch is two waves per SIMD
       (64 records per wave, four SIMDs per CU) */
    const uint32_t cus = duplex_run_chunk_cus();
    const bool runs = cus && (uint64_t)a.n_records >= 2ull * 4 * 64 * cus;
    KernelFn<UniformArgs> fn = chacha_uniform_fn(k, open, fast, ukey, a.vf != 0, runs);
    if (!fn) return NOISE_ERROR_INVALID_PARAM;
    if (k == 1 && fast) {
        /* one-lane kernels: balance = the launch is one generation (at most
           two 64-record waves per SIMD; chachapoly.hip solo_blocks2) */
        UniformArgs b = a;
        b.balance = cus && (uint64_t)a.n_records <= 2ull * 4 * 64 * cus;
        return launch(fn, a.n_records, k, b, s);
    }
    return launch(fn, a.n_records, k, a, s);
}

/* chachapoly_duplex_solo's run length: the device's CU count (one seal and
   one open block per CU); NOISE_AEAD_DUPLEX_RUNS=0 alternates block by
   block (A/B runs) */
static uint32_t duplex_run_chunk()
{
    static const uint32_t c = [] {
        const char *e = getenv("NOISE_AEAD_DUPLEX_RUNS");
        if (e && e[0] == '0') return 0u;
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return 0u;
        return (uint32_t)cus;
    }();
    return c;
}

int chacha_duplex(const UniformArgs &a, const UniformArgs &b, int k, bool ukey, hipStream_t s)
{
    const uint32_t sb = (uint32_t)(((uint64_t)a.n_records * k + 255) / 256);
    const uint32_t ob = (uint32_t)(((uint64_t)b.n_records * k + 255) / 256);
    if (k == 1) {
        /* balance: the launch is one generation (two waves per SIMD at most,
           256-thread blocks of four waves; chachapoly.hip solo_blocks2) */
        const uint32_t cus = duplex_run_chunk_cus();
        UniformArgs a1 = a, b1 = b;
        a1.balance = b1.balance = cus && (uint64_t)(sb + ob) <= 2ull * cus;
        worker_park_for_batch(sb + ob);
        hipLaunchKernelGGL(ukey ? chachapoly_duplex_solo<true> : chachapoly_duplex_solo<false>, dim3(sb + ob),
                           dim3(256), 0, s, a1, b1, sb, ob, duplex_run_chunk());
        return hip_rc(hipGetLastError());
    }
    void (*fn)(UniformArgs, UniformArgs, uint32_t, uint32_t);
    if (k == 4) fn = ukey ? chachapoly_duplex_staged<4, true> : chachapoly_duplex_staged<4, false>;
    else if (k == 8) fn = ukey ? chachapoly_duplex_staged<8, true> : chachapoly_duplex_staged<8, false>;
    else return NOISE_ERROR_INVALID_PARAM;
    worker_park_for_batch(sb + ob);
    hipLaunchKernelGGL(fn, dim3(sb + ob), dim3(256), 0, s, a, b, sb, ob);
    return hip_rc(hipGetLastError());
}

int chacha_ragged(const RaggedArgs &a, int k, bool open, bool fast, hipStream_t s)
{
    KernelFn<RaggedArgs> fn = chacha_ragged_fn(k, open, fast, a.vf != 0);
    if (!fn) return NOISE_ERROR_INVALID_PARAM;
    return launch(fn, a.n_records, k, a, s);
}

/* Resident workgroups of chachapoly_seg_ragged<open> on the current device,
   cached per device (a host may mix GPU models): the persistent
   grid and worker_park_for_batch take this count. */
template <typename F>
uint32_t seg_resident(bool open, F fn)
{
    constexpr int MAX_DEV = 64;
    static std::atomic<uint32_t> cache[MAX_DEV][2];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
    if (dev >= MAX_DEV) return resident_blocks(fn);
    std::atomic<uint32_t> &c = cache[dev][open ? 1 : 0];
    uint32_t v = c.load(std::memory_order_relaxed);
    if (!v) {
        v = resident_blocks(fn); /* idempotent: a racing thread stores the same value */
        c.store(v, std::memory_order_relaxed);
    }
    return v;
}

/* Ragged FAST batch through the segmented one-lane kernel: the plan (count,
   scan, place) in a stream-ordered scratch block, then the persistent
   kernel, then the scratch is freed (stream-ordered too). */
int chacha_ragged_seg(const RaggedArgs &a, bool open, hipStream_t s)
{
    if (a.n_records == 0) return NOISE_ERROR_NONE;
    const size_t bytes = SEG_MAP_OFF + (size_t)a.n_records * SEG_KMAX * sizeof(uint32_t);
    uint8_t *scratch = nullptr;
    if (hipMallocAsync((void **)&scratch, bytes, s) != hipSuccess) return NOISE_ERROR_NO_MEMORY;
    SegPlanHdr *p = (SegPlanHdr *)scratch;
#ifdef NA_SEG_DEBUG
    {
        uint64_t r[2] = {(uint64_t)(uintptr_t)scratch, (uint64_t)(uintptr_t)scratch + bytes};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_seg_arena), r, sizeof(r), 2 * sizeof(uint64_t),
                                     hipMemcpyHostToDevice, s);
    }
#endif
    uint32_t *map = (uint32_t *)(scratch + SEG_MAP_OFF);
    int rc = hip_rc(hipMemsetAsync(p, 0, sizeof(SegPlanHdr), s));
    const uint32_t pb = (a.n_records + 1023) / 1024;
    if (!rc) {
        hipLaunchKernelGGL(seg_plan_count, dim3(pb), dim3(1024), 0, s, a.recs, a.n_records, p);
        hipLaunchKernelGGL(seg_plan_scan, dim3(1), dim3(64), 0, s, p);
        hipLaunchKernelGGL(seg_plan_place, dim3(pb), dim3(1024), 0, s, a.recs, a.n_records, p, map, a.status);
        rc = hip_rc(hipGetLastError());
    }
    if (!rc) {
        auto fn = open ? chachapoly_seg_ragged<true> : chachapoly_seg_ragged<false>;
        const uint32_t res = seg_resident(open, fn);
        const uint64_t most = ((uint64_t)a.n_records * SEG_KMAX + 255) / 256; /* jobs / 4, at most */
        const uint32_t grid = (uint32_t)(res && most > res ? res : (most ? most : 1));
        if (!res) rc = NOISE_ERROR_SYSTEM;
        else {
            worker_park_for_batch(grid);
            hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, s, a, p, (const uint32_t *)map);
            rc = hip_rc(hipGetLastError());
        }
    }
    (void)hipFreeAsync(scratch, s);
    return rc;
}

} // namespace na

#ifdef NA_SEG_DEBUG
/* debug variant only: the caller's buffer range the segmented kernels may
   touch, and the accesses they skipped (address, kind << 56 | n << 40 | info) */
extern "C" int noise_aead_debug_seg_arena(uint64_t lo, uint64_t hi)
{
    uint64_t r[2] = {lo, hi};
    uint32_t z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(na::g_seg_arena), r, sizeof(r), 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(na::g_seg_nviol), &z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

extern "C" int noise_aead_debug_seg_viol(uint64_t *out, int n)
{
    uint32_t cnt = 0;
    if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(na::g_seg_nviol), sizeof(cnt), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (n > 64) n = 64;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(na::g_seg_viol), sizeof(uint64_t) * n, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return (int)cnt;
}
#endif

#ifdef NA_SEG_TL
/* debug variant only: the per-wave cycle accounts of the last persistent
   ragged launch (chachapoly_seg.hip SegTL), summed over waves into out[8];
   reset != 0 zeroes them afterwards.  Returns the waves that ran. */
extern "C" int noise_aead_debug_seg_tl(uint64_t *out, int reset)
{
    static unsigned long long h[4096][8];
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(na::g_seg_tlw), sizeof(h), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    int waves = 0;
    for (int k = 0; k < 8; ++k) out[k] = 0;
    for (int w = 0; w < 4096; ++w) {
        if (!h[w][0]) continue;
        ++waves;
        for (int k = 0; k < 8; ++k) out[k] += h[w][k];
    }
    if (reset) {
        static unsigned long long z[4096][8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(na::g_seg_tlw), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
            return -1;
    }
    return waves;
}
#endif
