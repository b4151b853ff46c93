/*
 * launch.h — the kernel launchers of each translation unit, as seen by the
 * C-ABI layer (aead_api.hip).  launch_chacha.hip holds the ChaChaPoly
 * kernels, launch_aes.hip the AES-GCM ones; they compile in parallel.
 * Internal (hidden visibility); the public ABI is include/noise_aead_hip.h.
 */
#pragma once
#include "noise_aead_hip.h"
#include "aead_kernels.h"
#include <hip/hip_runtime.h>

#define NA_HIDDEN __attribute__((visibility("hidden")))

namespace na {

inline int hip_rc(hipError_t e) { return e == hipSuccess ? NOISE_ERROR_NONE : NOISE_ERROR_SYSTEM; }

/* ---- worker.hip: before a batch launch of this many workgroups (asks the
   device's resident single-call workers to leave when it fills every CU) */
NA_HIDDEN void worker_park_for_batch(uint32_t workgroups);

/* ---- launch_chacha.hip.  k = lanes per record; every call returns a
   NOISE_ERROR_* code (NOISE_ERROR_INVALID_PARAM for an unsupported k). */
/* uniform batch; fast = FAST layout, ukey = every wave's records share one
   state; a.vf selects the two-pass open */
NA_HIDDEN int chacha_uniform(const UniformArgs &a, int k, bool open, bool fast, bool ukey, hipStream_t s);
/* one launch sealing job a and opening job b (k = 4 or 8, FAST layouts) */
NA_HIDDEN int chacha_duplex(const UniformArgs &a, const UniformArgs &b, int k, bool ukey, hipStream_t s);
NA_HIDDEN int chacha_ragged(const RaggedArgs &a, int k, bool open, bool fast, hipStream_t s);
/* FAST ragged batch through the segmented one-lane kernel (per-launch plan,
   chachapoly_seg.hip) */
NA_HIDDEN int chacha_ragged_seg(const RaggedArgs &a, bool open, hipStream_t s);

/* ---- launch_aes.hip */
/* S-box / T-table of the current device, built once (private stream) */
NA_HIDDEN hipError_t ensure_aes_tables();
NA_HIDDEN int aes_prepare(const uint8_t *raw_keys, uint32_t n_states, void *ctx, hipStream_t s);
/* staged = FAST layout with one state per GCM_WG_RECS records */
NA_HIDDEN int aes_uniform(const UniformArgs &a, bool open, bool ct, bool staged, hipStream_t s);
NA_HIDDEN int aes_duplex(const UniformArgs &a, const UniformArgs &b, bool ct, hipStream_t s);
/* wide = one record per workgroup (small batches, automatic lanes) */
NA_HIDDEN int aes_ragged(const RaggedArgs &a, bool open, bool fast, bool ct, bool wide, hipStream_t s);

} // namespace na
