/*
 * aead_kernels.h — kernel argument blocks shared by the HIP kernels and the
 * C-ABI launch layer (aead_api.hip).  Internal; the public ABI is
 * include/noise_aead_hip.h.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace na {

/* Uniform batch: record i belongs to state i / rps and uses nonce
   nonce_base[state] + i % rps (the nonce a run of single
   noise_cipherstate_encrypt() calls would use, cipherstate.c:325-326). */
struct UniformArgs {
    const uint8_t *keys;        /* per-state key context (ChaCha: 32 B raw key,
                                   AESGCM: AesCtx from the prepare kernel) */
    const uint64_t *nonce_base; /* per state */
    const uint8_t *in;
    uint8_t *out;
    const uint8_t *ad;
    uint8_t *status;            /* open: 0 ok / 1 MAC failure, per record */
    uint64_t in_stride, out_stride, ad_stride;
    uint32_t rps, n_records, len, ad_len;
    uint32_t balance;           /* the whole batch is one resident generation
                                   of waves (aead_device.h prio_by_progress) */
    uint32_t vf;                /* open: NOISE_AEAD_FLAG_VERIFY_FIRST — authenticate
                                   first, decrypt only verified records, write
                                   nothing (not even zeros) for a rejected one */
};

/* Ragged batch: one descriptor per record (variable lengths, states, AD).
   Layout identical to the public NoiseAeadRecord (include/noise_aead_hip.h). */
struct RecDesc {
    uint64_t in_off;   /* byte offset of the input record in `in`  */
    uint64_t out_off;  /* byte offset of the output record in `out` */
    uint64_t nonce;    /* the record's nonce (CipherState n at that call) */
    uint64_t ctx_off;  /* byte offset of the key context from `keys` */
    uint64_t ad_off;   /* byte offset of the AD in `ad` */
    uint32_t len;      /* plaintext / ciphertext length excluding the tag */
    uint32_t ad_len;
};

struct RaggedArgs {
    const uint8_t *keys;
    const RecDesc *recs;
    const uint8_t *in;
    uint8_t *out;
    const uint8_t *ad;
    uint8_t *status;   /* open: per record 0 ok / 1 MAC failure / 2 bad length;
                          seal (optional): 0 / 2 */
    uint32_t n_records;
    uint32_t vf;       /* as UniformArgs::vf */
};

/* A ragged descriptor's record longer than NOISE_MAX_PAYLOAD_LEN - 16 bytes
   (constants.h:151; cipherstate.c:307,313,382 refuse it) is not processed:
   nothing is written and status (when given) is 2.  The AES-GCM kernels
   also rely on it: their CTR counter stays below 2^16. */
constexpr uint32_t MAX_RECORD_LEN = 65535 - 16;
constexpr uint8_t STATUS_BAD_LENGTH = 2;

/* Called by every lane of record `rec` (the group leaves together). */
__device__ __forceinline__ bool reject_len(const RaggedArgs &a, uint32_t rec, uint32_t len,
                                           bool writer)
{
    if (len <= MAX_RECORD_LEN) return false;
    if (writer && a.status) a.status[rec] = STATUS_BAD_LENGTH;
    return true;
}

/* Length-balanced record order for a workgroup of a ragged batch.  A wave is
   as slow as its longest record, so the NREC records of the workgroup's
   window [base, base + NREC) are ranked by length (bitonic sort of
   len << 8 | index in LDS, every thread of the workgroup taking part) and
   record group g takes the g-th: the records sharing a wave then have
   near-equal lengths.  The result is a permutation of the window, so every
   record is still processed exactly once.  Returns the record of group g, or
   UINT32_MAX past the batch end.  Must be reached by the whole workgroup. */
template <int NREC>
__device__ __forceinline__ uint32_t window_rec(const RecDesc *recs, uint32_t n, uint32_t base,
                                               uint32_t g, uint32_t *keys)
{
    static_assert(NREC >= 2 && NREC <= 512 && (NREC & (NREC - 1)) == 0, "window");
    constexpr uint32_t IB = NREC <= 256 ? 8 : 9; /* index bits below the length */
    const uint32_t t = threadIdx.x, nt = blockDim.x;
    for (uint32_t i = t; i < (uint32_t)NREC; i += nt) {
        const uint32_t rec = base + i;
        keys[i] = rec < n ? (min(recs[rec].len, 65535u) << IB) | i : 0xFFFFFFFFu;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= (uint32_t)NREC; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < (uint32_t)NREC; i += nt) {
                const uint32_t p = i ^ j;
                if (p > i) {
                    const uint32_t x = keys[i], y = keys[p];
                    if ((x > y) == ((i & k) == 0)) {
                        keys[i] = y;
                        keys[p] = x;
                    }
                }
            }
            __syncthreads();
        }
    const uint32_t key = keys[g < (uint32_t)NREC ? g : 0];
    return (g < (uint32_t)NREC && key != 0xFFFFFFFFu) ? base + (key & ((1u << IB) - 1u)) : 0xFFFFFFFFu;
}

/* The rank in the sorted window of the p-th record of group g (of NG groups)
   when each group runs R records one after another: ranks g, 2NG-1-g, 2NG+g,
   ... — long records paired with short ones, so every group (and wave) of a
   workgroup carries about the same number of blocks, while the groups of one
   wave still see near-equal lengths at each p. */
template <int NG>
__device__ __forceinline__ uint32_t snake_rank(uint32_t g, int p)
{
    return (p & 1) ? (uint32_t)(p + 1) * NG - 1u - g : (uint32_t)p * NG + g;
}

/* AES-GCM per-state device context (prepared once per key). */
constexpr int GCM_LANES = 4;                    /* lanes per record */
constexpr int GCM_WG = 1024;                    /* threads per staged workgroup */
constexpr int GCM_WG_RECS = GCM_WG / GCM_LANES; /* records per staged workgroup */
constexpr int GHASH_TAB_ENTRIES = 32 * 16;      /* 4-bit positional table */
struct AesCtx {
    uint32_t rk[60];                            /* AES-256 round keys, BE words */
    uint32_t h[4];                              /* H = E_K(0^128), LE words */
    uint32_t pad_[12];
    /* tab[m]: multiply-by-H^(m+1) tables, m = 0..3 (H^4 is the Horner step) */
    uint32_t tab[GCM_LANES][GHASH_TAB_ENTRIES][4];
    /* hn[m]: H^(m+1) in the natural polynomial domain (constant-time GHASH) */
    uint32_t hn[GCM_LANES][4];
    /* H^8: the Horner step of 8-lane record groups (gcm_ragged_staged KL = 8),
       as a multiply table and in the natural domain */
    uint32_t tab8[GHASH_TAB_ENTRIES][4];
    uint32_t hn8[4];
};

} // namespace na
