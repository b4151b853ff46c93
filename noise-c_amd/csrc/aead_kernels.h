/*
 * aead_kernels.h — kernel argument blocks shared by the HIP kernels and the
 * C-ABI launch layer (aead_api.hip).  Internal; the public ABI is
 * include/noise_aead_hip.h.
 */
#pragma once
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
    uint8_t *status;
    uint32_t n_records;
};

/* AES-GCM per-state device context (prepared once per key). */
constexpr int GCM_LANES = 4;                    /* lanes per record */
constexpr int GHASH_TAB_ENTRIES = 32 * 16;      /* 4-bit positional table */
struct AesCtx {
    uint32_t rk[60];                            /* AES-256 round keys, BE words */
    uint32_t h[4];                              /* H = E_K(0^128), LE words */
    uint32_t pad_[12];
    /* tab[m]: multiply-by-H^(m+1) tables, m = 0..3 (H^4 is the Horner step) */
    uint32_t tab[GCM_LANES][GHASH_TAB_ENTRIES][4];
};

} // namespace na
