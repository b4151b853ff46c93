/*
 * pad.hip — noise_randstate_pad for a uniform batch of payloads (SURVEY.md
 * §8f rank 4), so that records padded to one length (examples/echo
 * echo-client -g, echo-client.c:400-410) feed the uniform seal path.
 *
 * Semantics: n calls noise_randstate_pad(state, payload_i, orig_i, padded,
 * mode) in record order (randstate.c:348-375).
 *  - ZERO: bytes [orig_i, padded) of every payload zeroed — independent per
 *    record, one workgroup each.
 *  - RANDOM (and unknown modes): noise_randstate_generate (:263-316) from a
 *    snapshot of the RandState generator — ChaCha key, 64-bit block counter,
 *    64-bit IV, reseed budget.  Each request takes 64-byte key-stream chunks
 *    (a partial last chunk spends a whole block), rekeys before chunk 16 and
 *    every 17 chunks after (NOISE_RAND_REKEY_COUNT), and rekeys once more at
 *    its end (:230-247: the next 40 key-stream bytes become key and IV,
 *    counter 0).  Every record's key depends on the previous record's last
 *    rekey, so one wave walks the records in order; its lanes compute a
 *    segment's (up to 17) blocks and the rekey block at once.  A request the
 *    reference could serve only after reseeding from OS entropy stops the
 *    walk there (*done = records padded) with the snapshot as of that point.
 */
#include "aead_device.h"

namespace na {

struct RandSnap {
    uint32_t key[8];
    uint64_t counter;
    uint64_t iv;
    uint64_t left;
};

constexpr uint32_t RAND_REKEY_COUNT = 16; /* randstate.c:63 */

__global__ __launch_bounds__(256) void pad_zero(uint8_t *p, uint64_t stride, const uint32_t *orig,
                                                uint32_t padded, uint32_t n, uint32_t *done)
{
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        const uint32_t o = orig[r];
        if (padded <= o) continue;
        uint8_t *q = p + (size_t)r * stride;
        for (uint32_t b = o + threadIdx.x; b < padded; b += 256) q[b] = 0;
    }
    if (done && blockIdx.x == 0 && threadIdx.x == 0) *done = n;
}

/* bytes [0, nb) of a 64-byte key-stream block, any alignment */
NA_DEV void put_block(uint8_t *q, uint32_t nb, const uint32_t x[16])
{
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t at = 4 * i;
        if (at < nb) st_bytes(q + at, x[i], nb - at >= 4 ? 4u : nb - at);
    }
}

__global__ __launch_bounds__(64) void pad_random(RandSnap *snap, uint8_t *p, uint64_t stride,
                                                 const uint32_t *orig, uint32_t padded, uint32_t n,
                                                 uint32_t *done)
{
    const uint32_t lane = threadIdx.x;
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = snap->key[i];
    uint64_t ctr = snap->counter, iv = snap->iv, left = snap->left;
    uint32_t r = 0;
    for (; r < n; ++r) {
        const uint32_t o = orig[r];
        if (padded <= o) continue; /* no padding: the state is not touched */
        const uint32_t len = padded - o;
        const uint64_t chunks = (len + 63) / 64;
        if (left < len || left < 64 * chunks) break; /* would reseed from the OS */
        left -= 64 * chunks;
        uint8_t *out = p + (size_t)r * stride + o;
        uint64_t c0 = 0;                    /* first chunk of the segment */
        uint64_t seg = RAND_REKEY_COUNT;    /* chunks before the next rekey */
        for (;;) {
            const uint32_t cnt = (uint32_t)min(seg, chunks - c0);
            /* lanes < cnt: the segment's chunks; lane cnt (and above, the
               same block): the rekey block after them */
            const uint32_t l = lane < cnt ? lane : cnt;
            const uint64_t cc = ctr + l;
            uint32_t x[16];
            chacha20_block(key, (uint32_t)cc, (uint32_t)(cc >> 32), (uint32_t)iv,
                           (uint32_t)(iv >> 32), x);
            if (lane < cnt) {
                const uint64_t at = 64 * (c0 + lane);
                put_block(out + at, (uint32_t)min((uint64_t)64, len - at), x);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) key[i] = (uint32_t)__shfl((int)x[i], (int)cnt, 64);
            iv = (uint64_t)(uint32_t)__shfl((int)x[8], (int)cnt, 64) |
                 ((uint64_t)(uint32_t)__shfl((int)x[9], (int)cnt, 64) << 32);
            ctr = 0;
            c0 += cnt;
            if (c0 == chunks) break;
            seg = RAND_REKEY_COUNT + 1;
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) snap->key[i] = key[i];
        snap->counter = ctr;
        snap->iv = iv;
        snap->left = left;
        if (done) *done = r;
    }
}

} // namespace na
