/*
 * worker.hip — the resident single-record engine of the CipherState calls.
 *
 * A per-record noise_cipherstate_encrypt/decrypt (src/protocol/cipherstate.c
 * :293-410, the call pattern of examples/echo) is one record of 1 B - 64 KiB.
 * Launching a kernel and waiting for it costs ~20 us on its own, 5x the
 * reference's whole ~4 us CPU call.  Instead, the first call on a device
 * starts ONE resident workgroup (256 threads) on a private stream; it polls
 * a request slot and serves records as they are posted.  The request (header
 * and input stream) sits in fine-grained device memory that the CPU writes
 * through the BAR where the device has a large BAR, else in pinned host
 * memory; results, status and the done word always go to pinned host memory,
 * so each side polls memory of its own and writes the other's:
 *
 *   host                                    worker (aead_worker)
 *   write AD || record || tag to data[]
 *   write op, cipher, ctx, nonce, lengths
 *   seq = k        (release, system)  --->  sees seq != last (acquire, system)
 *                                           copies AD || record into LDS,
 *                                           runs the record (the same device
 *                                           code as the ragged kernels),
 *                                           writes it back, fences,
 *   spins until done == k       <------     done = k (release, system)
 *   reads status, copies out
 *
 * The worker exits on its own after IDLE of no requests (and after at most
 * LIFETIME), or when the host sets stop; every exit path is reached by every
 * thread of the workgroup (one barrier-synchronised loop).  Before leaving it
 * sets `exiting` and looks at seq once more, so a request posted meanwhile
 * is either served or seen by the host (exiting set, done behind): the host
 * then waits for the stream and starts the worker again, which resumes at
 * the slot's `done`.
 *
 * Workers come in GROUPS: one kernel of S workgroups (request slots) on one
 * high-priority stream, so S calling threads share a hardware queue (a queue
 * runs nothing else while a resident kernel holds it).  A device runs one
 * group per high-priority queue but one (3 by default, the last left to the
 * application), S = ceil(8 / groups) slots each: 9 slots, one per calling
 * thread up to 9, each a workgroup on its own CU, claimed without waiting
 * while one is free.  A group leaves as a whole (aead_worker: the closing
 * word), for idleness only once all its slots are idle.  Batch launches that
 * fill every CU ask the resident groups to leave first
 * (worker_park_for_batch), so no batch workgroup waits for a worker's CU.
 *
 * Key material reaches the worker through the slot as well: the ChaCha key
 * itself, or for AES-GCM a pinned host copy of the state's device context
 * (made once per key).  A resident kernel never reads device memory that was
 * written after it started: another XCD's L2 would not be kept coherent with
 * its own, while host memory read after a system-scope acquire is always
 * current.
 *
 * Opens are two-pass (verify first, then decrypt): a rejected record's bytes
 * are never written back.  Records longer than WORKER_MAX_LEN, or any setup
 * failure, return NOISE_ERROR_NOT_APPLICABLE and the caller takes the
 * regular launch path.  NOISE_AEAD_WORKER=0 disables the worker.
 */
#include "launch.h"
#include "chachapoly.hip"
#define NA_NO_SETUP_KERNELS
#include "aesgcm.hip"
#include <cstddef>
#include <emmintrin.h>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <ctime>

namespace na {

constexpr uint32_t WORKER_MAX_LEN = 65535 - 16; /* whole records only */
constexpr uint32_t WORKER_MAX_AD = 256;
/* data area: ChaCha key (32 B) || AD (padded to 16) || record || tag */
constexpr uint32_t WORKER_DATA = 32 + WORKER_MAX_AD + 65536 + 64;
/* The request's input stream (key || AD padded to 16 || record || tag) is
   posted as 16-byte chunks of 12 stream bytes and the request's sequence
   number, each written with one 16-byte store: a chunk carries its own
   proof of freshness.  So the worker can read the first WORKER_SPEC chunks
   speculatively with every poll of the header (4 KiB per poll, one PCIe
   round trip for header and data together) and keep the ones stamped with
   the new number, re-reading only stale ones. */
constexpr uint32_t WCHUNK_BYTES = 12;
constexpr uint32_t WORKER_SPEC = 256; /* chunks read with every poll: one per thread */
constexpr uint32_t WORKER_HEAD = WORKER_SPEC * WCHUNK_BYTES; /* stream bytes sent as chunks */
/* the stream past the head (records over ~3 KiB) is posted raw, read after the header */
constexpr uint32_t WORKER_TAIL = WORKER_DATA - WORKER_HEAD;
static_assert(WORKER_HEAD % 16 == 0, "the raw tail lands 16-B aligned in LDS");
/* With the request in device memory the CPU's stores reach it through
   write-combining buffers, which may write a 16-byte store as two 8-byte
   pieces: there every 8-byte half carries the number, {4 stream bytes, seq}
   (header chunks {seq, field, seq, field}), so a chunk is 8 stream bytes. */
constexpr uint32_t VCHUNK_BYTES = 8;
constexpr uint32_t VWORKER_HEAD = WORKER_SPEC * VCHUNK_BYTES;
constexpr uint32_t VWORKER_TAIL = WORKER_DATA - VWORKER_HEAD;
/* AES-GCM contexts the worker keeps in LDS (an echo session uses two) */
constexpr int WORKER_CTX_SLOTS = 2;
constexpr uint32_t WORKER_CTX_BYTES = sizeof(AesCtx); /* rk, H, the H^1..H^4 and H^8 tables */

/* The request slot (host pinned, fine-grained).  The request header is four
   16-byte chunks, each starting with the request's sequence number; the host
   writes each chunk with one 16-byte store after the data area, and the
   worker takes the header only when all four chunks carry the same new
   number — one read round trip, no torn header.  The worker's words sit on
   their own 128-B line. */
struct alignas(128) WorkerSlot {
    /* host -> worker */
    uint32_t c0[4];    /* seq, op | ct << 8, len, ad_len */
    uint32_t c1[4];    /* seq, nonce lo, nonce hi, cipher */
    uint32_t c2[4];    /* seq, ctx lo, ctx hi, stop */
    uint32_t c3[4];    /* seq, ctx generation, 0, 0 */
    /* stop (word 0): its own chunk, written only by park / stop / launch —
       never by a request's header (a header written after a
       park used to carry stop = 0 and cancel it) */
    uint32_t c4[4];
    uint8_t pad0[128 - 80];
    /* worker -> host */
    uint64_t done;     /* last request completed */
    uint32_t status;   /* 0 ok, 1 MAC failure, 2 input never arrived */
    uint32_t exiting;  /* the worker is leaving (or has left) */
    uint32_t stamps[8]; /* debug: s_memrealtime (10 ns) of the last request's phases */
    uint32_t fstamps[8]; /* debug: s_memtime (cycles) through the latency-first path */
    uint32_t leave[4];   /* debug: the last leave's born, now (10 ns ticks, low words), lifetime, gen */
    uint8_t pad1[128 - 96];
};
static_assert(sizeof(WorkerSlot) == 256, "slot layout");

#define NA_SYS_LOAD(p) __hip_atomic_load((p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
#define NA_SYS_STORE(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM)

/* ---------------------------------------------- latency-first ChaChaPoly
 *
 * One record on the whole workgroup, built for the depth of its dependency
 * chains rather than its instruction count (a lone wave issues about one
 * instruction per 4.7 cycles, so depth and count both cost time):
 *  - ChaCha20 four lanes per block (quad q = block q, lane c = column c:
 *    words c, 4+c, 8+c, 12+c), the diagonal rounds by quad DPP rotations of
 *    rows b, c, d: ~330 instructions per lane instead of ~1000;
 *  - Poly1305 one 16-byte block per lane (AD blocks, CT blocks, the length
 *    block: n of them), right-justified in N = 2^ceil(log2 n) lanes, and the
 *    polynomial sum_i b_i r^(n-i) as a left-aligned tree: level L sets
 *    v_j = v_j r^L + v_{j+L} for j = 0 mod 2L (in-wave shuffles below 64,
 *    LDS for 64 and 128), then * r: log2(n) multiplies deep;
 *  - open verifies first and writes plaintext only on a match.
 * Records of up to WFAST_BLOCKS - 1 units with n <= 256 take it
 * (worker_fast_fits), longer ones worker_chacha_multi; the result equals
 * seal_il / open_il's bit for bit (the same Poly1305 value:
 * sum_i b_i r^(n-i+1) mod 2^130-5 + s). */
constexpr uint32_t WFAST_BLOCKS = 64; /* ChaCha blocks: 4 lanes each on 256 threads */

NA_DEV bool worker_fast_fits(uint32_t len, uint32_t ad_len)
{
    const uint32_t blocks = (len + 63) / 64 + 1;
    const uint32_t n = (ad_len + 15) / 16 + (len + 15) / 16 + 1;
    return blocks <= WFAST_BLOCKS && n <= 256;
}

template <int CTRL>
NA_DEV uint32_t quad_perm(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false); }

/* quad_perm controls: lane i of a quad reads lane perm[i] */
constexpr int QP_NEXT1 = 0x39; /* [1,2,3,0] */
constexpr int QP_NEXT2 = 0x4e; /* [2,3,0,1] */
constexpr int QP_NEXT3 = 0x93; /* [3,0,1,2] */

/* ChaCha20 block `ctr` on the four lanes of a quad; lane c returns words
   c, 4+c, 8+c, 12+c of the key stream (chacha.c:74-133 layout). */
NA_DEV void chacha_quad(const uint32_t key[8], uint32_t ctr, uint32_t n_lo, uint32_t n_hi, int c,
                        uint32_t &oa, uint32_t &ob, uint32_t &oc, uint32_t &od)
{
    const uint32_t a0 = c == 0 ? 0x61707865u : c == 1 ? 0x3320646eu : c == 2 ? 0x79622d32u : 0x6b206574u;
    const uint32_t b0 = c == 0 ? key[0] : c == 1 ? key[1] : c == 2 ? key[2] : key[3];
    const uint32_t c0 = c == 0 ? key[4] : c == 1 ? key[5] : c == 2 ? key[6] : key[7];
    const uint32_t d0 = c == 0 ? ctr : c == 1 ? 0u : c == 2 ? n_lo : n_hi;
    uint32_t a = a0, b = b0, cc = c0, d = d0;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        NA_QR(a, b, cc, d);                                   /* columns */
        b = quad_perm<QP_NEXT1>(b); cc = quad_perm<QP_NEXT2>(cc); d = quad_perm<QP_NEXT3>(d);
        NA_QR(a, b, cc, d);                                   /* diagonals */
        b = quad_perm<QP_NEXT3>(b); cc = quad_perm<QP_NEXT2>(cc); d = quad_perm<QP_NEXT1>(d);
    }
    oa = a + a0; ob = b + b0; oc = cc + c0; od = d + d0;
}

/* chacha_quad for two blocks at once (blocks ctr0 and ctr1 on the same
   quad): two independent dependency chains in one instruction stream, so a
   lone wave's issue slots fill with the other block's work (the multi-pass
   records' passes, two per step) */
NA_DEV void chacha_quad_x2(const uint32_t key[8], uint32_t ctr0, uint32_t ctr1, uint32_t n_lo, uint32_t n_hi,
                           int c, uint32_t o0[4], uint32_t o1[4])
{
    const uint32_t a0 = c == 0 ? 0x61707865u : c == 1 ? 0x3320646eu : c == 2 ? 0x79622d32u : 0x6b206574u;
    const uint32_t b0 = c == 0 ? key[0] : c == 1 ? key[1] : c == 2 ? key[2] : key[3];
    const uint32_t c0 = c == 0 ? key[4] : c == 1 ? key[5] : c == 2 ? key[6] : key[7];
    const uint32_t d0 = c == 0 ? ctr0 : c == 1 ? 0u : c == 2 ? n_lo : n_hi;
    const uint32_t d1 = c == 0 ? ctr1 : d0;
    uint32_t a = a0, b = b0, cc = c0, d = d0;
    uint32_t e = a0, f = b0, g = c0, h = d1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        NA_QR(a, b, cc, d);
        NA_QR(e, f, g, h);
        b = quad_perm<QP_NEXT1>(b); cc = quad_perm<QP_NEXT2>(cc); d = quad_perm<QP_NEXT3>(d);
        f = quad_perm<QP_NEXT1>(f); g = quad_perm<QP_NEXT2>(g); h = quad_perm<QP_NEXT3>(h);
        NA_QR(a, b, cc, d);
        NA_QR(e, f, g, h);
        b = quad_perm<QP_NEXT3>(b); cc = quad_perm<QP_NEXT2>(cc); d = quad_perm<QP_NEXT1>(d);
        f = quad_perm<QP_NEXT3>(f); g = quad_perm<QP_NEXT2>(g); h = quad_perm<QP_NEXT1>(h);
    }
    o0[0] = a + a0; o0[1] = b + b0; o0[2] = cc + c0; o0[3] = d + d0;
    o1[0] = e + a0; o1[1] = f + b0; o1[2] = g + c0; o1[3] = h + d1;
}

/* 16 bytes at p (16-B aligned LDS), bytes from `n` on cleared */
NA_DEV void lds_block(const uint8_t *p, uint32_t n, uint32_t w[4])
{
    const uint4 v = *(const uint4 *)p;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rem = (int)n - 4 * i;
        w[i] &= rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
    }
}

struct FastLds {
    uint32_t dbg[8];         /* s_memtime stamps of thread 0 (debug hook) */
    uint32_t rs[8];          /* r, s (key stream words 0..7 of block 0) */
    uint32_t v[4][5];        /* the tree's cross-wave partners (levels 64, 128) */
    uint32_t verdict;
};

/* v of lane t + L (the tree's partner) for L < 64: DPP where the partner is
   in the same row of 16 lanes, a lane shuffle otherwise */
template <uint32_t L>
NA_DEV uint32_t from_plus(uint32_t x, int lane)
{
    if constexpr (L == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xb1, 0xf, 0xf, false);  /* quad [1,0,3,2] */
    else if constexpr (L == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4e, 0xf, 0xf, false); /* quad [2,3,0,1] */
    else if constexpr (L == 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xf, 0xf, false); /* row_shl:4 */
    else if constexpr (L == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x108, 0xf, 0xf, false); /* row_shl:8 */
    else return (uint32_t)__shfl((int)x, lane + (int)L, 64);
}

/* One level of the Poly1305 tree: lanes j = 0 mod 2L set v_j = v_j r^L + v_{j+L};
   mP holds r^L on entry and r^(2L) on exit (when a next level exists). */
template <uint32_t L>
NA_DEV void tree_level(Fe &v, Mul &mP, int t, uint32_t N, FastLds &F)
{
    if (L >= N) return; /* uniform */
    const int lane = t & 63;
    Fe w;
    if constexpr (L < 64) {
        w.l0 = from_plus<L>(v.l0, lane);
        w.l1 = from_plus<L>(v.l1, lane);
        w.l2 = from_plus<L>(v.l2, lane);
        w.l3 = from_plus<L>(v.l3, lane);
        w.l4 = from_plus<L>(v.l4, lane);
    } else {
        /* partner t + L sits in another wave: through LDS */
        if (lane == 0 && (t & (int)(2 * L - 1)) == (int)L) {
            const int slot = t >> 6;
            F.v[slot][0] = v.l0; F.v[slot][1] = v.l1; F.v[slot][2] = v.l2;
            F.v[slot][3] = v.l3; F.v[slot][4] = v.l4;
        }
        __syncthreads();
        const int slot = min((t + (int)L) >> 6, 3); /* receivers: 1, 2 or 3 */
        w = Fe{F.v[slot][0], F.v[slot][1], F.v[slot][2], F.v[slot][3], F.v[slot][4]};
        __syncthreads();
    }
    const Mul cur = mP;
    if (2 * L < N) mP = mk_mul(fe_mul(mul_fe(cur), cur)); /* r^(2L), off the chain */
    if ((t & (int)(2 * L - 1)) == 0) v = fe_carry(fe_add(fe_mul(v, cur), w));
}

/* rec: len bytes (+ the tag for open) in LDS, 16-B aligned; ad: ad_len bytes
   (16-B aligned, padded).  256 threads, every one calls this. */
template <bool OPEN>
NA_DEV bool worker_chacha_fast(uint8_t *rec, const uint8_t *ad, uint32_t ad_len, uint32_t len,
                               const uint8_t *key8, uint64_t nonce, FastLds &F)
{
    const int t = (int)threadIdx.x, c = t & 3;
    const uint32_t q = (uint32_t)t >> 2; /* ChaCha block */
    const uint64_t c00 = __builtin_amdgcn_s_memtime();
#define NA_FSTAMP(k) do { if (t == 0) F.dbg[k] = (uint32_t)(__builtin_amdgcn_s_memtime() - c00); } while (0)
    uint32_t key[8];
    load_key(key8, key);
    const uint32_t n_lo = (uint32_t)nonce, n_hi = (uint32_t)(nonce >> 32);
    const uint32_t J = (len + 63) / 64; /* data blocks 1..J */
    uint32_t ks[4] = {0, 0, 0, 0};
    if (q <= J) chacha_quad(key, q, n_lo, n_hi, c, ks[0], ks[1], ks[2], ks[3]);
    if (q == 0) { F.rs[c] = ks[0]; F.rs[4 + c] = ks[1]; }
    NA_FSTAMP(0); /* ChaCha done (thread 0's quad) */
    /* data words 64(q-1) + 4c + 16i, i = 0..3: key stream word 4i + c */
    uint32_t pt[4] = {0, 0, 0, 0};
    if (q >= 1 && q <= J) {
        uint32_t *w = (uint32_t *)(rec + 64 * (q - 1) + 4 * c);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pt[i] = w[4 * i] ^ ks[i];
            if (!OPEN) w[4 * i] = pt[i]; /* CT; bytes past len are overwritten by the tag */
        }
    }
    __syncthreads();
    NA_FSTAMP(1); /* CT in LDS, r and s published */
    /* Poly1305 block of this lane, right-justified in N lanes */
    const uint32_t a = (ad_len + 15) / 16, m = (len + 15) / 16, n = a + m + 1;
    const uint32_t N = n <= 1 ? 1u : 1u << (32 - __builtin_clz(n - 1));
    const int i = t - (int)(N - n);
    Fe v = fe_zero();
    if (i >= 0 && (uint32_t)i < n) {
        uint32_t b[4];
        if ((uint32_t)i < a) {
            lds_block(ad + 16 * i, ad_len - 16 * i, b);
        } else if ((uint32_t)i < a + m) {
            const uint32_t j = (uint32_t)i - a;
            lds_block(rec + 16 * j, len - 16 * j, b);
        } else {
            b[0] = ad_len; b[1] = 0; b[2] = len; b[3] = 0;
        }
        fe_add_block(v, b[0], b[1], b[2], b[3]);
    }
    const Fe r = fe_clamp_r(F.rs[0], F.rs[1], F.rs[2], F.rs[3]);
    Mul mP = mk_mul(r); /* r^L */
    NA_FSTAMP(2); /* Poly block loaded */
    /* levels 1..8 by DPP (quad swaps, row shifts), 16 and 32 by lane
       shuffles, 64 and 128 through LDS; each level a uniform branch on N */
    tree_level<1>(v, mP, t, N, F);
    tree_level<2>(v, mP, t, N, F);
    tree_level<4>(v, mP, t, N, F);
    tree_level<8>(v, mP, t, N, F);
    tree_level<16>(v, mP, t, N, F);
    tree_level<32>(v, mP, t, N, F);
    tree_level<64>(v, mP, t, N, F);
    tree_level<128>(v, mP, t, N, F);
    NA_FSTAMP(3); /* tree done */
    /* thread 0: the tag; every lane of the group got the same tree, so
       only thread 0's value is the sum */
    if (t == 0) {
        v = fe_mul(v, mk_mul(r));
        const uint32_t s[4] = {F.rs[4], F.rs[5], F.rs[6], F.rs[7]};
        uint32_t tag[4];
        fe_finish(v, s, tag);
        if (OPEN) {
            uint32_t got[4];
            load16(rec + len, 16, got);
            F.verdict = tag_equal(tag, got) ? 1u : 0u;
        } else {
            store16(rec + len, 16, tag);
        }
    }
    NA_FSTAMP(4); /* tag */
    if (!OPEN) return true;
    __syncthreads();
    const bool ok = F.verdict != 0;
    if (ok && q >= 1 && q <= J) {
        uint32_t *w = (uint32_t *)(rec + 64 * (q - 1) + 4 * c);
#pragma unroll
        for (int i2 = 0; i2 < 4; ++i2) w[4 * i2] = pt[i2]; /* bytes past len: not copied out */
    }
    NA_FSTAMP(5);
#undef NA_FSTAMP
    return ok;
}

/* Records past one pass (more than 63 units, or a Poly1305 input of more
   than 256 blocks): the same layout over P = ceil((J + 1) / 64) ChaCha
   passes, and G = ceil(n / 256) Poly1305 blocks per lane — lane j runs
   Horner with r over its G consecutive blocks (right-justified chunks),
   then the tree of worker_chacha_fast sums the chunks with unit R = r^G:
     poly = (sum_j h_j R^(NL-1-j)) r,  h_j = sum_k b_(jG+k-pad) r^(G-1-k),
   which is sum_i b_i r^(n-i+1) again.  Seal XORs each pass into the record
   in LDS, then authenticates the ciphertext; open authenticates first (pass
   0 for r and s) and decrypts only a verified record.  A separate
   instantiation, so records of one pass keep worker_chacha_fast unchanged
   (round 3 measured a merged version costing them 0.3-0.8 us). */
/* XOR the key stream of blocks 1..J into the record in LDS: pass p holds
   blocks 64p + q (pass 0's key stream, ks0, computed already); the other
   passes two at a time (chacha_quad_x2) */
NA_DEV void multi_xor_one(uint8_t *rec, uint32_t v, uint32_t J, int c, const uint32_t ks[4])
{
    if (v >= 1 && v <= J) {
        uint32_t *w = (uint32_t *)(rec + 64 * (v - 1) + 4 * c);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[4 * i] ^= ks[i];
    }
}

NA_DEV void multi_xor_passes(uint8_t *rec, const uint32_t key[8], uint32_t n_lo, uint32_t n_hi, int c, uint32_t q,
                             uint32_t J, uint32_t P, const uint32_t ks0[4])
{
    multi_xor_one(rec, q, J, c, ks0);
    for (uint32_t p = 1; p < P; p += 2) {
        const uint32_t v0 = 64 * p + q, v1 = v0 + 64;
        uint32_t k0[4], k1[4];
        if (p + 1 < P) { /* uniform */
            chacha_quad_x2(key, v0, v1, n_lo, n_hi, c, k0, k1);
            multi_xor_one(rec, v0, J, c, k0);
            multi_xor_one(rec, v1, J, c, k1);
        } else {
            chacha_quad(key, v0, n_lo, n_hi, c, k0[0], k0[1], k0[2], k0[3]);
            multi_xor_one(rec, v0, J, c, k0);
        }
    }
}

template <bool OPEN>
NA_DEV bool worker_chacha_multi(uint8_t *rec, const uint8_t *ad, uint32_t ad_len, uint32_t len,
                                const uint8_t *key8, uint64_t nonce, FastLds &F)
{
    const int t = (int)threadIdx.x, c = t & 3;
    const uint32_t q = (uint32_t)t >> 2;
    const uint64_t c00 = __builtin_amdgcn_s_memtime();
#define NA_FSTAMP(k) do { if (t == 0) F.dbg[k] = (uint32_t)(__builtin_amdgcn_s_memtime() - c00); } while (0)
    uint32_t key[8];
    load_key(key8, key);
    const uint32_t n_lo = (uint32_t)nonce, n_hi = (uint32_t)(nonce >> 32);
    const uint32_t J = (len + 63) / 64, P = (J + 1 + 63) / 64; /* blocks 0..J in P passes */
    /* ChaCha pass p: block v = 64p + q; data words 64(v-1) + 4c + 16i */
    uint32_t ks0[4] = {0, 0, 0, 0}; /* pass 0 (open: XORed after the verdict) */
    chacha_quad(key, q, n_lo, n_hi, c, ks0[0], ks0[1], ks0[2], ks0[3]);
    if (q == 0) { F.rs[c] = ks0[0]; F.rs[4 + c] = ks0[1]; }
    if (!OPEN) multi_xor_passes(rec, key, n_lo, n_hi, c, q, J, P, ks0); /* CT; bytes past len: the tag overwrites */
    __syncthreads();
    NA_FSTAMP(0); /* seal: CT in LDS; both: r and s published */
    const uint32_t a = (ad_len + 15) / 16, m = (len + 15) / 16, n = a + m + 1;
    const uint32_t G = (n + 255) / 256, NL = (n + G - 1) / G, pad = NL * G - n;
    const uint32_t N = NL <= 1 ? 1u : 1u << (32 - __builtin_clz(NL - 1));
    const int j = t - (int)(N - NL); /* this lane's chunk */
    const Fe r = fe_clamp_r(F.rs[0], F.rs[1], F.rs[2], F.rs[3]);
    const Mul mr = mk_mul(r);
    Fe h = fe_zero();
    if (j >= 0 && (uint32_t)j < NL) {
        for (uint32_t k = 0; k < G; ++k) {
            const int idx = j * (int)G + (int)k - (int)pad; /* 0-based block of the Poly input */
            if (idx < 0) continue;                          /* leading padding of chunk 0 */
            uint32_t b[4];
            const uint32_t i = (uint32_t)idx;
            if (i < a) {
                lds_block(ad + 16 * i, ad_len - 16 * i, b);
            } else if (i < a + m) {
                const uint32_t jj = i - a;
                lds_block(rec + 16 * jj, len - 16 * jj, b);
            } else {
                b[0] = ad_len; b[1] = 0; b[2] = len; b[3] = 0;
            }
            h = fe_mul(h, mr);
            fe_add_block(h, b[0], b[1], b[2], b[3]);
        }
    }
    NA_FSTAMP(1); /* chunks' Horner done */
    /* R = r^G (G <= 17), square-and-multiply, the same in every lane */
    Fe R = r;
    {
        const int top = 31 - __builtin_clz(G);
        for (int bit = top - 1; bit >= 0; --bit) {
            R = fe_mul(R, mk_mul(R));
            if ((G >> bit) & 1u) R = fe_mul(R, mr);
        }
    }
    Mul mP = mk_mul(R);
    Fe vv = h;
    tree_level<1>(vv, mP, t, N, F);
    tree_level<2>(vv, mP, t, N, F);
    tree_level<4>(vv, mP, t, N, F);
    tree_level<8>(vv, mP, t, N, F);
    tree_level<16>(vv, mP, t, N, F);
    tree_level<32>(vv, mP, t, N, F);
    tree_level<64>(vv, mP, t, N, F);
    tree_level<128>(vv, mP, t, N, F);
    NA_FSTAMP(2); /* tree done */
    if (t == 0) {
        vv = fe_mul(vv, mr);
        const uint32_t s[4] = {F.rs[4], F.rs[5], F.rs[6], F.rs[7]};
        uint32_t tag[4];
        fe_finish(vv, s, tag);
        if (OPEN) {
            uint32_t got[4];
            load16(rec + len, 16, got);
            F.verdict = tag_equal(tag, got) ? 1u : 0u;
        } else {
            store16(rec + len, 16, tag);
        }
    }
    NA_FSTAMP(3); /* tag */
    if (!OPEN) return true;
    __syncthreads();
    const bool ok = F.verdict != 0;
    if (ok) multi_xor_passes(rec, key, n_lo, n_hi, c, q, J, P, ks0); /* decrypt the verified record in LDS */
    NA_FSTAMP(4);
#undef NA_FSTAMP
    return ok;
}

/* One 16-byte system-coherent load (a single request: the chunk is read
   whole, never half before and half after the host's 16-byte store). */
NA_DEV uint4 load_sys16(const uint32_t *p)
{
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                 : "=v"(v) : "v"(p) : "memory");
    return v;
}

/* two system-coherent 16-byte loads in one round trip */
NA_DEV void load_sys16x2(const uint32_t *p, const uint32_t *q, uint4 &a, uint4 &b)
{
    asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
                 "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(a), "=&v"(b) : "v"(p), "v"(q) : "memory");
}

NA_DEV uint32_t now10ns() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }

/* 16 raw stream bytes, system-coherent, as two 8-byte atomic loads the
   compiler schedules (no wait per load) */
NA_DEV uint4 load_sys16_raw(const uint8_t *p)
{
    const uint64_t *q = (const uint64_t *)p;
    const uint64_t a = NA_SYS_LOAD(q), b = NA_SYS_LOAD(q + 1);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

/* polls without a request after which only the header is polled: 20 us */
constexpr uint64_t POLL_BACKOFF = 2000;

/* A worker GROUP is one kernel of nslots workgroups on one high-priority
   stream, workgroup i serving request slot i: several calling threads per
   hardware queue (4 queues served at most 4 threads).  A group
   ends as a whole — a hardware queue runs nothing else until its kernel has
   left — so the workgroups agree on leaving through the group words (in the
   slots' placement, polled with the header in the same load instruction):
   word 0 `closing`, set by the first workgroup to leave (stop, idle,
   lifetime), after which every workgroup leaves between requests; words
   1..nslots the workgroups' last-request times.  A workgroup leaves for
   idleness only when every slot of the group has been idle that long.  Only
   the device writes the group words (`closing` is the number of the launch
   that closed, never reset by the host). */
constexpr int WORKER_MAX_SLOTS = 4;
struct WorkerSlotArgs {
    WorkerSlot *slot;      /* device view of the slot */
    const uint32_t *req;   /* the header chunks (4 in host memory; 8 in device memory, vram) */
    const uint4 *in;       /* the stream's stamped chunks */
    const uint8_t *tail;   /* the rest of the stream, raw */
    uint8_t *out;          /* results */
    uint32_t vram;
    uint32_t pad_;
};
struct WorkerArgs {
    WorkerSlotArgs s[WORKER_MAX_SLOTS];
    uint32_t *group;       /* the group words (8) */
    uint32_t nslots;
    uint32_t gen;          /* this launch's number: `closing` holds the number of the launch that closed */
    uint64_t idle, lifetime; /* s_memrealtime ticks (100 MHz) */
};

/* 256 threads per workgroup, one workgroup per slot. */
__global__ __launch_bounds__(256) void aead_worker(WorkerArgs a)
{
    const uint32_t me = blockIdx.x;
    WorkerSlot *const slot = a.s[me].slot;
    const uint32_t *const req = a.s[me].req;
    const uint4 *const in = a.s[me].in;
    const uint8_t *const tail = a.s[me].tail;
    uint8_t *const out = a.s[me].out;
    const uint32_t vram = a.s[me].vram;
    const uint64_t idle = a.idle, lifetime = a.lifetime;
    /* the last request served on this slot (a relaunched group starts where
       the one before it stopped: a request it left unserved is served) */
    uint32_t last = (uint32_t)NA_SYS_LOAD(&slot->done);
    const uint32_t head = vram ? VWORKER_HEAD : WORKER_HEAD, cbytes = vram ? VCHUNK_BYTES : WCHUNK_BYTES;
    __shared__ uint32_t te[256], sb[256];
    __shared__ __attribute__((aligned(16))) uint8_t cbuf[WORKER_CTX_SLOTS][WORKER_CTX_BYTES];
    __shared__ uint64_t ctag[WORKER_CTX_SLOTS]; /* host address of the cached context */
    __shared__ uint32_t cgen[WORKER_CTX_SLOTS], cuse[WORKER_CTX_SLOTS];
    __shared__ uint32_t hdr[16];
    __shared__ uint32_t s_cmd;          /* 0 wait, 1 serve, 2 leave */
    __shared__ uint32_t wl[40];         /* gcm_wide_record's verdict, E_K(J0), GHASH rows */
    __shared__ uint32_t s_stale;        /* chunks still stamped with an older request */
    __shared__ FastLds fast;
    __shared__ __attribute__((aligned(16))) uint8_t buf[WORKER_DATA];
    const uint32_t t = threadIdx.x;
    aes_table_entry(t, sb[t], te[t]);
    if (t < WORKER_CTX_SLOTS) {
        ctag[t] = 0;
        cgen[t] = 0;
        cuse[t] = 0;
    }
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    uint64_t quiet = born;
    /* the group word of this slot's last-request time is refreshed at most
       every idle / 8 (a system store the next poll would wait for: +0.7 us
       per call when written after every request); the idle test allows for
       the lag */
    uint64_t stamped = born;
    if (t == 0) NA_SYS_STORE(&a.group[1 + me], (uint32_t)born);
    bool leaving = false;
    uint32_t tick = 0;
    __shared__ uint32_t s_slow; /* backed-off polling (see below) */
    if (t == 0) s_slow = 0;
    __syncthreads();
    for (;;) {
        uint32_t t_seen = 0;
        /* every thread reads input chunk t; wave 0's lanes 0..3 (0..7 in
           device memory) hold the header (other lanes read a header chunk
           too: same round trip).  After POLL_BACKOFF without a request only
           wave 0 polls, the header alone (128 B instead of 8 KiB per poll:
           with the request in host memory every poll crosses PCIe), and a
           request then re-reads its chunks once (stamp 0 is never current).
           A wave may see the previous poll's setting: both are correct. */
        uint4 c = make_uint4(0, 0, 0, 0), mine = make_uint4(0, 0, 0, 0);
        /* lanes 14 and 15 of every 16 read the group words instead */
        const uint32_t *hp = (t & 15) >= 14 ? a.group + 4 * (t & 1) : req + 4 * (t & (vram ? 15 : 7));
        if (!s_slow) load_sys16x2(hp, (const uint32_t *)(in + t), c, mine);
        else if (t < 64) c = load_sys16(hp);
        if (t == 0) s_stale = 0;
        if (t < 64) {
            const uint32_t s0 = __shfl((int)c.x, 0, 64);
            uint32_t stop;
            bool fresh;
            if (!vram) { /* chunk k = {seq, A_k, B_k, C_k} */
                const uint32_t s1 = __shfl((int)c.x, 1, 64);
                const uint32_t s2 = __shfl((int)c.x, 2, 64), s3 = __shfl((int)c.x, 3, 64);
                stop = __shfl((int)c.x, 4, 64); /* chunk 4: the stop word */
                fresh = s0 != last && s0 == s1 && s0 == s2 && s0 == s3;
                if (t < 4) {
                    hdr[4 * t] = c.x; hdr[4 * t + 1] = c.y; hdr[4 * t + 2] = c.z; hdr[4 * t + 3] = c.w;
                }
            } else { /* chunk 2k = {seq, A_k, seq, B_k}, 2k + 1 = {seq, C_k, seq, 0} */
                stop = __shfl((int)c.x, 8, 64); /* chunk 8: the stop word */
                fresh = s0 != last && __all(t >= 8 || (c.x == s0 && c.z == s0));
                if (t < 8) {
                    const uint32_t k = t >> 1;
                    if (t & 1) {
                        hdr[4 * k + 3] = c.y;
                    } else {
                        hdr[4 * k] = c.x; hdr[4 * k + 1] = c.y; hdr[4 * k + 2] = c.w;
                    }
                }
            }
            /* the group words: closing, then the slots' last-request times */
            const bool closing = (uint32_t)__shfl((int)c.x, 14, 64) == a.gen;
            const uint32_t gq[WORKER_MAX_SLOTS] = {(uint32_t)__shfl((int)c.y, 14, 64),
                                                   (uint32_t)__shfl((int)c.z, 14, 64),
                                                   (uint32_t)__shfl((int)c.w, 14, 64),
                                                   (uint32_t)__shfl((int)c.x, 15, 64)};
            if (t == 0) {
                uint32_t cmd = 0;
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                bool group_idle = now - quiet > idle;
                for (uint32_t j = 0; j < a.nslots; ++j) /* 32-bit tick differences: idle < 2^31 */
                    if ((uint32_t)now - gq[j] <= (uint32_t)(idle + idle / 8)) group_idle = false;
                if (fresh) {
                    cmd = 1;
                } else if (leaving) {
                    cmd = 2;
                } else if (stop || closing || group_idle || now - born > lifetime) {
                    /* the group leaves with this workgroup; announce, then
                       poll once more: a request posted before that poll is
                       served; one posted after it finds `exiting` set and the
                       host starts the group again once all of it has left */
                    /* debug: why (stamps[7]: 1 stop, 2 closing, 4 idle, 8 lifetime) */
                    slot->stamps[7] = (stop ? 1u : 0u) | (closing ? 2u : 0u) | (group_idle ? 4u : 0u) |
                                      (now - born > lifetime ? 8u : 0u);
                    slot->leave[0] = (uint32_t)born;
                    slot->leave[1] = (uint32_t)now;
                    slot->leave[2] = (uint32_t)lifetime;
                    slot->leave[3] = a.gen;
                    NA_SYS_STORE(&a.group[0], a.gen);
                    NA_SYS_STORE(&slot->exiting, 1u);
                    leaving = true;
                } else if (now - quiet > POLL_BACKOFF) {
                    __builtin_amdgcn_s_sleep(8);
                } else {
                    __builtin_amdgcn_s_sleep(2);
                }
                s_slow = cmd == 0 && now - quiet > POLL_BACKOFF ? 1u : 0u;
                s_cmd = cmd;
                t_seen = (uint32_t)now;
            }
        }
        __syncthreads();
        const uint32_t cmd = s_cmd;
        if (cmd == 2) break;
        if (cmd == 0) {
            __syncthreads();
            continue;
        }
        /* serve request hdr[0]: the data area was written before the header;
           the acquire orders the reads below after the header's */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint32_t seq = hdr[0], op = hdr[1] & 0xff, ct = (hdr[1] >> 8) & 1;
        const uint32_t len = hdr[2], ad_len = hdr[3];
        const uint64_t nonce = (uint64_t)hdr[5] | ((uint64_t)hdr[6] << 32);
        const uint32_t cipher = hdr[7];
        const uint64_t ctx_addr = (uint64_t)hdr[9] | ((uint64_t)hdr[10] << 32);
        const uint32_t gen = hdr[13];
        const uint32_t ad_pad = (ad_len + 15) & ~15u;
        const uint32_t bytes = 32 + ad_pad + len + 16;
        const uint32_t t_fence = now10ns();
        /* the input stream: the head as stamped chunks (chunk t read
           speculatively with the poll, re-read while stale), the rest raw
           (written before the header, read after it) */
        const uint32_t total = 32 + ad_pad + len + (op ? 16u : 0u);
        const uint32_t nchunks = min((total + cbytes - 1) / cbytes, WORKER_SPEC);
        if (t < nchunks) {
            uint4 v = mine;
            for (uint32_t tries = 0; (v.w != seq || (vram && v.y != seq)) && tries < (1u << 20); ++tries)
                v = load_sys16((const uint32_t *)(in + t));
            if (v.w != seq || (vram && v.y != seq)) s_stale = 1; /* never in practice: written before the header */
            uint32_t *d = (uint32_t *)(buf + cbytes * t);
            if (vram) {
                d[0] = v.x; d[1] = v.z;
            } else {
                d[0] = v.x; d[1] = v.y; d[2] = v.z;
            }
        }
        for (uint32_t o = 16 * t; head + o < total; o += 16 * 256)
            *(uint4 *)(buf + head + o) = load_sys16_raw(tail + o);
        int cs = 0;
        if (cipher == NOISE_CIPHER_AESGCM) { /* the context: cached, or copied into the LRU slot */
            cs = ctag[0] == ctx_addr && cgen[0] == gen ? 0 : (ctag[1] == ctx_addr && cgen[1] == gen ? 1 : -1);
            if (cs < 0) {
                cs = cuse[0] <= cuse[1] ? 0 : 1;
                const uint8_t *src = (const uint8_t *)ctx_addr;
                for (uint32_t o = 16 * t; o < WORKER_CTX_BYTES; o += 16 * 256)
                    *(uint4 *)(cbuf[cs] + o) = *(const uint4 *)(src + o);
            }
        }
        __syncthreads();
        if (t == 0 && cipher == NOISE_CIPHER_AESGCM) {
            ctag[cs] = ctx_addr;
            cgen[cs] = gen;
            cuse[cs] = ++tick;
        }
        const uint32_t t_in = now10ns();
        if (t < 8) fast.dbg[t] = 0; /* the path's stamps: those it does not reach stay 0 */
        const uint64_t c_in = __builtin_amdgcn_s_memtime();
        uint8_t *key = buf, *ad = buf + 32, *rec = buf + 32 + ad_pad;
        bool ok = true;
        if (cipher == NOISE_CIPHER_CHACHAPOLY && worker_fast_fits(len, ad_len)) {
            ok = op ? worker_chacha_fast<true>(rec, ad, ad_len, len, key, nonce, fast)
                    : worker_chacha_fast<false>(rec, ad, ad_len, len, key, nonce, fast);
        } else if (cipher == NOISE_CIPHER_CHACHAPOLY) { /* past one pass */
            ok = op ? worker_chacha_multi<true>(rec, ad, ad_len, len, key, nonce, fast)
                    : worker_chacha_multi<false>(rec, ad, ad_len, len, key, nonce, fast);
        } else {
            const AesCtx *c = (const AesCtx *)cbuf[cs];
            const uint4 *h8 = (const uint4 *)c->tab8;
            if (ct) ok = op ? gcm_wide_record<true, true>(rec, rec, ad, ad_len, len, nonce, c, te, sb, h8, wl, nullptr, fast.dbg)
                            : gcm_wide_record<false, true>(rec, rec, ad, ad_len, len, nonce, c, te, sb, h8, wl, nullptr, fast.dbg);
            else ok = op ? gcm_wide_record<true, false>(rec, rec, ad, ad_len, len, nonce, c, te, sb, h8, wl, nullptr, fast.dbg)
                         : gcm_wide_record<false, false>(rec, rec, ad, ad_len, len, nonce, c, te, sb, h8, wl, nullptr, fast.dbg);
            if (t == 0) /* absolute s_memtime stamps -> cycles since c_in */
                for (int k = 0; k < 8; ++k) fast.dbg[k] = fast.dbg[k] ? fast.dbg[k] - (uint32_t)c_in : 0u;
        }
        __syncthreads();
        const uint32_t t_done = now10ns();
        const uint32_t c_run = (uint32_t)(__builtin_amdgcn_s_memtime() - c_in); /* shader cycles */
        /* results back: seal CT || tag, open the plaintext (only if verified);
           every storing wave drains its stores, then one system release and
           the flag (MI355X_MICROARCH.md, inter-workgroup visibility) */
        const bool stale = s_stale != 0;
        if (stale) ok = false;
        const uint32_t nout = op ? (ok ? len : 0u) : (stale ? 0u : len + 16);
        for (uint32_t o = 16 * t; o < ((nout + 15) & ~15u); o += 16 * 256)
            *(uint4 *)(out + o) = *(const uint4 *)(rec + o);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            const uint32_t t_out = now10ns();
            slot->status = stale ? 2u : (ok ? 0u : 1u);
            slot->stamps[0] = t_seen;
            slot->stamps[1] = t_fence;
            slot->stamps[2] = t_in;
            slot->stamps[3] = t_done;
            slot->stamps[4] = t_out;
            slot->stamps[6] = c_run;
            for (int k = 0; k < 8; ++k) slot->fstamps[k] = fast.dbg[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            slot->stamps[5] = now10ns();
            NA_SYS_STORE(&slot->done, (uint64_t)seq);
        }
        last = seq;
        quiet = __builtin_amdgcn_s_memrealtime();
        if (quiet - stamped > idle / 8) {
            if (t == 0) NA_SYS_STORE(&a.group[1 + me], (uint32_t)quiet);
            stamped = quiet;
        }
        /* scrub this record's bytes (and the key) from LDS before the next one;
           the kernels may have written whole 64-B units past len + 16 */
        for (uint32_t o = 16 * t; o < bytes + 64; o += 16 * 256) *(uint4 *)(buf + o) = make_uint4(0, 0, 0, 0);
        __syncthreads();
    }
    /* the cached AES-GCM contexts hold key material too */
    for (uint32_t o = 16 * t; o < WORKER_CTX_SLOTS * WORKER_CTX_BYTES; o += 16 * 256)
        *(uint4 *)(&cbuf[0][0] + o) = make_uint4(0, 0, 0, 0);
}

/* ------------------------------------------------------------- host side */

namespace {

struct WorkerGroup;

/* One request slot: served by one workgroup of its group's kernel. */
struct Worker {
    std::mutex mu;             /* held by the calling thread for a whole call */
    int state = 0;             /* 0 not set up, 1 usable, -1 failed */
    WorkerSlot *slot = nullptr; /* host view */
    WorkerSlot *dslot = nullptr; /* device view */
    /* the request (header chunks, stream): in fine-grained device memory the
       CPU writes through the BAR (vram), or in the host slot */
    bool vram = false;
    uint32_t *req = nullptr;    /* host view of the header chunks */
    const uint32_t *dreq = nullptr;
    void *vbase = nullptr;      /* the device allocation (vram) */
    uint4 *in = nullptr, *din = nullptr;       /* the stream's head: stamped chunks */
    uint8_t *tail = nullptr, *dtail = nullptr; /* the rest of the stream, raw */
    uint8_t *out = nullptr, *dout = nullptr;   /* raw results */
    uint32_t seq = 0;
    /* the AES-GCM contexts (host copies) sent to this slot's workgroup, whose
       LDS cache may hold them: only a group one of whose slots was sent a
       context is parked when the state is freed; past kCtxHist
       distinct ones since the group's launch, any free parks it */
    static constexpr int kCtxHist = 8;
    const void *ctx_hist[kCtxHist] = {};
    uint32_t ctx_n = 0;        /* written under mu (or at launch), read by forget() with atomics */
    WorkerGroup *g = nullptr;
};

/* One kernel on one high-priority stream: nslots workgroups, one per slot. */
struct WorkerGroup {
    std::mutex mu;             /* launch, drain, recover (taken after a slot's mu, never before) */
    int state = 0;             /* 0 unknown, 1 usable, -1 disabled, -2 draining (worker_abandon) */
    uint32_t launches = 0;     /* debug: kernels launched (noise_aead_debug_worker_launches) */
    int launch_fails = 0;      /* consecutive failed launches (3 disable the group) */
    hipStream_t stream = nullptr;
    bool launched = false;     /* written under mu, read by park() with atomics */
    uint32_t gen = 0;          /* launches so far (atomics): a relaunch happens once */
    uint32_t abandoned = 0;    /* slots whose request was abandoned: results scrubbed on recovery */
    uint32_t *words = nullptr; /* host view of the group words (8) */
    uint32_t *dwords = nullptr;
    bool words_vram = false;
    int nslots = 1;
    Worker slot[WORKER_MAX_SLOTS];
};

constexpr int kMaxDev = 64;
constexpr int kMaxGroups = 8;

/* A resident group never ends while calls keep coming (up to LIFETIME), so
   it must own its hardware queue: a kernel queued behind it on the same AQL
   queue waits for it to leave.  HIP maps streams onto GPU_MAX_HW_QUEUES
   queues per device and priority (4 by default), so the groups run on
   high-priority streams — a pool apart from the application's normal
   streams (tools/queue_probe.cpp: a memset on a new normal stream waited
   the worker's whole 5 s lifetime beside a normal-priority worker, 20-60 us
   beside high-priority ones) — and a device runs one group per queue of that
   pool but one: the last queue stays free for a high-priority stream of the
   application's own.  NOISE_AEAD_WORKER_QUEUES sets the number
   of queues the groups take instead (1..8; an application with several
   high-priority streams of its own lowers it, or raises GPU_MAX_HW_QUEUES).
   NOISE_AEAD_WORKER_PRIO=normal / low: the A/B placements. */
int worker_stream_prio()
{
    static const int v = [] {
        const char *e = getenv("NOISE_AEAD_WORKER_PRIO");
        if (!e) return 1;
        return !strcmp(e, "normal") ? 0 : (!strcmp(e, "low") ? -1 : 1);
    }();
    return v;
}

int hw_queues()
{
    const char *e = getenv("GPU_MAX_HW_QUEUES");
    const int q = e ? atoi(e) : 4;
    return q < 1 ? 4 : q;
}

int groups_per_dev()
{
    static const int v = [] {
        const char *e = getenv("NOISE_AEAD_WORKER_QUEUES");
        int g = e && atoi(e) > 0 ? atoi(e) : (hw_queues() > 1 ? hw_queues() - 1 : 1);
        return g < kMaxGroups ? g : kMaxGroups;
    }();
    return v;
}

/* Slots per group: enough for 8 calling threads over the groups
   (NOISE_AEAD_WORKER_SLOTS: 1..4).  A CipherState is single-owner with no
   locks (cipherstate.c:293-410), so N threads on N states run N calls at once
   on the CPU; here each calling thread gets a slot of its own (a workgroup on
   its own CU), claimed without waiting while one is free. */
int slots_per_group()
{
    static const int v = [] {
        const char *e = getenv("NOISE_AEAD_WORKER_SLOTS");
        int s = e && atoi(e) > 0 ? atoi(e) : (8 + groups_per_dev() - 1) / groups_per_dev();
        return s < WORKER_MAX_SLOTS ? s : WORKER_MAX_SLOTS;
    }();
    return v;
}

WorkerGroup g_group[kMaxDev][kMaxGroups];
std::atomic<uint32_t> g_next_pref{0};
thread_local int t_pref = -1;             /* this thread's first-choice slot (spread over groups first) */
thread_local Worker *t_last = nullptr;    /* the slot of this thread's last call (debug hooks) */
std::once_flag g_atexit_once;

constexpr uint64_t IDLE_TICKS = 200000;       /* 2 ms at 100 MHz */
/* Test hook: NOISE_AEAD_DEBUG_WORKER_IDLE_MS overrides the idle timeout. */
uint64_t idle_ticks()
{
    static const uint64_t v = [] {
        const char *e = getenv("NOISE_AEAD_DEBUG_WORKER_IDLE_MS");
        return e && atoi(e) > 0 ? (uint64_t)atoi(e) * 100000ull : IDLE_TICKS;
    }();
    return v;
}
constexpr uint64_t LIFETIME_TICKS = 500000000; /* 5 s */
/* The longest request (a 65519-B AES-GCM record) takes ~0.4 ms; a group
   that has not answered after this is taken for lost: the call falls back to
   the launch path and the group is drained before it is used again. */
constexpr uint64_t WAIT_LIMIT_NS = 2000000000ull; /* 2 s */

/* the stop word: chunk 4 of the host slot, chunk 8 of the device request
   area — a chunk of its own, apart from the request header the calls
   rewrite */
uint32_t *stop_word(Worker &w) { return w.vram ? &w.req[4 * 8] : &w.req[4 * 4]; }

void set_stops(WorkerGroup &g, uint32_t v)
{
    for (int i = 0; i < g.nslots; ++i)
        if (g.slot[i].state == 1) __atomic_store_n(stop_word(g.slot[i]), v, __ATOMIC_RELEASE);
    _mm_sfence();
}

/* Ask a launched group to leave (no wait).  A workgroup leaving scrubs its
   LDS; a request racing with the stop is either served or seen by its caller
   as `exiting` (the caller then starts the group again).  The stop words
   have chunks of their own, so no request header written meanwhile can undo
   them. */
void park_group(WorkerGroup &g)
{
    if (__atomic_load_n(&g.launched, __ATOMIC_ACQUIRE)) set_stops(g, 1u);
}

void park_device(int dev)
{
    for (int i = 0; i < kMaxGroups; ++i) park_group(g_group[dev][i]);
}

/* Did slot w (maybe) receive AES-GCM context h since its group's launch? */
bool worker_saw_ctx(const Worker &w, const void *h)
{
    const uint32_t n = __atomic_load_n(&w.ctx_n, __ATOMIC_ACQUIRE);
    if (n > (uint32_t)Worker::kCtxHist) return true; /* history overflowed */
    for (uint32_t i = 0; i < n; ++i)
        if (__atomic_load_n(&w.ctx_hist[i], __ATOMIC_RELAXED) == h) return true;
    return false;
}

/* (under w.mu) record that context h goes to slot w */
void worker_note_ctx(Worker &w, const void *h)
{
    const uint32_t n = w.ctx_n;
    if (n > (uint32_t)Worker::kCtxHist) return;
    for (uint32_t i = 0; i < n; ++i)
        if (w.ctx_hist[i] == h) return;
    if (n < (uint32_t)Worker::kCtxHist) __atomic_store_n(&w.ctx_hist[n], h, __ATOMIC_RELAXED);
    __atomic_store_n(&w.ctx_n, n + 1, __ATOMIC_RELEASE);
}

/* A request the group did not answer within WAIT_LIMIT_NS (under w.mu): the
   group is asked to leave and the request's header is made unservable — its
   first chunk no longer agrees with the others — so a late workgroup cannot
   take it; the group is drained (state -2) and made usable again once its
   stream is idle (worker_recover), when the slot's result area is scrubbed
   once more in case a late workgroup wrote it. */
void worker_abandon(Worker &w, uint32_t k)
{
    WorkerGroup &g = *w.g;
    /* the stop words and this slot's header first, without the group's
       lock: a caller holding it may be waiting in group_launch for this very
       group to leave */
    set_stops(g, 1u);
    const uint32_t bad = k ^ 0x80000000u;
    const __m128i c = w.vram ? _mm_set_epi32(0, (int)bad, 0, (int)bad) : _mm_set_epi32(0, 0, 0, (int)bad);
    _mm_store_si128((__m128i *)w.req, c);
    _mm_sfence();
    std::lock_guard<std::mutex> gl(g.mu);
    g.abandoned |= 1u << (int)(&w - g.slot);
    g.state = -2;
}

/* (under g.mu) a drained group whose stream has gone idle: the abandoned
   slots' results scrubbed, usable again (relaunched by the next call) */
void worker_recover(WorkerGroup &g)
{
    if (g.state != -2 || hipStreamQuery(g.stream) != hipSuccess) return;
    for (int i = 0; i < g.nslots; ++i)
        if (g.abandoned & (1u << i)) explicit_bzero(g.slot[i].out, WORKER_DATA);
    g.abandoned = 0;
    __atomic_store_n(&g.launched, false, __ATOMIC_RELEASE);
    g.state = 1;
}

void worker_stop_all()
{
    for (int d = 0; d < kMaxDev; ++d)
        for (int i = 0; i < kMaxGroups; ++i) {
            WorkerGroup &g = g_group[d][i];
            std::lock_guard<std::mutex> lk(g.mu);
            if ((g.state != 1 && g.state != -2) || !g.launched) continue;
            set_stops(g, 1u);
            (void)hipStreamSynchronize(g.stream);
            for (int s = 0; s < g.nslots; ++s) /* a late workgroup's results */
                if (g.abandoned & (1u << s)) explicit_bzero(g.slot[s].out, WORKER_DATA);
            __atomic_store_n(&g.launched, false, __ATOMIC_RELEASE);
        }
}

bool worker_enabled()
{
    static const int v = [] {
        const char *e = getenv("NOISE_AEAD_WORKER");
        return e && e[0] == '0' ? 0 : 1;
    }();
    return v != 0;
}

/* The request goes to device memory when the CPU can store to it (a large
   BAR: hipDeviceAttributeIsLargeBar): the worker then polls its own HBM and
   the host's stores arrive as posted PCIe writes, ordered behind each other
   (tools/microbench/doorbell.hip: 1 KiB request + doorbell -> acknowledgement
   3.2 us vs 4.9-5.5 us polling host memory).  NOISE_AEAD_WORKER_VRAM=0 keeps
   it in host memory. */
bool vram_wanted(int dev)
{
    const char *e = getenv("NOISE_AEAD_WORKER_VRAM");
    if (e && e[0] == '0') return false;
    int large_bar = 0;
    return hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) == hipSuccess && large_bar;
}

int slot_setup(Worker &w, int dev)
{
    if (w.state) return w.state;
    w.state = -1;
    const size_t in_bytes = (size_t)WORKER_SPEC * 16, tail_bytes = WORKER_TAIL + 64;
    const size_t total = sizeof(WorkerSlot) + in_bytes + tail_bytes + WORKER_DATA;
    if (hipHostMalloc((void **)&w.slot, total, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return -1;
    memset(w.slot, 0, total); /* chunk stamps 0: no request has that number */
    if (hipHostGetDevicePointer((void **)&w.dslot, w.slot, 0) != hipSuccess) return -1;
    w.in = (uint4 *)(w.slot + 1);
    w.din = (uint4 *)(w.dslot + 1);
    w.tail = (uint8_t *)(w.in + WORKER_SPEC);
    w.dtail = (uint8_t *)(w.din + WORKER_SPEC);
    w.out = w.tail + tail_bytes;
    w.dout = w.dtail + tail_bytes;
    w.req = w.slot->c0;
    w.dreq = w.dslot->c0;
    /* device-memory request: 8 header chunks and the stop chunk (256 B), the
       stamped chunks, then the raw tail */
    const size_t vbytes = 256 + in_bytes + VWORKER_TAIL + 64;
    if (vram_wanted(dev) && hipExtMallocWithFlags(&w.vbase, vbytes, hipDeviceMallocFinegrained) == hipSuccess) {
        memset(w.vbase, 0, vbytes); /* through the BAR mapping */
        _mm_sfence();
        w.vram = true;
        w.req = (uint32_t *)w.vbase;
        w.dreq = (const uint32_t *)w.vbase;
        w.in = w.din = (uint4 *)((uint8_t *)w.vbase + 256);
        w.tail = w.dtail = (uint8_t *)(w.in + WORKER_SPEC);
    }
    w.state = 1;
    return 1;
}

/* (under g.mu) the group's stream, words and slots, once */
int group_setup(WorkerGroup &g, int dev)
{
    if (g.state) return g.state;
    g.state = -1;
    g.nslots = slots_per_group();
    for (int i = 0; i < g.nslots; ++i) {
        g.slot[i].g = &g;
        if (slot_setup(g.slot[i], dev) != 1) return -1;
    }
    void *vw = nullptr;
    if (g.slot[0].vram && hipExtMallocWithFlags(&vw, 256, hipDeviceMallocFinegrained) == hipSuccess) {
        memset(vw, 0, 256);
        _mm_sfence();
        g.words = g.dwords = (uint32_t *)vw;
        g.words_vram = true;
    } else {
        if (hipHostMalloc((void **)&g.words, 256, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return -1;
        memset(g.words, 0, 256);
        if (hipHostGetDevicePointer((void **)&g.dwords, g.words, 0) != hipSuccess) return -1;
    }
    if (worker_stream_prio() == 0) {
        if (hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking) != hipSuccess) return -1;
    } else {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return -1;
        if (hipStreamCreateWithPriority(&g.stream, hipStreamNonBlocking,
                                        worker_stream_prio() > 0 ? greatest : least) != hipSuccess)
            return -1;
    }
    std::call_once(g_atexit_once, [] { atexit(worker_stop_all); });
    g.state = 1;
    return 1;
}

/* NOISE_ERROR_NONE, or NOISE_ERROR_NOT_APPLICABLE (the caller takes the
   launch path; three failures in a row retire the group) */
/* Test hook: NOISE_AEAD_DEBUG_WORKER_FAIL=1 makes every worker launch fail
   (tests/test_gpu_worker.py: the calls must then take the launch path). */
bool debug_launch_fails()
{
    static const bool v = [] {
        const char *e = getenv("NOISE_AEAD_DEBUG_WORKER_FAIL");
        return e && e[0] == '1';
    }();
    return v;
}

/* Test hook: NOISE_AEAD_DEBUG_WORKER_LEAVE=1 makes the group leave after a
   call has checked it is up and before it posts its request, so the wait
   loop must relaunch it (the mid-wait relaunch of ADVICE r5,
   tests/worker_mode_check.py --relaunch-free). */
bool debug_leave_before_post()
{
    static const bool v = [] {
        const char *e = getenv("NOISE_AEAD_DEBUG_WORKER_LEAVE");
        return e && e[0] == '1';
    }();
    return v;
}

/* NOISE_AEAD_WORKER_PARK=0: batch launches leave the workers resident (the
   A/B of tests/test_gpu_worker.py's batch-beside-worker measurement). */
bool park_enabled()
{
    static const bool v = [] {
        const char *e = getenv("NOISE_AEAD_WORKER_PARK");
        return !(e && e[0] == '0');
    }();
    return v;
}

/* (under g.mu, by the caller of slot `own`, whose mu it holds) start the
   group once the kernel before it has left: every slot's exiting and stop
   cleared, the closing word cleared.  Each workgroup starts at its slot's
   `done`, so a request a leaving group did not take is served now. */
int group_launch(WorkerGroup &g, Worker &own)
{
    (void)hipStreamSynchronize(g.stream); /* the kernel before has left (all its workgroups) */
    if (debug_launch_fails()) {
        if (++g.launch_fails >= 3) g.state = -1;
        return NOISE_ERROR_NOT_APPLICABLE;
    }
    WorkerArgs a = {};
    for (int i = 0; i < g.nslots; ++i) {
        Worker &w = g.slot[i];
        __atomic_store_n(&w.slot->exiting, 0u, __ATOMIC_RELEASE);
        __atomic_store_n(stop_word(w), 0u, __ATOMIC_RELEASE);
        /* a fresh group caches nothing: the history restarts for slots not
           in a call (a slot in a call may be noting a context right now) */
        if (&w == &own) {
            __atomic_store_n(&w.ctx_n, 0u, __ATOMIC_RELEASE);
        } else {
            std::unique_lock<std::mutex> l(w.mu, std::try_to_lock);
            if (l.owns_lock()) __atomic_store_n(&w.ctx_n, 0u, __ATOMIC_RELEASE);
        }
        a.s[i].slot = w.dslot;
        a.s[i].req = w.dreq;
        a.s[i].in = (const uint4 *)w.din;
        a.s[i].tail = (const uint8_t *)w.dtail;
        a.s[i].out = w.dout;
        a.s[i].vram = w.vram ? 1u : 0u;
    }
    _mm_sfence();
    a.group = g.dwords;
    a.gen = __atomic_load_n(&g.gen, __ATOMIC_RELAXED) + 1u; /* never 0: the words start zeroed */
    a.nslots = (uint32_t)g.nslots;
    a.idle = idle_ticks();
    a.lifetime = LIFETIME_TICKS;
    hipLaunchKernelGGL(aead_worker, dim3(g.nslots), dim3(256), 0, g.stream, a);
    if (hipGetLastError() != hipSuccess) {
        if (++g.launch_fails >= 3) g.state = -1;
        return NOISE_ERROR_NOT_APPLICABLE;
    }
    g.launch_fails = 0;
    __atomic_add_fetch(&g.launches, 1u, __ATOMIC_RELAXED);
    __atomic_store_n(&g.launched, true, __ATOMIC_RELEASE);
    __atomic_add_fetch(&g.gen, 1u, __ATOMIC_RELEASE);
    return NOISE_ERROR_NONE;
}

/* (by the caller of slot w, holding w.mu) make sure w's group runs: gen0 is
   the group generation read BEFORE the caller saw it gone or leaving; if a
   relaunch happened since, there is nothing to do. */
std::atomic<uint32_t> g_dbg_ensure[4]; /* debug: group_ensure calls by cause (0 not launched, 1 exiting at the
                                          call, 2 exiting while waiting), 3 of them launched nothing */

int group_ensure(Worker &w, uint32_t gen0, int cause)
{
    WorkerGroup &g = *w.g;
    std::lock_guard<std::mutex> gl(g.mu);
    g_dbg_ensure[cause].fetch_add(1, std::memory_order_relaxed);
    if (g.state != 1) return NOISE_ERROR_NOT_APPLICABLE;
    if (__atomic_load_n(&g.gen, __ATOMIC_ACQUIRE) != gen0 && __atomic_load_n(&g.launched, __ATOMIC_ACQUIRE)) {
        g_dbg_ensure[3].fetch_add(1, std::memory_order_relaxed);
        return NOISE_ERROR_NONE;
    }
    return group_launch(g, w);
}

/* (holding w.mu) is w's group usable: recovered if drained, set up once */
bool group_usable(Worker &w, WorkerGroup &g, int dev)
{
    std::lock_guard<std::mutex> gl(g.mu);
    worker_recover(g);
    (void)w;
    return group_setup(g, dev) == 1;
}

/* slot n of the device's flattened order: spread over the groups first */
Worker &slot_n(int dev, int n)
{
    const int ng = groups_per_dev(), ns = slots_per_group();
    n %= ng * ns;
    WorkerGroup &g = g_group[dev][n % ng];
    return g.slot[(n / ng) % ns];
}

/* A usable slot of device dev, locked: this thread's own if free, else the
   first free one, else wait for this thread's own.  nullptr: none usable
   (set up failed on all of them). */
Worker *claim_worker(int dev, std::unique_lock<std::mutex> &lk)
{
    const int ng = groups_per_dev(), nw = ng * slots_per_group();
    if (t_pref < 0) t_pref = (int)(g_next_pref.fetch_add(1, std::memory_order_relaxed) % (uint32_t)nw);
    for (int pass = 0; pass < 2; ++pass)
        for (int i = 0; i < nw; ++i) {
            const int n = (t_pref + i) % nw;
            WorkerGroup &g = g_group[dev][n % ng];
            Worker &w = slot_n(dev, n);
            std::unique_lock<std::mutex> l(w.mu, std::defer_lock);
            if (pass == 0) {
                if (!l.try_lock()) continue;
            } else {
                l.lock();
            }
            if (!group_usable(w, g, dev)) continue;
            lk = std::move(l);
            return &w;
        }
    return nullptr;
}

int g_cus[kMaxDev]; /* compute units per device (0: not read yet) */

} // namespace


extern "C" NA_HIDDEN int na_worker_enabled(void) { return worker_enabled() ? 1 : 0; }

/* A batch launch of `workgroups` workgroups on the current device: when it
   fills every CU, the resident workers of the device are asked to leave
   first.  A worker holds ~151 KB of its CU's LDS, so a batch workgroup
   placed on that CU could not start until it left (2 ms after its last
   request): the batch kernels are single generations per CU (C2: two
   one-lane workgroups per CU, C3: one AES-GCM workgroup), and one CU short
   would run a second generation on another CU. */
NA_HIDDEN void worker_park_for_batch(uint32_t workgroups)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return;
    int cus = __atomic_load_n(&g_cus[dev], __ATOMIC_RELAXED);
    if (!cus) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            return;
        __atomic_store_n(&g_cus[dev], cus, __ATOMIC_RELAXED);
    }
    if (workgroups >= (uint32_t)cus && park_enabled()) park_device(dev);
}

/* A state's AES-GCM context (its pinned host copy h_ctx) is being freed:
   every worker that was sent it since its launch — and so may hold it in its
   LDS cache — leaves, scrubbing its LDS on the way out; the others stay. */
extern "C" NA_HIDDEN void na_worker_forget_ctx(const void *h_ctx)
{
    for (int d = 0; d < kMaxDev; ++d)
        for (int i = 0; i < kMaxGroups; ++i) {
            WorkerGroup &g = g_group[d][i];
            for (int k = 0; k < WORKER_MAX_SLOTS; ++k)
                if (worker_saw_ctx(g.slot[k], h_ctx)) {
                    park_group(g);
                    break;
                }
        }
}

namespace {

bool ct_env()
{
    static const bool v = [] {
        const char *e = getenv("NOISE_AEAD_CT_GHASH");
        return e && e[0] == '1';
    }();
    return v;
}

} // namespace

/* 16-byte chunk store: one aligned SSE store, which the x86-64 hosts of
   MI355X (AVX-capable) perform atomically, so the worker never sees half of
   a chunk; the sequence number in every chunk catches a torn header */
static inline void store_chunk(uint32_t *dst, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    _mm_store_si128((__m128i *)dst, _mm_set_epi32((int)d, (int)c, (int)b, (int)a));
}

/* One record through the resident worker: data holds len bytes (+ the tag
   for open) and receives CT || tag (seal) or, verified, the plaintext.  key:
   the raw ChaCha key; h_ctx / gen: AES-GCM, the pinned host copy of the
   state's context and the generation it was written at.  Returns
   NOISE_ERROR_NONE, _MAC_FAILURE, _SYSTEM, or _NOT_APPLICABLE (take the
   launch path). */
/* host-side phase times of the last request (ns, CLOCK_MONOTONIC): packed,
   doorbell written, done seen, returned — relative to the call's start */
static thread_local uint64_t t_host[4];
static inline uint64_t host_ns()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

extern "C" NA_HIDDEN int na_worker_crypt(int cipher_id, const uint8_t *key, const void *h_ctx,
                                         uint32_t gen, uint64_t nonce, const uint8_t *ad,
                                         size_t ad_len, uint8_t *data, size_t len, int open)
{
    const uint64_t h0 = host_ns();
    if (cipher_id == NOISE_CIPHER_AESGCM && !h_ctx) return NOISE_ERROR_NOT_APPLICABLE;
    if (!worker_enabled() || len > WORKER_MAX_LEN || ad_len > WORKER_MAX_AD)
        return NOISE_ERROR_NOT_APPLICABLE;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return NOISE_ERROR_NOT_APPLICABLE;
    std::unique_lock<std::mutex> lk;
    Worker *wp = claim_worker(dev, lk);
    if (!wp) return NOISE_ERROR_NOT_APPLICABLE;
    Worker &w = *wp;
    t_last = wp;
    void *d_hctx = nullptr;
    if (h_ctx && hipHostGetDevicePointer(&d_hctx, (void *)h_ctx, 0) != hipSuccess)
        return NOISE_ERROR_NOT_APPLICABLE;
    const size_t ad_pad = (ad_len + 15) & ~(size_t)15;
    WorkerSlot *s = w.slot;
    WorkerGroup &g = *w.g;
    {   /* the generation first, then launched / exiting (group_ensure) */
        const uint32_t gen0 = __atomic_load_n(&g.gen, __ATOMIC_ACQUIRE);
        const bool up = __atomic_load_n(&g.launched, __ATOMIC_ACQUIRE);
        if (!up || __atomic_load_n(&s->exiting, __ATOMIC_ACQUIRE)) {
            const int rc = group_ensure(w, gen0, up ? 1 : 0);
            if (rc) return rc; /* nothing posted yet */
        }
    }
    /* after the launch (which starts the history afresh): this context may
       now sit in the workgroup's LDS cache */
    if (h_ctx) worker_note_ctx(w, h_ctx);
    if (debug_leave_before_post()) { /* test hook: the group leaves before k is posted */
        park_group(g);
        const uint64_t t0 = host_ns();
        while ((!__atomic_load_n(&s->exiting, __ATOMIC_ACQUIRE) || hipStreamQuery(g.stream) != hipSuccess) &&
               host_ns() - t0 < 1000000000ull)
            __builtin_ia32_pause();
    }
    const uint32_t k = ++w.seq;
    /* the input stream key || AD || pad || record (|| tag): its first head
       bytes as stamped chunks, the rest raw.  Host memory: 12 stream bytes +
       k per chunk; device memory: {4 bytes, k, 4 bytes, k} */
    const size_t in_len = len + (open ? 16 : 0), total = 32 + ad_pad + in_len;
    const size_t cbytes = w.vram ? VCHUNK_BYTES : WCHUNK_BYTES;
    const size_t hmax = w.vram ? VWORKER_HEAD : WORKER_HEAD;
    const size_t head = total < hmax ? total : hmax;
    const size_t nchunks = (head + cbytes - 1) / cbytes;
    const __m128i keep = _mm_set_epi32(0, -1, -1, -1), stamp = _mm_set_epi32((int)k, 0, 0, 0);
    const __m128i kk = _mm_set1_epi32((int)k);
    const __m128i vstamp = _mm_set_epi32((int)k, 0, (int)k, 0); /* a scrubbed device chunk */
    alignas(16) uint8_t tmp[WORKER_HEAD + 16];
    memset(tmp, 0, 32 + ad_pad);
    if (cipher_id == NOISE_CIPHER_CHACHAPOLY) memcpy(tmp, key, 32);
    if (ad_len) memcpy(tmp + 32, ad, ad_len);
    memcpy(tmp + 32 + ad_pad, data, head - 32 - ad_pad);
    memset(tmp + head, 0, 16); /* the last chunk's bytes past the stream */
    if (w.vram) {
        for (size_t c = 0; c < nchunks; ++c) {
            const __m128i v = _mm_loadl_epi64((const __m128i *)(tmp + VCHUNK_BYTES * c));
            _mm_store_si128((__m128i *)(w.in + c), _mm_unpacklo_epi32(v, kk)); /* {b0, k, b1, k} */
        }
    } else {
        for (size_t c = 0; c < nchunks; ++c) {
            const __m128i v = _mm_loadu_si128((const __m128i *)(tmp + WCHUNK_BYTES * c));
            _mm_store_si128((__m128i *)(w.in + c), _mm_or_si128(_mm_and_si128(v, keep), stamp));
        }
    }
    explicit_bzero(tmp, head);
    if (total > head) memcpy(w.tail, data + (head - 32 - ad_pad), total - head);
    const uint64_t ctx = (uint64_t)(uintptr_t)d_hctx;
    const uint64_t h1 = host_ns();
    /* the data area before the header: sfence drains the write-combining
       buffers (device memory) and orders the stores (both) */
    _mm_sfence();
    __atomic_thread_fence(__ATOMIC_RELEASE);
    const uint32_t f[4][3] = {{(open ? 1u : 0u) | (ct_env() ? 1u << 8 : 0u), (uint32_t)len, (uint32_t)ad_len},
                              {(uint32_t)nonce, (uint32_t)(nonce >> 32), (uint32_t)cipher_id},
                              {(uint32_t)ctx, (uint32_t)(ctx >> 32), 0u},
                              {gen, 0u, 0u}};
    for (int c = 0; c < 4; ++c) {
        if (w.vram) { /* chunk 2c = {k, A, k, B}, 2c + 1 = {k, C, k, 0} */
            store_chunk(w.req + 8 * c, k, f[c][0], k, f[c][1]);
            store_chunk(w.req + 8 * c + 4, k, f[c][2], k, 0u);
        } else {
            store_chunk(w.req + 4 * c, k, f[c][0], f[c][1], f[c][2]);
        }
    }
    _mm_sfence(); /* out of the write-combining buffer now, not later */
    const uint64_t h2 = host_ns();
    /* From here on every exit scrubs the shared memory below.  A failure the
       worker caused (a relaunch that fails, a stale input, no answer within
       WAIT_LIMIT_NS) is NOISE_ERROR_NOT_APPLICABLE: the caller runs the
       record through the launch path with the same nonce instead — the result
       is the same bytes, and the worker only ever writes w.out and the slot. */
    int st = NOISE_ERROR_NONE;
    uint64_t spins = 0;
    while (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) != k) {
        __builtin_ia32_pause();
        if ((++spins & 1023) != 0) continue;
        const uint32_t gen0 = __atomic_load_n(&g.gen, __ATOMIC_ACQUIRE);
        if (__atomic_load_n(&s->exiting, __ATOMIC_ACQUIRE) && __atomic_load_n(&s->done, __ATOMIC_ACQUIRE) != k) {
            /* the group left before this slot took k: start it again (its
               workgroup starts at done = k - 1 and serves k) */
            const int rc = group_ensure(w, gen0, 2);
            if (rc) {
                st = rc;
                break;
            }
            /* a relaunch by group_launch starts this slot's context history
               afresh, and the new workgroup serves k and caches h_ctx: note it
               again, or freeing the state would not park this group and the
               round keys would stay in its LDS */
            if (h_ctx) worker_note_ctx(w, h_ctx);
        }
        if (host_ns() - h2 > WAIT_LIMIT_NS) { /* no answer: drained, then reused */
            worker_abandon(w, k);
            st = NOISE_ERROR_NOT_APPLICABLE;
            break;
        }
    }
    const uint64_t h3 = host_ns();
    if (st == NOISE_ERROR_NONE) {
        const uint32_t status = s->status;
        st = status == 2 ? NOISE_ERROR_NOT_APPLICABLE : (status ? NOISE_ERROR_MAC_FAILURE : NOISE_ERROR_NONE);
        if (st == NOISE_ERROR_NONE) memcpy(data, w.out, open ? len : len + 16);
    }
    /* key, plaintext and results out of the shared host memory; the stamps
       stay (a zeroed chunk would carry number 0, which no request has).  The
       worker writes its results in 16-B pieces: up to roundup16(len + 16). */
    for (size_t c = 0; c < nchunks; ++c) _mm_store_si128((__m128i *)(w.in + c), w.vram ? vstamp : stamp);
    if (total > head) explicit_bzero(w.tail, total - head);
    if (w.vram) _mm_sfence();
    explicit_bzero(w.out, (len + 16 + 15) & ~(size_t)15);
    const uint64_t h4 = host_ns();
    t_host[0] = h1 - h0; t_host[1] = h2 - h0; t_host[2] = h3 - h0; t_host[3] = h4 - h0;
    return st;
}

/* Test hook: the phase stamps of this thread's last worker request, in
   10-ns ticks relative to the moment the worker saw it: [0] fence done, [1]
   record and context in LDS, [2] computed, [3] results written, [4] release
   done; n = 5. */
extern "C" void noise_aead_debug_worker_stamps(uint32_t *out, int n)
{
    const WorkerSlot *s = t_last ? t_last->slot : nullptr;
    for (int i = 0; i < n && i < 5; ++i) out[i] = s ? s->stamps[i + 1] - s->stamps[0] : 0;
}

/* Test hook: this thread's last worker call on the host (ns from its
   start): request packed, doorbell written, done seen, returned. */
extern "C" void noise_aead_debug_worker_host_ns(uint64_t *out, int n)
{
    for (int i = 0; i < n && i < 4; ++i) out[i] = t_host[i];
}

/* Test hook: the latency-first path's s_memtime stamps (cycles from its
   start: ChaCha, CT in LDS, Poly blocks loaded, tree, tag, open's write). */
extern "C" void noise_aead_debug_worker_fast_stamps(uint32_t *out, int n)
{
    const WorkerSlot *s = t_last ? t_last->slot : nullptr;
    for (int i = 0; i < n && i < 8; ++i) out[i] = s ? s->fstamps[i] : 0;
}

/* Test hook: the placement of this thread's last worker: 0 none set up, 1
   requests in pinned host memory, 2 in device memory. */
extern "C" int noise_aead_debug_worker_placement(void)
{
    const Worker *w = t_last;
    return !w || w->state != 1 || !w->g || w->g->state != 1 ? 0 : (w->vram ? 2 : 1);
}

/* Test hook: request slots of the current device whose group is resident
   (each slot is one workgroup of its group's kernel). */
extern "C" int noise_aead_debug_workers_resident(void)
{
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return -1;
    for (int i = 0; i < kMaxGroups; ++i) {
        WorkerGroup &g = g_group[dev][i];
        std::lock_guard<std::mutex> lk(g.mu);
        if (g.state == 1 && g.launched && hipStreamQuery(g.stream) == hipErrorNotReady) n += g.nslots;
    }
    return n;
}

/* Test hook: worker kernels launched on the current device so far (a
   parked worker that is called again is relaunched). */
extern "C" unsigned noise_aead_debug_worker_launches(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    unsigned n = 0;
    for (int i = 0; i < kMaxGroups; ++i) n += __atomic_load_n(&g_group[dev][i].launches, __ATOMIC_RELAXED);
    return n;
}

/* Test hook: per group of the current device, kernels launched (out[0..n)
   for groups 0..n-1), then the group_ensure counts by cause (debug). */
extern "C" unsigned noise_aead_debug_worker_leave_reason(int group, int slot)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev || group < 0 || group >= kMaxGroups ||
        slot < 0 || slot >= WORKER_MAX_SLOTS || !g_group[dev][group].slot[slot].slot)
        return 0;
    return g_group[dev][group].slot[slot].slot->stamps[7];
}

extern "C" void noise_aead_debug_worker_leave_info(int group, int slot, unsigned *out)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev || group < 0 || group >= kMaxGroups ||
        slot < 0 || slot >= WORKER_MAX_SLOTS || !g_group[dev][group].slot[slot].slot)
        return;
    for (int i = 0; i < 4; ++i) out[i] = g_group[dev][group].slot[slot].slot->leave[i];
}

extern "C" void noise_aead_debug_worker_group_launches(unsigned *out, int n)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return;
    for (int i = 0; i < n; ++i)
        out[i] = i < kMaxGroups ? __atomic_load_n(&g_group[dev][i].launches, __ATOMIC_RELAXED)
                                : (i - kMaxGroups < 4 ? g_dbg_ensure[i - kMaxGroups].load() : 0u);
}

/* Test hook: the shader clock (MHz) of the last worker request's compute
   phase (s_memtime cycles over s_memrealtime time). */
extern "C" double noise_aead_debug_worker_clock_mhz(void)
{
    const WorkerSlot *s = t_last ? t_last->slot : nullptr;
    if (!s || s->stamps[3] == s->stamps[2]) return 0.0;
    return (double)s->stamps[6] / ((double)(s->stamps[3] - s->stamps[2]) * 0.01);
}

} // namespace na
