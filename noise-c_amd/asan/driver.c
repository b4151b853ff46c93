/*
 * driver.c — SANITIZER TEST HARNESS ONLY (make -C noise-c_amd asan).
 *
 * Drives the host front end (cipherstate.c, wire.c, host_pool.c, errors.c),
 * built with -fsanitize=address,undefined over the CPU stubs, through the
 * public API: single calls, batches (mixed states and ciphers, AD, bad
 * lengths, nonce exhaustion, MAC failures and a run of forged records),
 * a batch larger than several pipeline chunks, and the wire paths (pageable
 * and pinned buffers, a tampered frame, a partial trailing frame).  Every
 * result is compared with the sequential semantics of the reference's
 * cipherstate.c:293-410 computed record by record with the oracle.  Any
 * sanitizer report aborts the run (-fno-sanitize-recover=all).
 */
#include "noise_aead_hip.h"
#include "noise_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);              \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

static uint64_t g_rng = 12345;
static uint32_t rnd(void) { return (uint32_t)oracle_splitmix64(g_rng++); }
static void fill(uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)rnd();
}

/* n of a state: the u64 at offset 16 of struct NoiseCipherState_s */
static uint64_t nonce_of(NoiseCipherState *st) { return *(uint64_t *)((uint8_t *)st + 16); }

typedef struct {
    int cipher, has_key;
    uint8_t key[32];
    uint64_t n;
} Model;

static NoiseCipherState *make_state(Model *m, int cipher, int keyed, uint64_t n0)
{
    NoiseCipherState *st;
    CHECK(noise_cipherstate_new_by_id(&st, cipher) == NOISE_ERROR_NONE);
    m->cipher = cipher;
    m->has_key = keyed;
    m->n = 0;
    if (keyed) {
        fill(m->key, 32);
        CHECK(noise_cipherstate_init_key(st, m->key, 32) == NOISE_ERROR_NONE);
        CHECK(noise_cipherstate_set_nonce(st, n0) == NOISE_ERROR_NONE);
        m->n = n0;
    }
    return st;
}

/* cipherstate.c:293-333 on the model; returns the code, updates buf/size */
static int model_encrypt(Model *m, const uint8_t *ad, size_t ad_len, uint8_t *data, size_t *size,
                         size_t max_size)
{
    if (*size > max_size) return NOISE_ERROR_INVALID_LENGTH;
    if (!m->has_key) return *size > 65535 ? NOISE_ERROR_INVALID_LENGTH : NOISE_ERROR_NONE;
    if (*size > 65535 - 16 || max_size - *size < 16) return NOISE_ERROR_INVALID_LENGTH;
    if (m->n == UINT64_MAX) return NOISE_ERROR_INVALID_NONCE;
    oracle_aead_encrypt(m->cipher, m->key, m->n++, ad, ad_len, data, *size);
    *size += 16;
    return NOISE_ERROR_NONE;
}

/* cipherstate.c:373-410 */
static int model_decrypt(Model *m, const uint8_t *ad, size_t ad_len, uint8_t *data, size_t *size,
                         size_t max_size)
{
    if (*size > max_size || *size > 65535) return NOISE_ERROR_INVALID_LENGTH;
    if (!m->has_key) return NOISE_ERROR_NONE;
    if (*size < 16) return NOISE_ERROR_INVALID_LENGTH;
    if (m->n == UINT64_MAX) return NOISE_ERROR_INVALID_NONCE;
    if (oracle_aead_decrypt(m->cipher, m->key, m->n, ad, ad_len, data, *size - 16))
        return NOISE_ERROR_MAC_FAILURE;
    ++m->n;
    *size -= 16;
    return NOISE_ERROR_NONE;
}

static void test_single(void)
{
    static const size_t lens[] = {0, 1, 15, 16, 17, 63, 64, 65, 1400, 4097, 65519};
    for (int c = 0; c < 2; ++c) {
        Model m;
        NoiseCipherState *st = make_state(&m, c ? NOISE_CIPHER_AESGCM : NOISE_CIPHER_CHACHAPOLY, 1, 5);
        for (size_t k = 0; k < sizeof(lens) / sizeof(lens[0]); ++k) {
            const size_t L = lens[k];
            uint8_t *a = (uint8_t *)malloc(L + 16), *b = (uint8_t *)malloc(L + 16);
            uint8_t ad[13];
            fill(a, L);
            fill(ad, sizeof ad);
            memcpy(b, a, L);
            NoiseBuffer buf;
            noise_buffer_set_inout(buf, a, L, L + 16);
            size_t sz = L;
            CHECK(noise_cipherstate_encrypt_with_ad(st, ad, sizeof ad, &buf) ==
                  model_encrypt(&m, ad, sizeof ad, b, &sz, L + 16));
            CHECK(buf.size == sz && !memcmp(a, b, sz) && nonce_of(st) == m.n);
            /* tamper: MAC failure, buffer and n untouched */
            NoiseCipherState *rx;
            Model mr = m;
            mr.n = m.n - 1;
            CHECK(noise_cipherstate_new_by_id(&rx, m.cipher) == 0);
            CHECK(noise_cipherstate_init_key(rx, m.key, 32) == 0);
            CHECK(noise_cipherstate_set_nonce(rx, mr.n) == 0);
            a[L / 2] ^= 4;
            memcpy(b, a, L + 16);
            noise_buffer_set_input(buf, a, L + 16);
            CHECK(noise_cipherstate_decrypt_with_ad(rx, ad, sizeof ad, &buf) == NOISE_ERROR_MAC_FAILURE);
            CHECK(!memcmp(a, b, L + 16) && nonce_of(rx) == mr.n);
            a[L / 2] ^= 4;
            sz = L + 16;
            memcpy(b, a, L + 16);
            CHECK(noise_cipherstate_decrypt_with_ad(rx, ad, sizeof ad, &buf) ==
                  model_decrypt(&mr, ad, sizeof ad, b, &sz, L + 16));
            CHECK(buf.size == L && !memcmp(a, b, L) && nonce_of(rx) == mr.n);
            noise_cipherstate_free(rx);
            free(a);
            free(b);
        }
        noise_cipherstate_free(st);
    }
}

#define NS 6
static void test_batch(size_t count, size_t max_len, int forged_run)
{
    Model m[NS], md[NS];
    NoiseCipherState *st[NS], *sd[NS];
    for (int s = 0; s < NS; ++s) {
        int cipher = s % 2 ? NOISE_CIPHER_AESGCM : NOISE_CIPHER_CHACHAPOLY;
        st[s] = make_state(&m[s], cipher, s != 5, s == 4 ? UINT64_MAX - 3 : rnd() % 1000);
    }
    NoiseCipherState **rs = (NoiseCipherState **)malloc(count * sizeof *rs);
    NoiseBuffer *bufs = (NoiseBuffer *)malloc(count * sizeof *bufs);
    uint8_t **mem = (uint8_t **)malloc(count * sizeof *mem), **exp = (uint8_t **)malloc(count * sizeof *exp);
    uint8_t **ads = (uint8_t **)malloc(count * sizeof *ads);
    size_t *ad_lens = (size_t *)malloc(count * sizeof *ad_lens), *max = (size_t *)malloc(count * sizeof *max);
    size_t *esz = (size_t *)malloc(count * sizeof *esz);
    int *res = (int *)malloc(count * sizeof *res), *eres = (int *)malloc(count * sizeof *eres);
    int *sidx = (int *)malloc(count * sizeof *sidx);
    for (size_t i = 0; i < count; ++i) {
        int s = forged_run ? 0 : (int)(rnd() % NS);
        size_t L = rnd() % (max_len + 1);
        if (!forged_run && rnd() % 40 == 0) L = 65535 - 16 + (rnd() % 2); /* max and max+1 */
        size_t mx = rnd() % 10 == 0 ? L + 3 : L + 16;
        sidx[i] = s;
        rs[i] = st[s];
        mem[i] = (uint8_t *)malloc(mx ? mx : 1);
        exp[i] = (uint8_t *)malloc(mx ? mx : 1);
        fill(mem[i], mx);
        memcpy(exp[i], mem[i], mx);
        max[i] = mx;
        ad_lens[i] = rnd() % 3 == 0 ? 1 + rnd() % 40 : 0;
        ads[i] = (uint8_t *)malloc(ad_lens[i] + 1);
        fill(ads[i], ad_lens[i]);
        noise_buffer_set_inout(bufs[i], mem[i], L, mx);
        esz[i] = L;
        eres[i] = model_encrypt(&m[s], ads[i], ad_lens[i], exp[i], &esz[i], mx);
    }
    CHECK(noise_cipherstate_encrypt_batch(rs, (const uint8_t *const *)ads, ad_lens, bufs, count, res) == 0);
    for (size_t i = 0; i < count; ++i) {
        CHECK(res[i] == eres[i]);
        CHECK(bufs[i].size == esz[i] && !memcmp(mem[i], exp[i], max[i]));
    }
    for (int s = 0; s < NS; ++s) CHECK(nonce_of(st[s]) == m[s].n);
    /* decrypt with fresh receive states: a few corrupt records, and with
       forged_run a long run of forged records on one state */
    for (int s = 0; s < NS; ++s) {
        sd[s] = make_state(&md[s], m[s].cipher, m[s].has_key, 0);
        if (m[s].has_key) {
            memcpy(md[s].key, m[s].key, 32);
            CHECK(noise_cipherstate_init_key(sd[s], md[s].key, 32) == 0);
        }
    }
    /* receive nonces: the sender's starting nonce of each state */
    for (size_t i = 0; i < count; ++i) {
        int s = sidx[i];
        rs[i] = sd[s];
        if (forged_run ? (i >= count / 4 && i < count / 2) : rnd() % 17 == 0)
            if (bufs[i].size) mem[i][rnd() % bufs[i].size] ^= 1;
        memcpy(exp[i], mem[i], max[i]);
        esz[i] = bufs[i].size;
    }
    {
        /* each receive state starts at its sender's first nonce */
        uint64_t n0[NS];
        for (int s = 0; s < NS; ++s) n0[s] = nonce_of(st[s]);
        for (size_t i = 0; i < count; ++i)
            if (eres[i] == NOISE_ERROR_NONE && m[sidx[i]].has_key) --n0[sidx[i]];
        for (int s = 0; s < NS; ++s) {
            md[s].n = n0[s];
            if (m[s].has_key) CHECK(noise_cipherstate_set_nonce(sd[s], n0[s]) == 0);
        }
    }
    for (size_t i = 0; i < count; ++i) {
        eres[i] = model_decrypt(&md[sidx[i]], ads[i], ad_lens[i], exp[i], &esz[i], max[i]);
        noise_buffer_set_inout(bufs[i], mem[i], bufs[i].size, max[i]);
    }
    CHECK(noise_cipherstate_decrypt_batch(rs, (const uint8_t *const *)ads, ad_lens, bufs, count, res) == 0);
    for (size_t i = 0; i < count; ++i) {
        CHECK(res[i] == eres[i]);
        CHECK(bufs[i].size == esz[i] && !memcmp(mem[i], exp[i], max[i]));
    }
    for (int s = 0; s < NS; ++s) CHECK(nonce_of(sd[s]) == md[s].n);
    if (forged_run) {
        uint64_t rounds, disp;
        noise_aead_debug_batch_stats(&rounds, &disp);
        CHECK(disp <= 3 * count);
    }
    for (size_t i = 0; i < count; ++i) {
        free(mem[i]);
        free(exp[i]);
        free(ads[i]);
    }
    for (int s = 0; s < NS; ++s) {
        noise_cipherstate_free(st[s]);
        noise_cipherstate_free(sd[s]);
    }
    free(rs); free(bufs); free(mem); free(exp); free(ads); free(ad_lens); free(max); free(esz);
    free(res); free(eres); free(sidx);
}

/* frames of examples/echo: 2-byte BE length || body */
static size_t build_frames(uint8_t *w, size_t nframes, size_t max_len, size_t *lens)
{
    size_t off = 0;
    for (size_t f = 0; f < nframes; ++f) {
        size_t L = rnd() % (max_len + 1);
        lens[f] = L;
        w[off] = (uint8_t)((L + 16) >> 8);
        w[off + 1] = (uint8_t)(L + 16);
        fill(w + off + 2, L);
        memset(w + off + 2 + L, 0, 16);
        off += 2 + L + 16;
    }
    return off;
}

static void test_wire(int pinned)
{
    enum { NF = 400 };
    size_t lens[NF];
    const size_t cap = NF * (2 + 3000 + 16) + 64;
    uint8_t *w = pinned ? (uint8_t *)noise_wire_alloc(cap) : (uint8_t *)malloc(cap);
    uint8_t *ref = (uint8_t *)malloc(cap);
    CHECK(w && ref);
    const size_t total = build_frames(w, NF, 3000, lens);
    memcpy(ref, w, total);
    Model ma, mb;
    NoiseCipherState *a = make_state(&ma, NOISE_CIPHER_CHACHAPOLY, 1, 7);
    NoiseCipherState *b = make_state(&mb, NOISE_CIPHER_AESGCM, 1, 9);
    size_t consumed, frames;
    /* seal, with a partial frame at the end */
    CHECK(noise_wire_seal(a, w, total - 5, &consumed, &frames) == 0);
    CHECK(frames == NF - 1);
    for (size_t f = 0, off = 0; f < NF - 1; ++f) {
        size_t sz = lens[f];
        CHECK(model_encrypt(&ma, NULL, 0, ref + off + 2, &sz, lens[f] + 16) == 0);
        off += 2 + lens[f] + 16;
    }
    CHECK(!memcmp(w, ref, consumed) && nonce_of(a) == ma.n);
    /* echo: open with a's receive side, seal with b */
    Model mra = ma;
    NoiseCipherState *ra;
    CHECK(noise_cipherstate_new_by_id(&ra, NOISE_CIPHER_CHACHAPOLY) == 0);
    CHECK(noise_cipherstate_init_key(ra, ma.key, 32) == 0);
    mra.n = 7;
    CHECK(noise_cipherstate_set_nonce(ra, 7) == 0);
    /* tamper frame 250: processing stops there */
    size_t off250 = 0;
    for (size_t f = 0; f < 250; ++f) off250 += 2 + lens[f] + 16;
    w[off250 + 2 + lens[250] / 2] ^= 0x20;
    memcpy(ref, w, total);
    CHECK(noise_wire_echo(ra, b, w, consumed, &consumed, &frames) == NOISE_ERROR_MAC_FAILURE);
    CHECK(frames == 250);
    for (size_t f = 0, off = 0; f < 250; ++f) {
        size_t sz = lens[f] + 16;
        CHECK(model_decrypt(&mra, NULL, 0, ref + off + 2, &sz, lens[f] + 16) == 0);
        sz = lens[f];
        CHECK(model_encrypt(&mb, NULL, 0, ref + off + 2, &sz, lens[f] + 16) == 0);
        off += 2 + lens[f] + 16;
    }
    CHECK(!memcmp(w, ref, total) && nonce_of(ra) == mra.n && nonce_of(b) == mb.n);
    noise_cipherstate_free(a);
    noise_cipherstate_free(b);
    noise_cipherstate_free(ra);
    if (pinned) noise_wire_free(w);
    else free(w);
    free(ref);
}

int main(void)
{
    test_single();
    test_batch(300, 5000, 0);
    test_batch(200, 600, 1);
    test_batch(1000, 9000, 0); /* > 4 MiB: several pipeline chunks */
    test_wire(0);
    test_wire(1);
    char buf[32];
    CHECK(noise_strerror(NOISE_ERROR_MAC_FAILURE, buf, sizeof buf) == 0 && !strcmp(buf, "MAC failure"));
    printf("asan driver ok\n");
    return 0;
}
