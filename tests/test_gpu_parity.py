"""GPU parity: the gfx950 kernels, called through the C ABI, against the oracle.

Bit-exact comparisons (integer/byte work): every ciphertext byte and tag must
equal the CPU oracle's (oracle/noise_oracle.c, itself pinned to the reference
by tests/test_oracle.py), and every decrypt must reproduce the reference's
accept/reject decision.  A rejected record is left untouched when opened in
place (the reference verifies before it decrypts); opened out of place, its
output is never written by an AES-GCM open or a NOISE_AEAD_FLAG_VERIFY_FIRST
one (both verify first) and zeroed by a one-pass ChaChaPoly open
(scrub_rejected: never unauthenticated plaintext).
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHACHA, AES = 0x4301, 0x4302
NONCE_MAX = 2**64 - 1


def _torch():
    import torch
    return torch


def dev(arr):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(arr)).to("cuda")


def stream():
    return _torch().cuda.current_stream().cuda_stream


def sync():
    _torch().cuda.synchronize()


# NOISE_AEAD_FLAG_*: verify-first is the default open order (round 6);
# ONE_PASS opts a ChaChaPoly FAST open into decrypt-while-authenticating
FLAG_CT_GHASH, FLAG_VERIFY_FIRST, FLAG_ONE_PASS = 2, 4, 8


def prepare(aead, cipher, keys):
    torch = _torch()
    keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, 32)
    d_keys = dev(keys.reshape(-1))
    ctx = torch.empty(keys.shape[0] * aead.dev_ctx_bytes(cipher), dtype=torch.uint8, device="cuda")
    assert aead.dev_prepare(cipher, d_keys.data_ptr(), keys.shape[0], ctx.data_ptr(), stream()) == 0
    return ctx, d_keys


def gpu_uniform(aead, open_, cipher, keys, nonce_base, rps, inp, in_stride, length, count,
                out_stride, lanes=0, ad=None, ad_stride=0, ad_len=0, out_init=0xA5, out=None,
                flags=0):
    torch = _torch()
    ctx, _k = prepare(aead, cipher, keys)
    d_nb = dev(np.asarray(nonce_base, dtype=np.uint64).view(np.int64))
    d_in = dev(inp)
    if out is None:
        d_out = torch.full((count * out_stride + 64,), out_init, dtype=torch.uint8, device="cuda")
    else:
        d_out = out
    d_st = torch.full((max(1, count),), 7, dtype=torch.uint8, device="cuda")
    d_ad = dev(ad) if ad is not None else None
    rc = aead.dev_uniform(open_, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                          inp=d_in.data_ptr(), out=d_out.data_ptr(), in_stride=in_stride,
                          out_stride=out_stride, length=length, n_records=count,
                          recs_per_state=rps, status=d_st.data_ptr(),
                          ad=d_ad.data_ptr() if d_ad is not None else 0, ad_stride=ad_stride,
                          ad_len=ad_len, lanes=lanes, flags=flags, stream=stream())
    assert rc == 0, hex(rc)
    sync()
    return d_out.cpu().numpy(), d_st.cpu().numpy()[:count]


def rejected_fill(cipher, out_init, flags=0):
    """What a rejected record's output holds after an out-of-place open:
    untouched (its prior fill) when the open verified first — every open by
    default since round 6 (aead_api.hip open_vf; every AES-GCM open always)
    — and zeroed after a ChaChaPoly open that opted into
    NOISE_AEAD_FLAG_ONE_PASS (VERIFY_FIRST overrides it)."""
    return 0 if (cipher == CHACHA and flags & FLAG_ONE_PASS and not flags & FLAG_VERIFY_FIRST) else out_init


def oracle_seal_records(oracle, cipher, keys, nonce_base, rps, pt, in_stride, length, count,
                        out_stride, ad=None, ad_stride=0, ad_len=0):
    out = np.full(count * out_stride + 64, 0xA5, dtype=np.uint8)
    for i in range(count):
        s = i // rps
        p = bytes(pt[i * in_stride: i * in_stride + length])
        a = bytes(ad[i * ad_stride: i * ad_stride + ad_len]) if ad_len else b""
        ct = oracle.encrypt(cipher, bytes(keys[s]), int(nonce_base[s]) + i % rps, p, a)
        out[i * out_stride: i * out_stride + length + 16] = np.frombuffer(ct, dtype=np.uint8)
    return out


# ------------------------------------------------------------------ KATs

def test_kat_through_device_api(aead, gpu, golden):
    kat, _ = golden
    for v in kat["vectors"]:
        key = np.frombuffer(bytes.fromhex(v["key"]), dtype=np.uint8).reshape(1, 32)
        pt = bytes.fromhex(v["pt"])
        ad = bytes.fromhex(v["ad"])
        L = len(pt)
        inp = np.frombuffer(pt + bytes(16), dtype=np.uint8)
        adv = np.frombuffer(ad or b"\0", dtype=np.uint8)
        out, _ = gpu_uniform(aead, False, v["cipher"], key, [v["nonce"]], 1, inp, L + 16, L, 1,
                             L + 16, ad=adv, ad_stride=len(ad), ad_len=len(ad))
        assert bytes(out[:L + 16]).hex() == v["ct"] + v["tag"], v["name"]
        back, st = gpu_uniform(aead, True, v["cipher"], key, [v["nonce"]], 1, out[:L + 16],
                               L + 16, L, 1, L + 16, ad=adv, ad_stride=len(ad), ad_len=len(ad))
        assert st[0] == 0 and bytes(back[:L]) == pt, v["name"]


# --------------------------------------------------- uniform vs the oracle

LENS = [0, 1, 15, 16, 17, 48, 56, 63, 64, 65, 127, 128, 129, 191, 192, 255, 256, 257,
        1023, 1400, 1401, 4096, 5000]


@pytest.mark.parametrize("cipher,lanes", [(CHACHA, 1), (CHACHA, 2), (CHACHA, 4), (CHACHA, 8),
                                          (CHACHA, 16), (CHACHA, 32), (CHACHA, 64), (AES, 0)])
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("rps", [13, 16])
def test_uniform_seal_open_vs_oracle(aead, gpu, oracle, cipher, lanes, packed, rps):
    """rps=13: states straddle waves; rps=16: every 4/8-lane wave holds one
    state (the wave-uniform-key kernels), the last wave partial.  The rps=13
    opens opt into NOISE_AEAD_FLAG_ONE_PASS, the rps=16 ones take the default
    (verify-first) order."""
    rng = np.random.default_rng(1000 + lanes + 7 * packed + (cipher & 3) + rps)
    oflags = FLAG_ONE_PASS if rps == 13 else 0
    for L in LENS:
        count = 37 if rps == 13 else 70  # the last state partial
        S = (count + rps - 1) // rps
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        nb = rng.integers(0, 2**63, S, dtype=np.uint64) * 2
        in_stride = L if packed else (L + 15) // 16 * 16 + 16
        out_stride = L + 16 if packed else (L + 16 + 15) // 16 * 16
        pt = rng.integers(0, 256, count * in_stride + 16, dtype=np.uint8)
        exp = oracle_seal_records(oracle, cipher, keys, nb, rps, pt, in_stride, L, count, out_stride)
        got, _ = gpu_uniform(aead, False, cipher, keys, nb, rps, pt, in_stride, L, count,
                             out_stride, lanes=lanes)
        assert np.array_equal(got, exp), f"seal mismatch len={L}"
        # open it back; tamper with a few records
        ct = got.copy()
        bad = sorted(set(rng.integers(0, count, 5).tolist()))
        for b in bad:
            pos = b * out_stride + int(rng.integers(0, L + 16))
            ct[pos] ^= 1 << int(rng.integers(0, 8))
        back, st = gpu_uniform(aead, True, cipher, keys, nb, rps, ct, out_stride, L, count,
                               in_stride, lanes=lanes, out_init=0x5A, flags=oflags)
        for i in range(count):
            seg = back[i * in_stride: i * in_stride + L]
            if i in bad:
                assert st[i] == 1, f"tamper not detected len={L} rec={i}"
                assert np.all(seg == rejected_fill(cipher, 0x5A, oflags)), "rejected record's output"
            else:
                assert st[i] == 0, f"valid record rejected len={L} rec={i}"
                assert np.array_equal(seg, pt[i * in_stride: i * in_stride + L])


@pytest.mark.parametrize("cipher,lanes", [(CHACHA, 0), (CHACHA, 1), (CHACHA, 4), (AES, 0)])
@pytest.mark.parametrize("oflags", [0, FLAG_ONE_PASS])
def test_uniform_staged_kernels(aead, gpu, oracle, cipher, lanes, oflags):
    """FAST layouts with one state per 256 records: the LDS-staged kernels
    (ChaChaPoly wave-uniform key at one and four lanes per record, AESGCM
    replicated T-tables) on a batch whose last workgroup is partial, every
    record vs the oracle, with AD; opens in the default (verify-first) order
    and with NOISE_AEAD_FLAG_ONE_PASS."""
    rng = np.random.default_rng(4242 + (cipher & 3) + 100 * lanes + oflags)
    rps, count = 256, 600
    S = (count + rps - 1) // rps
    for L, adl in [(0, 0), (1, 0), (15, 0), (16, 0), (17, 0), (100, 0), (1400, 0), (1401, 0),
                   (4096, 0), (1400, 13), (64, 32)]:
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        nb = rng.integers(0, 2**62, S, dtype=np.uint64)
        in_stride = (max(L, 1) + 63) // 64 * 64
        out_stride = (L + 16 + 63) // 64 * 64
        pt = rng.integers(0, 256, count * in_stride + 64, dtype=np.uint8)
        ad = rng.integers(0, 256, count * 48 + 64, dtype=np.uint8)
        kw = dict(ad=ad, ad_stride=48, ad_len=adl) if adl else {}
        exp = oracle_seal_records(oracle, cipher, keys, nb, rps, pt, in_stride, L, count,
                                  out_stride, **kw)
        got, _ = gpu_uniform(aead, False, cipher, keys, nb, rps, pt, in_stride, L, count,
                             out_stride, lanes=lanes, **kw)
        assert np.array_equal(got[:count * out_stride], exp[:count * out_stride]), f"len={L} ad={adl}"
        ct = got.copy()
        bad = sorted(set(int(x) for x in rng.integers(0, count, 7)))
        for b in bad:
            ct[b * out_stride + int(rng.integers(0, L + 16))] ^= 0x80
        back, st = gpu_uniform(aead, True, cipher, keys, nb, rps, ct, out_stride, L, count,
                               in_stride, out_init=0x3C, lanes=lanes, flags=oflags, **kw)
        for i in range(count):
            seg = back[i * in_stride: i * in_stride + L]
            if i in bad:
                assert st[i] == 1 and np.all(seg == rejected_fill(cipher, 0x3C, oflags)), f"len={L} rec={i}"
            else:
                assert st[i] == 0, f"len={L} rec={i}"
                assert np.array_equal(seg, pt[i * in_stride: i * in_stride + L]), f"len={L} rec={i}"


@pytest.mark.parametrize("cipher,lanes,rps,adl", [(CHACHA, 4, 256, 0), (CHACHA, 4, 13, 0),
                                                  (CHACHA, 8, 256, 0), (CHACHA, 8, 13, 0),
                                                  (CHACHA, 1, 16, 0), (CHACHA, 1, 256, 0),
                                                  (CHACHA, 1, 64, 21), (AES, 0, 256, 0),
                                                  (AES, 0, 13, 0), (CHACHA, 4, 256, 21),
                                                  (AES, 0, 256, 21)])
@pytest.mark.parametrize("oflags", [0, FLAG_ONE_PASS])
def test_open_in_place_rejects_leave_ciphertext(aead, gpu, oracle, cipher, lanes, rps, adl, oflags):
    """Open in place (in == out, one stride): every verified record becomes
    its plaintext and every rejected one reads exactly as given — CT and tag
    bytes — in the default (verify-first) order and in the single-pass
    ChaChaPoly kernels (NOISE_AEAD_FLAG_ONE_PASS), which write plaintext
    before the verdict and re-encrypt on failure; with and without associated
    data."""
    torch = _torch()
    rng = np.random.default_rng(808 + lanes + rps + (cipher & 3) + adl + oflags)
    for L, count in [(1400, 700), (0, 70), (17, 300), (4096, 40), (100, 257)]:
        S = (count + rps - 1) // rps
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        nb = rng.integers(0, 2**62, S, dtype=np.uint64)
        stride_ = (L + 16 + 63) // 64 * 64
        pt = rng.integers(0, 256, count * stride_ + 64, dtype=np.uint8)
        ad = rng.integers(0, 256, count * 32 + 64, dtype=np.uint8)
        akw = dict(ad=ad, ad_stride=32, ad_len=adl) if adl else {}
        ct = oracle_seal_records(oracle, cipher, keys, nb, rps, pt, stride_, L, count, stride_, **akw)
        bad = sorted(set(int(x) for x in rng.integers(0, count, 9)))
        for b in bad:
            ct[b * stride_ + int(rng.integers(0, L + 16))] ^= 0x21
        ctx, _k = prepare(aead, cipher, keys)
        d_nb = dev(nb.view(np.int64))
        d_buf = dev(ct)
        d_ad = dev(ad)
        d_st = torch.full((count,), 7, dtype=torch.uint8, device="cuda")
        assert aead.dev_uniform(True, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                                inp=d_buf.data_ptr(), out=d_buf.data_ptr(), in_stride=stride_,
                                out_stride=stride_, length=L, n_records=count, recs_per_state=rps,
                                status=d_st.data_ptr(), lanes=lanes, stream=stream(),
                                ad=d_ad.data_ptr() if adl else 0, ad_stride=32 if adl else 0,
                                ad_len=adl, flags=oflags) == 0
        sync()
        back, st = d_buf.cpu().numpy(), d_st.cpu().numpy()
        for i in range(count):
            o = i * stride_
            if i in bad:
                assert st[i] == 1 and np.array_equal(back[o:o + L + 16], ct[o:o + L + 16]), (L, i)
            else:
                assert st[i] == 0 and np.array_equal(back[o:o + L], pt[o:o + L]), (L, i)


DUPLEX_CASES = [((1400, 700, 350), (1400, 300, 100)), ((100, 64, 16), (1401, 513, 513)),
                ((0, 33, 16), (65, 1000, 16)), ((4096, 5, 5), (17, 0, 1))]
# one state per 256 records (the AES duplex kernel, the bench's wave-uniform
# keys) at the bench's 128-B record slots, last workgroup partial
SLOT_CASES = [((1400, 1024, 512), (1400, 768, 256)), ((1400, 512, 256), (1024, 2048, 1024)),
              ((1, 256, 256), (1400, 300, 256)), ((1400, 1000, 256), (4096, 256, 256))]


@pytest.mark.parametrize("cipher,lanes,layout,flags", [
    (CHACHA, 4, "fast", FLAG_ONE_PASS), (CHACHA, 8, "fast", FLAG_ONE_PASS), (CHACHA, 4, "packed", 0),
    (AES, 0, "fast", 0), (CHACHA, 1, "fast", FLAG_ONE_PASS), (CHACHA, 1, "slot128", FLAG_ONE_PASS),
    (CHACHA, 0, "slot128", FLAG_ONE_PASS), (CHACHA, 4, "slot128", FLAG_ONE_PASS),
    (CHACHA, 8, "slot128", FLAG_ONE_PASS), (AES, 0, "slot128", 0),
    (AES, 0, "slot128", FLAG_CT_GHASH), (CHACHA, 4, "slot128", FLAG_VERIFY_FIRST),
    (AES, 0, "slot128", FLAG_VERIFY_FIRST), (CHACHA, 1, "slot128", FLAG_VERIFY_FIRST),
    (CHACHA, 1, "fast", 0), (CHACHA, 0, "slot128", 0), (CHACHA, 4, "slot128", 0),
    (CHACHA, 1, "slot128", FLAG_ONE_PASS | FLAG_VERIFY_FIRST)])
def test_duplex_vs_oracle(aead, gpu, oracle, cipher, lanes, layout, flags):
    """noise_aead_dev_duplex_uniform: seal job A and open job B (other keys,
    nonces, length, record count; some records tampered) in one call must
    equal the two separate calls — i.e. the oracle — byte for byte.  ChaCha
    FAST layouts run the one-launch chachapoly_duplex_staged kernel; AES-GCM
    with one state per 256 records runs gcm_duplex_fused (plain and CT
    GHASH); a verify-first open (the default; VERIFY_FIRST also overrides
    ONE_PASS) shares the launch with the one-lane ChaCha kernel (AUTH + DEC
    passes) and the AES duplex kernels, the others run two launches.  A
    rejected record's output is zeroed (NOISE_AEAD_FLAG_ONE_PASS opens) or
    never written (verify-first)."""
    torch = _torch()
    rng = np.random.default_rng(3131 + lanes + (cipher & 3) + len(layout) + flags)
    for (La, na, rpsa), (Lb, nb_, rpsb) in (SLOT_CASES if layout == "slot128" else DUPLEX_CASES):
        def strides(L):
            if layout == "packed":
                return L, L + 16
            if layout == "slot128":
                return (max(L, 1) + 127) // 128 * 128, (L + 16 + 127) // 128 * 128
            return (max(L, 1) + 63) // 64 * 64, (L + 16 + 63) // 64 * 64
        ia, oa = strides(La)
        ib, ob = strides(Lb)
        Sa, Sb = (na + rpsa - 1) // rpsa, max(1, (nb_ + rpsb - 1) // rpsb)
        ka = rng.integers(0, 256, (Sa, 32), dtype=np.uint8)
        kb = rng.integers(0, 256, (Sb, 32), dtype=np.uint8)
        nba = rng.integers(0, 2**62, Sa, dtype=np.uint64)
        nbb = rng.integers(0, 2**62, Sb, dtype=np.uint64)
        pta = rng.integers(0, 256, na * ia + 64, dtype=np.uint8)
        ptb = rng.integers(0, 256, max(1, nb_) * ib + 64, dtype=np.uint8)
        exp_a = oracle_seal_records(oracle, cipher, ka, nba, rpsa, pta, ia, La, na, oa)
        ctb = oracle_seal_records(oracle, cipher, kb, nbb, rpsb, ptb, ib, Lb, nb_, ob)
        bad = sorted(set(int(x) for x in rng.integers(0, max(1, nb_), 4))) if nb_ else []
        for b in bad:
            ctb[b * ob + int(rng.integers(0, Lb + 16))] ^= 0x10
        ctxa, _k1 = prepare(aead, cipher, ka)
        ctxb, _k2 = prepare(aead, cipher, kb)
        d_nba, d_nbb = dev(nba.view(np.int64)), dev(nbb.view(np.int64))
        d_pta, d_ctb = dev(pta), dev(ctb)
        d_outa = torch.full((na * oa + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        d_outb = torch.full((max(1, nb_) * ib + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        d_st = torch.full((max(1, nb_),), 7, dtype=torch.uint8, device="cuda")
        sj = aead.uniform_job(ctx=ctxa.data_ptr(), nonce_base=d_nba.data_ptr(), inp=d_pta.data_ptr(),
                              out=d_outa.data_ptr(), in_stride=ia, out_stride=oa, length=La,
                              n_records=na, recs_per_state=rpsa, lanes=lanes,
                              flags=flags & FLAG_CT_GHASH)
        oj = aead.uniform_job(ctx=ctxb.data_ptr(), nonce_base=d_nbb.data_ptr(), inp=d_ctb.data_ptr(),
                              out=d_outb.data_ptr(), in_stride=ob, out_stride=ib, length=Lb,
                              n_records=nb_, recs_per_state=rpsb, status=d_st.data_ptr(),
                              lanes=lanes, flags=flags)
        assert aead.dev_duplex(cipher, sj, oj, stream()) == 0
        sync()
        got_a, back, st = d_outa.cpu().numpy(), d_outb.cpu().numpy(), d_st.cpu().numpy()
        assert np.array_equal(got_a[:na * oa], exp_a[:na * oa]), f"duplex seal len={La}"
        for i in range(nb_):
            seg = back[i * ib: i * ib + Lb]
            if i in bad:
                fill = rejected_fill(cipher, 0x5A, flags)
                assert st[i] == 1 and np.all(seg == fill), f"duplex open len={Lb} rec={i}"
            else:
                assert st[i] == 0, f"duplex open len={Lb} rec={i}"
                assert np.array_equal(seg, ptb[i * ib: i * ib + Lb]), f"len={Lb} rec={i}"
    # overlapping jobs are refused (the seal's output is the open's input)
    sj = aead.uniform_job(ctx=ctxa.data_ptr(), nonce_base=d_nba.data_ptr(), inp=d_pta.data_ptr(),
                          out=d_outa.data_ptr(), in_stride=64, out_stride=64, length=10,
                          n_records=4, recs_per_state=4)
    oj = aead.uniform_job(ctx=ctxa.data_ptr(), nonce_base=d_nba.data_ptr(), inp=d_outa.data_ptr(),
                          out=d_outb.data_ptr(), in_stride=64, out_stride=64, length=10,
                          n_records=4, recs_per_state=4, status=d_st.data_ptr())
    assert aead.dev_duplex(cipher, sj, oj, stream()) == 0x450B


@pytest.mark.parametrize("cipher,lanes", [(CHACHA, 1), (CHACHA, 4), (CHACHA, 8), (CHACHA, 32),
                                          (CHACHA, 64), (AES, 0)])
@pytest.mark.parametrize("rps", [4, 16])
def test_uniform_with_ad(aead, gpu, oracle, cipher, lanes, rps):
    rng = np.random.default_rng(77 + lanes + rps)
    for L in [0, 1, 64, 65, 1024, 1400]:
        for adl in [1, 12, 16, 32, 33, 100]:
            count = 2 * rps + 1
            S = 3
            keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
            nb = rng.integers(0, 2**40, S, dtype=np.uint64)
            stride = L + 16
            pt = rng.integers(0, 256, count * stride + 16, dtype=np.uint8)
            ad = rng.integers(0, 256, count * 128, dtype=np.uint8)
            exp = oracle_seal_records(oracle, cipher, keys, nb, rps, pt, stride, L, count, stride,
                                      ad=ad, ad_stride=128, ad_len=adl)
            got, _ = gpu_uniform(aead, False, cipher, keys, nb, rps, pt, stride, L, count, stride,
                                 lanes=lanes, ad=ad, ad_stride=128, ad_len=adl)
            assert np.array_equal(got, exp), f"len={L} ad={adl}"
            back, st = gpu_uniform(aead, True, cipher, keys, nb, rps, got, stride, L, count,
                                   stride, lanes=lanes, ad=ad, ad_stride=128, ad_len=adl)
            assert np.all(st == 0)


def test_nonce_edges(aead, gpu, oracle):
    rng = np.random.default_rng(5)
    for cipher in (CHACHA, AES):
        for base in [0, 2**32 - 2, 2**32 - 1, 2**63, NONCE_MAX - 4]:
            count, L = 3, 200
            keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
            pt = rng.integers(0, 256, count * L, dtype=np.uint8)
            exp = oracle_seal_records(oracle, cipher, keys, [base], count, pt, L, L, count, L + 16)
            got, _ = gpu_uniform(aead, False, cipher, keys, [base], count, pt, L, L, count, L + 16)
            assert np.array_equal(got, exp), hex(base)


def test_max_record(aead, gpu, oracle):
    """NOISE_MAX_PAYLOAD_LEN - 16 bytes of plaintext (constants.h:151)."""
    rng = np.random.default_rng(9)
    L = 65535 - 16
    for cipher, lanes in [(CHACHA, 8), (CHACHA, 1), (CHACHA, 16), (CHACHA, 64), (AES, 0)]:
        keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        pt = rng.integers(0, 256, 2 * L, dtype=np.uint8)
        exp = oracle_seal_records(oracle, cipher, keys, [123], 2, pt, L, L, 2, L + 16)
        got, _ = gpu_uniform(aead, False, cipher, keys, [123], 2, pt, L, L, 2, L + 16, lanes=lanes)
        assert np.array_equal(got, exp)


def test_in_place(aead, gpu, oracle):
    """in == out, as the reference encrypts/decrypts the buffer in place."""
    rng = np.random.default_rng(11)
    for cipher in (CHACHA, AES):
        L, count, stride = 1400, 50, 1424
        keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        pt = rng.integers(0, 256, count * stride, dtype=np.uint8)
        exp = oracle_seal_records(oracle, cipher, keys, [0], count, pt, stride, L, count, stride)
        ctx, _k = prepare(aead, cipher, keys)
        d_nb = dev(np.zeros(1, dtype=np.int64))
        buf = dev(pt)
        rc = aead.dev_uniform(False, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                              inp=buf.data_ptr(), out=buf.data_ptr(), in_stride=stride,
                              out_stride=stride, length=L, n_records=count, recs_per_state=count,
                              stream=stream())
        assert rc == 0
        sync()
        g = buf.cpu().numpy()
        for i in range(count):
            assert np.array_equal(g[i * stride: i * stride + L + 16],
                                  exp[i * stride: i * stride + L + 16])
        rc = aead.dev_uniform(True, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                              inp=buf.data_ptr(), out=buf.data_ptr(), in_stride=stride,
                              out_stride=stride, length=L, n_records=count, recs_per_state=count,
                              stream=stream())
        assert rc == 0
        sync()
        g = buf.cpu().numpy()
        for i in range(count):
            assert np.array_equal(g[i * stride: i * stride + L], pt[i * stride: i * stride + L])


# ------------------------------------------------------------ ragged kernel

@pytest.mark.parametrize("cipher,lanes", [(CHACHA, 0), (CHACHA, 4), (CHACHA, 8), (CHACHA, 16),
                                          (CHACHA, 32), (CHACHA, 64), (AES, 0), (AES, 4)])
def test_ragged_vs_oracle(aead, gpu, oracle, cipher, lanes):
    """lanes 0: the library's choice (wide groups for a batch this small)."""
    rng = np.random.default_rng(21 + (cipher & 3) + lanes)
    S, count = 5, 200
    keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
    torch = _torch()
    ctx, _k = prepare(aead, cipher, keys)
    cb = aead.dev_ctx_bytes(cipher)
    lens = rng.integers(0, 3000, count)
    lens[:10] = [0, 1, 15, 16, 17, 63, 64, 65, 1400, 16384]
    adls = rng.choice([0, 0, 0, 5, 32], count)
    recs = np.zeros(count, dtype=[("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"),
                                  ("ctx_off", "<u8"), ("ad_off", "<u8"), ("len", "<u4"),
                                  ("ad_len", "<u4")])
    inp_size = int(sum(int(l) + 16 + 3 for l in lens)) + 64
    inp = rng.integers(0, 256, inp_size, dtype=np.uint8)
    ad = rng.integers(0, 256, count * 64, dtype=np.uint8)
    off = 0
    exp = np.full(inp_size, 0xA5, dtype=np.uint8)
    for i in range(count):
        s = int(rng.integers(0, S))
        n = int(rng.integers(0, 2**62))
        recs[i] = (off + 3 * (i % 2), off, n, s * cb, 64 * i, lens[i], adls[i])
        # in_off deliberately misaligned for odd records (read from off+3)
        p = bytes(inp[off + 3 * (i % 2): off + 3 * (i % 2) + lens[i]])
        a = bytes(ad[64 * i: 64 * i + adls[i]])
        ct = oracle.encrypt(cipher, bytes(keys[s]), n, p, a)
        exp[off: off + lens[i] + 16] = np.frombuffer(ct, dtype=np.uint8)
        off += int(lens[i]) + 16 + 3
    d_recs = dev(recs.view(np.uint8))
    d_in, d_ad = dev(inp), dev(ad)
    d_out = torch.full((inp_size,), 0xA5, dtype=torch.uint8, device="cuda")
    rc = aead.dev_ragged(False, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                         inp=d_in.data_ptr(), out=d_out.data_ptr(), n_records=count,
                         ad=d_ad.data_ptr(), lanes=lanes, stream=stream())
    assert rc == 0
    sync()
    got = d_out.cpu().numpy()
    assert np.array_equal(got[:off], exp[:off])
    # open: out -> in positions swapped
    recs2 = recs.copy()
    recs2["in_off"], recs2["out_off"] = recs["out_off"], recs["out_off"]
    d_recs2 = dev(recs2.view(np.uint8))
    d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    rc = aead.dev_ragged(True, cipher, ctx_base=ctx.data_ptr(), recs=d_recs2.data_ptr(),
                         inp=d_out.data_ptr(), out=d_out.data_ptr(), n_records=count,
                         ad=d_ad.data_ptr(), status=d_st.data_ptr(), lanes=lanes, stream=stream())
    assert rc == 0
    sync()
    assert np.all(d_st.cpu().numpy() == 0)
    back = d_out.cpu().numpy()
    for i in range(count):
        o, io, L = int(recs["out_off"][i]), int(recs["in_off"][i]), int(lens[i])
        assert np.array_equal(back[o: o + L], inp[io: io + L])


@pytest.mark.parametrize("cipher,lanes", [(CHACHA, 0), (CHACHA, 4), (CHACHA, 8), (AES, 4),
                                          (AES, 0)])
@pytest.mark.parametrize("fast", [True, False])
def test_ragged_windows_states_and_tamper(aead, gpu, oracle, cipher, lanes, fast):
    """Many workgroup windows (records taken in length order inside each),
    per-state record runs of uneven size (so some windows hold 2 states,
    some 3+: the AES LDS state slots and the global-context path), 1/2 of
    the records in place, every 37th record tampered: each status, each
    verified plaintext and each rejected record's untouched bytes must match
    the oracle.  lanes 0 is the library's choice for a batch this small:
    64-lane ChaChaPoly groups, one AES-GCM record per workgroup (gcm_wide)."""
    torch = _torch()
    rng = np.random.default_rng(77 + (cipher & 3) + 10 * fast + lanes)
    count = 1500
    runs = []
    while sum(runs) < count:
        runs.append(int(rng.choice([1, 3, 40, 130, 300])))
    state_of = np.repeat(np.arange(len(runs)), runs)[:count]
    S = len(runs)
    keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
    ctx, _k = prepare(aead, cipher, keys)
    cb = aead.dev_ctx_bytes(cipher)
    lens = rng.integers(0, 4000, count)
    lens[::97] = 16384
    slot = lambda L: ((int(L) + 16 + 63) // 64) * 64 if fast else int(L) + 16 + 5
    offs = np.zeros(count, dtype=np.int64)
    offs[1:] = np.cumsum([slot(L) for L in lens])[:-1]
    total = int(offs[-1]) + slot(lens[-1]) + 64
    pt = rng.integers(0, 256, total, dtype=np.uint8)
    nonces = rng.integers(0, 2**62, count, dtype=np.int64).astype(np.uint64)
    dt = [("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
          ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")]
    recs = np.zeros(count, dtype=dt)
    recs["in_off"] = recs["out_off"] = offs
    recs["nonce"] = nonces
    recs["ctx_off"] = state_of.astype(np.uint64) * cb
    recs["len"] = lens
    d_recs = dev(recs.view(np.uint8))
    d_buf = dev(pt)
    flags = aead.FLAG_FAST if fast else 0
    assert aead.dev_ragged(False, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_buf.data_ptr(), out=d_buf.data_ptr(), n_records=count,
                           flags=flags, lanes=lanes, stream=stream()) == 0
    sync()
    sealed = d_buf.cpu().numpy().copy()
    for i in list(range(0, count, 7)) + [count - 1]:
        o, L = int(offs[i]), int(lens[i])
        exp = oracle.encrypt(cipher, bytes(keys[state_of[i]]), int(nonces[i]), bytes(pt[o:o + L]))
        assert bytes(sealed[o:o + L + 16]) == exp, i
    bad = np.arange(count) % 37 == 5
    tampered = sealed.copy()
    for i in np.nonzero(bad)[0]:
        o, L = int(offs[i]), int(lens[i])
        # ciphertext or tag byte: the single-pass opens write plaintext before
        # the verdict and must give back exactly these bytes in place
        tampered[o + int(rng.integers(0, L + 16))] ^= 0x40
    d_buf = dev(tampered)
    d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(True, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_buf.data_ptr(), out=d_buf.data_ptr(), n_records=count,
                           status=d_st.data_ptr(), flags=flags, lanes=lanes, stream=stream()) == 0
    sync()
    st = d_st.cpu().numpy()
    back = d_buf.cpu().numpy()
    assert np.array_equal(st != 0, bad)
    for i in range(count):
        o, L = int(offs[i]), int(lens[i])
        if bad[i]:
            assert np.array_equal(back[o:o + L + 16], tampered[o:o + L + 16]), i
        else:
            assert np.array_equal(back[o:o + L], pt[o:o + L]), i


@pytest.mark.parametrize("count,ct", [(70_000, False), (140_000, False), (70_000, True)])
def test_ragged_aes_paired_windows(aead, gpu, oracle, count, ct):
    """Ragged AES-GCM batches large enough for the paired shapes, where each
    record group runs a long and a short record one after the other
    (gcm_ragged_staged<.., R = 2>): 70 000 records take 256-record windows of
    8-lane groups (the H^8 Horner table), 140 000 take 512-record windows of
    4-lane groups.  Per-state runs of 300 records (windows holding 2 and 3
    states), out of place: a sample of records against the oracle, every
    record's round trip, and tampered records rejected with their output
    never written.  ct: the same through the constant-time GHASH (H^8 in the natural
    domain for the 8-lane groups)."""
    torch = _torch()
    rng = np.random.default_rng(4711 + count + ct)
    run = 300
    flags = aead.FLAG_FAST | (aead.FLAG_CT_GHASH if ct else 0)
    S = (count + run - 1) // run
    keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
    ctx, _k = prepare(aead, AES, keys)
    cb = aead.dev_ctx_bytes(AES)
    lens = rng.integers(0, 1200, count)
    lens[::211] = 9000
    slot = (lens + 16 + 63) // 64 * 64
    offs = np.zeros(count, dtype=np.int64)
    offs[1:] = np.cumsum(slot)[:-1]
    total = int(offs[-1] + slot[-1]) + 64
    pt = rng.integers(0, 256, total, dtype=np.uint8)
    nonces = rng.integers(0, 2**62, count, dtype=np.int64).astype(np.uint64)
    dt = [("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
          ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")]
    recs = np.zeros(count, dtype=dt)
    recs["in_off"] = recs["out_off"] = offs
    recs["nonce"] = nonces
    recs["ctx_off"] = (np.arange(count) // run).astype(np.uint64) * cb
    recs["len"] = lens
    d_recs = dev(recs.view(np.uint8))
    d_pt = dev(pt)
    d_ct = torch.zeros(total, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(False, AES, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_pt.data_ptr(), out=d_ct.data_ptr(), n_records=count,
                           flags=flags, stream=stream()) == 0
    sync()
    ct = d_ct.cpu().numpy()
    for i in list(rng.choice(count, 400, replace=False)) + list(range(0, count, 211)[:40]) + [count - 1]:
        o, L = int(offs[i]), int(lens[i])
        exp = oracle.encrypt(AES, bytes(keys[i // run]), int(nonces[i]), bytes(pt[o:o + L]))
        assert bytes(ct[o:o + L + 16]) == exp, i
    bad = np.arange(count) % 997 == 13
    for i in np.nonzero(bad)[0]:
        ct[int(offs[i]) + int(rng.integers(0, int(lens[i]) + 16))] ^= 0x08
    d_ct = dev(ct)
    d_back = torch.full((total,), 0x5A, dtype=torch.uint8, device="cuda")
    d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(True, AES, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_ct.data_ptr(), out=d_back.data_ptr(), n_records=count,
                           status=d_st.data_ptr(), flags=flags, stream=stream()) == 0
    sync()
    st, back = d_st.cpu().numpy(), d_back.cpu().numpy()
    assert np.array_equal(st != 0, bad) and set(np.unique(st)) <= {0, 1}
    keep = np.zeros(total, dtype=bool)
    for i in range(count):
        keep[int(offs[i]):int(offs[i]) + int(lens[i])] = True
    good_bytes = keep.copy()
    for i in np.nonzero(bad)[0]:
        o, L = int(offs[i]), int(lens[i])
        assert np.all(back[o:o + L] == 0x5A), i  # AES-GCM opens verify first: never written
        good_bytes[o:o + L] = False
    assert np.array_equal(back[good_bytes], pt[good_bytes])


# ------------------------------------------- the CipherState API on the GPU

def test_golden_grid_through_cipherstate(aead, gpu, oracle, golden):
    """All 500 reference-generated grid vectors through the single-record API."""
    _, grid = golden
    for c in grid["cases"]:
        rc, st = aead.CipherState.new_by_id(c["cipher"])
        assert rc == 0
        assert st.init_key(bytes.fromhex(c["key"])) == 0
        if c["nonce"]:
            assert st.set_nonce(c["nonce"]) == 0
        pt = oracle.fill(grid["seed_pt"], c["len"], c["pt_word0"])
        ad = oracle.fill(grid["seed_ad"], c["ad_len"], c["ad_word0"])
        out = st.seal(pt, ad)
        assert out[-16:].hex() == c["tag"], c
        if "ct" in c:
            assert out[:-16].hex() == c["ct"]
        import hashlib
        assert hashlib.sha256(out).hexdigest() == c["sha256"]
        st2 = aead.CipherState.new_by_id(c["cipher"])[1]
        st2.init_key(bytes.fromhex(c["key"]))
        if c["nonce"]:
            st2.set_nonce(c["nonce"])
        rc, back = st2.open(out, ad)
        assert rc == 0 and back == pt
        st.free()
        st2.free()


def _model_seq(oracle, ops):
    """Sequential semantics of cipherstate.c:293-410 on the oracle."""
    res = []
    for (m, kind, ad, data, size, max_size) in ops:
        data = bytearray(data)
        if kind == "enc":
            if size > max_size:
                res.append((0x450A, bytes(data), size)); continue
            if not m["has_key"]:
                res.append((0x450A if size > 65535 else 0, bytes(data), size)); continue
            if size > 65535 - 16 or max_size - size < 16:
                res.append((0x450A, bytes(data), size)); continue
            if m["n"] == NONCE_MAX:
                res.append((0x450D, bytes(data), size)); continue
            ct = oracle.encrypt(m["cipher"], m["key"], m["n"], bytes(data[:size]), ad)
            m["n"] += 1
            data[:size + 16] = ct
            res.append((0, bytes(data), size + 16))
        else:
            if size > max_size or size > 65535:
                res.append((0x450A, bytes(data), size)); continue
            if not m["has_key"]:
                res.append((0, bytes(data), size)); continue
            if size < 16:
                res.append((0x450A, bytes(data), size)); continue
            if m["n"] == NONCE_MAX:
                res.append((0x450D, bytes(data), size)); continue
            rc, pt = oracle.decrypt(m["cipher"], m["key"], m["n"], bytes(data[:size]), ad)
            if rc:
                res.append((0x4504, bytes(data), size)); continue
            m["n"] += 1
            data[:size - 16] = pt
            res.append((0, bytes(data), size - 16))
    return res


def test_batch_equals_sequential(aead, gpu, oracle):
    """encrypt_batch / decrypt_batch == the same calls made one by one,
    including no-key pass-through, bad lengths, MAC failures (nonce not
    advanced) and mixed ciphers (cipherstate.c:293-410)."""
    rng = np.random.default_rng(3)
    n_states = 6
    models, states = [], []
    for s in range(n_states):
        cipher = CHACHA if s % 2 == 0 else AES
        st = aead.CipherState.new_by_id(cipher)[1]
        key = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
        m = dict(cipher=cipher, key=key, has_key=s != 5, n=0)
        if m["has_key"]:
            st.init_key(key)
            n0 = int(rng.integers(0, 1000)) if s != 4 else NONCE_MAX - 3
            st.set_nonce(n0)
            m["n"] = n0
        models.append(m)
        states.append(st)
    # encrypt batch
    N = 60
    rec_state = rng.integers(0, n_states, N)
    mems, bufs, ads, ops = [], [], [], []
    for i in range(N):
        L = int(rng.choice([0, 5, 64, 100, 1400, 65535 - 16, 65535 - 15]))
        max_size = L + 16 if rng.random() > 0.1 else L + 3
        data = bytes(rng.integers(0, 256, L, dtype=np.uint8)) + bytes(max_size - L)
        mem = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        mems.append(mem)
        bufs.append(aead.NoiseBuffer.inout(mem, L, max_size))
        ad = bytes(rng.integers(0, 256, int(rng.choice([0, 0, 13])), dtype=np.uint8))
        ads.append(ad)
        ops.append((models[rec_state[i]], "enc", ad, data, L, max_size))
    exp = _model_seq(oracle, ops)
    rc, res = aead.encrypt_batch([states[s] for s in rec_state], bufs, ads)
    assert rc == 0
    for i in range(N):
        assert res[i] == exp[i][0], (i, hex(res[i]), hex(exp[i][0]))
        assert bufs[i].size == exp[i][2]
        assert bytes(mems[i])[:len(exp[i][1])] == exp[i][1][:len(bytes(mems[i]))]
    # decrypt the successful ones back with fresh states, corrupting some
    dstates, dmodels = [], []
    for s in range(n_states):
        st = aead.CipherState.new_by_id(models[s]["cipher"])[1]
        m = dict(models[s])
        if m["has_key"]:
            st.init_key(m["key"])
            n0 = m["n"] - int(sum(1 for i in range(N) if rec_state[i] == s and exp[i][0] == 0))
            st.set_nonce(n0)
            m["n"] = n0
        dstates.append(st)
        dmodels.append(m)
    dmems, dbufs, dops, dst = [], [], [], []
    for i in range(N):
        if exp[i][0] != 0:
            continue
        data = bytearray(exp[i][1][:exp[i][2]])
        if len(data) and rng.random() < 0.15:
            data[int(rng.integers(0, len(data)))] ^= 0x40
        mem = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        dmems.append(mem)
        dbufs.append(aead.NoiseBuffer.input(mem, len(data)))
        dops.append((dmodels[rec_state[i]], "dec", ads[i], bytes(data), len(data), len(data)))
        dst.append(dstates[rec_state[i]])
    dexp = _model_seq(oracle, dops)
    rc, dres = aead.decrypt_batch(dst, dbufs, [o[2] for o in dops])
    assert rc == 0
    for k in range(len(dops)):
        assert dres[k] == dexp[k][0], (k, hex(dres[k]), hex(dexp[k][0]))
        assert dbufs[k].size == dexp[k][2]
        assert bytes(dmems[k])[:dexp[k][2]] == dexp[k][1][:dexp[k][2]]
    for s in states + dstates:
        s.free()


def test_reference_unit_suite_on_gpu(aead, gpu, golden):
    """tests/unit/test-cipherstate.c:31-224 check_cipher, re-stated on our API."""
    kat, _ = golden
    names = {CHACHA: "ChaChaPoly", AES: "AESGCM"}
    for v in kat["vectors"]:
        cid, key = v["cipher"], bytes.fromhex(v["key"])
        pt, ct, tag, ad = (bytes.fromhex(v[x]) for x in ("pt", "ct", "tag", "ad"))
        nonce = v["nonce"]
        rc, st = aead.CipherState.new_by_id(cid)
        assert rc == 0 and st.cipher_id == cid and st.key_length == 32 and st.mac_length == 16
        assert not st.has_key
        buf = (C.c_uint8 * 512)()
        C.memmove(buf, pt, len(pt))
        nb = aead.NoiseBuffer.inout(buf, len(pt), 512)
        assert st.encrypt_with_ad(ad, nb) == 0 and nb.size == len(pt)
        assert bytes(buf)[:len(pt)] == pt
        assert st.set_nonce(nonce) == 0x450C  # INVALID_STATE before a key
        assert st.init_key(key) == 0 and st.set_nonce(nonce) == 0 and st.has_key
        nb = aead.NoiseBuffer.inout(buf, len(pt), 512)
        assert st.encrypt_with_ad(ad, nb) == 0 and nb.size == len(pt) + 16
        assert bytes(buf)[:len(pt)] == ct and bytes(buf)[len(pt):len(pt) + 16] == tag
        nb = aead.NoiseBuffer.input(buf, len(pt) + 16)
        assert st.decrypt_with_ad(ad, nb) == 0x4504  # nonce moved on
        assert st.set_nonce(nonce) == 0x450D
        assert st.set_nonce(NONCE_MAX - 1) == 0
        nb = aead.NoiseBuffer.inout(buf, len(pt), 512)
        assert st.encrypt_with_ad(ad, nb) == 0
        nb = aead.NoiseBuffer.inout(buf, len(pt), 512)
        assert st.encrypt_with_ad(ad, nb) == 0x450D
        assert st.init_key(key) == 0 and st.set_nonce(nonce) == 0
        C.memmove(buf, ct + tag, len(ct) + 16)
        nb = aead.NoiseBuffer.input(buf, len(pt) + 16)
        assert st.decrypt_with_ad(ad, nb) == 0 and nb.size == len(pt)
        assert bytes(buf)[:len(pt)] == pt
        assert st.set_nonce(NONCE_MAX - 1) == 0
        nb = aead.NoiseBuffer.input(buf, len(pt) + 16)
        assert st.decrypt_with_ad(ad, nb) == 0x4504
        nb = aead.NoiseBuffer.input(buf, len(pt) + 16)
        assert st.decrypt_with_ad(ad, nb) == 0x4504
        assert st.free() == 0
        rc, st = aead.CipherState.new_by_name(names[cid])
        assert rc == 0 and st.cipher_id == cid
        st.free()


# ------------------------------------- full BASELINE sizes: size-free checks

@pytest.mark.parametrize("cipher", [CHACHA, AES])
def test_full_size_config(aead, gpu, oracle, cipher):
    """Config 2/3 shape (64 Ki x 1400 B, one key): every lane split gives the
    same bytes, a sample of records equals the oracle, the open round trip
    restores every plaintext and flags exactly the tampered records."""
    torch = _torch()
    N, L = 65536, 1400
    in_stride, out_stride = 1408, 1424
    key = np.arange(32, dtype=np.uint8).reshape(1, 32)
    ctx, _k = prepare(aead, cipher, key)
    d_nb = dev(np.array([5], dtype=np.int64))
    d_pt = torch.empty(N * in_stride, dtype=torch.uint8, device="cuda")
    assert aead.dev_fill_splitmix(d_pt.data_ptr(), N * in_stride, 0x5EED, 0, stream()) == 0
    outs = []
    lane_opts = [1, 2, 4, 8] if cipher == CHACHA else [0]
    for lanes in lane_opts:
        d_ct = torch.zeros(N * out_stride, dtype=torch.uint8, device="cuda")
        rc = aead.dev_uniform(False, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                              inp=d_pt.data_ptr(), out=d_ct.data_ptr(), in_stride=in_stride,
                              out_stride=out_stride, length=L, n_records=N, recs_per_state=N,
                              lanes=lanes, stream=stream())
        assert rc == 0
        outs.append(d_ct)
    sync()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ct = outs[0]
    pt_h = d_pt.cpu().numpy()
    ct_h = ct.cpu().numpy()
    rng = np.random.default_rng(2)
    for i in list(rng.integers(0, N, 64)) + [0, N - 1]:
        i = int(i)
        exp = oracle.encrypt(cipher, bytes(key[0]), 5 + i, bytes(pt_h[i * in_stride: i * in_stride + L]))
        assert bytes(ct_h[i * out_stride: i * out_stride + L + 16]) == exp, i
    bad = sorted(set(int(x) for x in rng.integers(0, N, 100)))
    for b in bad:
        ct[b * out_stride + int(rng.integers(0, L + 16))] ^= 0x01
    d_back = torch.zeros(N * in_stride, dtype=torch.uint8, device="cuda")
    d_st = torch.full((N,), 9, dtype=torch.uint8, device="cuda")
    rc = aead.dev_uniform(True, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                          inp=ct.data_ptr(), out=d_back.data_ptr(), in_stride=out_stride,
                          out_stride=in_stride, length=L, n_records=N, recs_per_state=N,
                          status=d_st.data_ptr(), stream=stream())
    assert rc == 0
    sync()
    st = d_st.cpu().numpy()
    assert sorted(np.nonzero(st)[0].tolist()) == bad
    mask = np.ones(N, dtype=bool)
    mask[bad] = False
    back = d_back.cpu().numpy().reshape(N, in_stride)[:, :L]
    assert np.array_equal(back[mask], pt_h.reshape(N, in_stride)[:, :L][mask])
    assert np.all(back[~mask] == 0)


@pytest.mark.parametrize("cipher", [CHACHA, AES])
def test_interleaved_slots_one_buffer(aead, gpu, oracle, cipher):
    """Input and output slots alternating in one buffer with one stride
    (accepted since no two records meet): the seal writes every
    output slot, leaves every input slot as it was, and matches the oracle;
    the open back through the same interleaving restores the plaintext."""
    torch = _torch()
    rng = np.random.default_rng(2718 + (cipher & 3))
    L, count, slot = 1400, 300, 1536
    keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    nb = np.array([12345], dtype=np.uint64)
    buf = rng.integers(0, 256, 2 * slot * count + 64, dtype=np.uint8)
    pt = buf.copy()
    exp = oracle_seal_records(oracle, cipher, keys, nb, count, pt, 2 * slot, L, count, 2 * slot)
    ctx, _k = prepare(aead, cipher, keys)
    d_nb = dev(nb.view(np.int64))
    d = dev(buf)
    base = d.data_ptr()
    common = dict(ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(), in_stride=2 * slot,
                  out_stride=2 * slot, length=L, n_records=count, recs_per_state=count, stream=stream())
    assert aead.dev_uniform(False, cipher, inp=base, out=base + slot, **common) == 0
    sync()
    got = d.cpu().numpy()
    for i in range(count):
        o = 2 * slot * i
        assert np.array_equal(got[o:o + slot], pt[o:o + slot]), i  # input slot untouched
        assert np.array_equal(got[o + slot:o + slot + L + 16], exp[o:o + L + 16]), i
    st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    # open: read the output slots back into the input slots
    assert aead.dev_uniform(True, cipher, inp=base + slot, out=base, status=st.data_ptr(), **common) == 0
    sync()
    back = d.cpu().numpy()
    assert int(st.max().item()) == 0
    for i in range(count):
        o = 2 * slot * i
        assert np.array_equal(back[o:o + L], pt[o:o + L]), i


@pytest.mark.parametrize("flags", [FLAG_ONE_PASS, 0])
def test_duplex_solo_runs(aead, gpu, oracle, flags):
    """chachapoly_duplex_solo places the paired blocks in runs of the CU count
    (seal run, open run, ...) and the remainder block by block: job sizes
    that leave a partial run and a partial last block (300 x 256 + 17 seal
    records, 290 x 256 + 5 open records, one lane each).  The duplex output
    equals the separate launches byte for byte (both orders of open), and
    sampled records — every run boundary's neighbours among them — equal
    the oracle; tampered records are rejected."""
    torch = _torch()
    rng = np.random.default_rng(977 + flags)
    L, rps = 40, 64
    na, nb_ = 300 * 256 + 17, 290 * 256 + 5
    ins, outs = 64, 64
    Sa, Sb = (na + rps - 1) // rps, (nb_ + rps - 1) // rps
    ka = rng.integers(0, 256, (Sa, 32), dtype=np.uint8)
    kb = rng.integers(0, 256, (Sb, 32), dtype=np.uint8)
    nba = rng.integers(0, 2**62, Sa, dtype=np.uint64)
    nbb = rng.integers(0, 2**62, Sb, dtype=np.uint64)
    pta = rng.integers(0, 256, na * ins + 64, dtype=np.uint8)
    ptb = rng.integers(0, 256, nb_ * ins + 64, dtype=np.uint8)
    ctxa, _k1 = prepare(aead, CHACHA, ka)
    ctxb, _k2 = prepare(aead, CHACHA, kb)
    d_nba, d_nbb = dev(nba.view(np.int64)), dev(nbb.view(np.int64))
    d_pta, d_ptb = dev(pta), dev(ptb)
    # batch B sealed by the separate (oracle-checked) kernel, then tampered
    d_ctb = torch.full((nb_ * outs + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    assert aead.dev_uniform(False, CHACHA, ctx=ctxb.data_ptr(), nonce_base=d_nbb.data_ptr(),
                            inp=d_ptb.data_ptr(), out=d_ctb.data_ptr(), in_stride=ins, out_stride=outs,
                            length=L, n_records=nb_, recs_per_state=rps, lanes=1, stream=stream()) == 0
    bad = np.unique(rng.integers(0, nb_, 40))
    flat = d_ctb.view(-1)
    flat[torch.from_numpy(bad * outs + rng.integers(0, L + 16, len(bad))).to("cuda")] ^= 0x20
    # separate launches: the expected bytes
    exp_a = torch.full((na * outs + 64,), 0x11, dtype=torch.uint8, device="cuda")
    exp_b = torch.full((nb_ * ins + 64,), 0x22, dtype=torch.uint8, device="cuda")
    exp_st = torch.full((nb_,), 7, dtype=torch.uint8, device="cuda")
    assert aead.dev_uniform(False, CHACHA, ctx=ctxa.data_ptr(), nonce_base=d_nba.data_ptr(),
                            inp=d_pta.data_ptr(), out=exp_a.data_ptr(), in_stride=ins, out_stride=outs,
                            length=L, n_records=na, recs_per_state=rps, lanes=1, stream=stream()) == 0
    assert aead.dev_uniform(True, CHACHA, ctx=ctxb.data_ptr(), nonce_base=d_nbb.data_ptr(),
                            inp=d_ctb.data_ptr(), out=exp_b.data_ptr(), in_stride=outs, out_stride=ins,
                            length=L, n_records=nb_, recs_per_state=rps, status=exp_st.data_ptr(),
                            lanes=1, flags=flags, stream=stream()) == 0
    got_a = torch.full_like(exp_a, 0x11)
    got_b = torch.full_like(exp_b, 0x22)
    got_st = torch.full_like(exp_st, 7)
    sj = aead.uniform_job(ctx=ctxa.data_ptr(), nonce_base=d_nba.data_ptr(), inp=d_pta.data_ptr(),
                          out=got_a.data_ptr(), in_stride=ins, out_stride=outs, length=L,
                          n_records=na, recs_per_state=rps, lanes=1)
    oj = aead.uniform_job(ctx=ctxb.data_ptr(), nonce_base=d_nbb.data_ptr(), inp=d_ctb.data_ptr(),
                          out=got_b.data_ptr(), in_stride=outs, out_stride=ins, length=L,
                          n_records=nb_, recs_per_state=rps, status=got_st.data_ptr(), lanes=1,
                          flags=flags)
    assert aead.dev_duplex(CHACHA, sj, oj, stream()) == 0
    sync()
    assert torch.equal(got_a, exp_a)
    assert torch.equal(got_b, exp_b)
    assert torch.equal(got_st, exp_st)
    st = got_st.cpu().numpy()
    exp = np.zeros(nb_, dtype=np.uint8)
    exp[bad] = 1
    assert np.array_equal(st, exp)
    # sampled records against the oracle: every 997th plus the neighbours
    # of each 256-block run boundary (records 65536k - 1, 65536k)
    sample = sorted(set(list(range(0, na, 997)) + [na - 1] +
                        [r for k in range(1, na // 65536 + 1) for r in (65536 * k - 1, 65536 * k)
                         if r < na]))
    ga = got_a.cpu().numpy()
    for i in sample:
        s_ = i // rps
        ct = oracle.encrypt(CHACHA, bytes(ka[s_]), int(nba[s_]) + i % rps,
                            bytes(pta[i * ins:i * ins + L]), b"")
        assert bytes(ga[i * outs:i * outs + L + 16]) == ct, i
    gb = got_b.cpu().numpy()
    for i in range(0, nb_, 991):
        if i not in bad:
            assert np.array_equal(gb[i * ins:i * ins + L], ptb[i * ins:i * ins + L]), i
