"""The verify-first open order (the default of every open
since round 6; NOISE_AEAD_FLAG_VERIFY_FIRST requests it
explicitly).

The reference's ref backends authenticate first and decrypt only a record
whose tag verified (src/backend/ref/cipher-chachapoly.c:135-141,
cipher-aesgcm.c:172-188).  The opt-in NOISE_AEAD_FLAG_ONE_PASS FAST-layout
ChaChaPoly opens run in one pass and undo a rejected record's plaintext
before the kernel ends; in the default order (no flag) and with
VERIFY_FIRST no byte of a rejected record's output is ever written —
not plaintext, not zeros.  So out of place a rejected record's output still
holds its sentinel fill, and in place its CT || tag reads back as given; every
verified record equals the oracle's plaintext.  Uniform (staged and generic
kernels, both ciphers) and ragged (every ChaChaPoly lane width's two-pass
instantiation, AES-GCM windows of every launch shape) batches.
"""
import numpy as np
import pytest

from test_gpu_parity import AES, CHACHA, dev, oracle_seal_records, prepare, stream, sync

pytestmark = pytest.mark.gpu
VF, FAST = 4, 1
REC_DT = [("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
          ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")]


@pytest.mark.parametrize("cipher,lanes,rps", [(CHACHA, 4, 256), (CHACHA, 8, 256), (CHACHA, 4, 13),
                                              (CHACHA, 1, 16), (CHACHA, 1, 64), (CHACHA, 64, 16), (AES, 0, 256),
                                              (AES, 0, 13)])
@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("vflag", [VF, 0])
def test_uniform_verify_first(aead, gpu, oracle, cipher, lanes, rps, in_place, vflag):
    """vflag 0: no flag at all — the default open order must be the strict one."""
    import torch
    rng = np.random.default_rng(31 + lanes + rps + (cipher & 3) + 100 * in_place + vflag)
    for L, count, adl in [(1400, 600, 0), (0, 40, 0), (17, 300, 0), (4096, 30, 0), (1400, 257, 24)]:
        S = (count + rps - 1) // rps
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        nb = rng.integers(0, 2**62, S, dtype=np.uint64)
        ins = (max(L, 1) + 63) // 64 * 64
        outs = (L + 16 + 63) // 64 * 64
        stride_ct = outs
        pt = rng.integers(0, 256, count * ins + 64, dtype=np.uint8)
        ad = rng.integers(0, 256, count * 32 + 64, dtype=np.uint8)
        akw = dict(ad=ad, ad_stride=32, ad_len=adl) if adl else {}
        ct = oracle_seal_records(oracle, cipher, keys, nb, rps, pt, ins, L, count, stride_ct, **akw)
        bad = sorted(set(int(x) for x in rng.integers(0, count, 9)))
        for b in bad:
            ct[b * stride_ct + int(rng.integers(0, L + 16))] ^= 0x08
        ctx, _k = prepare(aead, cipher, keys)
        d_nb, d_ct, d_ad = dev(nb.view(np.int64)), dev(ct), dev(ad)
        if in_place:
            d_out, out_stride = d_ct, stride_ct
        else:
            d_out = torch.full((count * ins + 64,), 0xC3, dtype=torch.uint8, device="cuda")
            out_stride = ins
        d_st = torch.full((count,), 7, dtype=torch.uint8, device="cuda")
        assert aead.dev_uniform(True, cipher, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                                inp=d_ct.data_ptr(), out=d_out.data_ptr(), in_stride=stride_ct,
                                out_stride=out_stride, length=L, n_records=count, recs_per_state=rps,
                                status=d_st.data_ptr(), lanes=lanes, flags=vflag, stream=stream(),
                                ad=d_ad.data_ptr() if adl else 0, ad_stride=32 if adl else 0,
                                ad_len=adl) == 0
        sync()
        back, st = d_out.cpu().numpy(), d_st.cpu().numpy()
        for i in range(count):
            o = i * out_stride
            if i in bad:
                assert st[i] == 1, (L, i)
                if in_place:
                    assert np.array_equal(back[o:o + L + 16], ct[o:o + L + 16]), (L, i)
                else:
                    assert np.all(back[o:o + L] == 0xC3), (L, i)  # never written
            else:
                assert st[i] == 0 and np.array_equal(back[o:o + L], pt[i * ins:i * ins + L]), (L, i)


@pytest.mark.parametrize("cipher,lanes,count,maxlen", [
    (CHACHA, 0, 300, 9000), (CHACHA, 4, 1500, 3000), (CHACHA, 8, 1500, 3000), (CHACHA, 16, 200, 3000),
    (CHACHA, 64, 100, 16384), (AES, 0, 300, 5000), (AES, 4, 1500, 3000), (AES, 4, 70_000, 200),
    (AES, 4, 140_000, 100)])
@pytest.mark.parametrize("fast", [True, False])
def test_ragged_verify_first(aead, gpu, oracle, cipher, lanes, count, maxlen, fast):
    import torch
    rng = np.random.default_rng(61 + lanes + count + (cipher & 3) + 7 * fast)
    S = 5
    keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
    ctx, _k = prepare(aead, cipher, keys)
    cb = aead.dev_ctx_bytes(cipher)
    state_of = np.sort(rng.integers(0, S, count))
    lens = rng.integers(0, maxlen, count)
    slot = lambda L: ((int(L) + 16 + 63) // 64) * 64 if fast else int(L) + 16 + 3
    offs = np.zeros(count, dtype=np.int64)
    offs[1:] = np.cumsum([slot(L) for L in lens])[:-1]
    total = int(offs[-1]) + slot(lens[-1]) + 64
    pt = rng.integers(0, 256, total, dtype=np.uint8)
    nonces = rng.integers(0, 2**62, count, dtype=np.int64).astype(np.uint64)
    recs = np.zeros(count, dtype=REC_DT)
    recs["in_off"] = recs["out_off"] = offs
    recs["nonce"] = nonces
    recs["ctx_off"] = state_of.astype(np.uint64) * cb
    recs["len"] = lens
    d_recs = dev(recs.view(np.uint8))
    flags = FAST if fast else 0
    d_pt = dev(pt)
    d_ct = torch.zeros(total, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(False, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_pt.data_ptr(), out=d_ct.data_ptr(), n_records=count, flags=flags,
                           lanes=lanes, stream=stream()) == 0
    sync()
    ct = d_ct.cpu().numpy()
    for i in list(range(0, count, max(1, count // 60))) + [count - 1]:
        o, L = int(offs[i]), int(lens[i])
        exp = oracle.encrypt(cipher, bytes(keys[state_of[i]]), int(nonces[i]), bytes(pt[o:o + L]))
        assert bytes(ct[o:o + L + 16]) == exp, i
    bad = (np.arange(count) % 29) == 3
    for i in np.nonzero(bad)[0]:
        o, L = int(offs[i]), int(lens[i])
        ct[o + int(rng.integers(0, L + 16))] ^= 0x02
    d_ct = dev(ct)
    d_out = torch.full((total,), 0x3C, dtype=torch.uint8, device="cuda")
    d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(True, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_ct.data_ptr(), out=d_out.data_ptr(), n_records=count,
                           status=d_st.data_ptr(), flags=flags | VF, lanes=lanes,
                           stream=stream()) == 0
    sync()
    st, back = d_st.cpu().numpy(), d_out.cpu().numpy()
    assert np.array_equal(st != 0, bad)
    for i in range(count):
        o, L = int(offs[i]), int(lens[i])
        if bad[i]:
            assert np.all(back[o:o + L] == 0x3C), i  # never written
        else:
            assert np.array_equal(back[o:o + L], pt[o:o + L]), i
    # in place: the rejected records' bytes read back exactly as given
    d_st.fill_(9)
    assert aead.dev_ragged(True, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_ct.data_ptr(), out=d_ct.data_ptr(), n_records=count,
                           status=d_st.data_ptr(), flags=flags | VF, lanes=lanes,
                           stream=stream()) == 0
    sync()
    back = d_ct.cpu().numpy()
    assert np.array_equal(d_st.cpu().numpy() != 0, bad)
    for i in np.nonzero(bad)[0]:
        o, L = int(offs[i]), int(lens[i])
        assert np.array_equal(back[o:o + L + 16], ct[o:o + L + 16]), i
