"""Session key fan-out: noise_aead_dev_hkdf / _split.

The device HKDF must equal the reference's noise_hashstate_hkdf
(hashstate.c:476-516) byte for byte: against the reference's own outputs
(tests/golden/hkdf.json, gen_hkdf.py) and against the oracle on a large
random batch for each of the four Noise hashes.  The split keys then drive
the transport ciphers: a record sealed under noise_aead_dev_split's k1 must
equal the oracle's seal under the oracle's split of the same ck."""
import json
import os

import numpy as np
import pytest

HASHES = [0x4801, 0x4802, 0x4803, 0x4804]
HLEN = {0x4801: 32, 0x4802: 64, 0x4803: 32, 0x4804: 64}


def test_dev_hkdf_argument_rules(aead):
    """Validation before any launch (no GPU work): hashstate.c:496-497."""
    A = aead
    assert A.dev_hkdf(0x4899, keys=8, key_len=32, n=1, out1=8, out1_len=32, out2=8,
                      out2_len=32) == A.ERROR_UNKNOWN_ID
    assert A.dev_hkdf(0x4803, keys=8, key_len=32, n=1, out1=8, out1_len=33, out2=8,
                      out2_len=32) == A.ERROR_INVALID_LENGTH
    assert A.dev_hkdf(0x4803, keys=0, key_len=32, n=1, out1=8, out1_len=32, out2=8,
                      out2_len=32) == A.ERROR_INVALID_PARAM
    assert A.dev_hkdf(0x4803, keys=8, key_len=32, data=0, data_len=5, n=1, out1=8,
                      out1_len=32, out2=8, out2_len=32) == A.ERROR_INVALID_PARAM
    assert A.dev_hkdf(0x4804, keys=8, key_len=300, n=1, out1=8, out1_len=32, out2=8,
                      out2_len=32) == A.ERROR_INVALID_LENGTH
    assert A.dev_hkdf(0x4804, keys=8, key_len=64, n=0, out1=8, out1_len=32, out2=8,
                      out2_len=32) == A.ERROR_NONE


def _run_hkdf(A, torch, hid, keys, data, l1, l2):
    n, kl = keys.shape
    dl = data.shape[1] if data is not None else 0
    d_keys = torch.from_numpy(keys.reshape(-1).copy()).cuda()
    d_data = torch.from_numpy(data.reshape(-1).copy()).cuda() if dl else None
    o1 = torch.zeros(n * max(l1, 1), dtype=torch.uint8, device="cuda")
    o2 = torch.zeros(n * max(l2, 1), dtype=torch.uint8, device="cuda")
    assert A.dev_hkdf(hid, keys=d_keys.data_ptr(), key_len=kl,
                      data=d_data.data_ptr() if dl else 0, data_len=dl, n=n,
                      out1=o1.data_ptr(), out1_len=l1, out2=o2.data_ptr(), out2_len=l2,
                      stream=torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    return o1.cpu().numpy()[:n * l1].reshape(n, l1), o2.cpu().numpy()[:n * l2].reshape(n, l2)


@pytest.mark.gpu
def test_dev_hkdf_reference_golden(aead, gpu):
    import torch
    with open(os.path.join(os.path.dirname(__file__), "golden", "hkdf.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        key = np.frombuffer(bytes.fromhex(c["key"]), dtype=np.uint8)[None, :]
        data = bytes.fromhex(c["data"])
        dat = np.frombuffer(data, dtype=np.uint8)[None, :] if data else None
        l1, l2 = len(c["out1"]) // 2, len(c["out2"]) // 2
        o1, o2 = _run_hkdf(aead, torch, c["hash_id"], key, dat, l1, l2)
        assert bytes(o1[0]).hex() == c["out1"] and bytes(o2[0]).hex() == c["out2"], c


@pytest.mark.gpu
@pytest.mark.parametrize("hid", HASHES)
def test_dev_split_batch_matches_oracle(aead, gpu, oracle, hid):
    """4096 sessions (C4/C5's state count) through the split shape, plus a
    mix_key batch (HKDF(ck, 32-byte DH output) -> new ck and temp key)."""
    import torch
    rng = np.random.default_rng(hid)
    n, hl = 4096, HLEN[hid]
    ck = rng.integers(0, 256, (n, hl), dtype=np.uint8)
    d_ck = torch.from_numpy(ck.reshape(-1).copy()).cuda()
    k1 = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    k2 = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    assert aead.dev_split(hid, ck=d_ck.data_ptr(), n=n, k1=k1.data_ptr(), k2=k2.data_ptr()) == 0
    torch.cuda.synchronize()
    k1h, k2h = k1.cpu().numpy().reshape(n, 32), k2.cpu().numpy().reshape(n, 32)
    for i in list(range(0, n, 97)) + [n - 1]:
        e1, e2 = oracle.hkdf(hid, bytes(ck[i]), b"", 32, 32)
        assert bytes(k1h[i]) == e1 and bytes(k2h[i]) == e2, i
    dh = rng.integers(0, 256, (256, 32), dtype=np.uint8)
    o1, o2 = _run_hkdf(aead, torch, hid, ck[:256], dh, hl, hl)
    for i in range(0, 256, 17):
        e1, e2 = oracle.hkdf(hid, bytes(ck[i]), bytes(dh[i]), hl, hl)
        assert bytes(o1[i]) == e1 and bytes(o2[i]) == e2, i


@pytest.mark.gpu
@pytest.mark.parametrize("cipher", [0x4301, 0x4302])
def test_split_keys_drive_transport(aead, gpu, oracle, cipher):
    """split -> noise_aead_dev_prepare -> seal, all on the device; equal to
    the oracle's split + encrypt (the c1 direction, nonce 0..)."""
    import torch
    rng = np.random.default_rng(cipher)
    n, L = 64, 300
    ck = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d_ck = torch.from_numpy(ck.reshape(-1).copy()).cuda()
    k1 = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    k2 = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    assert aead.dev_split(0x4801, ck=d_ck.data_ptr(), n=n, k1=k1.data_ptr(), k2=k2.data_ptr(),
                          stream=sp) == 0
    ctx = torch.empty(n * aead.dev_ctx_bytes(cipher), dtype=torch.uint8, device="cuda")
    assert aead.dev_prepare(cipher, k1.data_ptr(), n, ctx.data_ptr(), sp) == 0
    pt = rng.integers(0, 256, (n, 320), dtype=np.uint8)
    d_pt = torch.from_numpy(pt.reshape(-1).copy()).cuda()
    d_ct = torch.zeros(n * 320, dtype=torch.uint8, device="cuda")
    nb = torch.zeros(n, dtype=torch.int64, device="cuda")
    assert aead.dev_uniform(False, cipher, ctx=ctx.data_ptr(), nonce_base=nb.data_ptr(),
                            inp=d_pt.data_ptr(), out=d_ct.data_ptr(), in_stride=320,
                            out_stride=320, length=L, n_records=n, recs_per_state=1,
                            stream=sp) == 0
    torch.cuda.synchronize()
    ct = d_ct.cpu().numpy().reshape(n, 320)
    for i in range(n):
        key1, _ = oracle.hkdf(0x4801, bytes(ck[i]), b"", 32, 32)
        assert bytes(ct[i, :L + 16]) == oracle.encrypt(cipher, key1, 0, bytes(pt[i, :L])), i


@pytest.mark.gpu
@pytest.mark.parametrize("cipher,hid", [(0x4301, 0x4801), (0x4302, 0x4803), (0x4301, 0x4804),
                                        (0x4302, 0x4802)])
def test_encrypt_and_hash_batch(aead, gpu, oracle, cipher, hid):
    """noise_symmetricstate_{encrypt,decrypt}_and_hash (symmetricstate.c
    :352-445) for 300 states at once: AD = h_i; h_i <- HASH(h_i || CT || tag);
    a record whose tag fails keeps its old h and its ciphertext."""
    import torch
    rng = np.random.default_rng(cipher + hid)
    n, hl = 300, HLEN[hid]
    keys = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d_keys = torch.from_numpy(keys.reshape(-1).copy()).cuda()
    cb = aead.dev_ctx_bytes(cipher)
    ctx = torch.empty(n * cb, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    assert aead.dev_prepare(cipher, d_keys.data_ptr(), n, ctx.data_ptr(), sp) == 0
    h0 = rng.integers(0, 256, (n, hl), dtype=np.uint8)
    lens = rng.integers(0, 1500, n)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens + 16 + 7)[:-1]
    total = int(offs[-1] + lens[-1] + 16 + 64)
    pt = rng.integers(0, 256, total, dtype=np.uint8)
    nonces = rng.integers(0, 2**40, n).astype(np.uint64)
    dt = [("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
          ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")]
    recs = np.zeros(n, dtype=dt)
    recs["in_off"] = recs["out_off"] = offs
    recs["nonce"] = nonces
    recs["ctx_off"] = np.arange(n, dtype=np.uint64) * cb
    recs["ad_off"] = np.arange(n, dtype=np.uint64) * hl
    recs["len"] = lens
    recs["ad_len"] = hl
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
    d_buf = torch.from_numpy(pt.copy()).cuda()
    d_h = torch.from_numpy(h0.reshape(-1).copy()).cuda()
    kw = dict(ctx_base=ctx.data_ptr(), h=d_h.data_ptr(), recs=d_recs.data_ptr(), inp=d_buf.data_ptr(),
              out=d_buf.data_ptr(), n_records=n, stream=sp)
    # job->ad must be the hashes
    assert aead.dev_and_hash(False, cipher, hid, **kw) == 0
    torch.cuda.synchronize()
    ct = d_buf.cpu().numpy()
    h1 = d_h.cpu().numpy().reshape(n, hl)
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        exp = oracle.encrypt(cipher, bytes(keys[i]), int(nonces[i]), bytes(pt[o:o + L]),
                             bytes(h0[i]))
        assert bytes(ct[o:o + L + 16]) == exp, i
        assert bytes(h1[i]) == oracle.hash(hid, bytes(h0[i]) + exp), i
    # the receiving side: same h0, tampered records fail and keep h0
    bad = np.arange(n) % 23 == 4
    tampered = ct.copy()
    for i in np.nonzero(bad)[0]:
        tampered[int(offs[i]) + int(lens[i]) + 3] ^= 1
    d_buf = torch.from_numpy(tampered.copy()).cuda()
    d_h = torch.from_numpy(h0.reshape(-1).copy()).cuda()
    d_st = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    kw.update(h=d_h.data_ptr(), inp=d_buf.data_ptr(), out=d_buf.data_ptr())
    assert aead.dev_and_hash(True, cipher, hid, status=d_st.data_ptr(), **kw) == 0
    torch.cuda.synchronize()
    st, back, h2 = d_st.cpu().numpy(), d_buf.cpu().numpy(), d_h.cpu().numpy().reshape(n, hl)
    assert np.array_equal(st != 0, bad)
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        if bad[i]:
            assert bytes(h2[i]) == bytes(h0[i]) and np.array_equal(back[o:o + L + 16],
                                                                   tampered[o:o + L + 16]), i
        else:
            assert np.array_equal(back[o:o + L], pt[o:o + L]), i
            assert bytes(h2[i]) == oracle.hash(hid, bytes(h0[i]) + bytes(ct[o:o + L + 16])), i
