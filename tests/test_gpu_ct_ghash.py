"""NOISE_AEAD_FLAG_CT_GHASH: the table-free GHASH (aesgcm.hip gh_mul_ct)
through every AES-GCM kernel, bit-exact against the oracle (itself pinned to
the reference's AES-GCM, tests/test_oracle.py) and equal to the default
table GHASH on the same inputs:

- the reference's KATs (uniform, one record per state: gcm_uniform);
- uniform FAST batches with one state per 256 records (gcm_staged), with AD;
- ragged multi-state windows with tampered records (gcm_ragged_staged, FAST
  and any-alignment) and a small ragged batch (gcm_wide);
- NOISE_AEAD_CT_GHASH=1 in the environment: the golden grid through the
  CipherState API in a child process (the variable is read once per process).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_parity import AES, dev, gpu_uniform, oracle_seal_records, prepare, stream, sync

pytestmark = pytest.mark.gpu


def test_ct_kats(aead, gpu, golden):
    kat, _ = golden
    n = 0
    for v in kat["vectors"]:
        if v["cipher"] != AES:
            continue
        key = np.frombuffer(bytes.fromhex(v["key"]), dtype=np.uint8).reshape(1, 32)
        pt, ad = bytes.fromhex(v["pt"]), bytes.fromhex(v["ad"])
        L = len(pt)
        inp = np.frombuffer(pt + bytes(16), dtype=np.uint8)
        adv = np.frombuffer(ad or b"\0", dtype=np.uint8)
        kw = dict(ad=adv, ad_stride=len(ad), ad_len=len(ad), flags=aead.FLAG_CT_GHASH)
        out, _ = gpu_uniform(aead, False, AES, key, [v["nonce"]], 1, inp, L + 16, L, 1, L + 16, **kw)
        assert bytes(out[:L + 16]).hex() == v["ct"] + v["tag"], v["name"]
        back, st = gpu_uniform(aead, True, AES, key, [v["nonce"]], 1, out[:L + 16], L + 16, L, 1,
                               L + 16, **kw)
        assert st[0] == 0 and bytes(back[:L]) == pt, v["name"]
        n += 1
    assert n > 0


@pytest.mark.parametrize("rps", [1, 256])
def test_ct_uniform_vs_oracle_and_tables(aead, gpu, oracle, rps):
    rng = np.random.default_rng(99 + rps)
    count = 600
    S = (count + rps - 1) // rps
    for L, adl in [(0, 0), (1, 0), (15, 0), (16, 0), (17, 0), (100, 0), (1400, 0), (1401, 0),
                   (4096, 0), (1400, 13), (64, 32), (0, 7)]:
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        nb = rng.integers(0, 2**62, S, dtype=np.uint64)
        in_stride = (max(L, 1) + 63) // 64 * 64
        out_stride = (L + 16 + 63) // 64 * 64
        pt = rng.integers(0, 256, count * in_stride + 64, dtype=np.uint8)
        ad = rng.integers(0, 256, count * 48 + 64, dtype=np.uint8)
        kw = dict(ad=ad, ad_stride=48, ad_len=adl) if adl else {}
        exp = oracle_seal_records(oracle, AES, keys, nb, rps, pt, in_stride, L, count, out_stride, **kw)
        got, _ = gpu_uniform(aead, False, AES, keys, nb, rps, pt, in_stride, L, count, out_stride,
                             flags=aead.FLAG_CT_GHASH, **kw)
        tab, _ = gpu_uniform(aead, False, AES, keys, nb, rps, pt, in_stride, L, count, out_stride, **kw)
        n = count * out_stride
        assert np.array_equal(got[:n], exp[:n]), f"len={L} ad={adl}"
        assert np.array_equal(got[:n], tab[:n])
        ct = got.copy()
        bad = sorted(set(int(x) for x in rng.integers(0, count, 7)))
        for b in bad:
            ct[b * out_stride + int(rng.integers(0, L + 16))] ^= 0x80
        back, st = gpu_uniform(aead, True, AES, keys, nb, rps, ct, out_stride, L, count, in_stride,
                               out_init=0x3C, flags=aead.FLAG_CT_GHASH, **kw)
        for i in range(count):
            seg = back[i * in_stride: i * in_stride + L]
            if i in bad:
                assert st[i] == 1 and np.all(seg == 0x3C), f"len={L} rec={i}"  # verified first: untouched
            else:
                assert st[i] == 0 and np.array_equal(seg, pt[i * in_stride: i * in_stride + L])


@pytest.mark.parametrize("lanes,count,fast", [(4, 1500, True), (4, 1500, False), (0, 300, False)])
def test_ct_ragged_vs_oracle(aead, gpu, oracle, lanes, count, fast):
    torch = __import__("torch")
    rng = np.random.default_rng(555 + lanes + count + fast)
    runs = []
    while sum(runs) < count:
        runs.append(int(rng.choice([1, 3, 40, 130, 300])))
    state_of = np.repeat(np.arange(len(runs)), runs)[:count]
    keys = rng.integers(0, 256, (len(runs), 32), dtype=np.uint8)
    ctx, _k = prepare(aead, AES, keys)
    cb = aead.dev_ctx_bytes(AES)
    lens = rng.integers(0, 3000, count)
    lens[:8] = [0, 1, 15, 16, 17, 64, 1400, 16384]
    adls = rng.choice([0, 0, 5, 32], count)
    slot = lambda L: ((int(L) + 16 + 63) // 64) * 64 if fast else int(L) + 16 + 5
    offs = np.zeros(count, dtype=np.int64)
    offs[1:] = np.cumsum([slot(L) for L in lens])[:-1]
    total = int(offs[-1]) + slot(lens[-1]) + 64
    pt = rng.integers(0, 256, total, dtype=np.uint8)
    ad = rng.integers(0, 256, count * 64, dtype=np.uint8)
    nonces = rng.integers(0, 2**62, count, dtype=np.int64).astype(np.uint64)
    dt = [("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
          ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")]
    recs = np.zeros(count, dtype=dt)
    recs["in_off"] = recs["out_off"] = offs
    recs["nonce"] = nonces
    recs["ctx_off"] = state_of.astype(np.uint64) * cb
    recs["ad_off"] = np.arange(count) * 64
    recs["len"] = lens
    recs["ad_len"] = adls
    d_recs, d_ad = dev(recs.view(np.uint8)), dev(ad)
    flags = (aead.FLAG_FAST if fast else 0) | aead.FLAG_CT_GHASH
    d_buf = dev(pt)
    kw = dict(ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(), n_records=count, ad=d_ad.data_ptr(),
              lanes=lanes, stream=stream())
    assert aead.dev_ragged(False, AES, inp=d_buf.data_ptr(), out=d_buf.data_ptr(), flags=flags, **kw) == 0
    sync()
    sealed = d_buf.cpu().numpy().copy()
    for i in range(count):
        o, L = int(offs[i]), int(lens[i])
        exp = oracle.encrypt(AES, bytes(keys[state_of[i]]), int(nonces[i]), bytes(pt[o:o + L]),
                             bytes(ad[64 * i: 64 * i + int(adls[i])]))
        assert bytes(sealed[o:o + L + 16]) == exp, i
    bad = np.arange(count) % 29 == 3
    tampered = sealed.copy()
    for i in np.nonzero(bad)[0]:
        tampered[int(offs[i]) + int(rng.integers(0, int(lens[i]) + 16))] ^= 0x04
    d_buf = dev(tampered)
    d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(True, AES, inp=d_buf.data_ptr(), out=d_buf.data_ptr(), flags=flags,
                           status=d_st.data_ptr(), **kw) == 0
    sync()
    st, back = d_st.cpu().numpy(), d_buf.cpu().numpy()
    assert np.array_equal(st != 0, bad)
    for i in range(count):
        o, L = int(offs[i]), int(lens[i])
        if bad[i]:
            assert np.array_equal(back[o:o + L + 16], tampered[o:o + L + 16]), i
        else:
            assert np.array_equal(back[o:o + L], pt[o:o + L]), i


_CHILD = r"""
import hashlib, json, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import noise_aead as A
from oracle import Oracle
grid = json.load(open(sys.argv[3]))
o = Oracle()
n = 0
for c in grid["cases"]:
    if c["cipher"] != 0x4302:
        continue
    st = A.CipherState.new_by_id(c["cipher"])[1]
    st.init_key(bytes.fromhex(c["key"]))
    if c["nonce"]:
        st.set_nonce(c["nonce"])
    pt = o.fill(grid["seed_pt"], c["len"], c["pt_word0"])
    ad = o.fill(grid["seed_ad"], c["ad_len"], c["ad_word0"])
    out = st.seal(pt, ad)
    assert hashlib.sha256(out).hexdigest() == c["sha256"], c
    st.free()
    n += 1
print("ok", n)
"""


def test_ct_env_through_cipherstate(gpu, tmp_path):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    grid = os.path.join(root, "tests", "golden", "grid.json")
    if not os.path.exists(grid):
        pytest.skip("grid fixture missing")
    env = dict(os.environ, NOISE_AEAD_CT_GHASH="1")
    r = subprocess.run([sys.executable, "-c", _CHILD, os.path.join(root, "noise-c_amd"),
                        os.path.join(root, "oracle"), grid],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[0] == "ok" and int(r.stdout.split()[1]) > 0
