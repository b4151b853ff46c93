"""Full-size bit-exactness of the bench workloads.

tests/golden/config_digests.json holds, for C2, C3 and C4 at N = 1, the
SHA-256 of the packed plaintexts and of the packed sealed records (ct || tag)
that the CPU oracle produces over bench.py's synthetic inputs (SplitMix64,
SURVEY.md §8d); every one of them (C2, C3, C4, C5, perf) was also
reproduced through the reference's own CipherState API, one call per record
(`reference_checked`; gen_config_digests.py --ref-check).  The GPU test regenerates the same
inputs in HBM, seals every record of the full batch with the gfx950 kernels,
and compares the digest of every output byte; the open then has to accept
every record and give back the plaintext digest.
"""
import hashlib
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED_PT, SEED_KEY = 0x7074, 0x6B6579


def _golden():
    with open(os.path.join(ROOT, "tests", "golden", "config_digests.json")) as f:
        return json.load(f)["configs"]


def test_oracle_reproduces_c2_digest(oracle):
    """CPU: the oracle regenerates C2's plaintext and sealed digests (2 s)."""
    c = _golden()["c2"]
    N, L, ins, outs = c["records"], c["len"], c["in_stride"], c["out_stride"]
    keys = np.frombuffer(oracle.fill(SEED_KEY, 32, 0), dtype=np.uint8).copy()
    pt = np.frombuffer(oracle.fill(SEED_PT, N * ins, 0), dtype=np.uint8).copy()
    assert hashlib.sha256(pt.reshape(N, ins)[:, :L].tobytes()).hexdigest() == c["pt_sha256"]
    ct = np.zeros(N * outs, dtype=np.uint8)
    oracle.seal_uniform(c["cipher"], keys, np.zeros(1, dtype=np.uint64), N, pt, ins, ct, outs, L, N)
    assert hashlib.sha256(ct.reshape(N, outs)[:, :L + 16].tobytes()).hexdigest() == c["sealed_sha256"]
    assert c.get("reference_checked")


def test_every_config_digest_reference_checked():
    """no full-size golden digest rests on the oracle
    alone — C3 (AES-GCM) and C4 (4096 states) were re-derived through the
    reference build too."""
    for name, c in _golden().items():
        assert c.get("reference_checked") is True, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c2", "c3", "c4"])
def test_full_config_digest_on_gpu(name):
    import torch

    import noise_aead as A
    A.lib()  # raises loudly if the gfx950 library is missing
    c = _golden()[name]
    N, L, S, ins, outs = c["records"], c["len"], c["states"], c["in_stride"], c["out_stride"]
    cipher = c["cipher"]
    sp = torch.cuda.current_stream().cuda_stream
    raw = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
    for k in range(S):
        assert A.dev_fill_splitmix(raw[32 * k:].data_ptr(), 32, SEED_KEY, 4 * k, sp) == 0
    ctx = torch.empty(S * A.dev_ctx_bytes(cipher), dtype=torch.uint8, device="cuda")
    assert A.dev_prepare(cipher, raw.data_ptr(), S, ctx.data_ptr(), sp) == 0
    nb = torch.zeros(S, dtype=torch.int64, device="cuda")
    pt = torch.empty(N * ins, dtype=torch.uint8, device="cuda")
    assert A.dev_fill_splitmix(pt.data_ptr(), pt.numel(), SEED_PT, 0, sp) == 0
    ct = torch.empty(N * outs, dtype=torch.uint8, device="cuda")
    rc = A.dev_uniform(False, cipher, ctx=ctx.data_ptr(), nonce_base=nb.data_ptr(),
                       inp=pt.data_ptr(), out=ct.data_ptr(), in_stride=ins, out_stride=outs,
                       length=L, n_records=N, recs_per_state=N // S, stream=sp)
    assert rc == 0
    sealed = ct.view(N, outs)[:, :L + 16].contiguous().cpu().numpy()
    assert hashlib.sha256(sealed.tobytes()).hexdigest() == c["sealed_sha256"], name
    del sealed
    back = torch.empty(N * ins, dtype=torch.uint8, device="cuda")
    st = torch.full((N,), 9, dtype=torch.uint8, device="cuda")
    rc = A.dev_uniform(True, cipher, ctx=ctx.data_ptr(), nonce_base=nb.data_ptr(),
                       inp=ct.data_ptr(), out=back.data_ptr(), in_stride=outs, out_stride=ins,
                       length=L, n_records=N, recs_per_state=N // S, status=st.data_ptr(),
                       stream=sp)
    assert rc == 0
    assert int(st.max().item()) == 0
    opened = back.view(N, ins)[:, :L].contiguous().cpu().numpy()
    assert hashlib.sha256(opened.tobytes()).hexdigest() == c["pt_sha256"], name


def _shard_golden():
    with open(os.path.join(ROOT, "tests", "golden", "shard_digests.json")) as f:
        return json.load(f)["configs"]


def _mask_t(off, lens, buf):
    """Mask of the bytes [off_i, off_i + lens_i) of every record of buf, built
    on the GPU (a +1/-1 boundary cumsum); records are in offset order, so
    buf[mask] is the records' bytes packed in record order."""
    import torch
    edge = torch.zeros(buf.numel() + 1, dtype=torch.int32, device=buf.device)
    o = torch.from_numpy(off).to(buf.device)
    e = o + torch.from_numpy(lens).to(buf.device)
    edge.index_add_(0, o, torch.ones_like(o, dtype=torch.int32))
    edge.index_add_(0, e, -torch.ones_like(e, dtype=torch.int32))
    return torch.cumsum(edge[:-1], 0) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("rank", range(8))
def test_c5_shard_digest_on_gpu(rank):
    """C5 rank by rank (bench.py run_mixed at rank r of the 8-GPU job, laid
    out on this one GPU): the mixed ChaChaPoly/AES-GCM ragged batch of rank
    r — 128 Ki records of 64 B-16 KiB over its 512 states, its own length
    mix, nonces, key ids and state parities — sealed with the FAST ragged
    kernels; every record's ct || tag, in record order, hashes to the digest
    of the reference build for that rank (tests/golden/shard_digests.json;
    rank 0 is also config_digests.json's), and the open accepts every record
    and restores every plaintext."""
    import torch

    import noise_aead as A
    from bench import CHACHA, AES, CONFIGS as BC, mixed_layout
    A.lib()
    want = _shard_golden()["c5"]["rank_sealed_sha256"][rank]
    R, S = BC["c5"]["records"], BC["c5"]["states"]
    if rank == 0:
        c = _golden()["c5"]
        assert (R, S) == (c["records"], c["states"]) and want == c["sealed_sha256"]
    lay = mixed_layout(R, S, rank)
    sp = torch.cuda.current_stream().cuda_stream
    rec_dt = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
                       ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")])
    pt = torch.empty(lay["total"], dtype=torch.uint8, device="cuda")
    assert A.dev_fill_splitmix(pt.data_ptr(), pt.numel(), SEED_PT, rank << 40, sp) == 0
    ct = torch.zeros_like(pt)
    back = torch.zeros_like(pt)
    groups = []
    for cipher, parity in ((CHACHA, 0), (AES, 1)):
        states = [s for s in range(S) if (rank * S + s) % 2 == parity]
        cb = A.dev_ctx_bytes(cipher)
        raw = torch.empty(len(states) * 32, dtype=torch.uint8, device="cuda")
        for i, s in enumerate(states):
            assert A.dev_fill_splitmix(raw[32 * i:].data_ptr(), 32, SEED_KEY, 4 * (rank * S + s), sp) == 0
        ctx = torch.empty(len(states) * cb, dtype=torch.uint8, device="cuda")
        assert A.dev_prepare(cipher, raw.data_ptr(), len(states), ctx.data_ptr(), sp) == 0
        slot_of = {s: i for i, s in enumerate(states)}
        idx = np.nonzero((lay["st_global"] % 2) == parity)[0]
        recs = np.zeros(len(idx), dtype=rec_dt)
        recs["in_off"] = lay["off"][idx]
        recs["out_off"] = lay["off"][idx]
        recs["nonce"] = lay["nonce"][idx]
        recs["ctx_off"] = np.array([slot_of[s] for s in lay["st_local"][idx]], dtype=np.uint64) * cb
        recs["len"] = lay["lens"][idx]
        d_recs = torch.from_numpy(recs.view(np.uint8)).to("cuda")
        st = torch.full((len(idx),), 9, dtype=torch.uint8, device="cuda")
        groups.append((cipher, ctx, d_recs, len(idx), st))
    for open_, src, dst in ((False, pt, ct), (True, ct, back)):
        for cipher, ctx, d_recs, n, st in groups:
            rc = A.dev_ragged(open_, cipher, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                              inp=src.data_ptr(), out=dst.data_ptr(), n_records=n,
                              status=st.data_ptr() if open_ else 0, flags=A.FLAG_FAST, stream=sp)
            assert rc == 0
    torch.cuda.synchronize()
    for g in groups:
        assert int(g[4].max().item()) == 0
    off, lens = lay["off"].astype(np.int64), lay["lens"].astype(np.int64)
    sealed = ct[_mask_t(off, lens + 16, ct)].cpu().numpy()
    assert hashlib.sha256(sealed.tobytes()).hexdigest() == want, rank
    del sealed
    m = _mask_t(off, lens, pt)
    assert torch.equal(back[m], pt[m])


@pytest.mark.gpu
@pytest.mark.parametrize("name,lanes,vf", [("c2", 0, False), ("c2", 4, False), ("c3", 0, False),
                                           ("c2", 0, True), ("c3", 0, True), ("c4", 0, False),
                                           ("c4", 0, True), ("perf", 0, True)])
def test_full_size_duplex_at_bench_slots(name, lanes, vf):
    """The kernels bench.py times: C2 / C3 at full size
    through noise_aead_dev_duplex_uniform at the bench's 128-B record slots
    (in_stride 1408, out_stride 1536), one state, recs_per_state 65 536 —
    chachapoly_duplex_solo<true> (the default: one lane per record; lanes=4
    the four-lane chachapoly_duplex_staged<4, true>) / gcm_duplex_fused<false>.  The seal
    half's sealed records hash to the golden digest (cipher-chachapoly.c
    :107-133 / cipher-aesgcm.c:156-170 bytes); the open half, over a batch
    sealed beforehand with 64 records tampered, accepts every other record
    with the plaintext digest and rejects (zeroes) exactly the tampered ones.
    vf: the open half in the default order — verify first since round 6,
    the bench's default line, still one launch: rejected records never
    written; not vf: the open half with NOISE_AEAD_FLAG_ONE_PASS (the bench's
    --one-pass line): rejected records zeroed.
    c4: the timed kernel of C4 — the one-lane duplex
    over 4096 states x 256 records; perf: the duplex of 1024-B records with
    32 B of AD each (both reference-checked digests, the perf one through
    the reference's own CipherState API)."""
    import torch

    import noise_aead as A
    A.lib()
    c = _golden()[name]
    N, L, cipher, S, AD = c["records"], c["len"], c["cipher"], c["states"], c.get("ad", 0)
    # bench.py SLOT_ALIGN = 128: strides roundup128(len), roundup128(len + 16)
    ins, outs = (L + 127) // 128 * 128, (L + 16 + 127) // 128 * 128
    # the golden plaintext is the SplitMix64 stream over 16-B slots
    gins = c["in_stride"]
    sp = torch.cuda.current_stream().cuda_stream
    raw = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
    for k in range(S):
        assert A.dev_fill_splitmix(raw[32 * k:].data_ptr(), 32, SEED_KEY, 4 * k, sp) == 0
    ctx = torch.empty(S * A.dev_ctx_bytes(cipher), dtype=torch.uint8, device="cuda")
    assert A.dev_prepare(cipher, raw.data_ptr(), S, ctx.data_ptr(), sp) == 0
    nb = torch.zeros(S, dtype=torch.int64, device="cuda")
    gpt = torch.empty(N * gins, dtype=torch.uint8, device="cuda")
    assert A.dev_fill_splitmix(gpt.data_ptr(), gpt.numel(), SEED_PT, 0, sp) == 0
    pt = torch.zeros(N * ins, dtype=torch.uint8, device="cuda")
    pt.view(N, ins)[:, :L] = gpt.view(N, gins)[:, :L]
    del gpt
    assert hashlib.sha256(pt.view(N, ins)[:, :L].contiguous().cpu().numpy().tobytes()).hexdigest() \
        == c["pt_sha256"]
    ad_kw = {}
    if AD:
        adb = torch.empty(N * AD, dtype=torch.uint8, device="cuda")
        assert A.dev_fill_splitmix(adb.data_ptr(), adb.numel(), 0x6164, 0, sp) == 0
        ad_kw = dict(ad=adb.data_ptr(), ad_stride=AD, ad_len=AD)
    common = dict(ctx=ctx.data_ptr(), nonce_base=nb.data_ptr(), length=L, n_records=N,
                  recs_per_state=N // S, lanes=lanes, **ad_kw)
    # batch B: sealed by the separate kernel, then tampered
    ct_b = torch.empty(N * outs, dtype=torch.uint8, device="cuda")
    assert A.dev_uniform(False, cipher, inp=pt.data_ptr(), out=ct_b.data_ptr(), in_stride=ins,
                         out_stride=outs, stream=sp, **common) == 0
    rng = np.random.default_rng(17 + (cipher & 3))
    bad = np.unique(rng.integers(0, N, 64))
    pos = torch.from_numpy(bad * outs + rng.integers(0, L + 16, len(bad))).to("cuda")
    flat = ct_b.view(-1)
    flat[pos] ^= 0x40
    # one duplex launch: seal A (same plaintext) while opening B
    ct_a = torch.empty(N * outs, dtype=torch.uint8, device="cuda")
    back = torch.full((N * ins,), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((N,), 9, dtype=torch.uint8, device="cuda")
    sj = A.uniform_job(inp=pt.data_ptr(), out=ct_a.data_ptr(), in_stride=ins, out_stride=outs, **common)
    oj = A.uniform_job(inp=ct_b.data_ptr(), out=back.data_ptr(), in_stride=outs, out_stride=ins,
                       status=st.data_ptr(), flags=0 if vf else A.FLAG_ONE_PASS, **common)
    assert A.dev_duplex(cipher, sj, oj, sp) == 0
    torch.cuda.synchronize()
    sealed = ct_a.view(N, outs)[:, :L + 16].contiguous().cpu().numpy()
    assert hashlib.sha256(sealed.tobytes()).hexdigest() == c["sealed_sha256"], name
    del sealed
    s = st.cpu().numpy()
    exp = np.zeros(N, dtype=np.uint8)
    exp[bad] = 1
    assert np.array_equal(s, exp), np.nonzero(s != exp)[0][:10]
    bv, pv = back.view(N, ins)[:, :L], pt.view(N, ins)[:, :L]
    good = torch.ones(N, dtype=torch.bool, device="cuda")
    good[torch.from_numpy(bad).to("cuda")] = False
    assert torch.equal(bv[good], pv[good])
    # rejected records: zeroed out of place (ONE_PASS ChaChaPoly) / never
    # written (verify-first: the default, and every AES-GCM open)
    fill = 0xA5 if (vf or cipher == A.AESGCM) else 0
    assert int(bv[~good].max().item()) == fill
    assert int(bv[~good].min().item()) == fill


@pytest.mark.gpu
@pytest.mark.parametrize("name,vf,in_place", [("c2", True, False), ("c2", True, True), ("c2", False, False),
                                              ("perf", True, False)])
def test_full_size_standalone_open_at_bench_slots(name, vf, in_place):
    """The standalone opens of the bench's per-direction pass and --mode
    separate at full size and the bench slots: since round 6 a verify-first
    open of 64 Ki FAST records runs four lanes per record
    (chachapoly_open_staged_vf<4, true>); with NOISE_AEAD_FLAG_ONE_PASS the
    one-pass chachapoly_open_staged<4, true>.  A batch sealed by the library
    (its sealed digest checked against the golden one) with 64 records
    tampered: every other record opens to the plaintext, the tampered ones
    get status 1 and are never written (verify-first: out of place the fill
    stays, in place the ciphertext stays) or zeroed (one pass, out of
    place)."""
    import torch

    import noise_aead as A
    A.lib()
    c = _golden()[name]
    N, L, cipher, S, AD = c["records"], c["len"], c["cipher"], c["states"], c.get("ad", 0)
    ins, outs = (L + 127) // 128 * 128, (L + 16 + 127) // 128 * 128
    gins = c["in_stride"]
    sp = torch.cuda.current_stream().cuda_stream
    raw = torch.empty(S * 32, dtype=torch.uint8, device="cuda")
    for k in range(S):
        assert A.dev_fill_splitmix(raw[32 * k:].data_ptr(), 32, SEED_KEY, 4 * k, sp) == 0
    ctx = torch.empty(S * A.dev_ctx_bytes(cipher), dtype=torch.uint8, device="cuda")
    assert A.dev_prepare(cipher, raw.data_ptr(), S, ctx.data_ptr(), sp) == 0
    nb = torch.zeros(S, dtype=torch.int64, device="cuda")
    gpt = torch.empty(N * gins, dtype=torch.uint8, device="cuda")
    assert A.dev_fill_splitmix(gpt.data_ptr(), gpt.numel(), SEED_PT, 0, sp) == 0
    pt = torch.zeros(N * ins, dtype=torch.uint8, device="cuda")
    pt.view(N, ins)[:, :L] = gpt.view(N, gins)[:, :L]
    del gpt
    ad_kw = {}
    if AD:
        adb = torch.empty(N * AD, dtype=torch.uint8, device="cuda")
        assert A.dev_fill_splitmix(adb.data_ptr(), adb.numel(), 0x6164, 0, sp) == 0
        ad_kw = dict(ad=adb.data_ptr(), ad_stride=AD, ad_len=AD)
    common = dict(ctx=ctx.data_ptr(), nonce_base=nb.data_ptr(), length=L, n_records=N,
                  recs_per_state=N // S, **ad_kw)
    ct = torch.empty(N * outs, dtype=torch.uint8, device="cuda")
    assert A.dev_uniform(False, cipher, inp=pt.data_ptr(), out=ct.data_ptr(), in_stride=ins,
                         out_stride=outs, stream=sp, **common) == 0
    torch.cuda.synchronize()
    sealed = ct.view(N, outs)[:, :L + 16].contiguous().cpu().numpy()
    assert hashlib.sha256(sealed.tobytes()).hexdigest() == c["sealed_sha256"], name
    del sealed
    rng = np.random.default_rng(29 + 2 * vf + in_place)
    bad = np.unique(rng.integers(0, N, 64))
    pos = torch.from_numpy(bad * outs + rng.integers(0, L + 16, len(bad))).to("cuda")
    ct.view(-1)[pos] ^= 0x40
    tampered = ct.clone()
    st = torch.full((N,), 9, dtype=torch.uint8, device="cuda")
    if in_place:
        out, out_stride = ct, outs
    else:
        out, out_stride = torch.full((N * ins,), 0xA5, dtype=torch.uint8, device="cuda"), ins
    assert A.dev_uniform(True, cipher, inp=ct.data_ptr(), out=out.data_ptr(), in_stride=outs,
                         out_stride=out_stride, status=st.data_ptr(),
                         flags=0 if vf else A.FLAG_ONE_PASS, stream=sp, **common) == 0
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    exp = np.zeros(N, dtype=np.uint8)
    exp[bad] = 1
    assert np.array_equal(s, exp), np.nonzero(s != exp)[0][:10]
    good = torch.ones(N, dtype=torch.bool, device="cuda")
    good[torch.from_numpy(bad).to("cuda")] = False
    bv = out.view(N, out_stride)
    assert torch.equal(bv[good][:, :L], pt.view(N, ins)[:, :L][good])
    if in_place:  # rejected: the ciphertext and tag as given
        tv = tampered.view(N, outs)[:, :L + 16]
        assert torch.equal(bv[~good][:, :L + 16], tv[~good])
    else:
        fill = 0xA5 if vf else 0
        assert int(bv[~good][:, :L].max().item()) == fill
        assert int(bv[~good][:, :L].min().item()) == fill
