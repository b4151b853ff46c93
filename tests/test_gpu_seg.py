"""GPU parity of the segmented one-lane ChaChaPoly kernels (chachapoly_seg.hip).

A record is cut into K contiguous segments, one lane each, whose Poly1305
chains are joined by r^e: the uniform K = 2 kernel (the standalone seal / open
of 64 Ki <= n < 128 Ki records) and the ragged kernel with its per-launch plan
(records bucketed by length, K from each record's length, persistent waves).
Every output byte is compared with the CPU oracle (oracle/noise_oracle.c,
pinned to the reference by tests/test_oracle.py): ciphertext and tag of every
record, the accept/reject decision of every open, the plaintext of accepted
records, and the bytes of rejected ones (in place: as given; out of place:
zeroed by a NOISE_AEAD_FLAG_ONE_PASS open, never written by a verify-first
one — the default order).
"""
import numpy as np
import pytest

from test_gpu_parity import CHACHA, dev, gpu_uniform, oracle_seal_records, prepare, stream, sync

pytestmark = pytest.mark.gpu

REC_DT = [("in_off", "<u8"), ("out_off", "<u8"), ("nonce", "<u8"), ("ctx_off", "<u8"),
          ("ad_off", "<u8"), ("len", "<u4"), ("ad_len", "<u4")]
EDGE_LENS = [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 129, 1400, 1983, 1984, 1985, 2047, 2048,
             4095, 4096, 4097, 8191, 8192, 16383, 16384, 16385, 30000, 40000, 65519]
REFUSED = [65520, 70000]


def _fast_slot(L):
    """a FAST slot: 16-B aligned, readable to roundup64(max(len, 1)), room for the tag"""
    return max(((max(int(L), 1) + 63) // 64) * 64, int(L) + 16) + 64


def _ragged_batch(rng, count, S):
    lens = rng.integers(0, 2600, count)
    big = rng.choice(count, count // 50, replace=False)
    lens[big] = rng.integers(2600, 16385, len(big))
    lens[:len(EDGE_LENS)] = EDGE_LENS
    lens[len(EDGE_LENS):len(EDGE_LENS) + len(REFUSED)] = REFUSED
    perm = rng.permutation(count)          # descriptors in no particular order
    lens = lens[perm]
    adls = np.where(rng.random(count) < 0.1, rng.integers(0, 48, count), 0)
    slots = np.array([_fast_slot(min(int(L), 65519)) for L in lens], dtype=np.int64)
    offs = np.zeros(count, dtype=np.int64)
    offs[1:] = np.cumsum(slots)[:-1]
    total = int(offs[-1] + slots[-1]) + 256
    recs = np.zeros(count, dtype=REC_DT)
    recs["in_off"] = recs["out_off"] = offs
    recs["nonce"] = rng.integers(0, 2**63, count, dtype=np.int64).astype(np.uint64)
    key_idx = rng.integers(0, S, count).astype(np.uint32)
    recs["ctx_off"] = key_idx.astype(np.uint64) * 32
    recs["ad_off"] = np.arange(count, dtype=np.uint64) * 64
    recs["len"] = lens
    recs["ad_len"] = adls
    return recs, key_idx, offs, lens, total


@pytest.mark.parametrize("vf", [False, True])
@pytest.mark.parametrize("inplace", [False, True, "mixed"])
def test_ragged_seg_vs_oracle(aead, gpu, oracle, vf, inplace):
    """20 000 records (past the segmented kernel's 16 384-record threshold):
    0 B - 64 KiB, the edge lengths of every segment count K = 1..16, two
    refused lengths (status 2, nothing written), AD on a tenth, 300 states,
    descriptors shuffled; seal out of place, then open (in place, out of
    place, or mixed — every other record's output in place, the rest in a
    second region of the same buffer, ADVICE r5 — one-pass or verify-first)
    with every 41st record tampered."""
    torch = __import__("torch")
    rng = np.random.default_rng(5150 + 2 * vf + (2 if inplace == "mixed" else int(inplace)))
    count, S = 20000, 300
    keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
    ctx, _k = prepare(aead, CHACHA, keys)
    recs, key_idx, offs, lens, total = _ragged_batch(rng, count, S)
    pt = rng.integers(0, 256, total, dtype=np.uint8)
    ad = rng.integers(0, 256, count * 64, dtype=np.uint8)
    exp = np.full(total, 0xA5, dtype=np.uint8)
    oracle.seal_ragged(CHACHA, np.ascontiguousarray(keys.reshape(-1)), key_idx, recs, pt, exp, ad)
    d_recs, d_pt, d_ad = dev(recs.view(np.uint8)), dev(pt), dev(ad)
    d_ct = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
    assert aead.dev_ragged(False, CHACHA, ctx_base=ctx.data_ptr(), recs=d_recs.data_ptr(),
                           inp=d_pt.data_ptr(), out=d_ct.data_ptr(), n_records=count,
                           ad=d_ad.data_ptr(), status=d_st.data_ptr(), flags=aead.FLAG_FAST,
                           stream=stream()) == 0
    sync()
    got = d_ct.cpu().numpy()
    refused = lens > 65519
    st = d_st.cpu().numpy()
    assert np.array_equal(st, np.where(refused, 2, 0)), np.nonzero(st != np.where(refused, 2, 0))[0][:8]
    if not np.array_equal(got, exp):
        bad = [i for i in range(count) if not refused[i] and not np.array_equal(
            got[offs[i]:offs[i] + lens[i] + 16], exp[offs[i]:offs[i] + lens[i] + 16])]
        pytest.fail(f"{len(bad)} records differ, e.g. {[(i, int(lens[i])) for i in bad[:6]]}")
    # open: tamper every 41st record (a CT or tag byte)
    tampered = got.copy()
    badm = (np.arange(count) % 41 == 7) & ~refused
    for i in np.nonzero(badm)[0]:
        tampered[offs[i] + int(rng.integers(0, lens[i] + 16))] ^= 0x08
    if inplace == "mixed":
        # one buffer: the ciphertext at [0, total), out-of-place outputs at
        # [total, 2 total); record i is in place when i is even
        ip = np.arange(count) % 2 == 0
        buf = np.concatenate([tampered, np.full(total, 0x5A, dtype=np.uint8)])
        d_in = d_out = dev(buf)
        orecs = recs.copy()
        orecs["out_off"] = np.where(ip, offs, offs + total).astype(np.uint64)
        d_orecs = dev(orecs.view(np.uint8))
        oo = np.where(ip, offs, offs + total)
    else:
        ip = np.full(count, bool(inplace))
        d_in = dev(tampered)
        d_out = d_in if inplace else torch.full((total,), 0x5A, dtype=torch.uint8, device="cuda")
        d_orecs = d_recs
        oo = offs
    d_st.fill_(9)
    flags = aead.FLAG_FAST | (0 if vf else aead.FLAG_ONE_PASS)  # vf: the default order
    assert aead.dev_ragged(True, CHACHA, ctx_base=ctx.data_ptr(), recs=d_orecs.data_ptr(),
                           inp=d_in.data_ptr(), out=d_out.data_ptr(), n_records=count,
                           ad=d_ad.data_ptr(), status=d_st.data_ptr(), flags=flags,
                           stream=stream()) == 0
    sync()
    st = d_st.cpu().numpy()
    want = np.where(refused, 2, np.where(badm, 1, 0))
    assert np.array_equal(st, want), np.nonzero(st != want)[0][:8]
    back = d_out.cpu().numpy()
    for i in range(count):
        o, L, q = int(offs[i]), int(lens[i]), int(oo[i])
        if refused[i]:
            seg = back[q:q + 16]
            assert np.array_equal(seg, tampered[o:o + 16] if ip[i] else np.full(16, 0x5A, np.uint8)), i
        elif badm[i]:
            if ip[i]:
                assert np.array_equal(back[q:q + L + 16], tampered[o:o + L + 16]), (i, L)
            else:
                assert np.all(back[q:q + L] == (0x5A if vf else 0)), (i, L)
        else:
            assert np.array_equal(back[q:q + L], pt[o:o + L]), (i, L)


LENS2 = [0, 1, 15, 16, 63, 64, 65, 127, 128, 191, 192, 1023, 1400, 1401, 4096, 5000, 65519]


@pytest.mark.parametrize("vf", [False, True])
@pytest.mark.parametrize("rps", [13, 64])
def test_uniform_seg2_vs_oracle(aead, gpu, oracle, vf, rps):
    """Two segments per record (lanes_per_record = 2 on a FAST layout): every
    length class of the split (a one-block record, the key block alone in the
    first segment, odd / even block counts, the 65519-byte maximum); rps 64 =
    one state per wave (scalar key), 13 = states straddling waves; open out of
    place with tampered records, then in place."""
    rng = np.random.default_rng(808 + 3 * vf + rps)
    for L in LENS2:
        count = 70 if L < 65519 else 9
        S = (count + rps - 1) // rps
        keys = rng.integers(0, 256, (S, 32), dtype=np.uint8)
        nb = rng.integers(0, 2**63, S, dtype=np.uint64)
        ins = ((max(L, 1) + 63) // 64) * 64 + 64
        outs = ins
        pt = rng.integers(0, 256, count * ins + 64, dtype=np.uint8)
        exp = oracle_seal_records(oracle, CHACHA, keys, nb, rps, pt, ins, L, count, outs)
        got, _ = gpu_uniform(aead, False, CHACHA, keys, nb, rps, pt, ins, L, count, outs, lanes=2)
        assert np.array_equal(got[:count * outs], exp[:count * outs]), f"seal len={L}"
        ct = got.copy()
        bad = sorted(set(rng.integers(0, count, 4).tolist()))
        for b in bad:
            ct[b * outs + int(rng.integers(0, L + 16))] ^= 0x20
        flags = aead.FLAG_VERIFY_FIRST if vf else aead.FLAG_ONE_PASS
        back, st = gpu_uniform(aead, True, CHACHA, keys, nb, rps, ct, outs, L, count, ins, lanes=2,
                               out_init=0x5A, flags=flags)
        for i in range(count):
            seg = back[i * ins: i * ins + L]
            if i in bad:
                assert st[i] == 1, (L, i)
                assert np.all(seg == (0x5A if vf else 0)), (L, i)
            else:
                assert st[i] == 0, (L, i)
                assert np.array_equal(seg, pt[i * ins: i * ins + L]), (L, i)
        # in place: rejected records read back as given
        torch = __import__("torch")
        buf = dev(ct)
        ctx, _k = prepare(aead, CHACHA, keys)
        d_nb = dev(nb.view(np.int64))
        d_st = torch.full((count,), 9, dtype=torch.uint8, device="cuda")
        assert aead.dev_uniform(True, CHACHA, ctx=ctx.data_ptr(), nonce_base=d_nb.data_ptr(),
                                inp=buf.data_ptr(), out=buf.data_ptr(), in_stride=outs, out_stride=outs,
                                length=L, n_records=count, recs_per_state=rps, status=d_st.data_ptr(),
                                lanes=2, flags=flags, stream=stream()) == 0
        sync()
        g = buf.cpu().numpy()
        for i in range(count):
            if i in bad:
                assert np.array_equal(g[i * outs: i * outs + L + 16], ct[i * outs: i * outs + L + 16]), (L, i)
            else:
                assert np.array_equal(g[i * outs: i * outs + L], pt[i * ins: i * ins + L]), (L, i)


def test_default_lanes_segmented(aead):
    """The library's choice: four lanes for a standalone 64 Ki-record
    ChaChaPoly job (two segments measured slower there), one lane from
    128 Ki, one lane in a duplex launch."""
    assert aead.dev_default_lanes(CHACHA, 65536) == 4
    assert aead.dev_default_lanes(CHACHA, 131072) == 1
    assert aead.dev_duplex_lanes(CHACHA, 65536) == 1
