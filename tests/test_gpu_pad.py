"""noise_aead_dev_pad on the GPU against the oracle's
restatement of noise_randstate_pad (pinned to the reference's RandState in
test_randstate.py), the contract cases of tests/unit/test-randstate.c:86-123,
and the echo-client -g flow: messages padded to one length with RANDOM
padding (echo-client.c:400-410), then sealed by the uniform batch path —
compared with the reference's own RandState + CipherState calls when the
reference library is present, and with the oracle otherwise."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import RandSnapshot, REF_FULL_SO

pytestmark = pytest.mark.gpu
ZERO, RANDOM = 0x4701, 0x4702
CHACHA = 0x4301


def _torch():
    import torch
    return torch


def _snap(seed):
    s = RandSnapshot()
    rng = np.random.default_rng(seed)
    for i in range(8):
        s.key[i] = int(rng.integers(0, 2**32))
    s.counter = int(rng.integers(0, 1000))
    s.iv = int(rng.integers(0, 2**63))
    s.left = 1_600_000
    return s


def _dev_snap(s):
    torch = _torch()
    return torch.frombuffer(bytearray(bytes(s)), dtype=torch.uint8).to("cuda")


def _host_snap(t):
    s = RandSnapshot()
    C.memmove(C.byref(s), bytes(t.cpu().numpy()), C.sizeof(s))
    return s


def run_pad(aead, snap, payloads, stride, orig, padded, mode):
    """Device pad of a flat payload array; returns (rc, bytes, snapshot, done)."""
    torch = _torch()
    d_p = torch.from_numpy(payloads.copy()).to("cuda")
    d_o = torch.from_numpy(np.asarray(orig, dtype=np.uint32)).to("cuda")
    d_s = _dev_snap(snap) if snap is not None else None
    d_done = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = aead.dev_pad(rand=d_s.data_ptr() if d_s is not None else 0, payloads=d_p.data_ptr(),
                      stride=stride, orig_lens=d_o.data_ptr(), padded_len=padded, n=len(orig),
                      mode=mode, done=d_done.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return (rc, d_p.cpu().numpy(), _host_snap(d_s) if d_s is not None else None,
            int(d_done.cpu().item()))


def oracle_pad(oracle, snap, payloads, stride, orig, padded, mode):
    out = bytearray(payloads.tobytes())
    s = snap.copy() if snap is not None else None
    rcs = []
    for i, o in enumerate(orig):
        rec = bytearray(out[i * stride:(i + 1) * stride])
        rcs.append(oracle.rand_pad(s, rec, o, padded, mode))
        out[i * stride:(i + 1) * stride] = rec
    return rcs, np.frombuffer(bytes(out), dtype=np.uint8), s


@pytest.mark.parametrize("mode", [ZERO, RANDOM, 0x4737])
@pytest.mark.parametrize("padded", [51, 1000, 1088, 5000])
def test_pad_batch_vs_oracle(aead, gpu, oracle, mode, padded):
    rng = np.random.default_rng(padded + (mode & 0xff))
    n, stride = 257, padded + 40
    orig = rng.integers(0, padded + 20, n).tolist()
    orig[:3] = [0, padded, padded - 1]
    payloads = rng.integers(0, 256, n * stride, dtype=np.uint8)
    snap = _snap(padded)
    rc, got, gsnap, done = run_pad(aead, snap, payloads, stride, orig, padded, mode)
    rcs, exp, esnap = oracle_pad(oracle, snap, payloads, stride, orig, padded, mode)
    assert rc == 0 and set(rcs) == {0} and done == n
    assert np.array_equal(got, exp)
    assert gsnap.words() == esnap.words()


def test_pad_contract_cases_on_device(aead, gpu, oracle):
    """test-randstate.c:86-123 through noise_aead_dev_pad, one record each."""
    snap = _snap(7)
    # ZERO 29 -> 51
    t = np.full(128, 0xAA, dtype=np.uint8)
    rc, got, s, _ = run_pad(aead, snap, t, 128, [29], 51, ZERO)
    assert rc == 0 and np.all(got[:29] == 0xAA) and np.all(got[29:51] == 0) and np.all(got[51:] == 0xAA)
    assert s.words() == snap.words()
    # RANDOM / unknown mode 29 -> 100: prefix and tail kept, padding random
    for mode, fill in ((RANDOM, 0x66), (0x4737, 0x55)):
        t = np.full(128, fill, dtype=np.uint8)
        rc, got, s, _ = run_pad(aead, snap, t, 128, [29], 100, mode)
        assert rc == 0 and np.all(got[:29] == fill) and np.all(got[100:] == fill)
        assert not np.all(got[29:100] == fill) and not np.all(got[29:100] == 0)
    # padded_len <= orig_len: nothing changes, not even the generator
    t = np.concatenate([np.full(29, 0x55, np.uint8), np.full(99, 0xAA, np.uint8)])
    rc, got, s, _ = run_pad(aead, snap, t, 128, [29], 28, RANDOM)
    assert rc == 0 and np.array_equal(got, t) and s.words() == snap.words()
    # NULL state: padding zeroed, INVALID_PARAM
    t = np.full(128, 0xAA, dtype=np.uint8)
    rc, got, _, _ = run_pad(aead, None, t, 128, [28], 128, RANDOM)
    assert rc == 0x450B and np.all(got[:28] == 0xAA) and np.all(got[28:] == 0)


def test_pad_stops_where_reference_would_reseed(aead, gpu, oracle):
    snap = _snap(9)
    snap.left = 64 * 40  # enough for a few records of 16 chunks
    n, padded, stride = 10, 1024, 1024
    payloads = np.full(n * stride, 0x11, dtype=np.uint8)
    rc, got, gsnap, done = run_pad(aead, snap, payloads, stride, [0] * n, padded, RANDOM)
    rcs, exp, esnap = oracle_pad(oracle, snap, payloads, stride, [0] * n, padded, RANDOM)
    first_bad = rcs.index(0x450C)
    assert rc == 0 and done == first_bad == 2
    assert np.array_equal(got[:done * stride], exp[:done * stride])
    assert np.all(got[done * stride:] == 0x11)  # later records untouched
    s = snap.copy()
    for i in range(done):  # the snapshot is the state after the last padded record
        oracle.rand_pad(s, bytearray(stride), 0, padded, RANDOM)
    assert gsnap.words() == s.words()


def test_echo_client_padding_feeds_uniform_seal(aead, gpu, oracle):
    """echo-client -g: every line padded with RANDOM bytes to max_line_len,
    then encrypted (echo-client.c:395-415).  On the GPU: one noise_aead_dev_pad
    over the batch, then one noise_aead_dev_seal_uniform of the now uniform
    records.  Expected: the reference's own noise_randstate_pad +
    CipherState sequence from the same RandState (its generator snapshot read
    from the reference object), or the oracle when the reference is absent."""
    torch = _torch()
    rng = np.random.default_rng(42)
    n, max_line = 300, 1000
    lines = [bytes(rng.integers(32, 127, int(rng.integers(1, 200)), dtype=np.uint8)) for _ in range(n)]
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    stride_in = (max_line + 63) // 64 * 64
    stride_out = (max_line + 16 + 15) // 16 * 16
    # the RandState: the reference's when present, else a synthetic snapshot
    ref = None
    if os.path.exists(REF_FULL_SO):
        from test_randstate import _ref_randstate, snapshot_of
        R, st = _ref_randstate()
        snap = snapshot_of(st)
        ref = (R, st)
    else:
        snap = _snap(42)
    payloads = np.zeros(n * stride_in, dtype=np.uint8)
    for i, m in enumerate(lines):
        payloads[i * stride_in:i * stride_in + len(m)] = np.frombuffer(m, np.uint8)
    d_p = torch.from_numpy(payloads).to("cuda")
    d_o = torch.tensor([len(m) for m in lines], dtype=torch.int32, device="cuda")
    d_s = _dev_snap(snap)
    sp = torch.cuda.current_stream().cuda_stream
    assert aead.dev_pad(rand=d_s.data_ptr(), payloads=d_p.data_ptr(), stride=stride_in,
                        orig_lens=d_o.data_ptr(), padded_len=max_line, n=n, mode=RANDOM,
                        stream=sp) == 0
    # the padded lines are a uniform batch: seal them with nonces 0..n-1
    d_key = torch.tensor(list(key), dtype=torch.uint8, device="cuda")
    ctx = torch.empty(aead.dev_ctx_bytes(CHACHA), dtype=torch.uint8, device="cuda")
    assert aead.dev_prepare(CHACHA, d_key.data_ptr(), 1, ctx.data_ptr(), sp) == 0
    nonce = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_ct = torch.empty(n * stride_out, dtype=torch.uint8, device="cuda")
    assert aead.dev_uniform(False, CHACHA, ctx=ctx.data_ptr(), nonce_base=nonce.data_ptr(),
                            inp=d_p.data_ptr(), out=d_ct.data_ptr(), in_stride=stride_in,
                            out_stride=stride_out, length=max_line, n_records=n,
                            recs_per_state=n, stream=sp) == 0
    torch.cuda.synchronize()
    ct = d_ct.cpu().numpy()
    # expected, message by message as echo-client does it
    s = snap.copy()
    for i, m in enumerate(lines):
        msg = bytearray(m) + bytearray(max_line - len(m))
        if ref is not None:
            R, st = ref
            buf = (C.c_uint8 * max_line).from_buffer_copy(bytes(msg))
            assert R.noise_randstate_pad(st, buf, len(m), max_line, RANDOM) == 0
            padded = bytes(buf)
            assert oracle.rand_pad(s, msg, len(m), max_line, RANDOM) == 0
            assert bytes(msg) == padded  # oracle == reference, record by record
        else:
            assert oracle.rand_pad(s, msg, len(m), max_line, RANDOM) == 0
            padded = bytes(msg)
        exp = oracle.encrypt(CHACHA, key, i, padded)
        assert bytes(ct[i * stride_out:i * stride_out + max_line + 16]) == exp, i
    assert _host_snap(d_s).words() == s.words()
    if ref is not None:
        ref[0].noise_randstate_free(ref[1])
