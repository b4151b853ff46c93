"""Transport wire path: noise_wire_{seal,open,echo}.

Frames are those of the reference's examples/echo (echo-common.c:643-688):
2-byte big-endian length || CT || tag.  Every sealed frame must equal the
oracle's encryption of its message under nonce n + k; open and echo must stop
exactly where the per-frame CipherState calls of the echo server
(echo-server.c:377-407) would, leaving the failing frame and everything after
it untouched.  The CPU tests cover the host-side rules that never reach the
GPU."""
import ctypes as C
import os

import numpy as np
import pytest

CHACHA, AES = 0x4301, 0x4302
NONCE_MAX = 2**64 - 1


def _state(A, cid, key, n=0):
    rc, st = A.CipherState.new_by_id(cid)
    assert rc == 0
    assert st.init_key(key) == 0
    if n:
        assert st.set_nonce(n) == 0
    return st


def _buf(data: bytes):
    return (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")


# ------------------------------------------------------------ CPU (no GPU)

def test_wire_host_rules(aead_built):
    A = aead_built
    L = A.lib()
    key = bytes(range(32))
    st = _state(A, CHACHA, key)
    other = _state(A, CHACHA, key)
    nokey = A.CipherState.new_by_id(CHACHA)[1]
    b = _buf(bytes(64))
    z = C.c_size_t()
    assert L.noise_wire_seal(None, b, 64, C.byref(z), C.byref(z)) == A.ERROR_INVALID_PARAM
    assert L.noise_wire_open(st.ptr, None, 64, C.byref(z), C.byref(z)) == A.ERROR_INVALID_PARAM
    assert A.wire_echo(st, st, b, 64)[0] == A.ERROR_INVALID_PARAM
    assert A.wire_seal(nokey, b, 64)[0] == A.ERROR_INVALID_STATE
    assert A.wire_echo(st, nokey, b, 64)[0] == A.ERROR_INVALID_STATE
    # empty, header-only and partial frames: nothing to do, no error
    assert A.wire_open(st, b, 0) == (0, 0, 0)
    assert A.wire_open(st, _buf(b"\x00"), 1) == (0, 0, 0)
    assert A.wire_open(st, _buf(b"\x00\x40" + bytes(10)), 12) == (0, 0, 0)
    # a first frame shorter than a tag: INVALID_LENGTH before any GPU work
    w = b"\x00\x0f" + bytes(15)
    for fn in (A.wire_seal, A.wire_open):
        assert fn(st, _buf(w), len(w)) == (A.ERROR_INVALID_LENGTH, 0, 0)
    assert A.wire_echo(st, other, _buf(w), len(w)) == (A.ERROR_INVALID_LENGTH, 0, 0)
    # exhausted nonce on the first frame
    st.set_nonce(NONCE_MAX)
    w = b"\x00\x10" + bytes(16)
    assert A.wire_open(st, _buf(w), len(w)) == (A.ERROR_INVALID_NONCE, 0, 0)
    assert A.wire_echo(other, st, _buf(w), len(w)) == (A.ERROR_INVALID_NONCE, 0, 0)
    assert st.nonce == NONCE_MAX and other.nonce == 0
    for s in (st, other, nokey):
        s.free()


@pytest.fixture(scope="module")
def aead_built():
    import noise_aead
    noise_aead.lib()
    return noise_aead


# ------------------------------------------------------------------- GPU

def _messages(rng, n, lo=0, hi=2000, extra=()):
    lens = list(rng.integers(lo, hi, n)) + list(extra)
    return [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in lens]


def _sealed_wire(oracle, cid, key, n0, msgs):
    out = bytearray()
    for k, m in enumerate(msgs):
        f = oracle.encrypt(cid, key, n0 + k, m)
        out += bytes((len(f) >> 8, len(f) & 0xFF)) + f
    return bytes(out)


@pytest.mark.gpu
@pytest.mark.parametrize("cid", [CHACHA, AES])
@pytest.mark.parametrize("pinned", [False, True])
def test_wire_seal_matches_oracle(aead, gpu, oracle, cid, pinned):
    A = aead
    rng = np.random.default_rng(cid + pinned)
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    n0 = 2**32 - 3
    # ~5.5 MB of frames: more than one pipeline chunk; includes the extremes
    msgs = _messages(rng, 3900, 0, 2800, extra=(0, 1, 15, 16, 17, 1400, 65519))
    img = A.frame_for_seal(msgs) + b"\x07\x00\x01"  # trailing partial frame
    st = _state(A, cid, key, n0)
    if pinned:
        pw = A.PinnedWire(len(img))
        C.memmove(pw.addr, img, len(img))
        rc, consumed, frames = A.wire_seal(st, pw.addr, len(img))
        got = bytes(pw.view)
        pw.close()
    else:
        b = _buf(img)
        rc, consumed, frames = A.wire_seal(st, b, len(img))
        got = bytes(b)[:len(img)]
    assert rc == 0 and frames == len(msgs) and consumed == len(img) - 3
    assert st.nonce == n0 + len(msgs)
    assert got == _sealed_wire(oracle, cid, key, n0, msgs) + b"\x07\x00\x01"
    st.free()


@pytest.mark.gpu
@pytest.mark.parametrize("cid", [CHACHA, AES])
@pytest.mark.parametrize("pinned", [False, True])
def test_wire_open_and_mac_failure(aead, gpu, oracle, cid, pinned):
    A = aead
    rng = np.random.default_rng(10 + cid + pinned)
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    msgs = _messages(rng, 4200, 0, 2400)
    wire = _sealed_wire(oracle, cid, key, 5, msgs)
    frames_at = A.parse_frames(wire)
    for bad in (None, 3700, 0):  # 3700 lies in the second pipeline chunk
        w = bytearray(wire)
        if bad is not None:
            off, L = frames_at[bad]
            w[off + L - 1] ^= 0x80  # flip a tag bit
        st = _state(A, cid, key, 5)
        if pinned:
            pw = A.PinnedWire(len(w))
            C.memmove(pw.addr, bytes(w), len(w))
            rc, consumed, frames = A.wire_open(st, pw.addr, len(w))
            got = bytes(pw.view)
            pw.close()
        else:
            b = _buf(w)
            rc, consumed, frames = A.wire_open(st, b, len(w))
            got = bytes(b)[:len(w)]
        upto = len(msgs) if bad is None else bad
        assert rc == (0 if bad is None else A.ERROR_MAC_FAILURE)
        assert frames == upto and st.nonce == 5 + upto
        for k in range(upto):
            off, L = frames_at[k]
            assert got[off:off + L - 16] == msgs[k], k
            assert got[off + L - 16:off + L] == w[off + L - 16:off + L]
        if upto < len(msgs):  # the failing frame and every later one untouched
            off = frames_at[upto][0] - 2
            assert got[off:] == bytes(w[off:])
            assert consumed == off
        st.free()


@pytest.mark.gpu
@pytest.mark.parametrize("cid", [CHACHA, AES])
def test_wire_echo_server_loop(aead, gpu, oracle, cid):
    """noise_wire_echo == the reference echo server applied frame by frame:
    decrypt with recv (c2s key), encrypt with send (s2c key)."""
    A = aead
    rng = np.random.default_rng(20 + cid)
    k_c2s = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    k_s2c = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    msgs = _messages(rng, 4000, 0, 1500, extra=(1024,) * 50)
    wire = _sealed_wire(oracle, cid, k_c2s, 0, msgs)
    frames_at = A.parse_frames(wire)
    for bad in (None, 3999, 17):
        w = bytearray(wire)
        if bad is not None:
            off, L = frames_at[bad]
            w[off] ^= 1  # corrupt ciphertext
        recv, send = _state(A, cid, k_c2s), _state(A, cid, k_s2c, 100)
        b = _buf(w)
        rc, consumed, frames = A.wire_echo(recv, send, b, len(w))
        got = bytes(b)[:len(w)]
        upto = len(msgs) if bad is None else bad
        assert rc == (0 if bad is None else A.ERROR_MAC_FAILURE)
        assert frames == upto and recv.nonce == upto and send.nonce == 100 + upto
        expect = _sealed_wire(oracle, cid, k_s2c, 100, msgs[:upto])
        assert got[:len(expect)] == expect and consumed == len(expect)
        assert got[len(expect):] == bytes(w[len(expect):])
        recv.free()
        send.free()


@pytest.mark.gpu
def test_wire_stops_at_short_frame_and_exhausted_nonce(aead, gpu, oracle):
    A = aead
    key = bytes(32)
    msgs = [bytes([i]) * (i * 7) for i in range(10)]
    wire = _sealed_wire(oracle, CHACHA, key, 0, msgs)
    bad = wire + b"\x00\x05" + bytes(5) + _sealed_wire(oracle, CHACHA, key, 10, msgs[:2])
    st = _state(A, CHACHA, key)
    b = _buf(bad)
    rc, consumed, frames = A.wire_open(st, b, len(bad))
    assert (rc, frames, consumed) == (A.ERROR_INVALID_LENGTH, 10, len(wire))
    assert st.nonce == 10
    st.free()
    # nonce runs out on frame 3 (n = 2^64-1 is never used, cipherstate.c:391-397)
    st = _state(A, CHACHA, key, NONCE_MAX - 3)
    img = A.frame_for_seal(msgs[:6])
    b = _buf(img)
    rc, consumed, frames = A.wire_seal(st, b, len(img))
    assert (rc, frames) == (A.ERROR_INVALID_NONCE, 3) and st.nonce == NONCE_MAX
    assert bytes(b)[:consumed] == _sealed_wire(oracle, CHACHA, key, NONCE_MAX - 3, msgs[:3])
    st.free()


@pytest.mark.gpu
@pytest.mark.parametrize("cipher", ["chachapoly", "aesgcm"])
def test_echo_loopback_tcp(aead, gpu, cipher):
    """Config C1's plumbing over a real 127.0.0.1 socket: bursts whose bytes
    reach the server in arbitrary recv() pieces (partial frames carried over),
    every echo decrypted by the client and compared with what it sent."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    import echo_loopback
    r = echo_loopback.run(messages=3000, size=1024, burst=700, cipher=cipher)
    assert r["verified"] and r["server_error"] == 0
    assert r["server_frames"] == 3000
