"""Padding for uniform batches: the oracle's
restatement of noise_randstate_pad (randstate.c:348-375 over the generator of
:230-316) pinned against the reference's own RandState, and the contract
cases of tests/unit/test-randstate.c:86-123.  CPU only; the device version
(noise_aead_dev_pad) is checked against this oracle in test_gpu_pad.py."""
import ctypes as C
import os

import pytest

from oracle import RandSnapshot, REF_FULL_SO

ZERO, RANDOM = 0x4701, 0x4702


def _ref_randstate():
    """A reference RandState (OS-seeded) and a snapshot of its generator:
    struct NoiseRandState_s {size_t size; size_t left; chacha_ctx chacha;}
    (randstate.c:47-58), chacha input words 4..15 = key, counter, IV."""
    if not os.path.exists(REF_FULL_SO):
        if not os.path.isdir("/root/reference/src"):
            pytest.skip("reference library not built (GPU box without oracle/_ref)")
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.dirname(REF_FULL_SO) + "/..", "full"], check=True)
    R = C.CDLL(REF_FULL_SO)
    R.noise_randstate_new.argtypes = [C.POINTER(C.c_void_p)]
    R.noise_randstate_pad.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int]
    R.noise_randstate_free.argtypes = [C.c_void_p]
    st = C.c_void_p()
    assert R.noise_randstate_new(C.byref(st)) == 0
    return R, st


def snapshot_of(st):
    w = (C.c_uint32 * 16).from_address(st.value + 16)
    s = RandSnapshot()
    for i in range(8):
        s.key[i] = w[4 + i]
    s.counter = w[12] | (w[13] << 32)
    s.iv = w[14] | (w[15] << 32)
    s.left = C.c_size_t.from_address(st.value + 8).value
    return s


def test_oracle_pad_equals_reference_randstate(oracle):
    R, st = _ref_randstate()
    snap = snapshot_of(st)
    assert snap.left > 1_000_000 and snap.counter == 0
    # lengths exercising partial chunks, the in-request rekey every 17 chunks
    # (NOISE_RAND_REKEY_COUNT), no-op calls and ZERO / unknown modes
    calls = [(29, 51, RANDOM), (0, 64, RANDOM), (10, 10, RANDOM), (5, 4, RANDOM),
             (0, 16 * 64, RANDOM), (3, 3 + 17 * 64 + 1, RANDOM), (100, 5000, RANDOM),
             (29, 51, ZERO), (7, 700, 0x4737), (0, 65535, RANDOM), (1, 2, RANDOM)]
    for orig, padded, mode in calls:
        size = max(orig, padded) + 8
        a = bytearray(b"\xa5" * size)
        b = (C.c_uint8 * size).from_buffer_copy(bytes(a))
        assert R.noise_randstate_pad(st, b, orig, padded, mode) == 0
        assert oracle.rand_pad(snap, a, orig, padded, mode) == 0
        assert bytes(a) == bytes(b), (orig, padded, mode)
        assert snap.words() == snapshot_of(st).words(), (orig, padded, mode)
    R.noise_randstate_free(st)


def test_pad_contract_cases(oracle):
    """tests/unit/test-randstate.c:86-123 on the oracle restatement."""
    snap = RandSnapshot()
    for i in range(8):
        snap.key[i] = 0x01020304 * (i + 1)
    snap.left = 1_600_000
    t = bytearray(b"\xaa" * 128)
    assert oracle.rand_pad(snap, t, 29, 51, ZERO) == 0
    assert t[:29] == b"\xaa" * 29 and t[29:51] == bytes(22) and t[51:] == b"\xaa" * 77
    for mode, fillb in ((RANDOM, 0x66), (0x4737, 0x55)):  # unknown mode -> RANDOM
        t = bytearray([fillb] * 128)
        assert oracle.rand_pad(snap, t, 29, 100, mode) == 0
        assert t[:29] == bytes([fillb]) * 29 and t[100:] == bytes([fillb]) * 28
        assert t[29:100] != bytes([fillb]) * 71 and t[29:100] != bytes(71)
    t = bytearray(b"\x55" * 29 + b"\xaa" * 99)
    before = snap.copy().words()
    assert oracle.rand_pad(snap, t, 29, 28, ZERO) == 0
    assert t == bytearray(b"\x55" * 29 + b"\xaa" * 99) and snap.words() == before
    # NULL state: the padding is zeroed and INVALID_PARAM returned
    t = bytearray(b"\xaa" * 128)
    assert oracle.rand_pad(None, t, 28, 128, RANDOM) == 0x450B
    assert t[:28] == b"\xaa" * 28 and t[28:] == bytes(100)
    # a request the reference would serve only after an OS reseed
    low = snap.copy()
    low.left = 100
    t = bytearray(b"\x11" * 300)
    assert oracle.rand_pad(low, t, 0, 150, RANDOM) == 0x450C
    assert t == bytearray(b"\x11" * 300) and low.left == 100
