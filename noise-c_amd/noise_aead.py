"""Python mirror of the noise-c CipherState interface over the gfx950 engine.

Thin ctypes layer over ``lib/libnoise_aead_hip.so`` (include/noise_aead_hip.h).
Names, argument meaning and return codes follow the reference C API
(include/noise/protocol/cipherstate.h:34-53) so tests read like
tests/unit/test-cipherstate.c: calls return the raw NOISE_ERROR_* code.

There is no fallback of any kind: if the shared library is missing this
module raises on import of ``lib()``; if no GPU is usable the crypto calls
return NOISE_ERROR_SYSTEM.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# NOISE_AEAD_LIB: another build of the same ABI (A/B measurements only)
LIB_PATH = os.environ.get("NOISE_AEAD_LIB") or os.path.join(HERE, "lib", "libnoise_aead_hip.so")
HEADER = os.path.join(HERE, "..", "include", "noise_aead_hip.h")


def NOISE_ID(ch: str, num: int) -> int:  # constants.h:31
    return (ord(ch) << 8) | num


CIPHER_NONE = 0
CHACHAPOLY = NOISE_ID("C", 1)
AESGCM = NOISE_ID("C", 2)
ERROR_NONE = 0
ERROR_NO_MEMORY = NOISE_ID("E", 1)
ERROR_UNKNOWN_ID = NOISE_ID("E", 2)
ERROR_UNKNOWN_NAME = NOISE_ID("E", 3)
ERROR_MAC_FAILURE = NOISE_ID("E", 4)
ERROR_SYSTEM = NOISE_ID("E", 6)
ERROR_INVALID_LENGTH = NOISE_ID("E", 10)
ERROR_INVALID_PARAM = NOISE_ID("E", 11)
ERROR_INVALID_STATE = NOISE_ID("E", 12)
ERROR_INVALID_NONCE = NOISE_ID("E", 13)
MAX_PAYLOAD_LEN = 65535
HASH_BLAKE2s = NOISE_ID("H", 1)  # constants.h:43-46
HASH_BLAKE2b = NOISE_ID("H", 2)
HASH_SHA256 = NOISE_ID("H", 3)
HASH_SHA512 = NOISE_ID("H", 4)
HASH_LEN = {HASH_BLAKE2s: 32, HASH_BLAKE2b: 64, HASH_SHA256: 32, HASH_SHA512: 64}


class NoiseBuffer(C.Structure):
    """include/noise/protocol/buffer.h:33-40"""
    _fields_ = [("data", C.c_void_p), ("size", C.c_size_t), ("max_size", C.c_size_t)]

    @classmethod
    def inout(cls, mem, size, max_size):  # noise_buffer_set_inout
        return cls(C.addressof(mem) if mem is not None else None, size, max_size)

    @classmethod
    def input(cls, mem, size):  # noise_buffer_set_input
        return cls(C.addressof(mem) if mem is not None else None, size, size)


class NoiseAeadUniform(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("nonce_base", C.c_void_p), ("in_", C.c_void_p),
                ("out", C.c_void_p), ("ad", C.c_void_p), ("status", C.c_void_p),
                ("in_stride", C.c_uint64), ("out_stride", C.c_uint64),
                ("ad_stride", C.c_uint64), ("recs_per_state", C.c_uint32),
                ("n_records", C.c_uint32), ("len", C.c_uint32), ("ad_len", C.c_uint32),
                ("lanes_per_record", C.c_uint32), ("flags", C.c_uint32)]


class NoiseAeadRecord(C.Structure):
    _fields_ = [("in_off", C.c_uint64), ("out_off", C.c_uint64), ("nonce", C.c_uint64),
                ("ctx_off", C.c_uint64), ("ad_off", C.c_uint64), ("len", C.c_uint32),
                ("ad_len", C.c_uint32)]


class NoiseAeadRagged(C.Structure):
    _fields_ = [("ctx_base", C.c_void_p), ("recs", C.c_void_p), ("in_", C.c_void_p),
                ("out", C.c_void_p), ("ad", C.c_void_p), ("status", C.c_void_p),
                ("n_records", C.c_uint32), ("lanes_per_record", C.c_uint32),
                ("flags", C.c_uint32), ("reserved_", C.c_uint32)]


FLAG_FAST = 1
FLAG_CT_GHASH = 2
FLAG_VERIFY_FIRST = 4  # the default open order since round 6 (accepted, overrides ONE_PASS)
FLAG_ONE_PASS = 8      # opt-in: ChaChaPoly FAST opens decrypt while authenticating
_LIB = None


def lib() -> C.CDLL:
    """Load the gfx950 library; raise loudly when it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run `make -C noise-c_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    # One HIP runtime per process: when PyTorch provides the device memory it
    # must be loaded first, so that our NEEDED libamdhip64.so.7 binds to the
    # copy torch already mapped (same SONAME) instead of a second runtime that
    # would not know torch's allocations.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz, i = C.c_void_p, C.c_size_t, C.c_int
    P = C.POINTER
    sigs = {
        "noise_cipherstate_new_by_id": (i, [P(vp), i]),
        "noise_cipherstate_new_by_name": (i, [P(vp), C.c_char_p]),
        "noise_cipherstate_free": (i, [vp]),
        "noise_cipherstate_get_cipher_id": (i, [vp]),
        "noise_cipherstate_get_key_length": (sz, [vp]),
        "noise_cipherstate_get_mac_length": (sz, [vp]),
        "noise_cipherstate_init_key": (i, [vp, vp, sz]),
        "noise_cipherstate_has_key": (i, [vp]),
        "noise_cipherstate_encrypt_with_ad": (i, [vp, vp, sz, P(NoiseBuffer)]),
        "noise_cipherstate_decrypt_with_ad": (i, [vp, vp, sz, P(NoiseBuffer)]),
        "noise_cipherstate_encrypt": (i, [vp, P(NoiseBuffer)]),
        "noise_cipherstate_decrypt": (i, [vp, P(NoiseBuffer)]),
        "noise_cipherstate_set_nonce": (i, [vp, C.c_uint64]),
        "noise_cipherstate_get_max_key_length": (i, []),
        "noise_cipherstate_get_max_mac_length": (i, []),
        "noise_chachapoly_new": (vp, []),
        "noise_aesgcm_new": (vp, []),
        "noise_cipherstate_encrypt_batch": (i, [P(vp), P(vp), P(sz), P(NoiseBuffer), sz, P(i)]),
        "noise_cipherstate_decrypt_batch": (i, [P(vp), P(vp), P(sz), P(NoiseBuffer), sz, P(i)]),
        "noise_wire_alloc": (vp, [sz]),
        "noise_wire_free": (None, [vp]),
        "noise_wire_seal": (i, [vp, vp, sz, P(sz), P(sz)]),
        "noise_wire_open": (i, [vp, vp, sz, P(sz), P(sz)]),
        "noise_wire_echo": (i, [vp, vp, vp, sz, P(sz), P(sz)]),
        "noise_aead_dev_hkdf": (i, [i, vp, C.c_uint32, vp, C.c_uint32, C.c_uint32, vp,
                                    C.c_uint32, vp, C.c_uint32, vp]),
        "noise_aead_dev_split": (i, [i, vp, C.c_uint32, vp, vp, vp]),
        "noise_aead_dev_encrypt_and_hash": (i, [i, i, vp, P(NoiseAeadRagged), vp]),
        "noise_aead_dev_decrypt_and_hash": (i, [i, i, vp, P(NoiseAeadRagged), vp]),
        "noise_aead_dev_ctx_bytes": (sz, [i]),
        "noise_aead_dev_prepare": (i, [i, vp, C.c_uint32, vp, vp]),
        "noise_aead_dev_seal_uniform": (i, [i, P(NoiseAeadUniform), vp]),
        "noise_aead_dev_open_uniform": (i, [i, P(NoiseAeadUniform), vp]),
        "noise_aead_dev_duplex_uniform": (i, [i, P(NoiseAeadUniform), P(NoiseAeadUniform), vp]),
        "noise_aead_dev_seal_ragged": (i, [i, P(NoiseAeadRagged), vp]),
        "noise_aead_dev_open_ragged": (i, [i, P(NoiseAeadRagged), vp]),
        "noise_aead_dev_default_lanes": (i, [i, C.c_uint32]),
        "noise_aead_dev_duplex_lanes": (i, [i, C.c_uint32]),
        "noise_aead_dev_pad": (i, [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_uint32, i, vp, vp]),
        "noise_strerror": (i, [i, C.c_char_p, sz]),
        "noise_perror": (None, [C.c_char_p, i]),
        "noise_aead_debug_batch_stats": (None, [P(C.c_uint64), P(C.c_uint64)]),
        "noise_aead_debug_last_freed_ctx": (vp, [P(sz)]),
        "noise_aead_dev_fill_splitmix": (i, [vp, C.c_uint64, C.c_uint64, C.c_uint64, vp]),
    }
    for name, (res, args) in sigs.items():
        if os.environ.get("NOISE_AEAD_LIB") and not hasattr(L, name):
            continue  # an older build under A/B: only the entry points it has
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


# ---------------------------------------------------------------- wire path
# Frames of examples/echo (echo-common.c:643-688): 2-byte BE length || body.

def frame_for_seal(messages) -> bytes:
    """Seal-ready wire image: each message as one frame whose header is the
    final length (len + 16) followed by the plaintext and 16 bytes of room."""
    out = bytearray()
    for m in messages:
        L = len(m) + 16
        if L > MAX_PAYLOAD_LEN:
            raise ValueError("message too long for one frame")
        out += bytes((L >> 8, L & 0xFF)) + bytes(m) + bytes(16)
    return bytes(out)


def parse_frames(wire: bytes, count=None):
    """[(offset of the body, L)] of the complete frames at the start of wire."""
    out, off = [], 0
    while off + 2 <= len(wire) and (count is None or len(out) < count):
        L = (wire[off] << 8) | wire[off + 1]
        if off + 2 + L > len(wire):
            break
        out.append((off + 2, L))
        off += 2 + L
    return out


def _wire_call(fn, states, buf, length):
    consumed, frames = C.c_size_t(), C.c_size_t()
    rc = fn(*[s.ptr for s in states], buf, length, C.byref(consumed), C.byref(frames))
    return rc, consumed.value, frames.value


def wire_seal(state, buf, length):
    """noise_wire_seal over a ctypes buffer / address; (rc, consumed, frames)."""
    return _wire_call(lib().noise_wire_seal, [state], buf, length)


def wire_open(state, buf, length):
    return _wire_call(lib().noise_wire_open, [state], buf, length)


def wire_echo(recv, send, buf, length):
    return _wire_call(lib().noise_wire_echo, [recv, send], buf, length)


class PinnedWire:
    """A noise_wire_alloc() buffer (pinned host memory), freed on close()."""

    def __init__(self, nbytes: int):
        self.n = nbytes
        self.addr = lib().noise_wire_alloc(nbytes)
        if not self.addr:
            raise MemoryError("noise_wire_alloc failed")
        self.view = (C.c_uint8 * nbytes).from_address(self.addr)

    def close(self):
        if self.addr:
            lib().noise_wire_free(self.addr)
            self.addr = None


def _bytes_ptr(b):
    if b is None:
        return None
    if isinstance(b, (bytes, bytearray)) and len(b) == 0:
        return None
    buf = (C.c_uint8 * len(b)).from_buffer_copy(bytes(b))
    return buf


class CipherState:
    """Object wrapper over a NoiseCipherState* (cipherstate.h:32)."""

    def __init__(self, ptr: int):
        self.ptr = C.c_void_p(ptr)

    @classmethod
    def new_by_id(cls, cid: int):
        p = C.c_void_p()
        rc = lib().noise_cipherstate_new_by_id(C.byref(p), cid)
        return rc, (cls(p.value) if p.value else None)

    @classmethod
    def new_by_name(cls, name):
        p = C.c_void_p()
        rc = lib().noise_cipherstate_new_by_name(
            C.byref(p), name.encode() if isinstance(name, str) else name)
        return rc, (cls(p.value) if p.value else None)

    def free(self) -> int:
        rc = lib().noise_cipherstate_free(self.ptr)
        self.ptr = C.c_void_p(None)
        return rc

    @property
    def cipher_id(self) -> int:
        return lib().noise_cipherstate_get_cipher_id(self.ptr)

    @property
    def key_length(self) -> int:
        return lib().noise_cipherstate_get_key_length(self.ptr)

    @property
    def mac_length(self) -> int:
        return lib().noise_cipherstate_get_mac_length(self.ptr)

    @property
    def has_key(self) -> int:
        return lib().noise_cipherstate_has_key(self.ptr)

    def init_key(self, key, key_len=None) -> int:
        k = _bytes_ptr(key) if key is not None else None
        return lib().noise_cipherstate_init_key(
            self.ptr, k, len(key) if key_len is None else key_len)

    @property
    def nonce(self) -> int:
        """n of the state: the u64 at offset 16 of struct NoiseCipherState_s
        (internal.h:58-146; there is no getter in the reference API)."""
        return C.c_uint64.from_address(self.ptr.value + 16).value

    def set_nonce(self, n: int) -> int:
        return lib().noise_cipherstate_set_nonce(self.ptr, n)

    def encrypt_with_ad(self, ad, buf: NoiseBuffer) -> int:
        a = _bytes_ptr(ad)
        return lib().noise_cipherstate_encrypt_with_ad(self.ptr, a, len(ad or b""), C.byref(buf))

    def decrypt_with_ad(self, ad, buf: NoiseBuffer) -> int:
        a = _bytes_ptr(ad)
        return lib().noise_cipherstate_decrypt_with_ad(self.ptr, a, len(ad or b""), C.byref(buf))

    # convenience: bytes in, bytes out (raises on error)
    def seal(self, pt: bytes, ad: bytes = b"") -> bytes:
        mem = (C.c_uint8 * (len(pt) + 16)).from_buffer_copy(bytes(pt) + bytes(16))
        nb = NoiseBuffer.inout(mem, len(pt), len(pt) + 16)
        rc = self.encrypt_with_ad(ad, nb)
        if rc:
            raise RuntimeError(f"encrypt failed: {rc:#x}")
        return bytes(mem)[: nb.size]

    def open(self, ct: bytes, ad: bytes = b""):
        mem = (C.c_uint8 * max(1, len(ct))).from_buffer_copy(bytes(ct) or b"\0")
        nb = NoiseBuffer.input(mem, len(ct))
        rc = self.decrypt_with_ad(ad, nb)
        return rc, bytes(mem)[: nb.size]


def _batch(fn_name, states, buffers, ads=None):
    n = len(states)
    st_arr = (C.c_void_p * max(1, n))(*[s.ptr.value if s else None for s in states])
    buf_arr = (NoiseBuffer * max(1, n))(*buffers)
    res = (C.c_int * max(1, n))()
    keep = []
    if ads is not None:
        ad_ptrs = []
        for a in ads:
            m = _bytes_ptr(a)
            keep.append(m)
            ad_ptrs.append(C.addressof(m) if m is not None else None)
        ad_arr = (C.c_void_p * max(1, n))(*ad_ptrs)
        len_arr = (C.c_size_t * max(1, n))(*[len(a or b"") for a in ads])
    else:
        ad_arr, len_arr = None, None
    rc = getattr(lib(), fn_name)(st_arr, ad_arr, len_arr, buf_arr, n, res)
    for i in range(n):
        buffers[i].size = buf_arr[i].size
    return rc, list(res[:n])


def encrypt_batch(states, buffers, ads=None):
    """noise_cipherstate_encrypt_batch: same results as sequential calls."""
    return _batch("noise_cipherstate_encrypt_batch", states, buffers, ads)


def decrypt_batch(states, buffers, ads=None):
    """noise_cipherstate_decrypt_batch: same results as sequential calls."""
    return _batch("noise_cipherstate_decrypt_batch", states, buffers, ads)


# ------------------------------------------------------------ device API

def dev_ctx_bytes(cipher: int) -> int:
    return lib().noise_aead_dev_ctx_bytes(cipher)


def dev_prepare(cipher: int, d_raw_keys: int, n_states: int, d_ctx: int, stream: int = 0) -> int:
    return lib().noise_aead_dev_prepare(cipher, d_raw_keys, n_states, d_ctx, stream or None)


def dev_uniform(open_: bool, cipher: int, *, ctx: int, nonce_base: int, inp: int, out: int,
                in_stride: int, out_stride: int, length: int, n_records: int,
                recs_per_state: int, status: int = 0, ad: int = 0, ad_stride: int = 0,
                ad_len: int = 0, lanes: int = 0, flags: int = 0, stream: int = 0) -> int:
    j = NoiseAeadUniform(ctx, nonce_base, inp, out, ad or None, status or None, in_stride,
                         out_stride, ad_stride, recs_per_state, n_records, length, ad_len,
                         lanes, flags)
    f = lib().noise_aead_dev_open_uniform if open_ else lib().noise_aead_dev_seal_uniform
    return f(cipher, C.byref(j), stream or None)


def uniform_job(*, ctx: int, nonce_base: int, inp: int, out: int, in_stride: int,
                out_stride: int, length: int, n_records: int, recs_per_state: int,
                status: int = 0, ad: int = 0, ad_stride: int = 0, ad_len: int = 0,
                lanes: int = 0, flags: int = 0) -> NoiseAeadUniform:
    return NoiseAeadUniform(ctx, nonce_base, inp, out, ad or None, status or None, in_stride,
                            out_stride, ad_stride, recs_per_state, n_records, length, ad_len,
                            lanes, flags)


def dev_duplex(cipher: int, seal_job: NoiseAeadUniform, open_job: NoiseAeadUniform,
               stream: int = 0) -> int:
    """noise_aead_dev_duplex_uniform: seal_job and open_job in one launch."""
    return lib().noise_aead_dev_duplex_uniform(cipher, C.byref(seal_job), C.byref(open_job),
                                               stream or None)


PADDING_ZERO, PADDING_RANDOM = NOISE_ID("G", 1), NOISE_ID("G", 2)


def dev_pad(*, rand: int, payloads: int, stride: int, orig_lens: int, padded_len: int, n: int,
            mode: int, done: int = 0, stream: int = 0) -> int:
    """noise_aead_dev_pad (device pointers; rand may be 0 = NULL state)."""
    return lib().noise_aead_dev_pad(rand or None, payloads, stride, orig_lens, padded_len, n, mode,
                                    done or None, stream or None)


def dev_ragged(open_: bool, cipher: int, *, ctx_base: int, recs: int, inp: int, out: int,
               n_records: int, status: int = 0, ad: int = 0, lanes: int = 0,
               flags: int = 0, stream: int = 0) -> int:
    j = NoiseAeadRagged(ctx_base or None, recs, inp, out, ad or None, status or None,
                        n_records, lanes, flags, 0)
    f = lib().noise_aead_dev_open_ragged if open_ else lib().noise_aead_dev_seal_ragged
    return f(cipher, C.byref(j), stream or None)


def dev_hkdf(hash_id: int, *, keys: int, key_len: int, data: int = 0, data_len: int = 0,
             n: int, out1: int, out1_len: int, out2: int, out2_len: int, stream: int = 0) -> int:
    return lib().noise_aead_dev_hkdf(hash_id, keys, key_len, data or None, data_len, n, out1,
                                     out1_len, out2, out2_len, stream or None)


def dev_and_hash(open_: bool, cipher: int, hash_id: int, *, ctx_base: int, h: int, recs: int,
                 inp: int, out: int, n_records: int, status: int = 0, flags: int = 0,
                 stream: int = 0) -> int:
    """noise_aead_dev_{en,de}crypt_and_hash: AD = the hashes at h; record
    ctx_off values are offsets from ctx_base (as dev_ragged)."""
    j = NoiseAeadRagged(ctx_base or None, recs, inp, out, h, status or None, n_records, 0,
                        flags, 0)
    f = (lib().noise_aead_dev_decrypt_and_hash if open_ else
         lib().noise_aead_dev_encrypt_and_hash)
    return f(cipher, hash_id, h, C.byref(j), stream or None)


def dev_split(hash_id: int, *, ck: int, n: int, k1: int, k2: int, stream: int = 0) -> int:
    return lib().noise_aead_dev_split(hash_id, ck, n, k1, k2, stream or None)


def dev_fill_splitmix(d_out: int, nbytes: int, seed: int, word0: int = 0, stream: int = 0) -> int:
    return lib().noise_aead_dev_fill_splitmix(d_out, nbytes, seed, word0, stream or None)


def dev_default_lanes(cipher: int, n_records: int) -> int:
    return lib().noise_aead_dev_default_lanes(cipher, n_records)


def dev_duplex_lanes(cipher: int, n_records: int) -> int:
    return lib().noise_aead_dev_duplex_lanes(cipher, n_records)
