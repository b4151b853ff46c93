"""ctypes bindings for the CPU oracle — TEST INFRASTRUCTURE ONLY.

Two checkers live behind this module:

* ``Oracle``   — the repo's own plain-C restatement (oracle/noise_oracle.c,
  built into oracle/_build/liboracle.so).
* ``RefLib``   — the reference noise-c itself, compiled from the sources under
  /root/reference into oracle/_ref/libnoiseref.so by oracle/Makefile.  Driven
  through its public CipherState API (include/noise/protocol/cipherstate.h:34-53).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product (noise-c_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libnoiseref.so")
REF_FULL_SO = os.path.join(HERE, "_ref", "libnoiseref_full.so")
REF_BENCH = os.path.join(HERE, "_ref", "ref_bench")

CHACHAPOLY = 0x4301  # constants.h:37
AESGCM = 0x4302      # constants.h:38
MAC_FAILURE = 0x4504  # constants.h:135


def build(ref: bool = True) -> None:
    """Compile the oracle (and, when /root/reference exists, oracle/_ref)."""
    targets = ["oracle"]
    if ref and os.path.isdir("/root/reference/src"):
        targets += ["hot", "full"]
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _buf(b):
    return (C.c_uint8 * len(b)).from_buffer(b) if len(b) else (C.c_uint8 * 1)()


class RandSnapshot(C.Structure):
    """OracleRand / NoiseRandSnapshot: the RandState generator's ChaCha key,
    64-bit block counter, 64-bit IV and reseed budget (randstate.c:47-58)."""
    _fields_ = [("key", C.c_uint32 * 8), ("counter", C.c_uint64), ("iv", C.c_uint64),
                ("left", C.c_uint64)]

    def copy(self):
        c = RandSnapshot()
        C.memmove(C.byref(c), C.byref(self), C.sizeof(self))
        return c

    def words(self):
        return (list(self.key), self.counter, self.iv, self.left)


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build(ref=False)
        L = C.CDLL(path)
        u8p, u64p, sz = C.c_void_p, C.c_void_p, C.c_size_t
        L.oracle_aead_encrypt.argtypes = [C.c_int, u8p, C.c_uint64, u8p, sz, u8p, sz]
        L.oracle_aead_decrypt.argtypes = [C.c_int, u8p, C.c_uint64, u8p, sz, u8p, sz]
        L.oracle_seal_uniform.argtypes = [C.c_int, u8p, u64p, C.c_uint32, u8p, sz,
                                          u8p, sz, C.c_uint32, C.c_uint32]
        L.oracle_open_uniform.argtypes = [C.c_int, u8p, u64p, C.c_uint32, u8p, sz,
                                          u8p, sz, C.c_uint32, C.c_uint32, u8p]
        L.oracle_seal_uniform_ad.argtypes = [C.c_int, u8p, u64p, C.c_uint32, u8p, sz,
                                             u8p, sz, C.c_uint32, C.c_uint32, u8p, sz, C.c_uint32]
        L.oracle_seal_ragged.argtypes = [C.c_int, u8p, u8p, u8p, C.c_uint32, u8p, u8p, u8p]
        L.oracle_chacha20_block.argtypes = [u8p, C.c_uint64, C.c_uint64, u8p]
        L.oracle_poly1305.argtypes = [u8p, u8p, sz, u8p]
        L.oracle_aes256_encrypt_block.argtypes = [u8p, u8p, u8p]
        L.oracle_gf128_mul.argtypes = [u8p, u8p, u8p]
        L.oracle_splitmix64.argtypes = [C.c_uint64]
        L.oracle_splitmix64.restype = C.c_uint64
        L.oracle_fill_splitmix.argtypes = [C.c_uint64, C.c_uint64, u8p, sz]
        L.oracle_hash.argtypes = [C.c_int, u8p, sz, u8p]
        L.oracle_hkdf.argtypes = [C.c_int, u8p, sz, u8p, sz, u8p, sz, u8p, sz]
        L.oracle_rand_pad.argtypes = [C.c_void_p, u8p, sz, sz, C.c_int]
        self.L = L

    @staticmethod
    def _p(b: bytearray):
        return C.addressof(_buf(b)) if len(b) else None

    def hash(self, hash_id: int, data: bytes) -> bytes:
        out = bytearray(64)
        d = bytearray(data)
        n = self.L.oracle_hash(hash_id, self._p(d), len(d), self._p(out))
        assert n > 0
        return bytes(out[:n])

    def hkdf(self, hash_id: int, key: bytes, data: bytes, l1: int, l2: int):
        """noise_hashstate_hkdf (hashstate.c:476-516)"""
        o1, o2 = bytearray(max(l1, 1)), bytearray(max(l2, 1))
        k, d = bytearray(key), bytearray(data)
        assert self.L.oracle_hkdf(hash_id, self._p(k), len(k), self._p(d), len(d),
                                  self._p(o1), l1, self._p(o2), l2) == 0
        return bytes(o1[:l1]), bytes(o2[:l2])

    def encrypt(self, cipher: int, key: bytes, n: int, pt: bytes, ad: bytes = b"") -> bytes:
        data = bytearray(pt) + bytearray(16)
        k, a = bytearray(key), bytearray(ad)
        self.L.oracle_aead_encrypt(cipher, self._p(k), n, self._p(a), len(a),
                                   self._p(data), len(pt))
        return bytes(data)

    def decrypt(self, cipher: int, key: bytes, n: int, ct_tag: bytes, ad: bytes = b""):
        data = bytearray(ct_tag)
        k, a = bytearray(key), bytearray(ad)
        rc = self.L.oracle_aead_decrypt(cipher, self._p(k), n, self._p(a), len(a),
                                        self._p(data), len(data) - 16)
        return rc, bytes(data[:-16])

    def chacha20_block(self, key: bytes, counter: int, iv: int) -> bytes:
        out, k = bytearray(64), bytearray(key)
        self.L.oracle_chacha20_block(self._p(k), counter, iv, self._p(out))
        return bytes(out)

    def poly1305(self, key: bytes, msg: bytes) -> bytes:
        out, k, m = bytearray(16), bytearray(key), bytearray(msg)
        self.L.oracle_poly1305(self._p(k), self._p(m), len(m), self._p(out))
        return bytes(out)

    def aes256(self, key: bytes, block: bytes) -> bytes:
        out, k, b = bytearray(16), bytearray(key), bytearray(block)
        self.L.oracle_aes256_encrypt_block(self._p(k), self._p(b), self._p(out))
        return bytes(out)

    def gf128_mul(self, x: bytes, h: bytes) -> bytes:
        out, xx, hh = bytearray(16), bytearray(x), bytearray(h)
        self.L.oracle_gf128_mul(self._p(xx), self._p(hh), self._p(out))
        return bytes(out)

    def rand_pad(self, snap, payload: bytearray, orig_len: int, padded_len: int, mode: int) -> int:
        """One noise_randstate_pad call on snapshot `snap` (a RandSnapshot,
        updated in place, or None) over `payload` (bytearray, in place)."""
        p = C.byref(snap) if snap is not None else None
        return self.L.oracle_rand_pad(p, self._p(payload), orig_len, padded_len, mode)

    def splitmix64(self, x: int) -> int:
        return self.L.oracle_splitmix64(x)

    def fill(self, seed: int, nbytes: int, word0: int = 0) -> bytes:
        out = bytearray(nbytes)
        self.L.oracle_fill_splitmix(seed, word0, self._p(out), nbytes)
        return bytes(out)

    # numpy-array batch helpers (arrays must be C-contiguous uint8 / uint64)
    def seal_uniform(self, cipher, keys, nonce_base, rps, inp, in_stride, out,
                     out_stride, length, count):
        self.L.oracle_seal_uniform(cipher, keys.ctypes.data, nonce_base.ctypes.data,
                                   rps, inp.ctypes.data, in_stride, out.ctypes.data,
                                   out_stride, length, count)

    def seal_uniform_ad(self, cipher, keys, nonce_base, rps, inp, in_stride, out,
                        out_stride, length, count, ad, ad_stride, ad_len):
        self.L.oracle_seal_uniform_ad(cipher, keys.ctypes.data, nonce_base.ctypes.data,
                                      rps, inp.ctypes.data, in_stride, out.ctypes.data,
                                      out_stride, length, count, ad.ctypes.data, ad_stride, ad_len)

    def seal_ragged(self, cipher, keys, key_idx, recs, inp, out, ad):
        """recs: structured array of the 48-B descriptors; key_idx: uint32 per record"""
        self.L.oracle_seal_ragged(cipher, keys.ctypes.data, key_idx.ctypes.data,
                                  recs.ctypes.data, len(recs), inp.ctypes.data, out.ctypes.data,
                                  ad.ctypes.data)

    def open_uniform(self, cipher, keys, nonce_base, rps, inp, in_stride, out,
                     out_stride, length, count, status):
        self.L.oracle_open_uniform(cipher, keys.ctypes.data, nonce_base.ctypes.data,
                                   rps, inp.ctypes.data, in_stride, out.ctypes.data,
                                   out_stride, length, count, status.ctypes.data)


class NoiseBuffer(C.Structure):
    """include/noise/protocol/buffer.h:33-40"""
    _fields_ = [("data", C.c_void_p), ("size", C.c_size_t), ("max_size", C.c_size_t)]


class RefLib:
    """The reference's CipherState API, compiled from /root/reference."""

    def __init__(self, path: str = REF_SO):
        L = C.CDLL(path)
        vp = C.c_void_p
        L.noise_cipherstate_new_by_id.argtypes = [C.POINTER(vp), C.c_int]
        L.noise_cipherstate_free.argtypes = [vp]
        L.noise_cipherstate_init_key.argtypes = [vp, vp, C.c_size_t]
        L.noise_cipherstate_set_nonce.argtypes = [vp, C.c_uint64]
        L.noise_cipherstate_encrypt_with_ad.argtypes = [vp, vp, C.c_size_t, C.POINTER(NoiseBuffer)]
        L.noise_cipherstate_decrypt_with_ad.argtypes = [vp, vp, C.c_size_t, C.POINTER(NoiseBuffer)]
        self.L = L

    def _state(self, cipher, key, n):
        st = vp = C.c_void_p()
        assert self.L.noise_cipherstate_new_by_id(C.byref(st), cipher) == 0
        k = (C.c_uint8 * 32).from_buffer_copy(key)
        assert self.L.noise_cipherstate_init_key(st, k, 32) == 0
        if n:
            assert self.L.noise_cipherstate_set_nonce(st, n) == 0
        return st

    def encrypt(self, cipher: int, key: bytes, n: int, pt: bytes, ad: bytes = b"") -> bytes:
        st = self._state(cipher, key, n)
        buf = (C.c_uint8 * (len(pt) + 16)).from_buffer_copy(bytes(pt) + bytes(16))
        nb = NoiseBuffer(C.addressof(buf), len(pt), len(pt) + 16)
        a = (C.c_uint8 * max(1, len(ad))).from_buffer_copy(bytes(ad) or b"\0")
        rc = self.L.noise_cipherstate_encrypt_with_ad(st, a if ad else None, len(ad), C.byref(nb))
        self.L.noise_cipherstate_free(st)
        assert rc == 0, hex(rc)
        return bytes(buf)[: nb.size]

    def decrypt(self, cipher: int, key: bytes, n: int, ct_tag: bytes, ad: bytes = b""):
        st = self._state(cipher, key, n)
        buf = (C.c_uint8 * len(ct_tag)).from_buffer_copy(bytes(ct_tag))
        nb = NoiseBuffer(C.addressof(buf), len(ct_tag), len(ct_tag))
        a = (C.c_uint8 * max(1, len(ad))).from_buffer_copy(bytes(ad) or b"\0")
        rc = self.L.noise_cipherstate_decrypt_with_ad(st, a if ad else None, len(ad), C.byref(nb))
        self.L.noise_cipherstate_free(st)
        return rc, bytes(buf)[: nb.size]
