"""The C-ABI library: it loads, exports every symbol include/*.h declares, its
structs have the documented layout, and the CipherState front end's host-side
rules (validation, nonce bookkeeping, error codes — src/protocol/cipherstate.c)
hold.  Nothing here launches a kernel: paths that would reach the GPU are not
called on CPU."""
import ctypes as C
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NONCE_MAX = 2**64 - 1


@pytest.fixture(scope="module")
def L(aead_built):
    return aead_built.lib()


@pytest.fixture(scope="module")
def aead_built():
    import noise_aead
    if not os.path.exists(noise_aead.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "noise-c_amd")], check=True)
    return noise_aead


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(noise_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_exports_every_declared_symbol(L):
    names = declared_functions()
    assert len(names) >= 27
    so = os.path.join(ROOT, "noise-c_amd", "lib", "libnoise_aead_hip.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = names - exported
    assert not missing, missing
    for n in names:
        assert hasattr(L, n)


def test_struct_layouts(aead_built):
    A = aead_built
    assert C.sizeof(A.NoiseAeadRecord) == 48
    assert C.sizeof(A.NoiseBuffer) == 24
    assert C.sizeof(A.NoiseAeadUniform) == 6 * 8 + 3 * 8 + 6 * 4
    assert A.dev_ctx_bytes(A.CHACHAPOLY) == 32
    assert A.dev_ctx_bytes(A.AESGCM) >= 240 + 16
    assert A.dev_ctx_bytes(0x4303) == 0


def test_cipherstate_errors(aead_built):
    """tests/unit/test-cipherstate.c:284-311 cipherstate_check_errors."""
    A = aead_built
    L = A.lib()
    assert L.noise_cipherstate_free(None) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_get_cipher_id(None) == A.CIPHER_NONE
    assert L.noise_cipherstate_get_key_length(None) == 0
    assert L.noise_cipherstate_get_mac_length(None) == 0
    assert L.noise_cipherstate_new_by_id(None, A.HASH_BLAKE2s) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_new_by_name(None, b"ChaChaPoly") == A.ERROR_INVALID_PARAM
    p = C.c_void_p(8)
    assert L.noise_cipherstate_new_by_id(C.byref(p), A.HASH_BLAKE2s) == A.ERROR_UNKNOWN_ID
    assert p.value is None
    p = C.c_void_p(8)
    assert L.noise_cipherstate_new_by_name(C.byref(p), None) == A.ERROR_INVALID_PARAM
    assert p.value is None
    p = C.c_void_p(8)
    assert L.noise_cipherstate_new_by_name(C.byref(p), b"ChaChaPony") == A.ERROR_UNKNOWN_NAME
    assert p.value is None
    assert L.noise_cipherstate_get_max_key_length() == 32
    assert L.noise_cipherstate_get_max_mac_length() == 16


@pytest.mark.parametrize("cid,name", [(0x4301, "ChaChaPoly"), (0x4302, "AESGCM")])
def test_cipherstate_host_rules(aead_built, cid, name):
    """The parts of check_cipher (test-cipherstate.c:31-224) that never reach
    the GPU: properties, no-key pass-through, key/nonce rules, bad args."""
    A = aead_built
    rc, st = A.CipherState.new_by_id(cid)
    assert rc == 0 and st.cipher_id == cid and st.key_length == 32 and st.mac_length == 16
    assert not st.has_key
    mem = (C.c_uint8 * 512)(*range(256), *range(256))
    before = bytes(mem)
    nb = A.NoiseBuffer.inout(mem, 100, 512)
    assert st.encrypt_with_ad(b"ad", nb) == 0 and nb.size == 100 and bytes(mem) == before
    nb = A.NoiseBuffer.input(mem, A.MAX_PAYLOAD_LEN + 1)
    assert st.encrypt_with_ad(b"ad", nb) == A.ERROR_INVALID_LENGTH
    nb = A.NoiseBuffer.inout(mem, 8, 512)
    assert st.encrypt_with_ad(b"ad", nb) == 0 and nb.size == 8
    nb = A.NoiseBuffer.input(mem, 116)
    assert st.decrypt_with_ad(b"ad", nb) == 0 and nb.size == 116
    nb = A.NoiseBuffer.input(mem, A.MAX_PAYLOAD_LEN + 1)
    assert st.decrypt_with_ad(b"ad", nb) == A.ERROR_INVALID_LENGTH
    nb = A.NoiseBuffer.input(mem, 8)
    assert st.decrypt_with_ad(b"ad", nb) == 0 and nb.size == 8
    assert st.set_nonce(5) == A.ERROR_INVALID_STATE
    key = bytes(range(32))
    assert st.init_key(key) == 0 and st.has_key
    assert st.set_nonce(5) == 0
    assert st.set_nonce(4) == A.ERROR_INVALID_NONCE
    assert st.set_nonce(NONCE_MAX) == 0
    # exhausted nonce: rejected before any GPU work (cipherstate.c:321-322, 394-395)
    nb = A.NoiseBuffer.inout(mem, 10, 512)
    assert st.encrypt_with_ad(None, nb) == A.ERROR_INVALID_NONCE
    nb = A.NoiseBuffer.input(mem, 40)
    assert st.decrypt_with_ad(None, nb) == A.ERROR_INVALID_NONCE
    # size checks with a key (cipherstate.c:312-315, 389-390)
    nb = A.NoiseBuffer.inout(mem, 65535 - 15, 65535 + 1)
    assert st.encrypt_with_ad(None, nb) == A.ERROR_INVALID_LENGTH
    nb = A.NoiseBuffer.inout(mem, 500, 510)
    assert st.encrypt_with_ad(None, nb) == A.ERROR_INVALID_LENGTH
    nb = A.NoiseBuffer.input(mem, 8)
    assert st.decrypt_with_ad(None, nb) == A.ERROR_INVALID_LENGTH
    nb = A.NoiseBuffer.inout(mem, 20, 10)
    assert st.encrypt_with_ad(None, nb) == A.ERROR_INVALID_LENGTH
    # re-keying resets the nonce (cipherstate.c:231-233)
    assert st.init_key(key) == 0 and st.set_nonce(0) == 0
    # parameter errors
    L = A.lib()
    k = (C.c_uint8 * 33)()
    assert L.noise_cipherstate_init_key(None, k, 32) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_init_key(st.ptr, None, 32) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_init_key(st.ptr, k, 31) == A.ERROR_INVALID_LENGTH
    assert L.noise_cipherstate_init_key(st.ptr, k, 33) == A.ERROR_INVALID_LENGTH
    assert L.noise_cipherstate_set_nonce(None, 1) == A.ERROR_INVALID_PARAM
    nb = A.NoiseBuffer.inout(mem, 10, 512)
    assert L.noise_cipherstate_encrypt_with_ad(None, None, 0, C.byref(nb)) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_encrypt_with_ad(st.ptr, None, 3, C.byref(nb)) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_encrypt_with_ad(st.ptr, None, 0, None) == A.ERROR_INVALID_PARAM
    nb.data = None
    assert L.noise_cipherstate_encrypt_with_ad(st.ptr, None, 0, C.byref(nb)) == A.ERROR_INVALID_PARAM
    nb = A.NoiseBuffer.input(mem, 40)
    assert L.noise_cipherstate_decrypt_with_ad(None, None, 0, C.byref(nb)) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_decrypt_with_ad(st.ptr, None, 3, C.byref(nb)) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_decrypt_with_ad(st.ptr, None, 0, None) == A.ERROR_INVALID_PARAM
    assert st.free() == 0
    rc, st = A.CipherState.new_by_name(name)
    assert rc == 0 and st.cipher_id == cid and not st.has_key
    assert st.free() == 0


def test_batch_host_rules(aead_built):
    """Batch entry points: argument errors and the records that never reach
    the GPU (no key, bad length, exhausted nonce) give per-record codes equal
    to the single-call ones."""
    A = aead_built
    L = A.lib()
    assert L.noise_cipherstate_encrypt_batch(None, None, None, None, 1, None) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_decrypt_batch(None, None, None, None, 1, None) == A.ERROR_INVALID_PARAM
    assert L.noise_cipherstate_encrypt_batch(None, None, None, None, 0, None) == 0
    nokey = A.CipherState.new_by_id(A.CHACHAPOLY)[1]
    spent = A.CipherState.new_by_id(A.AESGCM)[1]
    spent.init_key(bytes(32))
    spent.set_nonce(NONCE_MAX)
    mems = [(C.c_uint8 * 64)() for _ in range(4)]
    bufs = [A.NoiseBuffer.inout(mems[0], 10, 64), A.NoiseBuffer.inout(mems[1], 60, 64),
            A.NoiseBuffer.inout(mems[2], 10, 64), A.NoiseBuffer.inout(mems[3], 70, 64)]
    rc, res = A.encrypt_batch([nokey, spent, spent, nokey], bufs)
    assert rc == 0
    assert res == [0, A.ERROR_INVALID_LENGTH, A.ERROR_INVALID_NONCE, A.ERROR_INVALID_LENGTH]
    assert [b.size for b in bufs] == [10, 60, 10, 70]
    bufs = [A.NoiseBuffer.input(mems[0], 40), A.NoiseBuffer.input(mems[1], 8),
            A.NoiseBuffer.input(mems[2], 40)]
    rc, res = A.decrypt_batch([nokey, spent, spent], bufs)
    assert rc == 0 and res == [0, A.ERROR_INVALID_LENGTH, A.ERROR_INVALID_NONCE]
    nokey.free()
    spent.free()


def test_default_lane_policy(aead_built):
    """Lanes per record the library picks (aead_api.hip uniform_lanes /
    auto_lanes): a standalone seal or open takes one lane per record from
    128 Ki records (two waves per SIMD), 4 lanes from 64 Ki (two segments per
    record measured slower there, aead_api.hip seg_mode), 8 below, and wide
    groups (up to a wave per record) only for batches of at most 512 records
    — the latency regime; the jobs of a duplex launch take one lane per
    record from 64 Ki records (the BASELINE sizes, FAST layouts)."""
    A = aead_built
    lanes = lambda n: A.dev_default_lanes(A.CHACHAPOLY, n)
    duplex = lambda n: A.dev_duplex_lanes(A.CHACHAPOLY, n)
    assert lanes(65536) == 4 and lanes(131071) == 4 and lanes(131072) == 1 and lanes(1 << 20) == 1
    assert lanes(65535) == 8 and lanes(513) == 8
    assert lanes(512) == 64 and lanes(1) == 64
    assert duplex(65536) == 1 and duplex(1 << 20) == 1
    assert duplex(65535) == 8 and duplex(512) == 64
    assert A.dev_default_lanes(A.AESGCM, 1) == 4 and A.dev_duplex_lanes(A.AESGCM, 1 << 20) == 4


def test_device_api_argument_rules(aead_built):
    """The device-resident entry points reject bad jobs before any HIP call
    (aead_api.hip check_uniform / run_ragged), so these run without a GPU.
    The pointers are never dereferenced: every case fails validation."""
    A = aead_built
    fake = 1 << 20  # aligned, non-null, never touched
    ok = dict(ctx=fake, nonce_base=fake, inp=fake, out=fake + (1 << 30), in_stride=1408,
              out_stride=1424, length=1400, n_records=4, recs_per_state=4)
    for open_ in (False, True):
        for cid in (A.CHACHAPOLY, A.AESGCM):
            assert A.dev_uniform(open_, cid, **{**ok, "nonce_base": 0}) == A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**ok, "recs_per_state": 0}) == A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**ok, "ctx": fake + 8}) == A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**ok, "ad_len": 32}) == A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**ok, "length": 65520}) == A.ERROR_INVALID_LENGTH
        assert A.dev_uniform(open_, A.CHACHAPOLY, **{**ok, "lanes": 3}) == A.ERROR_INVALID_PARAM
        assert A.dev_uniform(open_, A.AESGCM, **{**ok, "lanes": 8}) == A.ERROR_INVALID_PARAM
        assert A.dev_uniform(open_, A.CHACHAPOLY, **{**ok, "n_records": 0}) == 0
        rg = dict(ctx_base=0, recs=fake, inp=fake, out=fake, n_records=4)
        for cid in (A.CHACHAPOLY, A.AESGCM):
            assert A.dev_ragged(open_, cid, **{**rg, "recs": 0}) == A.ERROR_INVALID_PARAM
            assert A.dev_ragged(open_, cid, **{**rg, "out": 0}) == A.ERROR_INVALID_PARAM
        assert A.dev_ragged(open_, A.CHACHAPOLY, **{**rg, "lanes": 5}) == A.ERROR_INVALID_PARAM
        assert A.dev_ragged(open_, 0x4399, **rg) == A.ERROR_UNKNOWN_ID
        # records must be exactly in place or disjoint: in == out
        # with two strides, or output shifted into the input, is refused
        for cid in (A.CHACHAPOLY, A.AESGCM):
            assert A.dev_uniform(open_, cid, **{**ok, "out": fake}) == A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**ok, "out": fake + 64, "out_stride": 1408}) \
                == A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**ok, "out": fake + 4 * 1408 - 16}) \
                == A.ERROR_INVALID_PARAM
            # one stride, input and output slots alternating in one buffer
            # (ADVICE r3): accepted while no two records meet, refused once
            # an output record reaches into an input record
            inter = {**ok, "in_stride": 2848, "out_stride": 2848}
            assert A.dev_uniform(open_, cid, **{**inter, "out": fake + 1424}) != A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**inter, "out": fake - 1424}) != A.ERROR_INVALID_PARAM
            assert A.dev_uniform(open_, cid, **{**inter, "out": fake + 1408}) \
                == (A.ERROR_INVALID_PARAM if open_ else A.dev_uniform(open_, cid, **{**inter, "out": fake + 1424}))
            assert A.dev_uniform(open_, cid, **{**inter, "out": fake + 1000}) == A.ERROR_INVALID_PARAM


def test_duplex_independence_rules(aead_built):
    """noise_aead_dev_duplex_uniform refuses jobs one of which writes what the
    other reads or writes: records, the open job's statuses, either AD
    (ADVICE r2).  Refused before any HIP call, so no GPU is needed."""
    A = aead_built
    G = 1 << 30
    base = dict(ctx=1 << 20, nonce_base=1 << 20, length=1400, n_records=4, recs_per_state=4)
    seal = dict(inp=2 * G, out=3 * G, in_stride=1408, out_stride=1536, **base)
    opn = dict(inp=4 * G, out=5 * G, in_stride=1536, out_stride=1408, status=6 * G, **base)
    for cid in (A.CHACHAPOLY, A.AESGCM):
        def duplex(s, o):
            return A.dev_duplex(cid, A.uniform_job(**s), A.uniform_job(**o))
        # the open reads the seal's output
        assert duplex(seal, {**opn, "inp": 3 * G}) == A.ERROR_INVALID_PARAM
        # outputs overlap
        assert duplex(seal, {**opn, "out": 3 * G + 100}) == A.ERROR_INVALID_PARAM
        # the open writes the seal's input
        assert duplex(seal, {**opn, "out": 2 * G}) == A.ERROR_INVALID_PARAM
        # the open's statuses land in the seal's output / input
        assert duplex(seal, {**opn, "status": 3 * G + 1536}) == A.ERROR_INVALID_PARAM
        assert duplex(seal, {**opn, "status": 2 * G + 8}) == A.ERROR_INVALID_PARAM
        # the open's AD sits in the seal's output; the seal's AD in the open's output
        assert duplex(seal, {**opn, "ad": 3 * G, "ad_len": 16, "ad_stride": 16}) == A.ERROR_INVALID_PARAM
        assert duplex({**seal, "ad": 5 * G + 32, "ad_len": 8, "ad_stride": 8}, opn) \
            == A.ERROR_INVALID_PARAM
        # the seal's AD sits in the open's status array
        assert duplex({**seal, "ad": 6 * G, "ad_len": 8, "ad_stride": 8}, opn) == A.ERROR_INVALID_PARAM


STRERROR = {0: "No error", 0x4501: "Out of memory", 0x4502: "Unknown identifier",
            0x4503: "Unknown name", 0x4504: "MAC failure", 0x4505: "Not applicable",
            0x4506: "System error", 0x4507: "Remote public key required",
            0x4508: "Local keypair required", 0x4509: "Pre shared key required",
            0x450A: "Invalid length", 0x450B: "Invalid parameter", 0x450C: "Invalid state",
            0x450D: "Invalid nonce", 0x450E: "Invalid private key", 0x450F: "Invalid public key",
            0x4510: "Invalid format", 0x4511: "Invalid signature"}


def _strerror(lib, err, size=64):
    buf = C.create_string_buffer(size)
    rc = lib.noise_strerror(err, buf, size)
    return rc, buf.value.decode()


def test_strerror_contract(L):
    """noise_strerror / noise_perror of the standalone library: the strings of
    src/protocol/errors.c:45-63, unknown codes, truncation, bad buffers."""
    for code, text in STRERROR.items():
        assert _strerror(L, code) == (0, text)
    for code in (0x4500, 0x4512, 0x4301, -1, 12345):
        assert _strerror(L, code) == (0, f"Unknown error 0x{code & 0xffffffff:x}")
    assert _strerror(L, 0x4504, 4) == (0, "MAC")  # truncated, NUL-terminated
    assert L.noise_strerror(0x4504, None, 16) == -1
    buf = C.create_string_buffer(4)
    assert L.noise_strerror(0x4504, buf, 0) == -1
    # noise_perror writes "<s>: <text>" to stderr
    code = ("import sys; sys.path.insert(0, %r); import noise_aead as A; "
            "A.lib().noise_perror(b'ctx', 0x450D); A.lib().noise_perror(None, 0x4599)"
            % os.path.join(ROOT, "noise-c_amd"))
    r = subprocess.run([os.sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert r.stderr.splitlines()[-2:] == ["ctx: Invalid nonce", "(null): Unknown error 0x4599"]


def test_strerror_matches_reference(L):
    """The same strings as the reference's own noise_strerror (compiled from
    /root/reference; build container only)."""
    ref = os.path.join(ROOT, "oracle", "_ref", "libnoiseref.so")
    if not os.path.exists(ref):
        pytest.skip("oracle/_ref not built")
    R = C.CDLL(ref)
    R.noise_strerror.argtypes = [C.c_int, C.c_char_p, C.c_size_t]
    for code in list(STRERROR) + [0x4500, 0x4512, 7]:
        for size in (64, 5):
            a, b = C.create_string_buffer(size), C.create_string_buffer(size)
            assert R.noise_strerror(code, a, size) == L.noise_strerror(code, b, size)
            assert a.value == b.value, hex(code)


def test_ad_longer_than_descriptor_field_refused(aead_built):
    """AD over 4 GiB cannot be described to the device (32-bit ad_len): the
    keyed encrypt/decrypt refuse it with INVALID_LENGTH before any GPU work
    (and leave n alone); a keyless pass-through does not look at AD."""
    A = aead_built
    L = A.lib()
    st = C.c_void_p()
    assert L.noise_cipherstate_new_by_id(C.byref(st), A.CHACHAPOLY) == 0
    data = (C.c_uint8 * 64)()
    ad = (C.c_uint8 * 1)()
    buf = A.NoiseBuffer(C.cast(data, C.c_void_p), 16, 64)
    # no key: pass-through, AD ignored
    assert L.noise_cipherstate_encrypt_with_ad(st, ad, 2**32, C.byref(buf)) == 0
    key = (C.c_uint8 * 32)(*range(32))
    assert L.noise_cipherstate_init_key(st, key, 32) == 0
    assert L.noise_cipherstate_encrypt_with_ad(st, ad, 2**32, C.byref(buf)) == A.ERROR_INVALID_LENGTH
    buf2 = A.NoiseBuffer(C.cast(data, C.c_void_p), 32, 64)
    assert L.noise_cipherstate_decrypt_with_ad(st, ad, 2**32 + 5, C.byref(buf2)) == A.ERROR_INVALID_LENGTH
    n = C.c_uint64()
    assert L.noise_cipherstate_set_nonce(st, 0) == 0  # n is still 0
    assert L.noise_cipherstate_free(st) == 0
