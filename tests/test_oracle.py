"""Pin the oracle: the repo's CPU restatement (oracle/noise_oracle.c) against
the reference's own KATs, published primitive vectors, the golden fixtures
generated from the reference itself, and (in the build container) the
reference library directly on random inputs."""
import hashlib
import os
import random

import pytest

CHACHA, AES = 0x4301, 0x4302


def test_kat_vectors(oracle, golden):
    """tests/unit/test-cipherstate.c:230-280 (RFC 7539 A.5, GCM TC13/14)."""
    kat, _ = golden
    assert len(kat["vectors"]) == 3
    for v in kat["vectors"]:
        key, pt, ad = (bytes.fromhex(v[x]) for x in ("key", "pt", "ad"))
        out = oracle.encrypt(v["cipher"], key, v["nonce"], pt, ad)
        assert out.hex() == v["ct"] + v["tag"], v["name"]
        rc, back = oracle.decrypt(v["cipher"], key, v["nonce"], out, ad)
        assert rc == 0 and back == pt


def test_grid_fixture(oracle, golden):
    """All 500 reference-generated grid cases (tests/golden/grid.json)."""
    _, grid = golden
    assert len(grid["cases"]) == 500
    for c in grid["cases"]:
        pt = oracle.fill(grid["seed_pt"], c["len"], c["pt_word0"])
        ad = oracle.fill(grid["seed_ad"], c["ad_len"], c["ad_word0"])
        out = oracle.encrypt(c["cipher"], bytes.fromhex(c["key"]), c["nonce"], pt, ad)
        assert out[-16:].hex() == c["tag"]
        assert hashlib.sha256(out).hexdigest() == c["sha256"]
        if "ct" in c:
            assert out[:-16].hex() == c["ct"]


def test_chacha20_block_rfc8439(oracle):
    """RFC 8439 §2.3.2: counter 1, nonce 00000009 0000004a 00000000 maps onto
    the 64/64 layout of chacha.c:111-133 as counter = 1 | 0x09000000<<32,
    IV = 0x4a000000."""
    key = bytes(range(32))
    out = oracle.chacha20_block(key, 1 | (0x09000000 << 32), 0x4a000000)
    assert out.hex() == (
        "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
        "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_poly1305_rfc8439(oracle):
    """RFC 8439 §2.5.2."""
    key = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    tag = oracle.poly1305(key, b"Cryptographic Forum Research Group")
    assert tag.hex() == "a8061dc1305136c6c22b8baf0c0127a9"


def test_aes256_fips197(oracle):
    """FIPS-197 Appendix C.3."""
    out = oracle.aes256(bytes(range(32)), bytes.fromhex("00112233445566778899aabbccddeeff"))
    assert out.hex() == "8ea2b7ca516745bfeafc49904b496089"


def test_gf128_mul_identity(oracle):
    """x^0 (0x80 00..00 in GCM bit order) is the multiplicative identity."""
    one = bytes([0x80]) + bytes(15)
    h = bytes(range(1, 17))
    assert oracle.gf128_mul(one, h) == h
    assert oracle.gf128_mul(h, one) == h


def test_decrypt_rejects_tamper(oracle):
    rng = random.Random(4)
    for cipher in (CHACHA, AES):
        key = bytes(rng.randrange(256) for _ in range(32))
        pt = bytes(rng.randrange(256) for _ in range(333))
        ct = bytearray(oracle.encrypt(cipher, key, 77, pt))
        for pos in (0, 100, len(ct) - 1):
            bad = bytearray(ct)
            bad[pos] ^= 1
            rc, _ = oracle.decrypt(cipher, key, 77, bytes(bad))
            assert rc == 0x4504
        rc, _ = oracle.decrypt(cipher, key, 78, bytes(ct))  # wrong nonce
        assert rc == 0x4504


def test_oracle_matches_reference_random(oracle, reflib):
    """Cross-check against the reference built from /root/reference (skipped
    where the sources are absent, e.g. on the GPU box)."""
    rng = random.Random(1)
    for _ in range(400):
        cipher = rng.choice([CHACHA, AES])
        L = rng.choice([0, 1, 15, 16, 17, 63, 64, 65, 1399, 1400, 1401, rng.randrange(3000)])
        ad = bytes(rng.randrange(256) for _ in range(rng.choice([0, 0, 1, 16, 32, 33])))
        key = bytes(rng.randrange(256) for _ in range(32))
        n = rng.choice([0, 1, 2**32 - 1, 2**32, 2**64 - 2, rng.getrandbits(63)])
        pt = bytes(rng.randrange(256) for _ in range(L))
        assert oracle.encrypt(cipher, key, n, pt, ad) == reflib.encrypt(cipher, key, n, pt, ad)


def test_splitmix_fill(oracle):
    """SplitMix64 generator of SURVEY.md §8d (first outputs of seed 0)."""
    assert oracle.splitmix64(0) == 0xE220A8397B1DCDAF
    b = oracle.fill(0, 16)
    assert int.from_bytes(b[:8], "little") == 0xE220A8397B1DCDAF


def test_hash_oracle_standard_vectors(oracle):
    """FIPS 180-4 / RFC 7693 'abc' vectors for the four Noise hashes
    (noise_oracle_hash.c)."""
    exp = {0x4803: "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
           0x4804: "ddaf35a193617abacc417349ae20413112e6fa4e89a97ea20a9eeee64b55d39a"
                   "2192992a274fc1a836ba3c23a3feebbd454d4423643ce80e2a9ac94fa54ca49f",
           0x4801: "508c5e8c327c14e2e1a72ba34eeb452f37458b209ed63a294d999b4c86675982",
           0x4802: "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
                   "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923"}
    for hid, h in exp.items():
        assert oracle.hash(hid, b"abc").hex() == h


def test_hkdf_oracle_vs_reference_golden(oracle):
    """tests/golden/hkdf.json: noise_hashstate_hkdf outputs of the reference
    itself (gen_hkdf.py), split and mix_key shapes, all four hashes."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "hkdf.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) == 40
    for c in cases:
        o1, o2 = oracle.hkdf(c["hash_id"], bytes.fromhex(c["key"]), bytes.fromhex(c["data"]),
                             len(c["out1"]) // 2, len(c["out2"]) // 2)
        assert (o1.hex(), o2.hex()) == (c["out1"], c["out2"]), c
