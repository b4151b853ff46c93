"""Generate tests/golden/hkdf.json from the reference noise-c itself.

Runs noise_hashstate_hkdf (src/protocol/hashstate.c:476-516) of the reference
library compiled from /root/reference by oracle/Makefile (target `full`,
oracle/_ref/libnoiseref_full.so) for the four Noise hashes, including the
split() shape of noise_symmetricstate_split (symmetricstate.c:530-533:
key = ck of hash_len bytes, empty data, two outputs of the 32-byte cipher
key length).  Build-container only; the JSON is the committed fixture.

Usage: python tests/golden/gen_hkdf.py
"""
import ctypes as C
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "..", "oracle", "_ref", "libnoiseref_full.so")
HASHES = {"BLAKE2s": 0x4801, "BLAKE2b": 0x4802, "SHA256": 0x4803, "SHA512": 0x4804}
HLEN = {0x4801: 32, 0x4802: 64, 0x4803: 32, 0x4804: 64}


def main():
    L = C.CDLL(LIB)
    L.noise_hashstate_new_by_id.argtypes = [C.POINTER(C.c_void_p), C.c_int]
    L.noise_hashstate_hkdf.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                       C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    L.noise_hashstate_free.argtypes = [C.c_void_p]
    rnd = random.Random(0x484B4446)
    cases = []
    for name, hid in HASHES.items():
        st = C.c_void_p()
        assert L.noise_hashstate_new_by_id(C.byref(st), hid) == 0
        hl = HLEN[hid]
        shapes = [(hl, 0, 32, 32, "split")] * 4 + [
            (hl, 32, hl, hl, "mix_key"), (hl, 56, hl, hl, "mix_key"),
            (32, 0, hl, hl, ""), (200, 10, hl, 16, ""), (hl, 200, 7, hl, ""), (1, 1, 1, 1, "")]
        for kl, dl, l1, l2, kind in shapes:
            key = bytes(rnd.getrandbits(8) for _ in range(kl))
            data = bytes(rnd.getrandbits(8) for _ in range(dl))
            o1, o2 = C.create_string_buffer(64), C.create_string_buffer(64)
            rc = L.noise_hashstate_hkdf(st, key, kl, data if dl else b"\0", dl, o1, l1, o2, l2)
            assert rc == 0
            cases.append({"hash": name, "hash_id": hid, "kind": kind, "key": key.hex(),
                          "data": data.hex(), "out1": o1.raw[:l1].hex(), "out2": o2.raw[:l2].hex()})
        L.noise_hashstate_free(st)
    with open(os.path.join(HERE, "hkdf.json"), "w") as f:
        json.dump({"source": "reference noise_hashstate_hkdf (libnoiseref_full.so)",
                   "cases": cases}, f, indent=1)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
