"""Regenerate the golden AEAD fixtures from the REFERENCE itself.

Run in the build container (needs /root/reference):
    make -C oracle hot && python tests/golden/gen_golden.py

Every expected output below is produced by the reference noise-c compiled from
/root/reference into oracle/_ref/libnoiseref.so, driven through its public
CipherState API (include/noise/protocol/cipherstate.h:34-53).  Inputs are
deterministic (SplitMix64) so the fixtures only need to carry
seeds for large records; small records carry their bytes as hex.

Outputs (data only — no reference source is copied):
  kat.json   the reference's own known-answer vectors
             (tests/unit/test-cipherstate.c:230-280), re-run through the ref
  grid.json  both ciphers x lengths x AD x nonces
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from oracle import AESGCM, CHACHAPOLY, Oracle, RefLib  # noqa: E402

# tests/unit/test-cipherstate.c:230-280 (data of the reference's own KATs)
KATS = [
    dict(name="rfc7539_A5", cipher=CHACHAPOLY,
         key="1c9240a5eb55d38af333888604f6b5f0473917c1402b80099dca5cbc207075c0",
         nonce=0x0807060504030201, ad="f33388860000000000004e91",
         pt=("496e7465726e65742d4472616674732061726520647261667420646f63756d65"
             "6e74732076616c696420666f722061206d6178696d756d206f6620736978206d"
             "6f6e74687320616e64206d617920626520757064617465642c207265706c6163"
             "65642c206f72206f62736f6c65746564206279206f7468657220646f63756d65"
             "6e747320617420616e792074696d652e20497420697320696e617070726f7072"
             "6961746520746f2075736520496e7465726e65742d4472616674732061732072"
             "65666572656e6365206d6174657269616c206f7220746f206369746520746865"
             "6d206f74686572207468616e206173202fe2809c776f726b20696e2070726f67"
             "726573732e2fe2809d"),
         ct=("64a0861575861af460f062c79be643bd5e805cfd345cf389f108670ac76c8cb2"
             "4c6cfc18755d43eea09ee94e382d26b0bdb7b73c321b0100d4f03b7f355894cf"
             "332f830e710b97ce98c8a84abd0b948114ad176e008d33bd60f982b1ff37c855"
             "9797a06ef4f0ef61c186324e2b3506383606907b6a7c02b0f9f6157b53c867e4"
             "b9166c767b804d46a59b5216cde7a4e99040c5a40433225ee282a1b0a06c523e"
             "af4534d7f83fa1155b0047718cbc546a0d072b04b3564eea1b422273f548271a"
             "0bb2316053fa76991955ebd63159434ecebb4e466dae5a1073a6727627097a10"
             "49e617d91d361094fa68f0ff77987130305beaba2eda04df997b714d6c6f2c29"
             "a6ad5cb4022b02709b"),
         tag="eead9d67890cbb22392336fea1851f38"),
    dict(name="gcm_tc13", cipher=AESGCM, key="00" * 32, nonce=0, ad="", pt="", ct="",
         tag="530f8afbc74536b9a963b4f1c4cb738b"),
    dict(name="gcm_tc14", cipher=AESGCM, key="00" * 32, nonce=0, ad="",
         pt="00" * 16, ct="cea7403d4d606b6e074ec5d3baf39d18",
         tag="d0d1c8a799996bf0265b98b5d48ab919"),
]

LENGTHS = [0, 1, 15, 16, 17, 31, 48, 56, 63, 64, 65, 127, 128, 129, 191, 255,
           256, 257, 1024, 1399, 1400, 1401, 4096, 16384, 65519]
ADS = [0, 32]
NONCES = [0, 1, 2**32 - 1, 2**32, 2**64 - 2]
HEX_MAX = 1500
SEED_KEY, SEED_PT, SEED_AD = 0x6B6579, 0x7074, 0x6164


def main():
    ref, orc = RefLib(), Oracle()
    kat_out = []
    for k in KATS:
        key, pt, ad = (bytes.fromhex(k[x]) for x in ("key", "pt", "ad"))
        got = ref.encrypt(k["cipher"], key, k["nonce"], pt, ad)
        assert got.hex() == k["ct"] + k["tag"], k["name"]
        kat_out.append(k)
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"source": "tests/unit/test-cipherstate.c:230-280, re-run "
                             "through oracle/_ref/libnoiseref.so", "vectors": kat_out},
                  f, indent=1)

    cases = []
    idx = 0
    for cipher in (CHACHAPOLY, AESGCM):
        for length in LENGTHS:
            for adl in ADS:
                for n in NONCES:
                    key = orc.fill(SEED_KEY, 32, 4 * idx)
                    pt = orc.fill(SEED_PT, length, idx << 16)
                    ad = orc.fill(SEED_AD, adl, idx << 8)
                    out = ref.encrypt(cipher, key, n, pt, ad)
                    c = dict(cipher=cipher, len=length, ad_len=adl, nonce=n,
                             key=key.hex(), pt_word0=idx << 16, ad_word0=idx << 8,
                             tag=out[-16:].hex(),
                             sha256=hashlib.sha256(out).hexdigest())
                    if length <= HEX_MAX:
                        c["ct"] = out[:-16].hex()
                    cases.append(c)
                    idx += 1
    with open(os.path.join(HERE, "grid.json"), "w") as f:
        json.dump({"source": "oracle/_ref/libnoiseref.so (reference noise-c, ref backend)",
                   "seed_key": SEED_KEY, "seed_pt": SEED_PT, "seed_ad": SEED_AD,
                   "cases": cases}, f, indent=0)
    print(f"kat: {len(kat_out)}  grid: {len(cases)}")


if __name__ == "__main__":
    main()
