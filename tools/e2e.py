"""End-to-end (host-memory) rate of the batch CipherState API — DESIGN.md §8.

Records start and end in pageable host memory, as a socket buffer would. One
call to noise_cipherstate_encrypt_batch (then decrypt_batch on the peer
state) covers:
- packing into the pinned staging buffer
- one H2D copy
- the kernel(s)
- one D2H copy
- unpacking
The timed loop calls the C entry points directly on prebuilt ctypes arrays,
so no Python per-record work is in it.

Usage: python tools/e2e.py [--records 65536] [--len 1400] [--cipher chachapoly|aesgcm] [--reps 5]
Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "noise-c_amd"))
import noise_aead as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=65536)
    ap.add_argument("--len", type=int, default=1400)
    ap.add_argument("--cipher", default="chachapoly", choices=["chachapoly", "aesgcm"])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    cid = A.CHACHAPOLY if args.cipher == "chachapoly" else A.AESGCM
    N, L = args.records, args.len
    slot = L + 16
    lib = A.lib()

    rng = np.random.default_rng(7)
    key = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    rc1, send = A.CipherState.new_by_id(cid)
    rc2, recv = A.CipherState.new_by_id(cid)
    assert rc1 == 0 and rc2 == 0
    assert send.init_key(key) == 0 and recv.init_key(key) == 0

    host = np.zeros(N * slot, dtype=np.uint8)
    pt = rng.integers(0, 256, (N, L), dtype=np.uint8)
    base = host.ctypes.data
    bufs = (A.NoiseBuffer * N)()
    states_s = (C.c_void_p * N)(*([send.ptr.value] * N))
    states_r = (C.c_void_p * N)(*([recv.ptr.value] * N))
    res = (C.c_int * N)()

    def load_plaintext():
        host.reshape(N, slot)[:, :L] = pt
        for i in range(N):
            bufs[i].data = base + i * slot
            bufs[i].size = L
            bufs[i].max_size = slot

    enc_t, dec_t = [], []
    for r in range(args.reps + 1):
        load_plaintext()
        t0 = time.perf_counter()
        rc = lib.noise_cipherstate_encrypt_batch(states_s, None, None, bufs, N, res)
        t1 = time.perf_counter()
        assert rc == 0 and all(x == 0 for x in res[:16]), (rc, res[:4])
        t2 = time.perf_counter()
        rc = lib.noise_cipherstate_decrypt_batch(states_r, None, None, bufs, N, res)
        t3 = time.perf_counter()
        assert rc == 0 and max(res) == 0 and min(res) == 0, rc
        if r:  # first pass warms allocations and the staging buffer
            enc_t.append(t1 - t0)
            dec_t.append(t3 - t2)
    assert np.array_equal(host.reshape(N, slot)[:, :L], pt), "round trip mismatch"
    gib = N * L / 2**30
    enc, dec = min(enc_t), min(dec_t)
    print(json.dumps({
        "metric": "GiB/s end-to-end host-buffer AEAD (batch CipherState API, PCIe-inclusive)",
        "cipher": args.cipher, "records": N, "record_len": L,
        "encrypt_gibs": round(gib / enc, 3), "decrypt_gibs": round(gib / dec, 3),
        "roundtrip_gibs": round(2 * gib / (enc + dec), 3),
        "encrypt_ms": round(enc * 1e3, 3), "decrypt_ms": round(dec * 1e3, 3),
        "reps": args.reps, "timing": "best of reps, wall clock around each C call",
    }))


if __name__ == "__main__":
    main()
