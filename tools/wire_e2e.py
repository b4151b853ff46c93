"""End-to-end rate of the transport wire path.

A buffer of N framed records (examples/echo wire format: 2-byte BE length ||
CT || tag) starts and ends in host memory, as a socket buffer does.  One call
of noise_wire_seal / noise_wire_open / noise_wire_echo covers the H2D copy,
the kernel(s) and the D2H copy, pipelined in chunks (csrc/wire.c).  Measured
for a pinned buffer (noise_wire_alloc: no staging copy) and for an ordinary
pageable buffer (staged through pinned memory by the host thread pool).

Usage: python tools/wire_e2e.py [--records 65536] [--len 1400] [--cipher chachapoly|aesgcm]
Prints one JSON line per (buffer kind); rates are GiB/s of payload.
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
    F = 2 + L + 16
    rng = np.random.default_rng(3)
    k1 = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    k2 = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    img = np.zeros((N, F), dtype=np.uint8)
    img[:, 0], img[:, 1] = (L + 16) >> 8, (L + 16) & 0xFF
    img[:, 2:2 + L] = rng.integers(0, 256, (N, L), dtype=np.uint8)
    img = img.reshape(-1)
    nbytes = img.size
    gib = N * L / 2**30
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            pw = A.PinnedWire(nbytes)
            view = np.frombuffer(pw.view, dtype=np.uint8)
            addr = pw.addr
        else:
            host = np.zeros(nbytes, dtype=np.uint8)
            view, addr = host, host.ctypes.data
        times = {"seal": [], "echo": [], "open": []}
        # one session: the key contexts are built on first use (hipMalloc +
        # key schedule), a per-session cost kept out of the per-buffer rate
        cli_send, srv_recv, srv_send, cli_recv = (A.CipherState.new_by_id(cid)[1] for _ in range(4))
        for s, k in ((cli_send, k1), (srv_recv, k1), (srv_send, k2), (cli_recv, k2)):
            assert s.init_key(k) == 0
        for r in range(args.reps + 1):
            view[:] = img
            t0 = time.perf_counter()
            rc1 = A.wire_seal(cli_send, addr, nbytes)
            t1 = time.perf_counter()
            rc2 = A.wire_echo(srv_recv, srv_send, addr, nbytes)
            t2 = time.perf_counter()
            rc3 = A.wire_open(cli_recv, addr, nbytes)
            t3 = time.perf_counter()
            for rc in (rc1, rc2, rc3):
                assert rc == (0, nbytes, N), rc
            assert np.array_equal(view.reshape(N, F)[:, 2:2 + L], img.reshape(N, F)[:, 2:2 + L])
            if r:
                times["seal"].append(t1 - t0)
                times["echo"].append(t2 - t1)
                times["open"].append(t3 - t2)
        for s in (cli_send, srv_recv, srv_send, cli_recv):
            s.free()
        if kind == "pinned":
            pw.close()
        best = {k: min(v) for k, v in times.items()}
        print(json.dumps({
            "metric": "GiB/s end-to-end wire-buffer AEAD (noise_wire_*, PCIe-inclusive)",
            "buffer": kind, "cipher": args.cipher, "frames": N, "record_len": L,
            "seal_gibs": round(gib / best["seal"], 3), "echo_gibs": round(gib / best["echo"], 3),
            "open_gibs": round(gib / best["open"], 3),
            "seal_ms": round(best["seal"] * 1e3, 3), "echo_ms": round(best["echo"] * 1e3, 3),
            "open_ms": round(best["open"] * 1e3, 3), "reps": args.reps,
            "check": "client seal -> server echo (open c2s, seal s2c) -> client open == plaintext",
            "timing": "best of reps, wall clock around each C call"}), flush=True)


if __name__ == "__main__":
    main()
