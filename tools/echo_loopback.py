"""Echo loopback over a real TCP socket (BASELINE config C1).

The reference's examples/echo in its transport phase: the client sends framed
ChaChaPoly messages (2-byte BE length || CT || tag, echo-common.c:643-688),
the server decrypts each with its receive CipherState, re-encrypts it with its
send CipherState and writes it back (echo-server.c:377-407), the client
decrypts the echo.  Here both ends move whole socket buffers through the GPU:
the client seals a burst of messages with noise_wire_seal, the server runs
noise_wire_echo on every complete frame it has received (a frame split across
recv() calls waits for its tail), the client checks the echoes with
noise_wire_open.  The handshake is out of scope: both sides
start from the same two transport keys, as after noise_handshakestate_split.

Usage: python tools/echo_loopback.py [--messages 65536] [--size 1024] [--burst 4096]
Prints one JSON line.
"""
import argparse
import json
import os
import socket
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "noise-c_amd"))
import noise_aead as A  # noqa: E402


def recv_exact(sock, view, n):
    got = 0
    while got < n:
        k = sock.recv_into(view[got:n], n - got)
        if not k:
            raise ConnectionError("peer closed")
        got += k
    return got


def server(sock, cid, k_c2s, k_s2c, cap, stats):
    recv = A.CipherState.new_by_id(cid)[1]
    send = A.CipherState.new_by_id(cid)[1]
    recv.init_key(k_c2s)
    send.init_key(k_s2c)
    pw = A.PinnedWire(cap)
    buf = memoryview(pw.view).cast("B")
    have = 0
    try:
        while True:
            k = sock.recv_into(buf[have:], cap - have)
            if not k:
                break
            have += k
            rc, consumed, frames = A.wire_echo(recv, send, pw.addr, have)
            if rc:
                stats["server_error"] = rc
                break
            if consumed:
                sock.sendall(buf[:consumed])
                stats["frames"] = stats.get("frames", 0) + frames
                stats["calls"] = stats.get("calls", 0) + 1
                buf[:have - consumed] = bytes(buf[consumed:have])  # keep the partial frame
                have -= consumed
    finally:
        pw.close()
        recv.free()
        send.free()
        sock.close()


def run(messages=65536, size=1024, burst=4096, cipher="chachapoly"):
    args = argparse.Namespace(messages=messages, size=size, burst=burst, cipher=cipher)
    cid = A.CHACHAPOLY if args.cipher == "chachapoly" else A.AESGCM
    rng = np.random.default_rng(11)
    k_c2s = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    k_s2c = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    F = 2 + args.size + 16
    burst_bytes = args.burst * F

    lsock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    lsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    lsock.bind(("127.0.0.1", 0))
    lsock.listen(1)
    port = lsock.getsockname()[1]
    stats = {}
    csock = socket.create_connection(("127.0.0.1", port))
    ssock, _ = lsock.accept()
    lsock.close()
    th = threading.Thread(target=server, args=(ssock, cid, k_c2s, k_s2c, 4 * burst_bytes, stats))
    th.start()

    send = A.CipherState.new_by_id(cid)[1]
    recv = A.CipherState.new_by_id(cid)[1]
    send.init_key(k_c2s)
    recv.init_key(k_s2c)
    out = A.PinnedWire(burst_bytes)
    back = A.PinnedWire(burst_bytes)
    ov, bv = memoryview(out.view).cast("B"), memoryview(back.view).cast("B")
    ok, sent, t_seal = True, 0, 0.0
    t0 = time.perf_counter()
    while sent < args.messages:
        n = min(args.burst, args.messages - sent)
        msgs = rng.integers(0, 256, (n, args.size), dtype=np.uint8)
        img = np.zeros((n, F), dtype=np.uint8)
        img[:, 0], img[:, 1] = (args.size + 16) >> 8, (args.size + 16) & 0xFF
        img[:, 2:2 + args.size] = msgs
        nb = n * F
        ov[:nb] = img.reshape(-1).tobytes()
        ts = time.perf_counter()
        rc = A.wire_seal(send, out.addr, nb)
        t_seal += time.perf_counter() - ts
        assert rc == (0, nb, n), rc
        # send and receive concurrently (the echo of a burst may exceed socket buffers)
        tx = threading.Thread(target=csock.sendall, args=(ov[:nb],))
        tx.start()
        recv_exact(csock, bv, nb)
        tx.join()
        rc = A.wire_open(recv, back.addr, nb)
        assert rc == (0, nb, n), rc
        ok &= np.array_equal(np.frombuffer(bv[:nb], dtype=np.uint8).reshape(n, F)[:, 2:2 + args.size], msgs)
        sent += n
    elapsed = time.perf_counter() - t0
    csock.shutdown(socket.SHUT_WR)
    th.join(timeout=60)
    csock.close()
    for x in (out, back):
        x.close()
    send.free()
    recv.free()
    return {
        "metric": "echo loopback (TCP 127.0.0.1), transport phase, messages echoed per second",
        "cipher": args.cipher, "messages": args.messages, "size": args.size, "burst": args.burst,
        "msgs_per_s": round(args.messages / elapsed, 1),
        "payload_gibs_round_trip": round(args.messages * args.size / elapsed / 2**30, 3),
        "server_echo_calls": stats.get("calls"), "server_frames": stats.get("frames"),
        "server_error": stats.get("server_error", 0), "verified": bool(ok),
        "note": "4 AEAD ops per message (client seal, server open+seal, client open), all on the GPU"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--messages", type=int, default=65536)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--burst", type=int, default=4096, help="messages per client send")
    ap.add_argument("--cipher", default="chachapoly", choices=["chachapoly", "aesgcm"])
    a = ap.parse_args()
    r = run(a.messages, a.size, a.burst, a.cipher)
    print(json.dumps(r), flush=True)
    if not r["verified"] or r["server_error"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
