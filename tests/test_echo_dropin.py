"""The reference's echo example (examples/echo) as a binary-level drop-in check.

oracle/Makefile's ``dropin`` target builds the reference's unmodified
echo-server and echo-client twice: ``-ref`` against the reference's own CPU
CipherState (src/protocol/cipherstate.c) and ``-hip`` against
libnoise_aead_hip.so, with the reference's handshake, DH and hash code in
both.  Every transport message of the echo session is then sealed or opened by
our GPU kernels in the ``-hip`` binaries
(examples/echo/echo-client/echo-client.c:396-440 and
examples/echo/echo-server/echo-server.c's echo loop call
noise_cipherstate_encrypt/decrypt per line).

Cross-connecting a GPU server with a CPU client (and the reverse) proves the
wire bytes are interchangeable: any bit of difference in a ciphertext or tag
makes the peer's decrypt fail with MAC_FAILURE and the session abort.

The binaries are test infrastructure built from /root/reference sources into
oracle/_ref/ (git-ignored, shipped to the GPU box with the tree); the tests
skip when they were not built.  ``ref``-only pairs run on CPU; any pair with a
``-hip`` side is ``-m gpu``.
"""
import base64
import os
import signal
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")

LINES = [b"hello\n", b"x" * 1000 + b"\n", b"the quick brown fox\n", b"\n",
         bytes(range(32, 127)) + b"\n"]


def _bin(name):
    p = os.path.join(REF, name)
    if not os.access(p, os.X_OK):
        pytest.skip(f"{name} not built (make -C oracle dropin)")
    return p


@pytest.fixture(scope="module")
def keydir(tmp_path_factory):
    """Keys laid out as examples/echo/echo-server/echo-server.c:258-277 loads them."""
    keygen = _bin("echo-keygen")
    d = tmp_path_factory.mktemp("echo_keys")
    for who in ("client", "server"):
        for curve in ("25519", "448"):
            subprocess.run([keygen, curve, f"{who}_key_{curve}",
                            f"{who}_key_{curve}.pub"], cwd=d, check=True,
                           timeout=60, capture_output=True)
    (d / "psk").write_bytes(base64.b64encode(os.urandom(32)) + b"\n")
    return d


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _listening(port):
    """Whether something LISTENs on ``port`` (without consuming the server's
    single accept, echo-common.c:389)."""
    hexport = f":{port:04X}"
    for f in ("/proc/net/tcp", "/proc/net/tcp6"):
        try:
            with open(f) as fh:
                next(fh)
                for line in fh:
                    parts = line.split()
                    if parts[1].endswith(hexport) and parts[3] == "0A":
                        return True
        except OSError:
            pass
    return False


def _children(pid):
    """Live (non-zombie) children: the server reaps exited sessions lazily."""
    try:
        with open(f"/proc/{pid}/task/{pid}/children") as fh:
            kids = [int(c) for c in fh.read().split()]
    except OSError:
        return []
    live = []
    for c in kids:
        try:
            with open(f"/proc/{c}/stat") as fh:
                if fh.read().rsplit(")", 1)[1].split()[0] != "Z":
                    live.append(c)
        except OSError:
            pass
    return live


def run_echo(server, client, keydir, protocol, *, client_args=(), lines=LINES,
             timeout=120):
    """One echo session.  echo-server forks a child per connection and keeps
    accepting (echo-common.c:389-560), so the server runs in its own process
    group: wait for the session child to finish, then end that group."""
    port = _free_port()
    srv = subprocess.Popen([server, f"--key-dir={keydir}", str(port)],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           start_new_session=True)
    try:
        t0 = time.time()
        while not _listening(port):
            if srv.poll() is not None or time.time() - t0 > 60:
                raise AssertionError("server did not listen")
            time.sleep(0.05)
        cl = subprocess.run([client, *client_args, protocol, "127.0.0.1",
                             str(port)], input=b"".join(lines),
                            capture_output=True, timeout=timeout, cwd=keydir)
        t0 = time.time()
        while _children(srv.pid) and time.time() - t0 < 60:
            time.sleep(0.05)
        session_done = not _children(srv.pid)
    finally:
        os.killpg(srv.pid, signal.SIGTERM)
        _, serr = srv.communicate(timeout=60)
    assert session_done, "server session child did not exit"
    return cl, serr


def _key_args(protocol):
    """Client-side key options the pattern needs (doc/example-echo.dox:280)."""
    parts = protocol.split("_")
    pattern, curve = parts[1], parts[2]
    args = []
    if pattern[0] in "KXI":
        args.append(f"--client-private-key=client_key_{curve}")
    if pattern[1:2] == "K":
        args.append(f"--server-public-key=server_key_{curve}.pub")
    if protocol.startswith("NoisePSK"):
        args.append("--psk=psk")
    return args


def check_session(cl, serr, protocol, lines=LINES):
    out = cl.stdout
    assert cl.returncode == 0, (protocol, cl.stderr.decode(), serr.decode())
    assert f"{protocol} handshake complete".encode() in out
    got = out.split(b"Received: ")[1:]
    assert got == lines, (protocol, got[:2])


PROTOCOLS = [
    "Noise_NN_25519_ChaChaPoly_BLAKE2s",
    "Noise_XX_25519_AESGCM_SHA256",
    "Noise_IK_448_ChaChaPoly_BLAKE2b",
    "Noise_KK_25519_AESGCM_SHA512",
    "NoisePSK_XX_25519_ChaChaPoly_SHA256",
]


@pytest.mark.parametrize("protocol", PROTOCOLS[:2])
def test_echo_ref_ref(keydir, protocol):
    """The harness itself, CPU both ends."""
    cl, serr = run_echo(_bin("echo-server-ref"), _bin("echo-client-ref"),
                        keydir, protocol, client_args=_key_args(protocol))
    check_session(cl, serr, protocol)


@pytest.mark.gpu
@pytest.mark.parametrize("pair", [("hip", "ref"), ("ref", "hip"), ("hip", "hip")])
@pytest.mark.parametrize("protocol", PROTOCOLS)
def test_echo_dropin(keydir, pair, protocol):
    server = _bin(f"echo-server-{pair[0]}")
    client = _bin(f"echo-client-{pair[1]}")
    cl, serr = run_echo(server, client, keydir, protocol,
                        client_args=_key_args(protocol))
    check_session(cl, serr, protocol)


@pytest.mark.gpu
@pytest.mark.parametrize("pair", [("hip", "ref"), ("ref", "hip")])
def test_echo_dropin_padding(keydir, pair):
    """--padding (echo-client.c:398-410): every record is max_line_len bytes,
    random-padded by the reference's RandState — long records through the GPU."""
    protocol = "Noise_XX_25519_AESGCM_BLAKE2b"
    cl, serr = run_echo(_bin(f"echo-server-{pair[0]}"),
                        _bin(f"echo-client-{pair[1]}"), keydir, protocol,
                        client_args=["--padding", *_key_args(protocol)])
    check_session(cl, serr, protocol)
