"""Drop-in proof: the reference's OWN test programs pass with this engine as
their CipherState.

oracle/Makefile `dropin` compiles the reference's tests/unit (test-noise:
11 suites, including test-cipherstate's KATs and nonce rules and
test-symmetricstate's encrypt_and_hash/split cross-checks) and tests/vector
(test-vector: 1392 handshake + transport vectors, cacophony, noise-c-basic,
-fallback, -hybrid) from /root/reference, with the reference's
cipherstate.c, internal.c and ref cipher backends left out and
libnoise_aead_hip.so linked instead.  Every CipherState the reference's
handshake, symmetric-state and test code creates is then one of ours, so
every AEAD of those programs — handshake payloads with AD = h, transport
messages, split keys — runs on the GPU.  The vector files are the
reference's own fixtures, stored gzipped under tests/golden/vectors/.
"""
import gzip
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
VECTORS = ["cacophony", "noise-c-basic", "noise-c-fallback", "noise-c-hybrid"]

pytestmark = pytest.mark.gpu


def _binary(name):
    path = os.path.join(REF, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not built (needs /root/reference: make -C oracle dropin)")
    return path


def test_reference_unit_suite_on_gpu_cipherstate(gpu):
    out = subprocess.run([_binary("test-noise-hip")], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "All tests succeeded" in out.stdout
    for suite in ("cipherstate", "handshakestate", "symmetricstate"):
        assert f"{suite} ... ok" in out.stdout


def test_reference_vectors_on_gpu_cipherstate(gpu, tmp_path):
    files = []
    for v in VECTORS:
        with gzip.open(os.path.join(ROOT, "tests", "golden", "vectors", v + ".txt.gz")) as f:
            p = tmp_path / (v + ".txt")
            p.write_bytes(f.read())
            files.append(str(p))
    out = subprocess.run([_binary("test-vector-hip")] + files, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    ok = sum(1 for line in out.stdout.splitlines() if line.endswith(" ... ok"))
    failed = [line for line in out.stdout.splitlines() if "... failed" in line]
    assert not failed, failed[:10]
    assert ok == 1392, ok
