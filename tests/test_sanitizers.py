"""Host C under AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r1
item 8; the reference keeps --enable-asan / --enable-ubsan builds,
configure.ac:102-115).  `make -C noise-c_amd asan` builds cipherstate.c,
wire.c, host_pool.c and errors.c with -fsanitize=address,undefined over CPU
stubs of the HIP runtime and of the device launchers (noise-c_amd/asan/; the
stub launchers compute with the oracle, this is test infrastructure only):

- asan_driver runs the host paths end to end — single calls, batches with
  mixed states / AD / bad lengths / exhausted nonces / MAC failures / a forged
  run, a multi-chunk batch, wire seal and echo on pageable and pinned buffers
  — against the sequential semantics, with leak checking;
- the Python host-rule tests (test_abi.py's CipherState rules,
  test_wire.py::test_wire_host_rules) run against the same sanitized library
  under LD_PRELOAD=libasan.
Any sanitizer report fails the test (-fno-sanitize-recover=all)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "noise-c_amd")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def asan_build():
    if not _runtime("libasan.so"):
        pytest.skip("gcc's libasan is not installed")
    subprocess.run(["make", "-s", "-C", LIB, "asan"], check=True)
    return os.path.join(LIB, "asan")


def test_asan_driver(asan_build):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(asan_build, "asan_driver")], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan driver ok" in r.stdout
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]


HOST_RULE_TESTS = [
    "tests/test_abi.py::test_cipherstate_errors",
    "tests/test_abi.py::test_strerror_contract",
    "tests/test_abi.py::test_ad_longer_than_descriptor_field_refused",
    "tests/test_wire.py::test_wire_host_rules",
    "tests/test_batch_host.py",
]


def test_python_host_rules_under_asan(asan_build):
    pre = ":".join(p for p in (_runtime("libasan.so"), _runtime("libubsan.so")) if p)
    env = dict(os.environ, LD_PRELOAD=pre, ASAN_OPTIONS="detect_leaks=0",
               NOISE_AEAD_LIB=os.path.join(asan_build, "libnoise_aead_asan.so"))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider"] + HOST_RULE_TESTS,
                       cwd=ROOT, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
