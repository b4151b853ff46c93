"""Shared test fixtures.

`-m "not gpu"` tests run in the CPU-only build container: the oracle against
the golden vectors, host-side logic, the C-ABI surface.  `-m gpu` tests call
the gfx950 library through its C ABI and compare with the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "noise-c_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    if not os.path.exists(O.ORACLE_SO):
        O.build(ref=False)
    return O.Oracle()


@pytest.fixture(scope="session")
def reflib():
    """The reference noise-c compiled from /root/reference (build container)."""
    import oracle as O
    if not os.path.exists(O.REF_SO):
        if not os.path.isdir("/root/reference/src"):
            pytest.skip("reference sources not present (GPU box): using committed fixtures")
        O.build(ref=True)
    return O.RefLib()


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "kat.json")) as f:
        kat = json.load(f)
    with open(os.path.join(d, "grid.json")) as f:
        grid = json.load(f)
    return kat, grid


@pytest.fixture(scope="session")
def aead():
    import noise_aead
    noise_aead.lib()  # raises loudly if the gfx950 library is missing
    return noise_aead


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test without a GPU")
    return torch.device("cuda:0")
