"""bench.py host logic (no GPU): the per-GPU efficiency field, the rehearsal
label, and the CPU-baseline core accounting."""
import io
import json
import os
import sys
from contextlib import redirect_stdout
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _finish(result, world, n1, rehearse=False):
    old = bench.REHEARSE
    bench.REHEARSE = rehearse
    try:
        buf = io.StringIO()
        with redirect_stdout(buf):
            bench.finish(SimpleNamespace(n1_value=n1), dict(result), 0, world, None)
        return json.loads(buf.getvalue())
    finally:
        bench.REHEARSE = old


def test_per_gpu_efficiency():
    r = _finish({"value": 7600.0, "roofline": {"frac": 0.3}}, 8, 1000.0)
    assert r["per_gpu_efficiency"] == 0.95 and r["n1_value"] == 1000.0
    assert "per_gpu_efficiency" not in _finish({"value": 1000.0}, 1, 1000.0)
    assert "per_gpu_efficiency" not in _finish({"value": 2000.0}, 2, None)


def test_rehearsal_drops_roofline_and_says_so():
    r = _finish({"value": 900.0, "roofline": {"frac": 0.2}}, 2, None, rehearse=True)
    assert "roofline" not in r
    assert "gloo" in r["rehearsal"] and "nccl" not in r["rehearsal"]


def test_host_cpu_counts():
    h = bench.host_cpu()
    assert h["usable_cpus"] >= 1
    assert h["physical_cores"] is None or 1 <= h["physical_cores"] <= h["usable_cpus"]
    assert bench.physical_cores([0]) in (None, 1)
