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


def test_default_layout_and_kernel_names():
    """The bench's default record slots (128 B) and the names of the kernels
    its roofline reads from profiles/traffic_<cfg>.json: every name the
    default C2/C3/C4/perf lines look up must be in the committed profile,
    or the line's traffic would silently read null."""
    import noise_aead as A

    assert bench.SLOT_ALIGN == 128
    assert (bench.stride(1400, 128), bench.stride(1416, 128)) == (1408, 1536)
    for cfg in ("c2", "c3", "c4", "perf"):
        c = bench.CONFIGS[cfg]
        n, s = c["records"], c["states"]
        ad = c.get("ad", 0)
        ins, outs = bench.stride(c["len"], 128), bench.stride(c["len"] + 16, 128)
        lanes = A.dev_duplex_lanes(c["cipher"], n)  # the library's choice for the timed duplex launch
        k = bench.kernel_name(c["cipher"], n, n // s, lanes, ins, outs, c["len"], duplex=True)
        assert "_duplex_" in k, (cfg, k)
        prof = bench.load_pmc(cfg, k)
        assert prof.get("hbm_bytes_per_launch"), (cfg, k)
        assert ad == 0 or cfg == "perf"


def test_c5_profile_names():
    """C5's dominant kernels as bench.run_mixed names them (the library's
    gcm_ragged_shape policy at 64 Ki AES records per GPU: 1024 threads, two
    records per 8-lane group; the segmented persistent ChaChaPoly kernel for
    64 Ki ragged FAST records) are in the committed C5 profile."""
    import json
    with open(os.path.join(ROOT, "profiles", "traffic_c5.json")) as f:
        kernels = json.load(f)["kernels"]
    for open_ in ("true", "false"):
        assert f"gcm_ragged_staged<{open_}, true, 1024, false, 2, 8>" in kernels
        assert f"chachapoly_seg_ragged<{open_}>" in kernels


def _bench(args, env=None, timeout=240):
    import subprocess
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=timeout, env=e)


def test_gpus_n_launches_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts the two
    ranks itself (a child torch.distributed.run on 127.0.0.1, gloo here) and
    relays rank 0's one line, which reports n_gpus 2.  --dry-run: the
    launcher and process-group plumbing without GPU work."""
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] and d["rank_env"]["WORLD_SIZE"] == "2"
    assert d["rank_env"]["MASTER_ADDR"] == "127.0.0.1"


def test_gpus_must_match_world_size():
    r = _bench(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    r = _bench(["--dry-run", "--steps", "1"])  # no launcher, no --gpus: one rank
    assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_shard_goldens_cover_every_rank():
    """bench.py verifies each rank's sealed shard against these digests."""
    for cfg in ("c2", "c3", "perf", "c5", "c5s"):
        for r in range(8):
            assert bench.shard_golden(cfg, r, 8, False), (cfg, r)
    for w in (1, 2, 4, 8):
        for r in range(w):
            assert bench.shard_golden("c4", r, w, True), (w, r)
    with open(os.path.join(ROOT, "tests", "golden", "config_digests.json")) as f:
        base = json.load(f)["configs"]
    assert bench.shard_golden("c2", 0, 1, False) == base["c2"]["sealed_sha256"]
    assert bench.shard_golden("c4", 0, 1, True) == base["c4"]["sealed_sha256"]


def test_bench_module_constants_exist():
    """Every noise_aead constant bench.py reads (A.FLAG_*, A.CHACHA ...) is
    defined: a run with a flag whose constant is missing would die on the GPU
    box after its setup, not here."""
    import re

    import noise_aead as A

    with open(os.path.join(ROOT, "bench.py")) as f:
        names = set(re.findall(r"\bA\.([A-Z][A-Z0-9_]+)\b", f.read()))
    assert names, "no constants found"
    missing = sorted(n for n in names if not hasattr(A, n))
    assert not missing, missing


def test_group_runs_keep_stdout_for_the_line():
    """A run with a process group points fd 1 at stderr (RCCL prints its
    banner on stdout when a communicator is made); the JSON line still goes
    to the original stdout, alone."""
    import subprocess
    code = ("import os, sys; sys.path.insert(0, %r); import bench; bench.keep_stdout_for_line(); "
            "os.write(1, b'RCCL version : x\\n'); print('stray'); bench.emit_line({'metric': 'm'})" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"metric": "m"}']
    assert "RCCL version" in r.stderr and "stray" in r.stderr
