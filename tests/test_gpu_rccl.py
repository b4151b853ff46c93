"""The N > 1 code path of bench.py on RCCL, on one GPU (VERDICT r4 weak #10:
the nccl process group and the RCCL scatter/gather legs had never run).

`bench.py --rccl` forms the nccl (RCCL) process group at WORLD_SIZE=1,
launched the way the driver launches N ranks (torch.distributed.run on
127.0.0.1), and runs the barrier / max-over-ranks timing and the SURVEY.md
8e scatter -> seal -> gather leg through it.  With one rank the scatter and
gather are RCCL's self send/recv: this checks the group's set-up, the
collectives' calls and the leg's verification on hardware, not xGMI
bandwidth (the 2/4/8-GPU runs are the driver's)."""
import json
import os
import signal
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _run(config, extra=(), rehearse_ranks=0):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    common = ["--config", config, "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--no-cpu-baseline",
              "--xfer-reps", "2", *extra]
    if rehearse_ranks:  # bench.py starts its own ranks, all on this GPU, gloo
        e["NOISE_BENCH_REHEARSE"] = "1"
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(rehearse_ranks), "--no-n1"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               os.path.join(ROOT, "bench.py"), "--gpus", "1", "--rccl"]
    cmd += common
    # its own process group, so that a hung run's ranks are all ended here
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e, cwd=ROOT,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=150)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        pytest.fail(f"bench.py {config} did not finish in 150 s; stderr tail:\n{err[-3000:]}")
    assert p.returncode == 0, err[-3000:]
    # stdout holds the one line only: RCCL's banner goes to stderr
    lines = out.strip().splitlines()
    assert len(lines) == 1 and lines[0].startswith('{"metric"'), out[-2000:]
    return json.loads(lines[0])


def _check(d):
    assert d["n_gpus"] == 1
    assert d["process_group"] == {"backend": "nccl", "world_size": 1}
    assert d["verified"] is True
    sg = d["scatter_gather"]
    assert "error" not in sg, sg
    assert "nccl" in sg["collective"]
    assert d["scatter_gather_ok"] is True
    assert [r["digest"] for r in d["verify"]["ranks"]] == ["match"]


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c2", "c5s"])
def test_two_rank_rehearsal_verifies_every_shard(config):
    """NOISE_BENCH_REHEARSE=1 --gpus 2: two ranks on this GPU over gloo, each
    sealing its own shard; the line's `verified` is both ranks' verdict, and
    each rank's set-0 output matches its golden shard digest
    (tests/golden/shard_digests.json, N = 2).  c5s: C5's mixed ragged layout
    (ChaChaPoly and AES-GCM states, 64 B-16 KiB records) at 16 Ki records per
    rank — full C5 took 67 s here (two ranks' ~1 GB slots through host
    memory); the reduced shards keep its ragged cross-rank verdict on
    hardware in a few seconds."""
    d = _run(config, rehearse_ranks=2)
    assert d["n_gpus"] == 2 and "rehearsal" in d
    assert d["verified"] is True
    assert [r["digest"] for r in d["verify"]["ranks"]] == ["match", "match"]
    assert d["scatter_gather_ok"] is True


@pytest.mark.gpu
def test_rccl_group_uniform_c2():
    _check(_run("c2"))


@pytest.mark.gpu
def test_rccl_group_mixed_c5():
    _check(_run("c5"))
