"""Multi-rank record sharding (bench.py / SURVEY.md §8e), world_size 2 on gloo.

Each rank derives its shard with bench.shard() exactly as the GPU ranks do,
seals its records with the oracle and all_gathers (key id, nonce, tag)
triples.  Rank 0 checks that the union is the single-GPU global stream
record for record, and that no (key, nonce) pair is used twice across ranks
— the property that makes sharding without a collective safe."""
import hashlib
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _records(rank, world, R, S):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    from oracle import Oracle
    o = Oracle()
    sh = bench.shard(R, S, rank, world)
    out = []
    for i in range(sh["count"]):
        s = i // sh["rps"]
        kid = sh["key_ids"][s]
        n = sh["nonce_base"][s] + i % sh["rps"]
        key = o.fill(0x6B6579, 32, 4 * kid)
        g = sh["first"] + i
        pt = o.fill(0x7074, 64, g * 8)
        tag = o.encrypt(0x4301, key, n, pt)[-16:]
        out.append((kid, n, int.from_bytes(hashlib.sha256(tag).digest()[:7], "little")))
    return out


def _worker(rank, world, port, R, S, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = torch.tensor(_records(rank, world, R, S), dtype=torch.int64)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank == 0:
        q.put(torch.cat(parts).tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("S", [1, 4])
def test_two_rank_shards_equal_global_stream(S):
    world, R = 2, 32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000 + S
    procs = [ctx.Process(target=_worker, args=(r, world, port, R, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the same records computed rank by rank in one process
    expect = []
    for r in range(world):
        expect += [list(t) for t in _records(r, world, R, S)]
    assert got == expect
    pairs = {(k, n) for k, n, _ in got}
    assert len(pairs) == world * R, "a (key, nonce) pair was reused across ranks"
    if S == 1:  # one logical CipherState: nonces run 0..world*R-1 across ranks
        assert sorted(n for _, n, _ in got) == list(range(world * R))


def _xfer_worker(rank, world, port, R, L, q):
    """The bench.py scatter -> per-rank seal -> gather leg on gloo/CPU, the
    per-rank seal done by the oracle over the rank's records (nonce = global
    record index, one logical CipherState as in C2)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "noise-c_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from distribute import scatter_records, gather_records
    from oracle import Oracle
    o = Oracle()
    key = o.fill(0x6B6579, 32, 0)
    shard_in, shard_out = R * L, R * (L + 16)
    full_in = full_out = None
    if rank == 0:
        full_in = torch.frombuffer(bytearray(o.fill(0x7074, world * shard_in, 0)), dtype=torch.uint8)
        full_out = torch.zeros(world * shard_out, dtype=torch.uint8)
    local_in = torch.empty(shard_in, dtype=torch.uint8)
    scatter_records(local_in, full_in, src=0)
    raw = bytes(local_in.numpy())
    assert raw == o.fill(0x7074, world * shard_in, 0)[rank * shard_in:(rank + 1) * shard_in]
    sealed = b"".join(o.encrypt(0x4301, key, rank * R + i, raw[i * L:(i + 1) * L]) for i in range(R))
    local_out = torch.frombuffer(bytearray(sealed), dtype=torch.uint8)
    gather_records(local_out, full_out, dst=0)
    if rank == 0:
        q.put(bytes(full_out.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_scatter_seal_gather():
    world, R, L = 2, 8, 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_xfer_worker, args=(r, world, port, R, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    o = Oracle()
    key = o.fill(0x6B6579, 32, 0)
    pt = o.fill(0x7074, world * R * L, 0)
    expect = b"".join(o.encrypt(0x4301, key, i, pt[i * L:(i + 1) * L]) for i in range(world * R))
    assert got == expect
