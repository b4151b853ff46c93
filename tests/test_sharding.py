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


def _xfer_v_worker(rank, world, port, sizes, q):
    """Variable-size scatter/gather (C5's ragged shards) on gloo: shards
    packed back to back, no padding; every rank transforms its shard (byte
    + rank + 1) and rank 0 gathers them back."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "noise-c_amd"))
    from distribute import gather_records_v, scatter_records_v
    total = sum(sizes)
    full_in = full_out = None
    if rank == 0:
        full_in = torch.arange(total, dtype=torch.int64).remainder(251).to(torch.uint8)
        full_out = torch.zeros(total, dtype=torch.uint8)
    local = torch.full((max(sizes) + 5,), 0xEE, dtype=torch.uint8)  # larger than the shard
    scatter_records_v(local, full_in, sizes, src=0)
    off = sum(sizes[:rank])
    exp = torch.arange(off, off + sizes[rank], dtype=torch.int64).remainder(251).to(torch.uint8)
    assert torch.equal(local[:sizes[rank]], exp)
    assert int(local[sizes[rank]:].min()) == 0xEE  # nothing past the shard written
    local[:sizes[rank]] += rank + 1
    gather_records_v(local, full_out, sizes, dst=0)
    if rank == 0:
        q.put(bytes(full_out.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [[1000, 1737], [0, 64, 5, 300]])
def test_variable_size_scatter_gather(sizes):
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000 + 7 * world
    procs = [ctx.Process(target=_xfer_v_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = bytearray()
    for r, n in enumerate(sizes):
        off = sum(sizes[:r])
        expect += bytes(((i % 251) + r + 1) % 256 for i in range(off, off + n))
    assert got == bytes(expect)


def test_c4_strong_shards_equal_one_gpu_layout():
    """C4 is strong scaling (bench.py: records and states divided by N): the
    ranks' (state key id, nonce) sets of N = 2 and 4 are exactly the N = 1
    layout's, each state's whole nonce run on one rank."""
    sys.path.insert(0, ROOT)
    import bench
    N, S = 1024, 64  # 1 Mi / 4096 scaled down, 16 records per state
    one = bench.shard(N, S, 0, 1)
    ref = {(one["key_ids"][i // one["rps"]], one["nonce_base"][i // one["rps"]] + i % one["rps"])
           for i in range(N)}
    for world in (2, 4):
        got, owner = set(), {}
        for r in range(world):
            sh = bench.shard(N // world, S // world, r, world)
            assert sh["rps"] == one["rps"]
            for i in range(sh["count"]):
                kid = sh["key_ids"][i // sh["rps"]]
                assert owner.setdefault(kid, r) == r, "a state's records split over ranks"
                got.add((kid, sh["nonce_base"][i // sh["rps"]] + i % sh["rps"]))
        assert got == ref


def _c5_records(rank, world, R, S, sample):
    """(global record, len, global state, nonce, cipher, tag hash) of a sample
    of rank's C5 records, sealed by the oracle as the GPU rank would."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    from oracle import Oracle
    o = Oracle()
    lay = bench.mixed_layout(R, S, rank)
    out = []
    for j in sample:
        L, st, n = int(lay["lens"][j]), int(lay["st_global"][j]), int(lay["nonce"][j])
        cipher = 0x4301 if st % 2 == 0 else 0x4302
        key = o.fill(bench.SEED_KEY, 32, 4 * st)
        # plaintext at the rank's own byte offset of its own SplitMix64 stream
        pt = o.fill(bench.SEED_PT, lay["off"][j] + L + 8, rank << 40)[lay["off"][j]:lay["off"][j] + L]
        tag = o.encrypt(cipher, key, n, pt)[-16:]
        out.append((rank * R + j, L, st, n, cipher,
                    int.from_bytes(hashlib.sha256(tag).digest()[:7], "little")))
    return out


def _c5_worker(rank, world, port, R, S, sample, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = torch.tensor(_c5_records(rank, world, R, S, sample), dtype=torch.int64)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank == 0:
        q.put(torch.cat(parts).tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_c5_ragged_shards():
    """C5 (mixed ChaChaPoly/AESGCM, 64 B-16 KiB records): rank r's shard is
    records [rR, (r+1)R) and states [rS, (r+1)S) of the global job; record
    lengths, state, cipher and nonce of every record equal those of the
    one-process layout of the whole job (mixed_layout over 2R records, 2S
    states), and the sampled records' oracle tags agree, gathered over gloo."""
    sys.path.insert(0, ROOT)
    import bench
    world, R, S = 2, 64, 8
    whole = bench.mixed_layout(world * R, world * S, 0)
    for r in range(world):
        lay = bench.mixed_layout(R, S, r)
        sl = slice(r * R, (r + 1) * R)
        assert (lay["lens"] == whole["lens"][sl]).all()
        assert (lay["st_global"] == whole["st_global"][sl]).all()
        assert (lay["nonce"] == whole["nonce"][sl]).all()
    sample = [0, 1, R // S - 1, R // S, R - 1]  # state edges
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + os.getpid() % 1000
    procs = [ctx.Process(target=_c5_worker, args=(r, world, port, R, S, sample, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = []
    for r in range(world):
        expect += [list(t) for t in _c5_records(r, world, R, S, sample)]
    assert got == expect
    # every (state, nonce) pair is used once over the whole job
    pairs = {(int(whole["st_global"][i]), int(whole["nonce"][i])) for i in range(world * R)}
    assert len(pairs) == world * R
