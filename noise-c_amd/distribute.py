"""Multi-GPU data movement for a sharded record batch.

Records are independent given (key, nonce), so the AEAD itself needs no
collective: each rank seals/opens the contiguous record range of its shard
(bench.shard).  The only exchange is at the edges of the path, when the batch
starts on one device (the rank holding the socket buffers) and must come back
to it:

- ``scatter_records``: the source rank splits its ``world`` equal shard slices
  of a flat byte buffer over the ranks (its own slice stays local);
- ``gather_records``: the reverse, every rank's output slice lands at its
  offset of the destination rank's flat buffer.

- ``scatter_records_v`` / ``gather_records_v``: the same for shards of
  different sizes (C5's ragged shards), packed back to back in the flat
  buffer — one point-to-point send/receive per peer in one batch, so no
  shard travels padded to the largest one's size.

The equal-size pair are single ``torch.distributed`` scatter/gather calls, which the nccl
backend (RCCL on ROCm) runs as grouped ncclSend/ncclRecv over xGMI — one
point-to-point transfer per peer, all peers in flight at once, matching the
"scatter inputs / gather outputs" shape the north star names.  On CPU tensors
with the gloo backend the same calls back the world_size-2 tests.
"""
from __future__ import annotations

from typing import Optional


def _slices(full, world: int, shard_bytes: int):
    if full.numel() < world * shard_bytes:
        raise ValueError(f"flat buffer of {full.numel()} B < {world} x {shard_bytes} B shards")
    return [full[r * shard_bytes:(r + 1) * shard_bytes] for r in range(world)]


def scatter_records(local, full: Optional[object], src: int = 0, group=None) -> None:
    """Fill ``local`` (this rank's shard, a flat uint8 tensor of S bytes) with
    slice ``rank`` of ``full`` (world x S bytes, only read on ``src``)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if local.dim() != 1 or not local.is_contiguous():
        raise ValueError("local shard must be a flat contiguous tensor")
    parts = None
    if rank == src:
        if full is None:
            raise ValueError("the source rank must pass the full buffer")
        parts = _slices(full, world, local.numel())
    dist.scatter(local, scatter_list=parts, src=src, group=group)


def gather_records(local, full: Optional[object], dst: int = 0, group=None) -> None:
    """Write every rank's ``local`` shard into slice ``rank`` of ``full`` on
    ``dst`` (``full`` is ignored elsewhere)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if local.dim() != 1 or not local.is_contiguous():
        raise ValueError("local shard must be a flat contiguous tensor")
    parts = None
    if rank == dst:
        if full is None:
            raise ValueError("the destination rank must pass the full buffer")
        parts = _slices(full, world, local.numel())
    dist.gather(local, gather_list=parts, dst=dst, group=group)


def _offsets(sizes):
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += int(n)
    return offs, o


def _p2p(ops) -> None:
    import torch.distributed as dist
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def scatter_records_v(local, full: Optional[object], sizes, src: int = 0, group=None) -> None:
    """Variable-size scatter: rank r receives ``sizes[r]`` bytes into
    ``local[:sizes[r]]`` from offset sum(sizes[:r]) of ``full`` (the shards
    packed back to back, read on ``src`` only).  Every rank calls it (one
    batched send per peer on ``src``, one receive elsewhere)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(sizes) != world:
        raise ValueError(f"{len(sizes)} shard sizes for {world} ranks")
    if local.dim() != 1 or not local.is_contiguous() or local.numel() < int(sizes[rank]):
        raise ValueError("local shard must be a flat contiguous tensor of at least its size")
    offs, total = _offsets(sizes)
    ops = []
    if rank == src:
        if full is None or full.numel() < total:
            raise ValueError("the source rank must pass the packed buffer of every shard")
        for r in range(world):
            if r != src and sizes[r]:
                ops.append(dist.P2POp(dist.isend, full[offs[r]:offs[r] + int(sizes[r])], r, group))
        local[:int(sizes[src])].copy_(full[offs[src]:offs[src] + int(sizes[src])])
    elif sizes[rank]:
        ops.append(dist.P2POp(dist.irecv, local[:int(sizes[rank])], src, group))
    _p2p(ops)


def gather_records_v(local, full: Optional[object], sizes, dst: int = 0, group=None) -> None:
    """Variable-size gather: ``local[:sizes[r]]`` of every rank r lands at
    offset sum(sizes[:r]) of ``full`` on ``dst`` (packed, no padding)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(sizes) != world:
        raise ValueError(f"{len(sizes)} shard sizes for {world} ranks")
    if local.dim() != 1 or not local.is_contiguous() or local.numel() < int(sizes[rank]):
        raise ValueError("local shard must be a flat contiguous tensor of at least its size")
    offs, total = _offsets(sizes)
    ops = []
    if rank == dst:
        if full is None or full.numel() < total:
            raise ValueError("the destination rank must pass the packed buffer of every shard")
        for r in range(world):
            if r != dst and sizes[r]:
                ops.append(dist.P2POp(dist.irecv, full[offs[r]:offs[r] + int(sizes[r])], r, group))
        full[offs[dst]:offs[dst] + int(sizes[dst])].copy_(local[:int(sizes[dst])])
    elif sizes[rank]:
        ops.append(dist.P2POp(dist.isend, local[:int(sizes[rank])], dst, group))
    _p2p(ops)
