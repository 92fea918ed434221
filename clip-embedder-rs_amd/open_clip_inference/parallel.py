"""Data-parallel sharding across ranks (one process per GPU) — SURVEY.md §8e.

The batch is split into contiguous row blocks in rank order; each rank embeds its
block on its own GPU; one all-gather of the [B/G, E] f32 embedding rows assembles [B, E]
in input order on every rank.  On GPUs the collective is the engine's own RCCL
communicator inside the C ABI (``init_engine_comm`` + ``Engine.embed_*_gather_device``:
ncclAllGather over xGMI); ``torch.distributed`` (gloo) is only the control plane that
carries the 128-byte RCCL unique id, barriers and timings.  ``all_gather_rows`` is the
same gather through torch.distributed (CPU tests, gloo).  Ragged batches (B % G != 0) are
padded to the largest shard for that collective and trimmed afterwards.  torch is
imported lazily (plumbing only).
"""
from __future__ import annotations

from typing import Callable


def shard_range(B: int, rank: int, world: int):
    """Contiguous [b0, b1) of rank `rank` (same split as the engine's multi-device path)."""
    return (B * rank) // world, (B * (rank + 1)) // world


def shard_rows(B: int, world: int):
    """Block sizes of every rank (the `rows` argument of the gathered entry points)."""
    return [shard_range(B, r, world)[1] - shard_range(B, r, world)[0] for r in range(world)]


def init_engine_comm(engine, group=None):
    """Join this rank's one-device engine to an RCCL communicator over all ranks of `group`:
    rank 0 draws the unique id (clipgpu_comm_unique_id), the control plane broadcasts it, every
    rank calls clipgpu_comm_init_rank (collective)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    box = [engine.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    engine.comm_init_rank(box[0], world, rank)
    return world, rank


def all_gather_rows(local, B: int, group=None):
    """Gather each rank's [b1-b0, E] rows into [B, E] in rank (= input) order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    E = local.shape[1]
    sizes = [shard_range(B, r, world)[1] - shard_range(B, r, world)[0] for r in range(world)]
    cap = max(sizes)
    buf = torch.zeros((cap, E), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    out = torch.empty((world * cap, E), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = [out[r * cap: r * cap + sizes[r]] for r in range(world)]
    return torch.cat(parts, 0)


def embed_data_parallel(embed_fn: Callable, batch, group=None):
    """Run `embed_fn` on this rank's shard of `batch` (indexable, len B) and all-gather.

    embed_fn(shard) -> torch tensor [n, E] on this rank's device.
    """
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    B = len(batch)
    b0, b1 = shard_range(B, rank, world)
    local = embed_fn(batch[b0:b1])
    return all_gather_rows(local, B, group)
