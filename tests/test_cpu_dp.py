"""Multi-rank data-parallel path on CPU (gloo, world_size 2 and 3): contiguous row
shards in rank order + one all-gather reproduce the single-process result row for
row, including ragged batches.  The per-rank embedding function is the tiny oracle
tower (the GPU path runs the same helper with the nccl/RCCL backend in bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from open_clip_inference.parallel import embed_data_parallel, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import clip_ref, weights
    from oracle.model_spec import TINY_CFG, vision_spec_from_cfg
    v = vision_spec_from_cfg(TINY_CFG["model_cfg"])
    P = weights.vision_weights(v, 1234)
    rng = np.random.default_rng(0)
    px = rng.standard_normal((B, 3, v.image_size, v.image_size)).astype(np.float32)

    def embed(shard):
        if len(shard) == 0:
            return torch.zeros((0, v.embed_dim))
        return torch.from_numpy(clip_ref.encode_image(P, v, shard, dtype=np.float64)).float()

    out = embed_data_parallel(embed, px)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 5), (2, 4), (3, 7), (2, 1)])
def test_dp_gather_matches_single_process(world, B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from oracle import clip_ref, weights
    from oracle.model_spec import TINY_CFG, vision_spec_from_cfg
    v = vision_spec_from_cfg(TINY_CFG["model_cfg"])
    rng = np.random.default_rng(0)
    px = rng.standard_normal((B, 3, v.image_size, v.image_size)).astype(np.float32)
    ref = clip_ref.encode_image(weights.vision_weights(v, 1234), v, px).astype(np.float32)
    assert got.shape == ref.shape
    assert np.allclose(got, ref, atol=1e-6)


def test_shard_ranges_cover_batch_in_order():
    for B in range(0, 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(B, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == B
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


class _FakeEngine:
    """Records what the RCCL bootstrap hands the C ABI (no GPU here)."""

    def __init__(self, rank):
        self.rank = rank
        self.got = None

    def comm_unique_id(self):
        assert self.rank == 0, "only rank 0 draws the unique id"
        return bytes(range(128))

    def comm_init_rank(self, uid, nranks, rank):
        self.got = (uid, nranks, rank)


def _comm_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from open_clip_inference.parallel import init_engine_comm, shard_rows
    e = _FakeEngine(rank)
    assert init_engine_comm(e) == (world, rank)
    q.put((rank, e.got, shard_rows(10, world)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_engine_comm_bootstrap_over_the_control_plane(world):
    """bench.py's N > 1 path: rank 0's 128-byte RCCL unique id reaches every rank over the gloo
    control plane, and each rank joins with its own rank number (clipgpu_comm_init_rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r, (rank, (uid, nranks, rk), rows) in enumerate(got):
        assert rank == r and rk == r and nranks == world and uid == bytes(range(128))
        assert sum(rows) == 10 and len(rows) == world
