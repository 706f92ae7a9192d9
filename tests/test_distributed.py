"""Multi-process data-parallel path on CPU (gloo, world_size 2).

The stage-b step shards rays by rank (each rank renders its own image's rays) and averages
the flat gradient with ONE all-reduce (`trainer.reduce_gradients`).  These tests pin that
average against torch DistributedDataParallel (what the reference wraps the model in,
imaginaire/trainers/utils/get_trainer.py:81), so the N-GPU run over RCCL (same code path,
backend "nccl") updates every replica with the DDP gradient.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mli_nerf_amd import layout, shard
from mli_nerf_amd.trainer import reduce_gradients

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        # 1. flat-buffer average over ranks
        n = layout.trainable_layout()[1]
        g = torch.Generator().manual_seed(100 + rank)
        grad = torch.randn(n, generator=g)
        mine = grad.clone()
        reduce_gradients(grad, WORLD)
        # 2. the same average as DDP on a module whose grads are rank-specific
        torch.manual_seed(0)
        lin = torch.nn.Linear(16, 4)
        ddp = torch.nn.parallel.DistributedDataParallel(lin)
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(rank))
        ddp(x).square().sum().backward()
        ddp_grad = torch.cat([p.grad.reshape(-1) for p in lin.parameters()])
        lin2 = torch.nn.Linear(16, 4)
        lin2.load_state_dict(lin.state_dict())
        lin2(x).square().sum().backward()
        local = torch.cat([p.grad.reshape(-1) for p in lin2.parameters()])
        reduce_gradients(local, WORLD)
        results[rank] = (mine, grad, ddp_grad, local)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gradient_average_matches_ddp_world2():
    port = _free_port()
    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    results = manager.dict()
    mp.start_processes(_worker, args=(port, results), nprocs=WORLD, join=True, start_method="spawn")
    mine = [results[r][0] for r in range(WORLD)]
    avg = sum(mine) / WORLD
    for r in range(WORLD):
        torch.testing.assert_close(results[r][1], avg, rtol=0, atol=1e-6)
        # identical on every rank (replicas stay in sync after the optimizer step)
        assert torch.equal(results[r][1], results[0][1])
        torch.testing.assert_close(results[r][3], results[r][2], rtol=1e-6, atol=1e-6)


def test_single_rank_is_identity():
    g = torch.randn(10)
    h = g.clone()
    assert reduce_gradients(h, 1) is h and torch.equal(h, g)


def _tile_worker(rank, port, results, n):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        lo, hi, _ = shard.shard_range(n, rank, WORLD)
        # each ray's 15 channels = a function of its pixel index (stands in for the render)
        pix = torch.arange(lo, hi, dtype=torch.float32)[:, None]
        local = pix * 100 + torch.arange(shard.N_CHANNELS, dtype=torch.float32)[None]
        results[rank] = shard.gather_tiles(local, n, WORLD)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [640, 641])
def test_inference_tiles_gather_world2(n):
    """config 5 sharding: contiguous tiles per rank, ONE all_gather rebuilds the frame
    (uneven n: the last tile is padded and the padding dropped)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_tile_worker, args=(port, results, n), nprocs=WORLD, join=True, start_method="spawn")
    full = torch.arange(n, dtype=torch.float32)[:, None] * 100 + torch.arange(shard.N_CHANNELS)[None]
    for r in range(WORLD):
        assert torch.equal(results[r], full)


def test_shard_ranges_cover_frame():
    for n, world in [(640000, 8), (97, 8), (5, 8), (10, 1)]:
        spans = [shard.shard_range(n, r, world)[:2] for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        packed = torch.randn(7, shard.N_CHANNELS)
        back = shard.pack(shard.unpack(packed))
        assert torch.equal(back, packed)
