"""Stage b over two ranks with the real HIP engine (gloo, both ranks on cuda:0): the per-dW-class
all-reduce overlapped with the backward (trainer.OverlappedGradReduce, DDP's buckets,
imaginaire/trainers/utils/get_trainer.py:81-88) against the single collective after the backward
(grad_overlap False).  A two-rank sum is exact in any order, so with the deterministic
(fixed-order) weight gradients both forms give the same flat parameters, moments and metrics bit
for bit, on both ranks; and the ranks did average (the result differs from one rank's own)."""
import pytest
import torch

from mli_nerf_amd import synthetic
from mli_nerf_amd.configs import preset

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _two_steps_b(world, overlap, frame):
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    cfg = preset("syn_hotdog_b", rays=256, n_coarse=32, n_fine=8, log2T=14)
    cfg.trainer["deterministic"] = True   # fixed-order weight-gradient sums: bit-reproducible
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=14))
    model = model.to(DEV)
    tr = Trainer(cfg, is_inference=False, model=model, world_size=world)
    tr.grad_overlap = overlap
    tr.current_iteration = 10000
    for s in range(2):
        b = synthetic.make_batch(256, frame=frame + 10 * s)
        u = synthetic.stratified_uniforms(256, 32, seed=frame + 10 * s)   # the same draws in both forms
        tr.train_step({k: v.to(DEV) for k, v in b.items()}, u=u.to(DEV))
    torch.cuda.synchronize()
    return dict(flat=model.flat.detach().cpu().clone(), m=tr.optim.m.cpu().clone(), v=tr.optim.v.cpu().clone(),
                psnr=tr.metrics["psnr"].detach().cpu().clone())


def _worker(rank, port, results):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        results[(rank, "overlap")] = _two_steps_b(2, True, 3 + rank)
        results[(rank, "serial")] = _two_steps_b(2, False, 3 + rank)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_stage_b_world2_on_one_gpu_overlap_equals_serial():
    _need_gpu()
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_worker, args=(port, results), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        for k in ("flat", "m", "v", "psnr"):
            assert torch.equal(results[(r, "overlap")][k], results[(r, "serial")][k]), (r, k)
            assert torch.equal(results[(r, "overlap")][k], results[(0, "overlap")][k]), (r, k)
    assert not torch.equal(results[(0, "overlap")]["flat"], _two_steps_b(1, None, 3)["flat"])   # averaged
