"""GPU parity of the stage-a training step (syn_hotdog_a: LumenRGB mode 'rgb', coarse-to-fine
hash grid, every parameter trained) against the CPU oracle's autograd.

The GPU step runs through the C ABI (Trainer.compute_grads_a: rays, sampler, FIELD, the
single head, composite, fused losses, then mli_composite_bwd_geo -> mli_geo_bwd ->
mli_sdf_bwd -> mli_hash_bwd -> split-K dW -> weight-norm backward).  The oracle
(oracle/render.py, pinned to the reference by tests/golden/hotdog_a_*) is given the
fp16-rounded hash table the GPU gathers and the GPU's hierarchical samples (the sampler is
chaotic; it is parity-tested round by round in test_gpu_parity.py).

Tolerances (fp16 MFMA operands, fp32 accumulation, fp16 gradient images with a power-of-two
loss scale; the reference computes in fp32 / TF32):
* loss terms: 1e-3 relative;
* every parameter gradient: cosine similarity >= 0.995 and relative L2 error <= 10 %
  per tensor (s_var: relative error <= 2 %);
* hash-table gradient: cosine >= 0.995 over the whole table, identical support on the
  levels the coarse-to-fine mask leaves active, exactly zero on the masked levels.
"""
import pytest
import torch

from mli_nerf_amd import synthetic
from margins import check
from mli_nerf_amd.configs import preset
from oracle import render as o_render

pytestmark = pytest.mark.gpu

DEV = "cuda:0"

# (R, Nc, Nf, iteration): iteration 20000 -> 8 active levels, tap eps of level 2;
# 80000 -> 15 active levels, tap eps of level 14
CASES = [(64, 16, 4, 20000), (32, 64, 16, 80000)]


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _setup(R, Nc, Nf, it, log2T=14, s_var=3.0):
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    cfg = preset("syn_hotdog_a", rays=R, n_coarse=Nc, n_fine=Nf, log2T=log2T)
    model = Model(cfg.model, cfg.data)
    sd = synthetic.make_state_dict(log2T=log2T, s_var=s_var, heads="rgb")
    model.load_state_dict(sd)
    model = model.to(DEV)
    trainer = Trainer(cfg, is_inference=False, model=model)
    trainer.current_iteration = it
    trainer._start_of_iteration()
    data = synthetic.make_batch(R, frame=3)
    u = synthetic.stratified_uniforms(R, Nc, seed=5)
    return cfg, model, trainer, sd, data, u


def _oracle(sd, model, trainer, data, u, dists, R, Nc, Nf, log2T=14):
    sdf = model.neural_sdf
    pcfg = o_render.PathCfg(n_coarse=Nc, n_fine=Nf, log2T=log2T, rgb_mode="rgb",
                            active_levels=int(sdf.active_levels), anneal_levels=int(sdf.anneal_levels))
    sd16 = dict(sd)
    sd16["neural_sdf.tcnn_encoding.params"] = sd["neural_sdf.tcnn_encoding.params"].half().float()
    sd16 = {k: v.clone().requires_grad_(True) for k, v in sd16.items()}
    out = o_render.forward(sd16, pcfg, data, u=u, training=True, progress=model.progress, dists=dists)
    total, losses, psnr = o_render.stage_a_losses(out, data, trainer.weights["curvature"])
    total.backward()
    return out, total, losses, {k: v.grad for k, v in sd16.items()}


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-300))


@pytest.mark.parametrize("R,Nc,Nf,it", CASES)
def test_stage_a_gradients_match_oracle(R, Nc, Nf, it):
    _need_gpu()
    cfg, model, trainer, sd, data, u = _setup(R, Nc, Nf, it)
    st, lv = trainer.compute_grads_a({k: v.to(DEV) for k, v in data.items()}, u=u.to(DEV))
    torch.cuda.synchronize()
    dists = model.outputs(st)["dists"].detach().cpu()
    out, total, losses, og = _oracle(sd, model, trainer, data, u, dists, R, Nc, Nf)
    lv = lv.cpu()
    for i, k in enumerate(("render", "eikonal", "curvature")):
        i = {"render": 0, "eikonal": 1, "curvature": 2}[k]
        ref = losses[k].item()
        check("loss %s rel" % k, abs(lv[i].item() - ref) / (abs(ref) + 1e-4), 1e-3, "<=")
    g_flat = trainer._grad.cpu()
    report = {}
    for name, shape, off in model._layout_items():
        g = g_flat[off:off + max(1, int(torch.tensor(shape).prod()))].reshape(og[name].shape)
        ref = og[name]
        if name == "s_var":
            rel = abs(g.item() - ref.item()) / max(abs(ref.item()), 1e-12)
            report[name] = rel
            check("grad rel s_var", rel, 2e-2, "<=")
            continue
        cos = _cos(g, ref)
        rel = float((g - ref).norm() / ref.norm().clamp_min(1e-30))
        report[name] = (round(cos, 5), round(rel, 4))
        check("grad cos " + name, cos, 0.995, ">=")
        check("grad rel " + name, rel, 0.10, "<=")
    gt = trainer._grad_table.cpu()
    rt = og["neural_sdf.tcnn_encoding.params"]
    cos = _cos(gt, rt)
    report["table"] = cos
    check("table grad cos", cos, 0.995, ">=")
    # masked levels carry exactly no gradient; active levels: same support
    from mli_nerf_amd.hashgrid import level_table
    table, _ = level_table(log2T=14)
    act = int(model.neural_sdf.active_levels)
    for lvl, (scale, res, size, offset) in enumerate(table):
        seg = slice(offset * 8, (offset + size) * 8)
        if lvl >= act:
            assert gt[seg].abs().max().item() == 0.0, lvl
        else:
            nz_g, nz_r = gt[seg] != 0, rt[seg] != 0
            assert (nz_g ^ nz_r).float().mean().item() < 1e-3, lvl
    print(report)


def test_stage_a_training_reduces_loss():
    """A few fused stage-a steps (AdamW on the MLPs and the table, fp16 shadow refresh)
    move the loss down on a fixed batch, and the table shadow stays equal to the table."""
    _need_gpu()
    cfg, model, trainer, sd, data, u = _setup(64, 16, 4, 6000)
    batch = {k: v.to(DEV) for k, v in data.items()}
    losses = []
    for _ in range(30):
        trainer.train_step(batch, u=u.to(DEV))
        losses.append(trainer.losses["total"].item())
    torch.cuda.synchronize()
    assert all(l == l for l in losses)
    assert sum(losses[-5:]) / 5 < sum(losses[:5]) / 5, losses
    table = model.neural_sdf.tcnn_encoding.params.detach()
    assert torch.equal(model.engine.table16, table.half())


def test_stage_a_autograd_path_matches_fused():
    """Model.forward under torch autograd (the reference trainer's way: losses on the output
    dict incl. gradients / hessians, total.backward()) gives the fused path's gradients."""
    _need_gpu()
    from mli_nerf_amd.trainer import stage_b_losses
    cfg, model, trainer, sd, data, u = _setup(64, 16, 4, 20000)
    batch = {k: v.to(DEV) for k, v in data.items()}
    trainer.compute_grads_a(batch, u=u.to(DEV))
    g_fused, t_fused = trainer._grad[:model.flat.numel()].clone(), trainer._grad_table.clone()
    model.train()
    table = model.neural_sdf.tcnn_encoding.params
    for p in model.parameters():
        p.grad = None
    out = model(batch, u=u.to(DEV))
    total, losses, _ = stage_b_losses(out, batch, trainer.weights)
    total.backward()
    torch.cuda.synchronize()
    for name, shape, off in model._layout_items():
        n = max(1, int(torch.tensor(shape).prod()))
        a, b = model.flat_grad_from_params()[off:off + n].cpu(), g_fused[off:off + n].cpu()
        assert _cos(a, b) > 0.99999 and float((a - b).norm() / b.norm().clamp_min(1e-30)) < 1e-3, name
    assert _cos(table.grad.cpu(), t_fused.cpu()) > 0.99999


def _two_steps_a(world=1, chunk=None, overlap=True, frame=3, zero=False):
    from mli_nerf_amd.trainer import FusedAdamW, ZeroTableAdamW
    cfg, model, trainer, sd, data, u = _setup(32, 16, 4, 100000)
    trainer.world_size = world
    trainer.table_overlap = overlap
    if chunk:
        trainer.table_chunk = chunk
    trainer.model.deterministic = True   # bit-reproducible gradients (fixed-order sums)
    t = model.neural_sdf.tcnn_encoding.params
    o = cfg.optim.params
    if zero:   # the sharded table optimizer (ZeroTableAdamW), else the replicated one
        import torch.distributed as dist
        trainer.optim_table = ZeroTableAdamW(t, world, dist.get_rank(), lr=o.lr, weight_decay=o.weight_decay)
    else:
        trainer.optim_table = FusedAdamW(t, lr=o.lr, weight_decay=o.weight_decay)
    for s in range(2):
        b = synthetic.make_batch(32, frame=frame + 10 * s)
        trainer.train_step({k: v.to(DEV) for k, v in b.items()}, u=u.to(DEV))
    trainer.sync_table()
    torch.cuda.synchronize()
    mv = trainer._table_full_moments if zero else (trainer.optim_table.m, trainer.optim_table.v)
    return dict(table=t.detach().cpu().clone(), table16=model.engine.table16.cpu().clone(),
                m=mv[0].cpu().clone(), v=mv[1].cpu().clone(),
                flat=model.flat.detach().cpu().clone(), gtab=trainer._grad_table.cpu().clone())


def test_table_step_chunked_equals_single_launch():
    """The table AdamW issued chunk by chunk (the overlapped reduction's form, here at world 1
    through FusedAdamW.step(ranges=...)) equals the single launch bit for bit."""
    _need_gpu()
    from mli_nerf_amd.trainer import FusedAdamW, table_chunks
    g = torch.Generator().manual_seed(3)
    n = 3 * (1 << 20) + 123
    p0 = torch.randn(n, generator=g).to(DEV)
    grads = [torch.randn(n, generator=g).to(DEV) for _ in range(3)]
    outs = []
    for chunked in (False, True):
        p = p0.clone()
        opt = FusedAdamW(p)
        p16 = torch.empty(n, dtype=torch.float16, device=DEV)
        for gr in grads:
            opt.step(gr, 1e-3, p16=p16, ranges=table_chunks(n, 1 << 18) if chunked else None)
        torch.cuda.synchronize()
        outs.append((p.cpu(), p16.cpu(), opt.m.cpu(), opt.v.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _world2_worker(rank, port, results):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        results[(rank, "overlap")] = _two_steps_a(2, chunk=1 << 16, overlap=True, frame=3 + rank)
        results[(rank, "serial")] = _two_steps_a(2, overlap=False, frame=3 + rank)
        results[(rank, "zero")] = _two_steps_a(2, frame=3 + rank, zero=True)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_stage_a_world2_on_one_gpu_overlap_equals_serial():
    """Two ranks (gloo, both on cuda:0, different rays) run two stage-a steps with the real HIP
    engine: the overlapped chunked table reduction (chunk i's AdamW behind chunk i's all-reduce)
    and the ZeRO-sharded table (reduce-scatter, AdamW on the rank's shard, all-gather of the fp16
    shadow; the fp32 master and moments gathered by sync_table) give the same table, fp16 shadow,
    moments and MLP buffer as the serial single all-reduce, bit for bit, and the replicas agree."""
    _need_gpu()
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_world2_worker, args=(port, results), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        for k in ("table", "table16", "m", "v", "flat", "gtab"):
            assert torch.equal(results[(r, "overlap")][k], results[(r, "serial")][k]), (r, k)
            assert torch.equal(results[(r, "overlap")][k], results[(0, "overlap")][k]), (r, k)
            if k != "gtab":   # (the sharded path's gradient buffer holds this rank's own sum)
                assert torch.equal(results[(r, "zero")][k], results[(r, "serial")][k]), (r, k)
    assert not torch.equal(results[(0, "overlap")]["table"], _two_steps_a(1)["table"])   # the ranks averaged


def test_consumed_gradients_left_zero():
    """ABI 17: the fused stage-a step issues no fill for its accumulators.  The table AdamW leaves
    the table gradient it consumed all zero (mli_adamw zero_grad stores 0 only where the entry was
    not), and the weight-norm assemble leaves the split-K dW buffer zero (zero_dw): after a step
    both are exactly zero, so the next step's scatter / atomics add into clean buffers.  The next
    step's table gradient then equals one accumulated into a freshly zeroed buffer (support
    identical; values to fp32 atomic-order noise)."""
    _need_gpu()
    cfg, model, trainer, sd, data, u = _setup(64, 16, 4, 100000)
    batch = {k: v.to(DEV) for k, v in data.items()}
    trainer.train_step(batch, u=u.to(DEV))
    torch.cuda.synchronize()
    eng = model.engine
    assert eng.table_grad_clean == trainer._grad_table.data_ptr()
    assert not bool(trainer._grad_table.any())
    assert not bool(eng._bufs["dw_a"].any())
    b2 = {k: v.to(DEV) for k, v in synthetic.make_batch(64, frame=11).items()}
    trainer.compute_grads_a(b2, u=u.to(DEV))            # into the buffer the AdamW cleaned
    g_clean = trainer._grad_table.clone()
    eng.table_grad_clean = None                         # force the dense fill
    trainer.compute_grads_a(b2, u=u.to(DEV))
    torch.cuda.synchronize()
    g_fill = trainer._grad_table
    assert torch.equal(g_clean != 0, g_fill != 0)
    assert _cos(g_clean.cpu(), g_fill.cpu()) > 0.9999999
    check("consumed table grad rel", float((g_clean - g_fill).norm() / g_fill.norm()), 1e-6, "<=")


def test_stage_b_dw_left_zero():
    """Stage b: every dW / db element the weight-norm assemble reads is left zero by it (no fill
    in the next step).  (The packed layer-0 columns a head has no input for -- mlp_r's SH rows --
    are never read; WIDE writes them through its slab sum, so their content is never used.)"""
    _need_gpu()
    import numpy as np
    from mli_nerf_amd import layout
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    cfg = preset("syn_hotdog_b", rays=512, n_coarse=32, n_fine=8, log2T=14)
    m = Model(cfg.model, cfg.data)
    m.load_state_dict(synthetic.make_state_dict(log2T=14))
    tr = Trainer(cfg, is_inference=False, model=m.to(DEV))
    tr.current_iteration = 10000
    for f in range(2):
        tr.train_step({k: v.to(DEV) for k, v in synthetic.make_batch(512, frame=f).items()})
        torch.cuda.synchronize()
        eng = m.engine
        dw = eng._bufs["dw"].cpu()
        assert eng._dw_zero == eng._bufs["dw"].data_ptr()
        off = 0
        for hdx, (name, k_in, k_out) in enumerate(layout.HEADS):
            for li in range(5):
                mm, kk = eng._dw_sizes()[hdx * 5 + li]
                w, b = dw[off:off + mm * kk].view(mm, kk), dw[off + mm * kk:off + mm * kk + mm]
                off += mm * kk + mm
                cols = torch.from_numpy(layout.head_kinv(name, k_in).astype(np.int64)) if li == 0 else slice(None)
                assert not bool(w[:, cols].any()) and not bool(b.any()), (name, li)
        assert torch.isfinite(m.flat.grad).all() and float(m.flat.grad.abs().sum()) > 0
