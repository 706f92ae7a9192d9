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


# ----------------------------------------------------------------------------------------
# Trainer / Model.inference at world size 2 behind the CPU stub engine (tests/stub_engine.py):
# the product's step and sharding plumbing, with the render kernels stubbed out
# ----------------------------------------------------------------------------------------
def _stub_setup():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import stub_engine
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    cfg = preset("syn_hotdog_b", rays=32, n_coarse=16, n_fine=4, log2T=12)
    m = Model(cfg.model, cfg.data)
    m.load_state_dict(synthetic.make_state_dict(log2T=12))
    return stub_engine, cfg, m


def _step_result(tr, m):
    head = m.neural_rgb.mlp.linears[0].bias
    return dict(flat=m.flat.clone(), grad=m.flat.grad.clone(), head_grad=head.grad.clone(),
                head_grad_is_view=head.grad.untyped_storage().data_ptr() == m.flat.grad.untyped_storage().data_ptr(),
                world=tr.world_size,
                psnr=float(tr.metrics["psnr"]), total=float(tr.losses["total"]), render=float(tr.losses["render"]))


def _train_worker(rank, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from mli_nerf_amd import synthetic
        from mli_nerf_amd.trainer import Trainer
        stub, cfg, m = _stub_setup()
        stub.install()
        tr = Trainer(cfg, is_inference=False, model=m)   # world size from the process group
        tr.current_iteration = 10000
        tr.train_step(synthetic.make_batch(32, frame=rank))
        results[rank] = _step_result(tr, m)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_trainer_step_world2_stub_engine(monkeypatch):
    """One fused stage-b step on 2 ranks with different rays: the flat gradient AND the loss /
    PSNR metrics are averaged by the one all-reduce, the replicas stay bit-identical, and every
    named Parameter's .grad is a view of the averaged flat gradient."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_train_worker, args=(port, results), nprocs=WORLD, join=True, start_method="spawn")
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.trainer import Trainer
    local = []
    for r in range(WORLD):   # each rank's own step, world size 1, same init
        stub, cfg, m = _stub_setup()
        stub.install(monkeypatch)
        tr = Trainer(cfg, is_inference=False, model=m, world_size=1)
        tr.current_iteration = 10000
        tr.train_step(synthetic.make_batch(32, frame=r))
        local.append(_step_result(tr, m))
    mean_grad = sum(x["grad"] for x in local) / WORLD
    for r in range(WORLD):
        res = results[r]
        assert res["world"] == WORLD
        torch.testing.assert_close(res["grad"], mean_grad, rtol=0, atol=1e-7)
        assert torch.equal(res["flat"], results[0]["flat"])
        for k in ("psnr", "total", "render"):
            assert abs(res[k] - sum(x[k] for x in local) / WORLD) < 1e-5, k
        assert res["head_grad_is_view"]
    assert not torch.equal(local[0]["grad"], local[1]["grad"])  # the ranks' rays differ


def _stub_setup_a():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import stub_engine
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    cfg = preset("syn_hotdog_a", rays=32, n_coarse=16, n_fine=4, log2T=12)
    m = Model(cfg.model, cfg.data)
    m.load_state_dict(synthetic.make_state_dict(log2T=12, heads="rgb"))
    return stub_engine, cfg, m


def _step_result_a(tr, m):
    table = m.neural_sdf.tcnn_encoding.params
    return dict(flat=m.flat.detach().clone(), grad=tr._grad[:m.flat.numel()].clone(),
                table=table.detach().clone(), table16=m.engine.table16.clone(),
                gtab=tr._grad_table.clone(), m_tab=tr.optim_table.m.clone(), v_tab=tr.optim_table.v.clone(),
                total=float(tr.losses["total"]), world=tr.world_size)


def _run_a(frame, world, overlap=True, chunk=1 << 14, steps=2, monkeypatch=None, install=True, consume=False):
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.trainer import Trainer
    stub, cfg, m = _stub_setup_a()
    if install:
        stub.install(monkeypatch)
    cfg.trainer.zero_table = False   # the replicated table path (ZeRO: test_stage_a_zero_table_matches_replicated)
    tr = Trainer(cfg, is_inference=False, model=m, world_size=world)
    tr.table_overlap, tr.table_chunk = overlap, chunk
    tr.table_grad_consume = consume   # False: the averaged table gradient stays readable (gtab)
    tr.current_iteration = 100000   # past the coarse-to-fine ramp
    grads = []
    for s in range(steps):
        tr.train_step(synthetic.make_batch(32, frame=frame + 10 * s))
        grads.append(_step_result_a(tr, m))
    return grads


def _train_a_worker(rank, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        results[(rank, "overlap")] = _run_a(rank, WORLD, overlap=True)
        results[(rank, "serial")] = _run_a(rank, WORLD, overlap=False, install=False)
        results[(rank, "consume")] = _run_a(rank, WORLD, overlap=True, install=False, consume=True)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_stage_a_step_world2_stub_engine(monkeypatch):
    """Stage a (f1) on 2 ranks with different rays: both the flat MLP
    gradient and the 1.46 GB-class hash-table gradient are the means of the per-rank gradients
    (DDP over every parameter, get_trainer.py:80-88); after the AdamW steps the table, its fp16
    gather shadow and the table moments are bit-identical on both ranks; the overlapped chunked
    table reduction (chunk i stepped while i+1 reduces) equals the serial single all-reduce
    bit for bit."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_train_a_worker, args=(port, results), nprocs=WORLD, join=True, start_method="spawn")
    # per-rank gradients of the first step (same init, world size 1)
    local = [_run_a(r, 1, steps=1, monkeypatch=monkeypatch)[0] for r in range(WORLD)]
    assert not torch.equal(local[0]["gtab"], local[1]["gtab"])   # the ranks' rays differ
    mean_gtab = (local[0]["gtab"] + local[1]["gtab"]) / WORLD
    mean_grad = (local[0]["grad"] + local[1]["grad"]) / WORLD
    n_chunks = -(-mean_gtab.numel() // (1 << 14))
    assert n_chunks >= 4
    for r in range(WORLD):
        for mode in ("overlap", "serial"):
            first = results[(r, mode)][0]
            assert first["world"] == WORLD
            torch.testing.assert_close(first["gtab"], mean_gtab, rtol=0, atol=1e-6)
            torch.testing.assert_close(first["grad"], mean_grad, rtol=0, atol=1e-7)
        for s in range(2):
            a, b = results[(r, "overlap")][s], results[(0, "overlap")][s]
            c = results[(r, "serial")][s]
            z = results[(r, "consume")][s]
            for k in ("table", "table16", "m_tab", "v_tab", "flat", "gtab"):
                assert torch.equal(a[k], b[k]), (r, s, k)   # replicas in sync
                assert torch.equal(a[k], c[k]), (r, s, k)   # overlapped == serial, bitwise
                if k != "gtab":   # the consumed gradient: left zero for the next scatter (ABI 17)
                    assert torch.equal(a[k], z[k]), (r, s, k)
            assert not bool(z["gtab"].any())
            assert torch.equal(a["table16"], a["table"].half())


def _run_zero(frame, world, zero, tmpdir, steps=2):
    """Stage-a steps with the table sharded (ZeroTableAdamW) or replicated (serial all-reduce);
    returns per-step results with the table state gathered (sync_table, every rank) and the
    path of a checkpoint saved through the Checkpointer after the last step."""
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.trainer import Trainer, ZeroTableAdamW
    stub, cfg, m = _stub_setup_a()
    stub.install(None)
    cfg.trainer["zero_table"] = zero
    cfg["logdir"] = os.path.join(tmpdir, "zero" if zero else "serial")
    tr = Trainer(cfg, is_inference=False, model=m, world_size=world)
    assert isinstance(tr.optim_table, ZeroTableAdamW) == zero
    tr.table_overlap = False
    tr.current_iteration = 100000
    out = []
    for s in range(steps):
        tr.train_step(synthetic.make_batch(32, frame=frame + 10 * s))
        tr.sync_table()
        table = m.neural_sdf.tcnn_encoding.params
        mt, vt = tr._table_full_moments if zero else (tr.optim_table.m, tr.optim_table.v)
        out.append(dict(flat=m.flat.detach().clone(), table=table.detach().clone(),
                        table16=m.engine.table16.clone(), m_tab=mt.clone(), v_tab=vt.clone()))
    path = tr.checkpointer.save(1, tr.current_iteration)
    return out, path


def _zero_worker(rank, world, port, tmpdir, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        results[(rank, True)] = _run_zero(rank, world, True, tmpdir)
        results[(rank, False)] = _run_zero(rank, world, False, tmpdir)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_stage_a_zero_table_matches_replicated(world, tmp_path):
    """Stage a with the hash table's optimizer state sharded ZeRO-style (VERDICT r4 item 5:
    reduce-scatter of the table gradient, AdamW on the rank's shard, all-gather of the fp16 gather
    shadow) against the replicated form (one all-reduce, the whole AdamW on every rank), two steps
    on ranks with different rays: the fp32 table (gathered), its fp16 shadow, the table moments
    and the MLP buffer are bit-identical at world size 2 (a two-term sum is exact in any order)
    and equal to fp32 rounding at world size 4 (the ring's summation order); the fp16 shadow is
    the same on every rank; and the checkpoint saved through the Checkpointer (the gather is a
    collective of every rank) equals the replicated run's file, optimizer moments included."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_zero_worker, args=(world, port, str(tmp_path), results), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        (zr, zpath), (sr, spath) = results[(r, True)], results[(r, False)]
        for s in range(2):
            for k in ("table", "table16", "m_tab", "v_tab", "flat"):
                if world == 2:
                    assert torch.equal(zr[s][k], sr[s][k]), (r, s, k)
                else:
                    torch.testing.assert_close(zr[s][k].float(), sr[s][k].float(), rtol=1e-5, atol=1e-7)
            assert torch.equal(zr[s]["table16"], results[(0, True)][0][s]["table16"])
            assert torch.equal(zr[s]["table16"], zr[s]["table"].half())
    zc = torch.load(results[(0, True)][1], weights_only=True)
    sc = torch.load(results[(0, False)][1], weights_only=True)
    key = "module.neural_sdf.tcnn_encoding.params"
    tol = dict(rtol=0, atol=0) if world == 2 else dict(rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(zc["model"][key], sc["model"][key], **tol)
    assert set(zc["optim"]["state"]) == set(sc["optim"]["state"])
    for i, st in sc["optim"]["state"].items():
        for k in ("exp_avg", "exp_avg_sq"):
            torch.testing.assert_close(zc["optim"]["state"][i][k], st[k], **tol)


def test_table_chunks_cover():
    from mli_nerf_amd.trainer import table_chunks
    for n, c in [(10, 3), (9, 3), (1, 5), (45724048 * 8, 1 << 25)]:
        ch = table_chunks(n, c)
        assert ch[0][0] == 0 and sum(k for _, k in ch) == n
        assert all(a[0] + a[1] == b[0] for a, b in zip(ch, ch[1:]))
        assert all(0 < k <= c for _, k in ch)


def _infer_worker(rank, port, results, size):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        results[rank] = _infer(size, install=True)
    finally:
        dist.destroy_process_group()


def _infer(size, install=False, monkeypatch=None):
    from mli_nerf_amd import synthetic
    stub, cfg, m = _stub_setup()
    stub.install(monkeypatch)
    stub.install_cpu_streams()
    m.image_size_val = list(size)
    m.rand_rays_val = 8
    b = synthetic.make_batch(1, frame=2)
    out = m.inference(dict(pose=b["pose"], intr=b["intr"], pose_light=b["pose_light"]))
    return {k: out[k].clone() for k in ("rgb_map", "o_r_map", "o_s_map", "depth_map", "normal_map", "opacity_map")}


@pytest.mark.timeout(300)
def test_model_inference_world2_stub_engine(monkeypatch):
    """Model.inference under a world-2 process group: each rank renders one contiguous tile in
    padded rand_rays_val chunks and ONE all_gather rebuilds every map on every rank, equal to the
    single-process render (7 x 9 frame: ragged tiles and chunks)."""
    size = (7, 9)
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_infer_worker, args=(port, results, size), nprocs=WORLD, join=True, start_method="spawn")
    saved = (torch.cuda.current_stream, torch.cuda.Stream, torch.cuda.stream, torch.Tensor.record_stream)
    try:
        ref = _infer(size, monkeypatch=monkeypatch)
    finally:
        torch.cuda.current_stream, torch.cuda.Stream, torch.cuda.stream, torch.Tensor.record_stream = saved
    for r in range(WORLD):
        for k, v in ref.items():
            assert torch.equal(results[r][k], v), (r, k)
    assert ref["rgb_map"].shape == (1, 3) + size


# ----------------------------------------------------------------------------------------
# bench.py --gpus N without a launcher: the spawn path
# ----------------------------------------------------------------------------------------
_WORKER = r'''
import json, os, sys
import torch, torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
if sys.argv[1:] == ["--fail"] and rank == 1:
    sys.exit(3)
dist.init_process_group("gloo")
t = torch.tensor([float(rank + 1)])
dist.all_reduce(t)
if rank == 0:
    print(json.dumps({"n_gpus": world, "sum": t.item(), "argv": sys.argv[1:]}))
dist.destroy_process_group()
'''


@pytest.mark.timeout(300)
def test_bench_launcher_world2(tmp_path, capfd):
    """bench.launch_workers: N processes with torchrun's environment, rank 0's line on stdout,
    exit code 0; a failing rank stops the others (they would block in a collective) and its
    exit code is returned."""
    import bench
    w = tmp_path / "worker.py"
    w.write_text(_WORKER)
    assert bench.launch_workers(WORLD, ["--steps", "3"], script=str(w)) == 0
    out = capfd.readouterr().out.strip().splitlines()
    import json
    line = json.loads(out[-1])
    assert line == {"n_gpus": WORLD, "sum": 3.0, "argv": ["--steps", "3"]}
    assert bench.launch_workers(WORLD, ["--fail"], script=str(w)) == 3


def _zero_guard_worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mli_nerf_amd import synthetic
        from mli_nerf_amd.trainer import Trainer, ZeroTableAdamW
        stub, cfg, m = _stub_setup_a()
        stub.install(None)
        cfg.trainer["zero_table"] = True
        tr = Trainer(cfg, is_inference=False, model=m, world_size=world)
        assert isinstance(tr.optim_table, ZeroTableAdamW)
        tr.table_overlap = False
        tr.current_iteration = 100000
        got = {}
        tr.train_step(synthetic.make_batch(32, frame=rank))
        tr.sync_table()
        tr.optim_state_dict()            # gathered: fine
        tr.train_step(synthetic.make_batch(32, frame=rank + 10))
        tr.train_step(synthetic.make_batch(32, frame=rank + 20))   # two steps without a sync
        for what, fn in (("optim_state_dict", tr.optim_state_dict),
                         ("save_checkpoint", lambda: tr.save_checkpoint("/nonexistent-not-written")),
                         ("prepare", lambda: (setattr(m, "engine", None), setattr(m, "_sdf_version", None),
                                              m.prepare()))):
            try:
                fn()
                got[what] = "no error"
            except RuntimeError as e:
                got[what] = "sync_table" in str(e)
        stub.install(None)   # (the prepare probe dropped the engine)
        tr.sync_table()      # collective: every rank
        tr.optim_state_dict()
        m.prepare()
        got["after_sync"] = True
        results[rank] = got
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_zero_table_stale_state_guards():
    """with the table ZeRO-sharded, the fp32 master outside this rank's shard and the
    gathered moments are only valid right after sync_table().  Two steps without a sync must make
    optim_state_dict, save_checkpoint and an engine rebuild (Model.prepare re-casting the fp16
    shadow from the fp32 master) raise instead of returning stale state or reverting the other
    ranks' updates; after sync_table() all three work again."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_zero_guard_worker, args=(2, port, results), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        assert results[r] == {"optim_state_dict": True, "save_checkpoint": True, "prepare": True,
                              "after_sync": True}, results[r]


def _overlap_worker(rank, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from mli_nerf_amd import synthetic
        from mli_nerf_amd.trainer import Trainer
        for overlap in (True, False):
            stub, cfg, m = _stub_setup()
            stub.install()
            tr = Trainer(cfg, is_inference=False, model=m)
            tr.grad_overlap = overlap
            tr.current_iteration = 10000
            calls = []
            if overlap:
                real = tr._grad_reducer

                def spy(model, real=real):
                    red = real(model)
                    orig = red.__call__

                    class Spy:
                        def __call__(self, cls):
                            calls.append(cls)
                            orig(cls)

                        def finish(self, off):
                            calls.append("finish")
                            return red.finish(off)
                    return Spy()
                tr._grad_reducer = spy
            for s in range(2):
                tr.train_step(synthetic.make_batch(32, frame=rank + 10 * s))
            res = _step_result(tr, m)
            res["calls"] = calls
            results[(rank, overlap)] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_trainer_grad_allreduce_overlap_world2():
    """the stage-b gradient average issued per dW class as each class's layers
    complete (DDP-bucket style, overlapped with the next class's dW) is bit-identical to the single
    all-reduce after the backward, on 2 ranks with different rays over two steps: gradient, every
    parameter after the AdamW step, and the averaged loss / PSNR metrics; the classes go out in the
    backward's launch order, then the metric slots."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    results = ctx.Manager().dict()
    mp.start_processes(_overlap_worker, args=(port, results), nprocs=WORLD, join=True, start_method="spawn")
    for r in range(WORLD):
        a, b = results[(r, True)], results[(r, False)]
        assert a["calls"] == ["out", "big", "wide", "finish"] * 2, a["calls"]
        assert torch.equal(a["grad"], b["grad"])
        assert torch.equal(a["flat"], b["flat"])
        assert torch.equal(a["flat"], results[(0, True)]["flat"])
        for k in ("psnr", "total", "render"):
            assert a[k] == b[k], k
    assert not torch.equal(results[(0, True)]["grad"], torch.zeros_like(results[(0, True)]["grad"]))


def test_grad_class_ranges_cover_the_flat_buffer():
    """The per-class ranges of OverlappedGradReduce tile the stage-b flat gradient exactly once."""
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import grad_class_ranges
    cfg = preset("syn_hotdog_b", rays=32, n_coarse=16, n_fine=4, log2T=12)
    m = Model(cfg.model, cfg.data)
    rng = grad_class_ranges(m._trainable_items())
    assert sorted(rng) == ["big", "out", "wide"]
    cover = torch.zeros(m.flat.numel(), dtype=torch.int32)
    for c, lst in rng.items():
        for o, k in lst:
            cover[o:o + k] += 1
    assert bool((cover == 1).all())
    assert len(rng["out"]) == 3 and len(rng["big"]) == 3 and len(rng["wide"]) == 3
