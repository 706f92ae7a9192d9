"""Checkpoint bridge, CPU: the imaginaire file layout
(``epoch_{:05}_iteration_{:09}_checkpoint.pt`` + ``latest_checkpoint.txt``,
imaginaire/trainers/base.py:570-607), ``module.``-prefixed keys, a stage-a checkpoint
warm-starting stage b (NeuralLumen/trainer.py:27-42: strict=False, tcnn flat params carried
over), and stage-a resume with the hash-table optimizer moments.  The fp16 table shadow the
GPU gathers is rebuilt from the loaded fp32 params (tests/test_gpu_video.py)."""
import os

import torch

from mli_nerf_amd import synthetic
from mli_nerf_amd.configs import preset


def _model(stage, seed=0):
    from mli_nerf_amd.model import Model
    name = "syn_hotdog_a" if stage == "a" else "syn_hotdog_b"
    cfg = preset(name, rays=32, n_coarse=16, n_fine=4, log2T=12)
    m = Model(cfg.model, cfg.data)
    m.load_state_dict(synthetic.make_state_dict(log2T=12, s_var=3.0 + seed, heads="rgb" if stage == "a" else "rgb_r_s",
                                                seed=seed))
    return cfg, m


def test_checkpoint_layout_and_round_trip(tmp_path):
    from mli_nerf_amd.trainer import Trainer
    cfg, m = _model("b")
    tr = Trainer(cfg, is_inference=False, model=m)
    tr.current_iteration, tr.current_epoch = 1234, 5
    tr.optim.m.uniform_()
    tr.optim.v.uniform_()
    tr.optim.step_count = 1234
    path = tr.save_checkpoint(str(tmp_path))
    assert os.path.basename(path) == "epoch_00005_iteration_000001234_checkpoint.pt"
    assert (tmp_path / "latest_checkpoint.txt").read_text().strip() == os.path.basename(path)
    ck = torch.load(path, weights_only=True)
    assert all(k.startswith("module.") for k in ck["model"])
    assert "module.neural_sdf.tcnn_encoding.params" in ck["model"]
    cfg2, m2 = _model("b", seed=1)
    tr2 = Trainer(cfg2, is_inference=False, model=m2)
    tr2.load_checkpoint(str(tmp_path / "latest_checkpoint.txt"))
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    assert torch.equal(tr2.optim.m, tr.optim.m) and tr2.current_iteration == 1234 and tr2.current_epoch == 5


def test_stage_a_checkpoint_warm_starts_stage_b(tmp_path):
    from mli_nerf_amd.trainer import Trainer
    cfg_a, ma = _model("a", seed=2)
    tra = Trainer(cfg_a, is_inference=False, model=ma)
    tra.optim_table.v.uniform_()
    tra.optim.step_count = tra.optim_table.step_count = 500000
    tra.current_iteration = 500000
    path = tra.save_checkpoint(str(tmp_path / "a"))
    # resume stage a: table moments come back
    cfg_a2, ma2 = _model("a", seed=3)
    tra2 = Trainer(cfg_a2, is_inference=False, model=ma2)
    tra2.load_checkpoint(path)
    assert torch.equal(tra2.optim_table.v, tra.optim_table.v)
    # warm start stage b (no resume): SDF, table and s_var from stage a; heads stay
    cfg_b, mb = _model("b", seed=4)
    heads_before = {k: v.clone() for k, v in mb.state_dict().items() if k.startswith("neural_rgb")}
    trb = Trainer(cfg_b, is_inference=False, model=mb)
    res = trb.load_pre_trained(path)
    sa, sb = ma.state_dict(), mb.state_dict()
    for k in ("neural_sdf.tcnn_encoding.params", "neural_sdf.mlp.linears.0.weight_v", "neural_sdf.mlp.linear_sdf.bias",
              "s_var"):
        assert torch.equal(sa[k], sb[k]), k
    assert trb.current_iteration == 0
    # the stage-a single head ('neural_rgb.mlp') has the stage-b key names of its first head
    for k, v in heads_before.items():
        if k in sa and sa[k].shape == v.shape:
            assert torch.equal(sb[k], sa[k]), k
        else:
            assert torch.equal(sb[k], v), k
    assert not res.unexpected_keys or all(k.startswith("neural_rgb") for k in res.unexpected_keys)


def test_prefetch_is_a_no_op_outside_the_fused_stage_b_path():
    """Trainer.prefetch only pipelines the fused stage-b step: in stage a (the geometry is being
    trained, so the next batch's sampling depends on this step's update) and for loss configs the
    fused kernel does not cover it issues nothing, and train_step finds no prefetched geometry."""
    from mli_nerf_amd.trainer import Trainer
    cfg_a, ma = _model("a")
    tra = Trainer(cfg_a, is_inference=False, model=ma)
    batch = synthetic.make_batch(32, frame=1)
    tra.prefetch(batch)
    assert tra._pending == [] and tra._take_prefetched(batch) is None
    cfg_b, mb = _model("b")
    trb = Trainer(cfg_b, is_inference=False, model=mb)
    trb.weights["unfused_term"] = 1.0
    trb.prefetch(batch)
    assert trb._pending == []


def test_checkpointer_adapter_as_test_py_calls_it(tmp_path):
    """trainer.checkpointer.load(args.checkpoint, args.resume, load_sch=False, load_opt=False)
    (test.py:93 over imaginaire/trainers/base.py:609-652): an explicit path loads the model only
    (resume False) or the metadata too (resume True); resume with no path takes cfg.logdir's
    latest_checkpoint.txt; no path and no resume trains from scratch; a missing file raises."""
    import pytest
    from mli_nerf_amd.trainer import Trainer
    cfg, m = _model("b")
    cfg["logdir"] = str(tmp_path)
    tr = Trainer(cfg, is_inference=False, model=m)
    path = tr.checkpointer.save(3, 777)
    assert os.path.basename(path) == "epoch_00003_iteration_000000777_checkpoint.pt"
    assert (tmp_path / "latest_checkpoint.txt").read_text().strip() == os.path.basename(path)
    cfg2, m2 = _model("b", seed=1)
    cfg2["logdir"] = str(tmp_path)
    tr2 = Trainer(cfg2, is_inference=True, model=m2)
    assert tr2.checkpointer.load(None, False) is None          # from scratch
    tr2.checkpointer.load(path, False, load_sch=False, load_opt=False)
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    assert tr2.current_iteration == 0 and tr2.checkpointer.eval_iteration == 777
    cfg3, m3 = _model("b", seed=2)
    cfg3["logdir"] = str(tmp_path)
    tr3 = Trainer(cfg3, is_inference=False, model=m3)
    tr3.checkpointer.load(None, True)                          # latest of cfg.logdir
    assert tr3.current_iteration == 777 and tr3.current_epoch == 3 and tr3.checkpointer.resume_iteration == 777
    assert torch.equal(m3.s_var, m.s_var)
    with pytest.raises(FileNotFoundError):
        tr3.checkpointer.load(str(tmp_path / "nope.pt"), False)


def test_adam_ranges_follow_partial_grad():
    """The fused AdamW steps exactly the optimized parameters whose requires_grad is on
    (NeuralLumen/trainer.py:44-54): the whole flat buffer by default (one launch), the named head
    alone with partial_grad = ['neural_rgb.mlp_r'], adjacent parameters merged into one range."""
    from mli_nerf_amd.trainer import Trainer
    cfg, m = _model("b")
    tr = Trainer(cfg, is_inference=False, model=m)
    assert tr.adam_ranges() is None
    cfg2, m2 = _model("b")
    cfg2.trainer["partial_grad"] = ["neural_rgb.mlp_r"]
    tr2 = Trainer(cfg2, is_inference=False, model=m2)
    items = {n: (off, k) for n, _, off, k in m2._trainable_items()}
    mine = sorted(v for n, v in items.items() if n.startswith("neural_rgb.mlp_r."))
    lo, hi = mine[0][0], mine[-1][0] + mine[-1][1]
    assert tr2.adam_ranges() == [(lo, hi - lo)]
    assert hi - lo == sum(k for _, k in mine)          # the head's parameters are contiguous
    cfg3, m3 = _model("a")
    cfg3.trainer["partial_grad"] = ["neural_rgb"]       # stage a with the SDF frozen: no table step
    tr3 = Trainer(cfg3, is_inference=False, model=m3)
    assert not tr3.table_trains() and tr3.adam_ranges() is not None


def test_train_py_surface_stub_engine(tmp_path, monkeypatch):
    """The calls train.py:81-101 / test.py:104-121 make on cfg.trainer.type (VERDICT r3 missing 4):
    set_data_loader, checkpointer.load, init_wandb, train (the imaginaire loop: DataLoader
    batches, start_of_iteration, train_step, checkpoints at save_iter and max_iter), finalize,
    test_save -- here behind the CPU stub engine (tests/stub_engine.py)."""
    import json
    import sys
    import numpy as np
    from PIL import Image
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import stub_engine
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    root = tmp_path / "set"
    (root / "img").mkdir(parents=True)
    rng = np.random.default_rng(0)
    frames = []
    for cam in range(2):
        for light in range(2):
            name = "c%02dl%02d.png" % (cam, light)
            Image.fromarray(rng.integers(0, 256, (12, 16, 3), dtype=np.uint8)).save(str(root / "img" / name))
            c2w = [[1, 0, 0, 0.1 * cam], [0, 1, 0, 0], [0, 0, 1, 3.0], [0, 0, 0, 1]]
            frames.append({"file_path": "img/" + name, "transform_matrix": c2w, "transform_matrix_light": c2w,
                           "camera_index": cam, "light_index": light})
    meta = {"fl_x": 20.0, "fl_y": 20.0, "cx": 8.0, "cy": 6.0, "sk_x": 0.0, "sk_y": 0.0, "frames": frames}
    for split in ("train", "val"):
        (root / (split + "_transforms.json")).write_text(json.dumps(meta))
    over = {"data": {"root": str(root), "type": "projects.NeuralLumen.data", "white_background": False,
                     "train": {"image_size": [12, 16]}, "val": {"image_size": [12, 16], "subset": None}},
            "max_iter": 5, "checkpoint": {"save_iter": 2}, "logdir": str(tmp_path / "logs")}
    cfg = preset("syn_hotdog_b", rays=32, n_coarse=16, n_fine=4, log2T=12, overrides=over)
    cfg.trainer.loss_weight = {"render": 1.0}   # no pseudo labels in this set
    stub_engine.install(monkeypatch)
    m = Model(cfg.model, cfg.data)
    m.load_state_dict(synthetic.make_state_dict(log2T=12))
    tr = Trainer(cfg, is_inference=False, model=m, world_size=1)
    tr.set_data_loader(cfg, split="train")
    tr.set_data_loader(cfg, split="val")
    assert len(tr.train_data_loader.dataset) == 4 and len(tr.eval_data_loader.dataset) == 4
    tr.checkpointer.load(None, False, load_sch=True, load_opt=True)
    tr.init_wandb(cfg, project="p", mode="disabled", resume=False, use_group=True)
    flat0 = m.flat.detach().clone()
    tr.train(cfg, tr.train_data_loader, single_gpu=True, profile=False, show_pbar=False)
    tr.finalize(cfg)
    assert tr.current_iteration == 5 and not torch.equal(m.flat.detach(), flat0)
    names = sorted(os.listdir(cfg.logdir))
    assert "epoch_00001_iteration_000000004_checkpoint.pt" in names
    assert "epoch_00001_iteration_000000005_checkpoint.pt" in names   # max_iter
    assert open(os.path.join(cfg.logdir, "latest_checkpoint.txt")).read().strip() == \
        "epoch_00001_iteration_000000005_checkpoint.pt"
    ck = torch.load(os.path.join(cfg.logdir, names[0]), weights_only=True)
    assert ck["iteration"] == 2 and "module.neural_rgb.mlp.linears.0.weight_v" in ck["model"]
    # set_data_loader's drop_last (train) and subset_indices (val) reach the loader (base.py:96-99)
    tr.set_data_loader(cfg, split="val", subset_indices=[0, 2])
    assert len(tr.eval_data_loader.dataset) == 2
    tr.set_data_loader(cfg, split="train", drop_last=False)
    assert tr.train_data_loader.drop_last is False
    # --profile: one more iteration under the profiler, its trace at <logdir>/trace.json (base.py:501-521)
    cfg.max_iter = 6
    tr.train(cfg, tr.train_data_loader, single_gpu=True, profile=True, show_pbar=False)
    assert tr.current_iteration == 6 and os.path.getsize(os.path.join(cfg.logdir, "trace.json")) > 0


def test_optim_state_keeps_moments_of_a_parameter_frozen_after_stepping():
    """A parameter the optimizer stepped and that is frozen later keeps its AdamW state in the
    saved optimizer state dict, as torch.optim.AdamW keeps it; a parameter never
    stepped (frozen from the start) has no entry."""
    from mli_nerf_amd.trainer import Trainer
    cfg, m = _model("b")
    cfg.trainer["partial_grad"] = ["neural_rgb.mlp_r"]
    tr = Trainer(cfg, is_inference=False, model=m)
    g = torch.zeros_like(m.flat)

    def fake_step(grad, lr, ranges=None, **kw):          # the HIP AdamW is not the subject here
        tr.optim.step_count += 1
    tr.optim.step = fake_step
    tr._step_flat(g, 1e-3)                               # steps mlp_r only
    names = [n for n, *_ in tr._moment_views()]
    sd = tr.optim_state_dict()
    assert {names[i] for i in sd["state"]} == {n for n in names if n.startswith("neural_rgb.mlp_r.")}
    for n, p in m.named_parameters():                    # freeze mlp_r, train mlp_s from now on
        p.requires_grad_(n.startswith("neural_rgb.mlp_s."))
    sd = tr.optim_state_dict()
    kept = {names[i] for i in sd["state"]}
    assert {n for n in names if n.startswith("neural_rgb.mlp_r.")} <= kept
    assert not any(n.startswith("neural_rgb.mlp.") for n in kept)
