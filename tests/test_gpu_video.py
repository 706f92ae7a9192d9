"""End-to-end video on the GPU renderer: Blender-layout files on disk ->
Dataset -> interpolated camera + light poses -> Model.inference per frame (the HIP path) ->
labelled collage -> mirrored sequence -> file.  The rendered tile of the first frame equals a
direct Model.inference at the first endpoint's pose (ratio 0)."""
import json
import os

import numpy as np
import pytest
import torch

from mli_nerf_amd import synthetic, video as V
from mli_nerf_amd.config import to_attr
from mli_nerf_amd.configs import preset

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _blender_dir(root, H, W, n=3):
    from PIL import Image
    rng = np.random.default_rng(0)
    frames = []
    for i in range(n):
        os.makedirs(os.path.join(root, "val"), exist_ok=True)
        Image.fromarray(rng.integers(0, 256, (H, W, 4), dtype=np.uint8)).save(os.path.join(root, f"val/r_{i}_Img.png"))
        pose = synthetic.look_at_w2c(synthetic.camera_positions()[i * 7])
        c2w = torch.eye(4)
        R, t = pose[:, :3], pose[:, 3:]
        c2w[:3, :3], c2w[:3, 3:] = R.t(), -R.t() @ t
        c2w = c2w * torch.tensor([1.0, -1.0, -1.0, 1.0])   # cv -> gl (the Dataset flips back)
        frames.append({"file_path": f"./val/r_{i}_", "transform_matrix": c2w.tolist(),
                       "pl_pos": list(synthetic.light_positions()[i * 7])})
    meta = {"camera_angle_x": 0.69, "frames": frames}
    for split in ("train", "val"):
        with open(os.path.join(root, f"{split}_transforms.json"), "w") as f:
            json.dump(meta, f)


def test_render_video_end_to_end(tmp_path):
    _need_gpu()
    from mli_nerf_amd.data import Dataset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    H, W = 12, 16
    _blender_dir(str(tmp_path), 24, 32)
    cfg = preset("syn_hotdog_b", rays=64, n_coarse=16, n_fine=4, log2T=14,
                 overrides={"data": {"val": {"image_size": [H, W]}}})
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=14, s_var=3.0))
    model = model.to(DEV)
    model.rand_rays_val = 96
    trainer = Trainer(cfg, is_inference=False, model=model)
    dcfg = to_attr({"data": {"root": str(tmp_path), "type": "projects.NeuralLumen.data_blender",
                             "white_background": True,
                             "train": {"image_size": [H, W]}, "val": {"image_size": [H, W], "subset": None}},
                    "model": {"render": {"rand_rays": 64}}})
    ds = Dataset(dcfg, is_inference=True)
    path = V.render_video(model, ds, 0, 2, str(tmp_path / "out"), trainer=trainer, n_frames=3,
                          video_content=("rgb", "gt", "o_r", "o_s"))
    assert os.path.exists(path)
    # frame 0 = ratio sin(-pi/2)/2 + 1/2 = 0: the first endpoint's camera and light
    s0, s2 = ds[0], ds[2]
    r0 = V.frame_ratio(0)
    assert float(r0) == 0.0
    pose = V.interpolate_pose(s0["pose"], s2["pose"], r0)
    light = V.interpolate_pose(s0["pose_light"], s2["pose_light"], r0)
    torch.testing.assert_close(pose, s0["pose"], rtol=0, atol=1e-6)
    out = model.inference(dict(intr=s0["intr"][None].to(DEV), pose=pose[None].to(DEV),
                               pose_light=light[None].to(DEV)))
    tile = V.img_to_np(out["rgb_map"][0], True, "Image (render)")
    if path.endswith(".gif"):
        from PIL import Image
        fdir = str(tmp_path / "out" / "render" / "0_2_frames")
        names = sorted(os.listdir(fdir))
        assert len(names) == 6
        f0 = np.asarray(Image.open(os.path.join(fdir, names[0])).convert("RGB"))
        f5 = np.asarray(Image.open(os.path.join(fdir, names[5])).convert("RGB"))
        assert f0.shape == (2 * tile.shape[0], 2 * tile.shape[1] + 5, 3)  # 4 tiles: 2x2 collage
        assert np.array_equal(f0, f5)                                     # mirrored sequence
        assert np.array_equal(f0[:tile.shape[0], :tile.shape[1]], tile)


def test_checkpoint_table_shadow_rebuilt(tmp_path):
    """Checkpoint bridge: a stage-a checkpoint's tcnn flat fp32 params, loaded into a model on
    the GPU, are what the fp16 gather shadow (engine.table16) holds at the next render, and a
    stage-a fused step keeps the shadow equal to the updated params."""
    _need_gpu()
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    cfg = preset("syn_hotdog_a", rays=64, n_coarse=16, n_fine=4, log2T=14)
    src = Model(cfg.model, cfg.data)
    src.load_state_dict(synthetic.make_state_dict(log2T=14, s_var=3.0, heads="rgb", seed=7))
    path = Trainer(cfg, is_inference=False, model=src).save_checkpoint(str(tmp_path))
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=14, s_var=3.0, heads="rgb", seed=8))
    model = model.to(DEV)
    tr = Trainer(cfg, is_inference=False, model=model)
    tr.current_iteration = 100000
    batch = {k: v.to(DEV) for k, v in synthetic.make_batch(64, frame=1).items()}
    tr.train_step(batch)                       # shadow built from the seed-8 table
    tr.load_checkpoint(path, resume=False)     # in-place copy into the fp32 params
    model.prepare()
    table = model.neural_sdf.tcnn_encoding.params.detach()
    assert torch.equal(table.cpu(), src.neural_sdf.tcnn_encoding.params.detach())
    assert torch.equal(model.engine.table16, table.half())
    tr.train_step(batch)
    torch.cuda.synchronize()
    assert torch.equal(model.engine.table16, model.neural_sdf.tcnn_encoding.params.detach().half())
