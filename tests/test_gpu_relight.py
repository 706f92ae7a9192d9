"""``Trainer.test_all_light`` end to end on the GPU render.

Reference: ``projects/NeuralLumen/trainer.py:216-316``.  A synthetic ReNe-layout transforms set
(3 cameras x 2 lights, 18 x 24 frames, written to tmp) is enumerated in the ``unpair`` and
``limitedlights`` modes; every (camera, light) pair is one ``Model.inference`` with the light
visibility pass on (sampling, FIELD, heads, composite, sphere-traced camera and light rays).
``results_all.pt`` is reloaded with ``weights_only=True`` and checked for the keys and shapes
``scripts/pseudo_label.py:294-410`` reads ({camera: {light: {normal [1,3,H,W], normal_x_light
[1,1,H,W], rgb_render [1,3,H,W], visibility [1,1,H,W], inter_mask [1,1,H,W]}}}, string keys), and
one (camera, light) entry is compared with ``Model.inference`` called directly on the same
inputs: bit-identical.  The enumeration itself is pinned to the reference in tests/test_relight.py.
"""
import copy
import json
import math
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
H, W = 18, 24
VIS = dict(enabled=True, camera_ray_type="blend_z_sphere_tracing", type="sphere_tracing",
           visibility_bounding_type="sphere", visibility_sphere_radius=0.95)


def _c2w(ang, y=0.3, r=2.5):
    c, s = math.cos(ang), math.sin(ang)
    return [[c, 0.0, s, r * s], [0.0, 1.0, 0.0, y], [-s, 0.0, c, r * c], [0, 0, 0, 1]]


def _write_set(root):
    """ReNe layout (NeuralLumen/data.py:12-140): camera_index / light_index / pl_index per frame."""
    import numpy as np
    from PIL import Image
    rng = np.random.default_rng(3)
    frames = []
    os.makedirs(os.path.join(root, "img"), exist_ok=True)
    for cam in range(3):
        for light in range(2):
            name = "c%02dl%02d.png" % (cam, light)
            Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(os.path.join(root, "img", name))
            frames.append({"file_path": "img/" + name, "transform_matrix": _c2w(0.4 * cam),
                           "transform_matrix_light": _c2w(1.3 + 1.7 * light, y=1.5, r=3.0),
                           "camera_index": cam, "light_index": light, "pl_index": light})
    meta = {"fl_x": 22.0, "fl_y": 22.0, "cx": W / 2, "cy": H / 2, "sk_x": 0.0, "sk_y": 0.0, "frames": frames}
    for split in ("train", "val"):
        with open(os.path.join(root, split + "_transforms.json"), "w") as f:
            json.dump(meta, f)


def _setup(root):
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.data import Dataset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    over = {"model": {"light_visibility": VIS, "render": {"rand_rays_val": 256}},
            "data": {"root": str(root), "type": "projects.NeuralLumen.data", "white_background": False,
                     "train": {"image_size": [H, W]}, "val": {"image_size": [H, W], "subset": None}}}
    cfg = preset("syn_hotdog_b", n_coarse=16, n_fine=4, log2T=14, overrides=over)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=14, s_var=6.0))
    model = model.to(DEV)
    tr = Trainer(cfg, is_inference=True, model=model)
    return cfg, model, tr, Dataset(cfg, is_inference=True)


@pytest.mark.parametrize("mode,sample_num,n_cams,n_lights", [("unpair", 2, 6, 2), ("limitedlights", 2, 6, 2)])
def test_all_light_gpu_render(tmp_path, mode, sample_num, n_cams, n_lights):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mli_nerf_amd import relight
    _write_set(str(tmp_path / "set"))
    cfg, model, tr, ds = _setup(tmp_path / "set")
    out_dir = str(tmp_path / "out")
    tr.test_all_light(ds, out_dir, mode="test", dataset_type=mode, sample_num=sample_num)
    torch.cuda.synchronize()
    res = torch.load(os.path.join(out_dir, "results_all.pt"), weights_only=True)
    assert sorted(res) == sorted(str(c) for c in range(n_cams))
    shapes = {"normal": (1, 3, H, W), "normal_x_light": (1, 1, H, W), "rgb_render": (1, 3, H, W),
              "visibility": (1, 1, H, W), "inter_mask": (1, 1, H, W)}
    seen_vis = []
    for cam, lights in res.items():
        assert sorted(lights) == [str(li) for li in range(n_lights)]
        for li, r in lights.items():
            assert {k: tuple(v.shape) for k, v in r.items()} == shapes, (cam, li)
            assert all(v.device.type == "cpu" and torch.isfinite(v.float()).all() for v in r.values())
            # pseudo_label.py reads the maps as [0,1] images and boolean-like masks
            assert r["rgb_render"].min() >= 0 and r["rgb_render"].max() <= 1
            assert set(r["visibility"].unique().tolist()) <= {0.0, 1.0}
            seen_vis.append(r["visibility"])
            for name in ("rgb_render", "normal", "visibility", "inter_mask", "normal_x_light", "pseudo_shading",
                         "inter_dist"):
                assert os.path.exists(os.path.join(out_dir, cam, li + "_" + name + ".png"))
    # the visibility pass decides something (not all shadowed, not all lit over every map)
    allv = torch.cat([v.flatten() for v in seen_vis])
    assert 0 < allv.mean() < 1
    # one (camera, light) pair against Model.inference called directly on the same inputs
    info = relight.index_info(ds, mode, sample_num, 999)
    cam = 1
    data = ds[cam]
    data["pose_light"] = ds.get_light(1)            # light 1 of a non-pair enumeration
    data = {k: v[None] if torch.is_tensor(v) else v for k, v in copy.deepcopy(data).items()}
    data = tr.start_of_iteration(data, current_iteration=sys.maxsize)
    tr._start_of_iteration()
    direct = model.inference(data)
    torch.cuda.synchronize()
    assert 1 in info[cam]
    got = res[str(cam)]["1"]
    for key, mk in (("visibility", "visibility_map"), ("normal_x_light", "normal_x_light_map"),
                    ("rgb_render", "rgb_map"), ("normal", "normal_map"), ("inter_mask", "inter_mask_map")):
        assert torch.equal(got[key], direct[mk].detach().cpu()), key
