"""``Trainer.test_all_light`` enumerations against the reference's own
``test_all_light`` (``projects/NeuralLumen/trainer.py:216-316``), pinned by
``tests/golden/relight_index.json`` (tests/golden/make_golden_relight.py ran the reference with a
stand-in model that encodes the requested camera frame and light into its maps).  CPU only: the
stand-in model replaces ``Model.inference``; the GPU render is tests/test_gpu_relight.py."""
import json
import os
import types

import pytest
import torch

from mli_nerf_amd import relight

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "relight_index.json")))
H = W = GOLD["H"]


class FakeDataset:
    """Frame f: pose_light translation x = 100 + f, image = f (as the golden generator's)."""

    def __init__(self, frames):
        self.list = frames
        self.sample_train_rays = True

    def __len__(self):
        return len(self.list)

    def get_light(self, idx):
        p = torch.zeros(3, 4)
        p[:3, :3] = torch.eye(3)
        p[0, 3] = 100.0 + idx
        return p

    def __getitem__(self, idx):
        return dict(idx=idx, image=torch.full((3, H, W), float(idx)), pose=torch.zeros(3, 4),
                    intr=torch.eye(3), pose_light=self.get_light(idx))


class FakeModel:
    pcfg = types.SimpleNamespace(light_visibility=dict(camera_ray_type="blend_z_sphere_tracing"))

    def eval(self):
        return self

    def inference(self, data):
        frame = float(data["image"].flatten()[0])
        light = float(data["pose_light"][0, 0, 3])
        m1 = torch.zeros(1, 1, H, W)
        return dict(rgb_map=torch.full((1, 3, H, W), frame), normal_map=torch.full((1, 3, H, W), light),
                    visibility_map=m1, inter_dist_map=m1 + 1, inter_mask_map=m1, normal_x_light_map=m1)


class FakeTrainer:
    def __init__(self):
        self.model = FakeModel()
        self.current_iteration = 7
        self.iters = []

    def start_of_iteration(self, data, current_iteration):
        self.current_iteration = current_iteration
        return data

    def _start_of_iteration(self):
        self.iters.append(self.current_iteration)


def decode(results):
    out = {}
    for cam, lights in results.items():
        out[cam] = {}
        for li, r in lights.items():
            tgt = int(r["rgb_target"].flatten()[0]) if "rgb_target" in r else -1
            out[cam][li] = [int(r["rgb_render"].flatten()[0]), int(r["normal"].flatten()[0]) - 100, tgt]
    return out


def test_random_other_index_matches_reference():
    for key, want in GOLD["random_other_index"].items():
        n, k, seed = (int(x) for x in key.split("_"))
        assert relight.get_random_other_index(n, k, seed) == want


@pytest.mark.parametrize("name", sorted(GOLD["cases"]))
def test_all_light_enumeration_matches_reference(name, tmp_path):
    case = GOLD["cases"][name]
    ds = FakeDataset(GOLD["frames"][case["frames"]])
    tr = FakeTrainer()
    loader = types.SimpleNamespace(dataset=ds)   # a DataLoader's .dataset, as test.py passes it
    kw = dict(output_dir=str(tmp_path), mode="test", dataset_type=case["dataset_type"],
              sample_num=case["sample_num"], seed=case["seed"])
    if "error" in case["results"]:
        with pytest.raises(ValueError):
            relight.test_all_light(tr, loader, **kw)
        return
    relight.test_all_light(tr, loader, **kw)
    res = torch.load(os.path.join(str(tmp_path), "results_all.pt"), weights_only=True)
    assert decode(res) == case["results"]
    # the layout scripts/pseudo_label.py:294-410 reads
    for cam, lights in res.items():
        for li, r in lights.items():
            keys = {"normal", "normal_x_light", "rgb_render", "visibility", "inter_mask"}
            if case["dataset_type"] == "pair":
                keys.add("rgb_target")
            assert set(r) == keys and r["normal"].shape == (1, 3, H, W) and r["visibility"].shape == (1, 1, H, W)
            assert os.path.exists(os.path.join(str(tmp_path), cam, li + "_pseudo_shading.png"))
            # trainer.py:270-274 squeezes the batch dim before preprocess_image: one-channel maps
            # stay single-channel 'L' PNGs (no colormap), levels int(v * 255)
            from PIL import Image
            for name, mode in (("visibility", "L"), ("inter_mask", "L"), ("normal_x_light", "L"),
                               ("pseudo_shading", "L"), ("inter_dist", "L"), ("rgb_render", "RGB"), ("normal", "RGB")):
                im = Image.open(os.path.join(str(tmp_path), cam, li + "_" + name + ".png"))
                assert im.mode == mode and im.size == (W, H), (name, im.mode)
            im = Image.open(os.path.join(str(tmp_path), cam, li + "_normal.png"))
            light = int(r["normal"].flatten()[0])   # normal map = light x (from range (-1, 1): clamped to 1)
            assert im.getpixel((0, 0)) == (255, 255, 255) if light >= 1 else True
    import sys
    assert tr.iters and all(i == sys.maxsize for i in tr.iters)   # mode 'test': iteration sys.maxsize
    assert tr.current_iteration == 7 and ds.sample_train_rays is False


def test_index_info_pair_and_unpair():
    ds = FakeDataset(GOLD["frames"]["pair"])
    info = relight.index_info(ds, "pair")
    for fi, fr in enumerate(ds.list):
        assert info[fr["camera_index"]][fr["light_index"]] == fi
    ds = FakeDataset(GOLD["frames"]["unpair"])
    info = relight.index_info(ds, "unpair", 4, 999)
    assert [list(info[c].values()) for c in sorted(info)] == GOLD["random_other_index"]["7_4_999"]
    with pytest.raises(NotImplementedError):
        relight.index_info(ds, "grid")


def test_all_light_needs_visibility():
    tr = FakeTrainer()
    tr.model.pcfg = types.SimpleNamespace(light_visibility=None)
    with pytest.raises(ValueError):
        relight.test_all_light(tr, FakeDataset(GOLD["frames"]["pair"]), output_dir=None)
