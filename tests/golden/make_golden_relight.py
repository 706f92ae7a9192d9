#!/usr/bin/env python
"""Golden vectors for ``Trainer.test_all_light`` from the REFERENCE's own
``projects/NeuralLumen/trainer.py:216-316`` (and ``get_random_other_index``,
``projects/NeuralLumen/utils/utils.py:230-252``).

The reference trainer is imported with its absent dependencies (wandb, torchinfo, termcolor, cv2,
torchvision, pynvml, tinycudann, apex) replaced by ``unittest.mock`` modules, and
``Trainer.test_all_light`` is called as an unbound function on a stand-in ``self`` whose model's
``inference`` encodes what it was asked to render: ``rgb_map`` = the frame index of the camera
sample, ``normal_map`` = the x translation of ``pose_light`` (the light), ``rgb_target`` = the
frame index the dataset returned.  The ``results_all.pt`` it writes is decoded into
{camera: {light: [frame of the rendered camera sample, light id, target frame or -1]}} for the
enumerations ``pair``, ``unpair`` (4 lights, seed 999), ``limitedlights`` (4) and the
``singlelight`` mode (limitedlights, 1), on small synthetic frame lists.
Output: tests/golden/relight_index.json (data only).

Runs only in the build container (needs /root/reference, read-only).
Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_relight.py
"""
import json
import os
import sys
import tempfile
import types
from unittest import mock

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("MLI_REFERENCE", "/root/reference")
H = W = 4


def frame_lists():
    """Frame lists of the three dataset layouts the enumerations read."""
    # ReNe-style grid, 3 cameras x 4 lights, stored in a scrambled order (pair mode)
    order = [5, 0, 11, 3, 8, 1, 10, 6, 2, 9, 4, 7]
    pair = [dict(camera_index=k // 4, light_index=k % 4) for k in order]
    # synthetic sets: 7 frames, pl_index cycling over 4 light positions (limited lights)
    pl = [dict(pl_index=p) for p in (2, 0, 3, 1, 2, 0, 3)]
    # one light position for every frame (the singlelight mode's datasets)
    single = [dict(pl_index=0) for _ in range(5)]
    return dict(pair=pair, unpair=[dict() for _ in range(7)], limited=pl, single=single)


class FakeDataset:
    """Frame f: pose_light translation x = 100 + f, image = f; the attributes test_all_light uses."""

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
    def eval(self):
        return self

    def inference(self, data):
        frame = float(data["image"].flatten()[0])
        light = float(data["pose_light"][0, 0, 3])
        m1 = torch.zeros(1, 1, H, W)
        return dict(rgb_map=torch.full((1, 3, H, W), frame), normal_map=torch.full((1, 3, H, W), light),
                    visibility_map=m1, inter_dist_map=m1 + 1, inter_mask_map=m1, normal_x_light_map=m1)


def decode(results):
    out = {}
    for cam, lights in results.items():
        out[cam] = {}
        for li, r in lights.items():
            tgt = int(r["rgb_target"].flatten()[0]) if "rgb_target" in r else -1
            out[cam][li] = [int(r["rgb_render"].flatten()[0]), int(r["normal"].flatten()[0]) - 100, tgt]
    return out


def main():
    for n in ("wandb", "torchinfo", "termcolor", "cv2", "torchvision", "torchvision.transforms",
              "torchvision.transforms.functional", "torchvision.utils", "pynvml", "tinycudann", "apex",
              "apex.optimizers"):
        sys.modules[n] = mock.MagicMock(name=n)
    sys.path.insert(0, REF)
    import projects.NeuralLumen.trainer as T
    from projects.NeuralLumen.utils.utils import get_random_other_index

    fl = frame_lists()
    cases = [("pair", "pair", 4), ("unpair", "unpair", 4), ("limitedlights", "limited", 4),
             ("singlelight", "single", 1), ("singlelight_mixed", "limited", 1)]
    golden = {"H": H, "W": W, "frames": fl, "cases": {},
              "random_other_index": {"7_4_999": get_random_other_index(7, 4, 999),
                                     "5_3_0": get_random_other_index(5, 3, 0)}}
    for name, frames, sample_num in cases:
        ds = FakeDataset(fl[frames])
        loader = types.SimpleNamespace(dataset=ds)
        me = types.SimpleNamespace(
            cfg=types.SimpleNamespace(trainer=types.SimpleNamespace(ema_config=types.SimpleNamespace(enabled=False))),
            model=types.SimpleNamespace(module=FakeModel()), current_iteration=0,
            start_of_iteration=lambda data, current_iteration: data)
        dtype = {"pair": "pair", "unpair": "unpair"}.get(name, "limitedlights")
        with tempfile.TemporaryDirectory() as d:
            try:
                T.Trainer.test_all_light(me, loader, output_dir=d, mode="test", dataset_type=dtype,
                                         sample_num=sample_num, seed=999)
                res = decode(torch.load(os.path.join(d, "results_all.pt"), weights_only=True))
            except ValueError as e:   # a frame whose light is not among the first sample_num frames'
                res = {"error": type(e).__name__}
        golden["cases"][name] = dict(dataset_type=dtype, frames=frames, sample_num=sample_num, seed=999,
                                     results=res)
    path = os.path.join(HERE, "relight_index.json")
    with open(path, "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
