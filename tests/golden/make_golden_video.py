#!/usr/bin/env python
"""Golden vectors for the video helpers from the REFERENCE's own
``projects/NeuralLumen/utils/utils.py`` (``interpolate_pose`` :12-33, ``create_collage``
:177-199) and the frame-ratio expression of ``projects/nerf/trainers/base.py:297``.

Runs only in the build container (needs /root/reference, read-only).  ``cv2`` is absent and
only imported at module top by utils.py: replaced by an empty module (the two functions
used here never touch it).  Output: tests/golden/video_helpers.pt (tensors only, loaded
with weights_only=True).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_video.py
"""
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("MLI_REFERENCE", "/root/reference")


def poses():
    """Two w2c poses (camera and light) per end, from seeded rotations."""
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(4)
    out = []
    for _ in range(4):
        R = Rotation.from_rotvec(rng.normal(size=3) * 1.2).as_matrix().astype(np.float32)
        t = rng.normal(size=(3, 1)).astype(np.float32) * 2
        out.append(torch.from_numpy(np.concatenate([R, t], 1)))
    return out


def main():
    sys.modules["cv2"] = types.ModuleType("cv2")
    sys.path.insert(0, REF)
    from projects.NeuralLumen.utils import utils as U
    p = poses()
    n = 60
    ratios, cams, lights = [], [], []
    for i in range(n):
        ratio = torch.sin(torch.Tensor([((i / n) - 0.5) * torch.pi])) * 0.5 + 0.5   # base.py:297
        ratios.append(ratio)
        cams.append(U.interpolate_pose(p[0], p[1], ratio))
        lights.append(U.interpolate_pose(p[2], p[3], ratio))
    rng = np.random.default_rng(5)
    collages = {}
    for k in (1, 2, 3, 4, 5):
        tiles = [rng.integers(0, 256, (7, 9, 3), dtype=np.uint8) for _ in range(k)]
        collages[f"tiles_{k}"] = torch.from_numpy(np.stack(tiles))
        collages[f"collage_{k}"] = torch.from_numpy(U.create_collage(tiles))
    out = dict(pose_ends=torch.stack(p), ratios=torch.cat(ratios), cam=torch.stack(cams),
               light=torch.stack(lights), **collages)
    torch.save(out, os.path.join(HERE, "video_helpers.pt"))
    print("wrote video_helpers.pt", {k: tuple(v.shape) for k, v in out.items()})


if __name__ == "__main__":
    main()
