"""FIELD / sampling kernels alone at the bench shape (for rocprofv3 --pmc passes).

Usage (GPU box): rocprofv3 --pmc <counters> -- python tools/field_probe.py [--reps 5]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mli_nerf_amd import synthetic  # noqa: E402
from mli_nerf_amd.configs import preset  # noqa: E402
from mli_nerf_amd.model import Model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rays", type=int, default=4096)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
cfg = preset("syn_hotdog_b", rays=args.rays)
model = Model(cfg.model, cfg.data)
model.load_state_dict(synthetic.make_state_dict(log2T=22))
model = model.to("cuda:0")
model.train()
model.prepare()
eng = model.engine
batch = {k: v.to("cuda:0") for k, v in synthetic.make_batch(args.rays, frame=0).items()}
rays = eng.rays(batch["pose"], batch["intr"], batch["pose_light"], batch["ray_idx"], model.image_size_train[1])
for _ in range(args.reps):
    dists = eng.sample(rays)
    eng.field(rays, dists, True)
torch.cuda.synchronize()
print("ok")
