"""Dump one FIELD pass (encoding image, sdf, grad, h0) at a fixed seed, for bitwise A/B of two
library builds: python tools/r4/field_dump.py out.pt  (MLI_HIP_LIB picks the build)."""
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, HERE)
import torch  # noqa: E402
from mli_nerf_amd import synthetic  # noqa: E402
from mli_nerf_amd.configs import preset  # noqa: E402
from mli_nerf_amd.model import Model  # noqa: E402

DEV = "cuda:0"
out = {}
for config, R, active in (("syn_hotdog_b", 4096, 16), ("syn_hotdog_a", 1024, 11)):
    cfg = preset(config, rays=R)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22, heads="rgb" if config.endswith("_a") else "rgb_r_s"))
    model = model.to(DEV)
    model.train()
    model.prepare()
    eng = model.engine
    eng.active_levels = active
    data = {k: v.to(DEV) for k, v in synthetic.make_batch(R, frame=3).items()}
    rays = eng.rays(data["pose"], data["intr"], data["pose_light"], data["ray_idx"], cfg.data.train.image_size[1])
    dists = eng.sample(rays)
    fld = eng.field(rays, dists, True)
    torch.cuda.synchronize()
    for k in ("enc", "sdf", "grad", "h0"):
        out["%s/%s" % (config, k)] = fld[k].cpu().clone()
    out["%s/dists" % config] = dists.cpu().clone()
torch.save(out, sys.argv[1])
print("saved", sys.argv[1])
