"""Debug helper: per-tensor gradient agreement GPU vs oracle (conditioned on the GPU samples).
python tools/grad_report.py [small|config2]"""
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from oracle import render as o_render  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "small"
if case == "small":
    from test_gpu_parity import build, to_dev, DEV, fp16_table_sd, _gpu_total  # noqa: E402
    model, sd, data, pcfg, (Hh, W) = build("syn_hotdog_b", 64, 64, 16, 4, 14, 6.0)
    sd16 = fp16_table_sd(sd)
    model.train()
    u = torch.rand(1, 64, 64)
    out = model(to_dev(data), u=u.to(DEV))
    _gpu_total(out, to_dev(data), pcfg).backward()
    loss_o = lambda o: o_render.stage_b_losses(o, data, pcfg)[0]  # noqa: E731
else:
    from test_gpu_fullsize import _setup, _subset, DEV  # noqa: E402
    cfg, model, sd16, data, pcfg, (Hh, W) = _setup("syn_hotdog_b", 4096, 16)
    idx = torch.arange(0, 4096, 16)
    data = _subset(data, idx)
    u = torch.rand(1, 4096, 64, generator=torch.Generator().manual_seed(7))[:, idx]
    model.train()
    out = model({k: v.to(DEV) for k, v in data.items()}, u=u.to(DEV))
    (F.l1_loss(out["rgb"], data["image_sampled"].to(DEV)) * 3).backward()
    loss_o = lambda o: F.l1_loss(o["rgb"], data["image_sampled"]) * 3  # noqa: E731
g_flat = model.flat_grad_from_params().detach().cpu()
sd_o = {k: v.clone().requires_grad_(k.startswith("neural_rgb")) for k, v in sd16.items()}
o_out = o_render.forward(sd_o, pcfg, data, u=u, training=True, progress=0.0, width=W, height=Hh,
                         dists=out["dists"].detach().cpu())
loss_o(o_out).backward()
for name, shape, off in model._layout_items():
    n = int(np.prod(shape))
    g = g_flat[off:off + n].view(*shape)
    o = sd_o[name].grad
    if o is None or o.norm() == 0:
        print("%-40s (no oracle gradient)  |g| %.3e" % (name, g.norm()))
        continue
    cos = F.cosine_similarity(g.flatten(), o.flatten(), dim=0).item()
    rel = ((g - o).norm() / o.norm()).item()
    print("%-40s cos %8.5f rel %.3e  |g| %.3e |o| %.3e" % (name, cos, rel, g.norm(), o.norm()))
