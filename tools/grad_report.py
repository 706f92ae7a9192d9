"""Debug helper: per-tensor gradient agreement GPU vs oracle for one small case."""
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from test_gpu_parity import build, to_dev, DEV, fp16_table_sd, _gpu_total  # noqa: E402
from oracle import render as o_render  # noqa: E402
model, sd, data, pcfg, (Hh, W) = build("syn_hotdog_b", 64, 64, 16, 4, 14, 6.0)
model.train()
u = torch.rand(1, 64, 64)
out = model(to_dev(data), u=u.to(DEV))
_gpu_total(out, to_dev(data), pcfg).backward()
g_flat = model.flat.grad.detach().cpu()
sd_o = {k: v.clone().requires_grad_(k.startswith("neural_rgb")) for k, v in fp16_table_sd(sd).items()}
o_out = o_render.forward(sd_o, pcfg, data, u=u, training=True, progress=0.0, width=W, height=Hh)
o_render.stage_b_losses(o_out, data, pcfg)[0].backward()
for name, shape, off in model.engine.tlayout:
    n = int(np.prod(shape))
    g = g_flat[off:off + n].view(*shape)
    o = sd_o[name].grad
    cos = F.cosine_similarity(g.flatten(), o.flatten(), dim=0).item()
    print("%-40s cos %8.5f  |g| %.3e |o| %.3e" % (name, cos, g.norm(), o.norm()))
    if name.endswith("linears.0.weight_v"):
        # per reference column block agreement
        for a, b in ((0, 3), (3, 19), (19, 22), (22, 278), (278, shape[1])):
            if b <= shape[1] and a < b:
                cc = F.cosine_similarity(g[:, a:b].flatten(), o[:, a:b].flatten(), dim=0).item()
                print("      cols %3d..%3d cos %.4f" % (a, b, cc))
