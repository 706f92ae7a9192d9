"""Debug helper: stored training activations (x0T, X1..X4) vs the oracle."""
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from test_gpu_parity import build, to_dev, DEV, fp16_table_sd  # noqa: E402
from oracle import render as o_render  # noqa: E402
model, sd, data, pcfg, (Hh, W) = build("syn_hotdog_b", 64, 64, 16, 4, 14, 6.0)
model.train()
u = torch.rand(1, 64, 64)
out = model(to_dev(data), u=u.to(DEV))
rays, dists, fld, hd, comp = model._last_state
torch.cuda.synchronize()
N, R = dists.shape
S = N * R
d_g = dists.t().cpu()[None, :, :, None]
c_g, v_g = rays["center"].cpu()[None], rays["ray_unit"].cpu()[None]
pts = c_g[..., None, :] + v_g[..., None, :] * d_g
sd16 = fp16_table_sd(sd)
_, feat = o_render.sdf_net(sd16, pcfg, pts, with_feat=True)      # [1,R,N,256]
feat_t = feat[0].reshape(S, 256).t()                              # [256, S] tile order m = r*N+k
from mli_nerf_amd import layout  # noqa: E402
x0T = layout.unfrag(hd["x0T"], 304).float().cpu()  # fragment image -> [304][S]
e = (x0T[:256] - feat_t).abs()
print("x0T feat rows: max err %.3e (max |feat| %.3e)" % (e.max(), feat_t.abs().max()))
p = pts[0].reshape(S, 3).t()
print("x0T p rows err %.3e" % (x0T[256:259] - p).abs().max())
g = fld["grad"].permute(1, 0, 2).cpu().reshape(S, 3)
nrm = F.normalize(g, dim=-1).t()
print("x0T n rows err %.3e" % (x0T[259:262] - nrm).abs().max())
print("x0T pad rows max %.3e" % x0T[262:272].abs().max())
light = o_render.sh16(rays["pts_light"].cpu()).repeat_interleave(N, 0).t()
view = o_render.sh16(v_g[0]).repeat_interleave(N, 0).t()
print("x0T light err %.3e view err %.3e" % ((x0T[272:288] - light).abs().max(), (x0T[288:304] - view).abs().max()))
# X1..X4 of head 0 from the oracle
xin = torch.cat([pts, o_render.sh16(v_g[..., None, :].expand_as(pts)), F.normalize(g.reshape(1, R, N, 3), dim=-1), feat,
                 o_render.sh16(rays["pts_light"].cpu()[None, :, None, :].expand_as(pts))], -1)[0].reshape(S, -1)
h = xin
for li in range(hd["xT"].shape[1]):
    pre = "neural_rgb.mlp.linears.%d" % li
    h = F.relu(F.linear(h, o_render.wn(sd, pre), sd[pre + ".bias"]))
    xg = layout.unfrag(hd["xT"][0, li], 256).float().cpu()
    print("head0 X%d err %.3e (max %.3e)" % (li + 1, (xg - h.t()).abs().max(), h.abs().max()))
torch.set_printoptions(precision=4, linewidth=200, sci_mode=False)
print("gpu x0T rows 256..263, samples 0..5:\n", x0T[256:264, :6])
print("gpu x0T rows 264..271, samples 0..5:\n", x0T[264:272, :6])
print("ref p rows:\n", p[:, :6])
print("ref n rows:\n", nrm[:, :6])
print("gpu light rows 272..275:\n", x0T[272:276, :6], "\nref\n", light[:4, :6])
