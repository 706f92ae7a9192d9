"""The training images the heads forward stores for the weight gradients (ABI 15 fragment images
``[S/32][k-steps][64][8]`` in ACC order: the x0 image -- 19 k-steps per tile -- and X1..X3, read
back through ``layout.unfrag``) against the oracle's activations at the same samples.

x0T rows: 0..255 the SDF feature (layer 1 of the SDF MLP, fp16 MFMA against the fp32 oracle:
4e-3 of its range), 256..258 the point, 259..261 the normal, 262..271 zero padding, 272..287 SH16
of the light position, 288..303 SH16 of the view direction -- fp16 roundings of fp32 values, so
within 2^-10 of their range.  X1..X3 (head 0, PQ mode stores X1..X3): the ReLU chain through
fp16 operands, 5e-3 of their range.  Layout errors would show as O(1) mismatches."""
import pytest
import torch
import torch.nn.functional as F

from margins import check
from oracle import render as o_render

pytestmark = pytest.mark.gpu


def test_stored_activations_match_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mli_nerf_amd import layout
    from test_gpu_parity import build, to_dev, DEV, fp16_table_sd
    model, sd, data, pcfg, _ = build("syn_hotdog_b", 64, 64, 16, 4, 14, 6.0)
    model.train()
    u = torch.rand(1, 64, 64, generator=torch.Generator().manual_seed(3))
    model(to_dev(data), u=u.to(DEV))
    rays, dists, fld, hd, _ = model._last_state
    torch.cuda.synchronize()
    N, R = dists.shape
    S = N * R
    d_g = dists.t().cpu()[None, :, :, None]
    c_g, v_g = rays["center"].cpu()[None], rays["ray_unit"].cpu()[None]
    pts = c_g[..., None, :] + v_g[..., None, :] * d_g
    _, feat = o_render.sdf_net(fp16_table_sd(sd), pcfg, pts, with_feat=True)   # [1, R, N, 256]
    x0T = layout.unfrag(hd["x0T"], layout.K0).float().cpu()                    # [304][S], tile order
    feat_t = feat[0].reshape(S, 256).t()
    check("x0T feat rows max abs / range", (x0T[:256] - feat_t).abs().max().item() / feat_t.abs().max().item(), 4e-3)
    p = pts[0].reshape(S, 3).t()
    check("x0T point rows max abs / range", (x0T[256:259] - p).abs().max().item() / p.abs().max().item(), 2.0 ** -10)
    g = fld["grad"].permute(1, 0, 2).cpu().reshape(S, 3)
    nrm = F.normalize(g, dim=-1).t()
    check("x0T normal rows max abs", (x0T[259:262] - nrm).abs().max().item(), 2.0 ** -10)
    check("x0T pad rows max abs", x0T[262:272].abs().max().item(), 0.0)
    light = o_render.sh16(rays["pts_light"].cpu()).repeat_interleave(N, 0).t()
    view = o_render.sh16(v_g[0]).repeat_interleave(N, 0).t()
    check("x0T light SH rows max abs / range", (x0T[272:288] - light).abs().max().item() / light.abs().max().item(),
          2.0 ** -10)
    check("x0T view SH rows max abs / range", (x0T[288:304] - view).abs().max().item() / view.abs().max().item(),
          2.0 ** -10)
    # head 0: X1..X3 from the oracle's ReLU chain on the same inputs
    xin = torch.cat([pts, o_render.sh16(v_g[..., None, :].expand_as(pts)),
                     F.normalize(g.reshape(1, R, N, 3), dim=-1), feat,
                     o_render.sh16(rays["pts_light"].cpu()[None, :, None, :].expand_as(pts))], -1)[0].reshape(S, -1)
    h = xin
    n_stored = hd["xT"].shape[1]
    assert n_stored == 3  # PQ mode: X4's contraction happens in registers
    for li in range(n_stored):
        pre = "neural_rgb.mlp.linears.%d" % li
        h = F.relu(F.linear(h, o_render.wn(sd, pre), sd[pre + ".bias"]))
        xg = layout.unfrag(hd["xT"][0, li], 256).float().cpu()
        check("head0 X%d max abs / range" % (li + 1), (xg - h.t()).abs().max().item() / h.abs().max().item(), 5e-3)

