"""Oracle: fp32 PyTorch-CPU restatement of the MLI-NeRF stage-b hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Each function cites the
reference function it restates (paths relative to the MLI-NeRF checkout).  Weights are a
flat dict keyed by the reference state-dict names (without the DDP ``module.`` prefix).
"""
import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from oracle import hashgrid

SH_C = dict(
    c0=0.28209479177387814,
    c1=0.4886025119029199,
    c2=(1.0925484305920792, -1.0925484305920792, 0.31539156525252005,
        -1.0925484305920792, 0.5462742152960396),
    c3=(-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
        -0.4570457994644658, 1.445305721320277, -0.5900435899266435),
)

HEAD_NAMES = ("mlp", "mlp_r", "mlp_s")


@dataclass
class PathCfg:
    """The knobs of the hot path (defaults = syn_hotdog_b on neuralangelo/configs/base.yaml)."""
    n_coarse: int = 64              # base.yaml:107
    n_fine: int = 16                # base.yaml:108
    n_hier: int = 4                 # base.yaml:110
    white_bg: bool = True           # syn_hotdog_b.yaml:79
    bounding: str = "sphere"        # syn_hotdog_b.yaml:56 ("box" -> rene)
    aabb: tuple = (-1.0, -1.0, -1.0, 1.0, 1.0, 1.0)
    outside_val: float = 1000.0     # neuralangelo/model.py:38
    anneal_end: float = 0.1         # base.yaml:83
    levels: int = 16                # base.yaml:57-63
    log2T: int = 22
    min_logres: int = 5
    max_logres: int = 11
    vol_range: tuple = (-2.0, 2.0)
    loss_w: dict = field(default_factory=lambda: dict(
        render=1.0, eikonal=0.1, curvature=5e-4, intrinsic=1.0, regularize_re=1.0))
    intrinsic_ranges: tuple = ((0.0, 1.0), (0.0, 1.0))   # syn_hotdog_b.yaml:10-16
    re_factors: tuple = (10.0, 1.0, 1.0)                   # syn_hotdog_b.yaml:19-22
    rgb_mode: str = "rgb_r_s"       # LumenRGB network_mode; "rgb" = stage a (modules.py:50-55)
    active_levels: int = None       # coarse-to-fine mask (modules.py:91-113); None = all levels
    anneal_levels: int = None       # tap epsilon level (modules.py:102-107); None = all levels
    light_visibility: dict = None   # model.light_visibility when enabled (NeuralLumen/model.py:25-35)
    scale_rule: str = "fp32"        # hash-grid level scale rule (oracle/hashgrid.py level_table)

    @property
    def n_samples(self):
        return self.n_coarse + self.n_fine * self.n_hier

    def growth_rate(self):
        r_min, r_max = 2 ** self.min_logres, 2 ** self.max_logres
        return np.exp((np.log(r_max) - np.log(r_min)) / (self.levels - 1))

    def normal_eps(self):
        # neuralangelo/utils/modules.py:51-54 (resolutions) + :102-107 (c2f: resolution of
        # level anneal_levels - 1; disabled in stage b -> the finest level)
        g = self.growth_rate()
        res = [np.floor(2 ** self.min_logres * g ** lv).astype(int) + 1 for lv in range(self.levels)]
        lv = self.levels if self.anneal_levels is None else self.anneal_levels
        return 1.0 / res[lv - 1]

    def table(self):
        return hashgrid.level_table(self.levels, self.log2T, 2 ** self.min_logres, self.growth_rate(),
                                    scale_rule=self.scale_rule)


# --------------------------------------------------------------------------------------
# rays (projects/nerf/utils/camera.py, projects/NeuralLumen/utils/utils.py)
# --------------------------------------------------------------------------------------
def invert_pose(pose):
    """camera.py:46-52  [R|t] -> [R^T | -R^T t]."""
    rot, trans = pose[..., :3], pose[..., 3:]
    rot_t = rot.transpose(-1, -2)
    return torch.cat([rot_t, -(rot_t @ trans)], dim=-1)


def pixel_rays(pose, intr, ray_idx, width, height=None):
    """camera.py:283-311 get_center_and_ray over the FULL pixel grid, then
    nerf_util.py:127-131 slice_by_ray_idx (the gather is kept: computing only the sampled
    pixels changes BLAS blocking by an ulp, which the 4-tap normals amplify ~1e4x).
    pose [B,3,4] (w2c), intr [B,3,3], ray_idx [B,R] flat y*W+x -> center, ray [B,R,3]."""
    height = height or width
    ys = torch.arange(height, dtype=torch.float32).add_(0.5)
    xs = torch.arange(width, dtype=torch.float32).add_(0.5)
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    pix = torch.stack([gx, gy], dim=-1).view(-1, 2).repeat(pose.shape[0], 1, 1)
    hom = lambda v: torch.cat([v, torch.ones_like(v[..., :1])], dim=-1)  # noqa: E731
    cam = hom(pix) @ intr.inverse().transpose(-1, -2)                  # img2cam :259-260
    c2w_t = invert_pose(pose).transpose(-1, -2)                         # [B,4,3]
    world = hom(cam) @ c2w_t                                            # cam2world :263-266
    center = hom(torch.zeros_like(cam)) @ c2w_t
    ray = world - center
    bidx = torch.arange(pose.shape[0])[:, None].expand_as(ray_idx)
    return center[bidx, ray_idx], ray[bidx, ray_idx]


def light_points(pose_light, n_rays):
    """NeuralLumen/utils/utils.py:61-79 get_center: cam2world(0, pose_light) per ray."""
    c2w_t = invert_pose(pose_light).transpose(-1, -2)                   # [B,4,3]
    origin = torch.zeros(pose_light.shape[0], n_rays, 3)
    return torch.cat([origin, torch.ones_like(origin[..., :1])], dim=-1) @ c2w_t


def sphere_bounds(center, ray_unit, radius=1.0):
    """nerf_util.py:199-205 + neuralangelo/model.py:426-429."""
    ctc = (center * center).sum(-1, keepdim=True)
    ctv = (center * ray_unit).sum(-1, keepdim=True)
    disc = ctv ** 2 - (ctc - radius ** 2)
    near = (-ctv - disc.sqrt()).relu()
    far = -ctv + disc.sqrt()
    outside = near.isnan()
    near = torch.where(outside, torch.ones_like(near), near)
    far = torch.where(outside, torch.full_like(far, 1.2), far)
    return near, far, outside


def aabb_bounds(center, ray_unit, aabb):
    """NeuralLumen/utils/utils.py:86-123 (slab test) + neuralangelo/model.py:422-424."""
    box = torch.tensor(aabb, dtype=center.dtype)
    t0 = (box[:3] - center) / ray_unit
    t1 = (box[3:] - center) / ray_unit
    tmin = torch.minimum(t0, t1).amax(-1, keepdim=True).clamp(0, 1e10)
    tmax = torch.maximum(t0, t1).amin(-1, keepdim=True).clamp(0, 1e10)
    outside = tmax <= tmin
    near = torch.where(outside, torch.ones_like(tmin), tmin)
    far = torch.where(outside, torch.full_like(tmax, 1.2), tmax)
    return near, far, outside


# --------------------------------------------------------------------------------------
# neural SDF (projects/neuralangelo/utils/{modules,mlp}.py)
# --------------------------------------------------------------------------------------
# matmul operand precision: None = fp32, "tf32" = the reference's own GEMM arithmetic
# (imaginaire/trainers/base.py:172-178 sets torch.backends.cuda.matmul.allow_tf32): operands
# rounded to TF32's 10-bit mantissa, fp32 accumulate, in the forward and in both backward GEMMs.
MATMUL_OPERANDS = None


def tf32_round(x):
    """Round fp32 to TF32 (10-bit mantissa, fp32 exponent), nearest-even, as a value."""
    i = x.detach().contiguous().view(torch.int32)
    r = (i + 0x0FFF + ((i >> 13) & 1)) & ~0x1FFF
    return r.view(torch.float32)


class _Tf32Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        x2 = tf32_round(x.reshape(-1, x.shape[-1]))
        y = x2 @ tf32_round(w).t() + b
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        g2 = tf32_round(gy.reshape(-1, gy.shape[-1]))
        x2 = tf32_round(x.reshape(-1, x.shape[-1]))
        gx = (g2 @ tf32_round(w)).reshape(x.shape)
        return gx, g2.t() @ x2, gy.reshape(-1, gy.shape[-1]).sum(0)


def linear(x, w, b):
    """F.linear at the oracle's matmul precision (MATMUL_OPERANDS)."""
    if MATMUL_OPERANDS == "tf32":
        return _Tf32Linear.apply(x, w, b)
    return F.linear(x, w, b)


def wn(weights, prefix):
    """torch weight_norm(dim=0): W = g * v / ||v||_row (nerf_util.py:177-178, mlp.py:42-43)."""
    v, g = weights[prefix + ".weight_v"], weights[prefix + ".weight_g"]
    return torch._weight_norm(v, g, 0)


def softplus100(x):
    """misc.py:92-107 activ softplus with beta=100 (torch threshold 20)."""
    return F.softplus(x, beta=100)


def sdf_net(weights, cfg, pts, with_feat):
    """NeuralSDF.forward/encode (modules.py:68-95) + MLPforNeuralSDF.forward (mlp.py:55-69).
    pts [...,3] -> sdf [...,1], feat [...,256] | None."""
    shape = pts.shape[:-1]
    flat = pts.reshape(-1, 3)
    lo, hi = cfg.vol_range
    x01 = (flat - lo) / (hi - lo)
    table, _ = cfg.table()
    enc = hashgrid.encode(x01, weights["neural_sdf.tcnn_encoding.params"], table)
    if cfg.active_levels is not None:
        # coarse-to-fine mask (modules.py:91-93,110-113): levels >= active_levels -> 0
        mask = torch.zeros_like(enc)
        mask[..., :cfg.active_levels * 8] = 1
        enc = enc * mask
    inp = torch.cat([flat, enc], dim=-1)
    h0 = softplus100(linear(inp, wn(weights, "neural_sdf.mlp.linears.0"),
                              weights["neural_sdf.mlp.linears.0.bias"]))
    sdf = linear(h0, weights["neural_sdf.mlp.linear_sdf.weight"],
                   weights["neural_sdf.mlp.linear_sdf.bias"])
    feat = None
    if with_feat:
        feat = softplus100(linear(h0, wn(weights, "neural_sdf.mlp.linears.1"),
                                    weights["neural_sdf.mlp.linears.1.bias"]))
        feat = feat.reshape(*shape, -1)
    return sdf.reshape(*shape, 1), feat


def sdf_taps(weights, cfg, pts, sdf_center, training):
    """NeuralSDF.compute_gradients numerical taps=4 (modules.py:157-175)."""
    eps = cfg.normal_eps() / np.sqrt(3)
    ks = [torch.tensor(k, dtype=pts.dtype) for k in ((1, -1, -1), (-1, -1, 1), (-1, 1, -1), (1, 1, 1))]
    taps = [sdf_net(weights, cfg, pts + k * eps, with_feat=False)[0] for k in ks]
    grad = sum(k * s for k, s in zip(ks, taps)) / (4.0 * eps)
    hess = None
    if training:
        h = ((taps[0] + taps[1] + taps[2] + taps[3]) / 2.0 - 2 * sdf_center) / eps ** 2
        hess = torch.cat([h, h, h], dim=-1) / 3.0
    return grad, hess


# --------------------------------------------------------------------------------------
# sampling (projects/nerf/utils/nerf_util.py, projects/neuralangelo/model.py)
# --------------------------------------------------------------------------------------
def stratified_dists(near, far, n, u=None):
    """nerf_util.py:20-38 sample_dists; u [B,R,n] injected uniforms (None -> 0.5)."""
    if u is None:
        u = torch.full((*near.shape[:2], n), 0.5)
    t = (u + torch.arange(n, dtype=torch.float32)) / n
    return (t * (far - near) + near)[..., None]                       # [B,R,n,1]


def exclusive_transmittance_weights(alpha):
    """render.py:87-99 alpha_compositing_weights -> [B,R,N,1]."""
    shifted = torch.cat([torch.zeros_like(alpha[..., :1]), alpha[..., :-1]], dim=2)
    return (alpha * (1 - shifted).cumprod(dim=2))[..., None]


def inverse_cdf(bins, w, n_fine):
    """nerf_util.py:41-68 sample_dists_from_pdf (midpoint quantiles, searchsorted right)."""
    pdf = F.normalize(w, p=1, dim=-1)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), pdf.cumsum(-1)], dim=-1)
    grid = torch.linspace(0, 1, n_fine + 1)
    u = (0.5 * (grid[:-1] + grid[1:])).repeat(*cdf.shape[:-1], 1)
    idx = torch.searchsorted(cdf, u, right=True)
    lo = (idx - 1).clamp(min=0)
    hi = idx.clamp(max=cdf.shape[-1] - 1)
    b = bins[..., 0]
    d0, d1 = b.gather(2, lo), b.gather(2, hi)
    c0, c1 = cdf.gather(2, lo), cdf.gather(2, hi)
    t = (u - c0) / (c1 - c0 + 1e-8)
    return (d0 + t * (d1 - d0))[..., None]


def section_pdf_samples(dists, sdfs, inv_s, n_fine):
    """neuralangelo/model.py:467-484 sample_dists_hierarchical (robust=True)."""
    s = sdfs[..., 0]
    d = dists[..., 0]
    ds = d[..., 1:] - d[..., :-1]
    mid = (s[..., :-1] + s[..., 1:]) * 0.5
    cos = (s[..., 1:] - s[..., :-1]) / (ds + 1e-5)
    prev = torch.cat([torch.zeros_like(cos[..., :1]), cos[..., :-1]], dim=-1)
    cos = torch.minimum(prev, cos)
    cdf_prev = ((mid - cos * ds * 0.5) * inv_s).sigmoid()
    cdf_next = ((mid + cos * ds * 0.5) * inv_s).sigmoid()
    alpha = ((cdf_prev - cdf_next) / (cdf_prev + 1e-5)).clip(0.0, 1.0)
    w = exclusive_transmittance_weights(alpha)
    return inverse_cdf(dists, w[..., 0], n_fine)


@torch.no_grad()
def hierarchical_dists(weights, cfg, center, ray_unit, near, far, u=None):
    """neuralangelo/model.py:449-465 sample_dists_all."""
    dists = stratified_dists(near, far, cfg.n_coarse, u)
    pts = center[..., None, :] + ray_unit[..., None, :] * dists
    sdfs = sdf_net(weights, cfg, pts, with_feat=False)[0]
    for h in range(cfg.n_hier):
        fine = section_pdf_samples(dists, sdfs, 64 * 2 ** h, cfg.n_fine)
        dists, order = torch.cat([dists, fine], dim=2).sort(dim=2)
        if h != cfg.n_hier - 1:
            pts = center[..., None, :] + ray_unit[..., None, :] * fine
            s_fine = sdf_net(weights, cfg, pts, with_feat=False)[0]
            sdfs = torch.cat([sdfs, s_fine], dim=2).gather(2, order)
    return dists


# --------------------------------------------------------------------------------------
# light-conditioned colour heads (projects/NeuralLumen/utils/modules.py)
# --------------------------------------------------------------------------------------
def sh16(v):
    """spherical_harmonics.py:47-84, levels=3 -> 16 coefficients."""
    x, y, z = v.unbind(-1)
    xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
    c1, c2, c3 = SH_C["c1"], SH_C["c2"], SH_C["c3"]
    cols = [
        torch.full_like(x, SH_C["c0"]),
        -c1 * y, c1 * z, -c1 * x,
        c2[0] * xy, c2[1] * yz, c2[2] * (2.0 * zz - xx - yy), c2[3] * xz, c2[4] * (xx - yy),
        c3[0] * y * (3 * xx - yy), c3[1] * xy * z, c3[2] * y * (4 * zz - xx - yy),
        c3[3] * z * (2 * zz - 3 * xx - 3 * yy), c3[4] * x * (4 * zz - xx - yy),
        c3[5] * z * (xx - yy), c3[6] * x * (xx - 3 * yy),
    ]
    return torch.stack(cols, dim=-1)


def head_mlp(weights, name, x):
    """MLPwithSkipConnection.forward (nerf_util.py:186-196): 4x(Linear+ReLU), Linear."""
    h = x
    for li in range(5):
        pre = "neural_rgb.%s.linears.%d" % (name, li)
        h = linear(h, wn(weights, pre), weights[pre + ".bias"])
        if li < 4:
            h = F.relu(h)
    return h


def rgb_heads(weights, pts, normals, rays_unit, feats, pts_light, mode="rgb_r_s"):
    """LumenRGB.forward, network_mode 'rgb_r_s' (NeuralLumen/utils/modules.py:106-163), or
    the single-head mode 'rgb' of stage a (:164-174, same input order as 'mlp').
    Quirk kept: SH of the raw (un-normalised) light position (:109)."""
    view = sh16(rays_unit)
    light = sh16(pts_light)
    x_rgb = torch.cat([pts, view, normals, feats, light], dim=-1)
    if mode == "rgb":
        return head_mlp(weights, "mlp", x_rgb).sigmoid(), None, None
    x_r = torch.cat([pts, normals, feats], dim=-1)
    x_s = torch.cat([pts, normals, feats, light], dim=-1)
    return (head_mlp(weights, "mlp", x_rgb).sigmoid(),
            head_mlp(weights, "mlp_r", x_r).sigmoid(),
            head_mlp(weights, "mlp_s", x_s).sigmoid())


# --------------------------------------------------------------------------------------
# NeuS alphas + compositing (neuralangelo/model.py, nerf/utils/render.py, NeuralLumen/model.py)
# --------------------------------------------------------------------------------------
def neus_alphas(s_var, ray_unit, sdfs, grads, dists, far, progress, anneal_end):
    """neuralangelo/model.py:492-515 compute_neus_alphas + _get_iter_cos."""
    s = sdfs[..., 0]
    inv_s = s_var.exp()
    cos = (ray_unit[..., None, :] * grads).sum(-1)
    a = min(progress / anneal_end, 1.0)
    iter_cos = -((-cos * 0.5 + 0.5).relu() * (1.0 - a) + (-cos).relu() * a)
    d = torch.cat([dists, far[..., None]], dim=2)[..., 0]
    step = d[..., 1:] - d[..., :-1]
    cdf_prev = ((s - iter_cos * step * 0.5) * inv_s).sigmoid()
    cdf_next = ((s + iter_cos * step * 0.5) * inv_s).sigmoid()
    return ((cdf_prev - cdf_next) / (cdf_prev + 1e-5)).clip(0.0, 1.0)


def render_rays(weights, cfg, center, ray_unit, pts_light, u=None, training=True, progress=0.0,
                dists=None, geometry=None, geometry_st=None):
    """NeuralLumen/model.py:232-336 render_rays_lumen + :338-403 render_rays_object_lumen,
    network_mode 'rgb_r_s', no background NeRF, no light visibility.  ``dists`` (test hook)
    replaces the hierarchical sampler's output, to condition downstream comparisons;
    ``geometry`` (test hook, with ``dists``) replaces the SDF network's outputs at those samples
    -- dict(sdfs [B,R,N,1] (outside already overwritten), grads [B,R,N,3], feats [B,R,N,256],
    hess or None) -- so that only the heads, the compositing and the losses are the oracle's.
    ``geometry_st`` (test hook, same keys): the forward VALUES of the SDF network's outputs are
    the given ones, the backward runs through the oracle's own graph (straight-through,
    v + (given - v).detach()): the stage-a gradients conditioned on another forward's geometry."""
    with torch.no_grad():
        if cfg.bounding == "box":
            near, far, outside = aabb_bounds(center, ray_unit, cfg.aabb)
        else:
            near, far, outside = sphere_bounds(center, ray_unit)
        if dists is None:
            dists = hierarchical_dists(weights, cfg, center, ray_unit, near, far, u)
    pts = center[..., None, :] + ray_unit[..., None, :] * dists
    if geometry is None:
        sdfs, feats = sdf_net(weights, cfg, pts, with_feat=True)
        sdfs = torch.where(outside[..., None].expand_as(sdfs), torch.full_like(sdfs, cfg.outside_val), sdfs)
        grads, hess = sdf_taps(weights, cfg, pts, sdfs, training)
        if geometry_st is not None:
            st = lambda v, g: v + (g.to(v.dtype) - v).detach()   # noqa: E731
            sdfs, grads, feats = st(sdfs, geometry_st["sdfs"]), st(grads, geometry_st["grads"]), \
                st(feats, geometry_st["feats"])
            if hess is not None and geometry_st.get("hess") is not None:
                hess = st(hess, geometry_st["hess"])
    else:
        sdfs, grads, feats, hess = geometry["sdfs"], geometry["grads"], geometry["feats"], geometry.get("hess")
    normals = F.normalize(grads, dim=-1)
    rays_n = ray_unit[..., None, :].expand_as(pts)
    light_n = pts_light[..., None, :].expand_as(pts)
    rgbs, o_r, o_s = rgb_heads(weights, pts, normals, rays_n, feats, light_n, cfg.rgb_mode)
    alphas = neus_alphas(weights["s_var"], ray_unit, sdfs, grads, dists, far, progress, cfg.anneal_end)
    w = exclusive_transmittance_weights(alphas)
    rgb = (rgbs * w).sum(2)
    opacity = w.sum(2)
    if cfg.rgb_mode == "rgb":  # NeuralLumen/model.py:300-303
        acc_r = acc_s = o_re = None
        if cfg.white_bg:
            rgb = rgb + (1 - opacity)
    else:
        acc_r = (o_r * w).sum(2)
        acc_s = (o_s * w).sum(2)
        if cfg.white_bg:
            rgb, acc_r, acc_s = rgb + (1 - opacity), acc_r + (1 - opacity), acc_s + (1 - opacity)
        o_re = rgb - acc_r * acc_s
    out = dict(rgb=rgb, o_r=acc_r, o_s=acc_s, o_re=o_re,
               outside=outside, dists=dists, weights=w, gradients=grads, hessians=hess,
               sdfs=sdfs, alphas=alphas, rgbs=rgbs, rgbs_r=o_r, rgbs_s=o_s,
               opacity=None, gradient=None)
    if not training:
        out["opacity"] = opacity
        out["gradient"] = (grads * w).sum(2)
    return out


# --------------------------------------------------------------------------------------
# light visibility for the pseudo labels (NeuralLumen/model.py:133-184, test_all_light)
# --------------------------------------------------------------------------------------
def sphere_trace(weights, cfg, center, ray_unit, near, far, iters=20, dist_start=None):
    """neuralangelo/model.py:298-325 sphere_tracing_intersection (the SDF network's forward:
    no outside overwrite).  center/ray_unit [B,R,3], near/far/dist_start [B,R,1]."""
    dist = near.clone() if dist_start is None else dist_start.clone()
    mask = torch.ones_like(dist, dtype=torch.bool)
    for _ in range(iters):
        pts = center + ray_unit * dist
        sdfs = sdf_net(weights, cfg, pts, with_feat=False)[0]
        dist[mask] += sdfs[mask]
        mask[dist > far] = False
        mask[dist < near] = False
    dist = torch.clamp(dist, near, far)
    return dist, center + ray_unit * dist, mask


def light_visibility(weights, cfg, vis, center, ray_unit, pts_light, near, far, out):
    """NeuralLumen/model.py:133-184 get_light_visibility, method 'sphere_tracing' (the one the
    configs use), camera ray types blend_z_sphere_tracing / blend_z / sphere_tracing; visibility
    bounds :186-199 (box: the model's bounding_box_aabb, as the reference reads it).
    ``vis``: dict(camera_ray_type, bounding, radius, aabb, gamma)."""
    with torch.no_grad():
        kind = vis["camera_ray_type"]
        blend = (out["dists"] * out["weights"]).sum(2)                       # render.composite
        if kind == "blend_z_sphere_tracing":
            inter_dist, inter_pts, inter_mask = sphere_trace(weights, cfg, center, ray_unit, near, far,
                                                             dist_start=blend)
        elif kind == "blend_z":
            inter_dist = blend
            inter_pts = center + ray_unit * inter_dist
            inter_mask = inter_dist > 0.0
        elif kind == "sphere_tracing":
            inter_dist, inter_pts, inter_mask = sphere_trace(weights, cfg, center, ray_unit, near, far)
        else:
            raise NotImplementedError(kind)
        light_ray = inter_pts - pts_light
        light_unit = F.normalize(light_ray, dim=-1)
        if vis["bounding"] == "box":
            near_l, far_l, outside_l = aabb_bounds(pts_light, light_unit, vis["aabb"])
        else:
            near_l, far_l, outside_l = sphere_bounds(pts_light, light_unit, vis["radius"])
        far_t = light_ray.norm(dim=-1, keepdim=True) - 1e-3
        inside = (near_l < far_t) & (far_t < far_l) & ~outside_l
        _, _, mask_l = sphere_trace(weights, cfg, pts_light, light_unit, near_l, far_t)
        visibility = (~mask_l) | (~inside)
        normal = F.normalize(-out["gradient"], dim=-1)
        nxl = (normal * light_unit).sum(dim=-1, keepdim=True).relu()
        shading = nxl * visibility.float()
        if vis.get("gamma"):
            shading = torch.pow(shading, 1.0 / vis["gamma"])
    return dict(visibility=visibility, normal_x_light=nxl, pseudo_shading=shading, inter_dist=inter_dist,
                inter_mask=inter_mask)


def forward(weights, cfg, data, u=None, training=True, progress=0.0, width=512, height=None, dists=None,
            geometry=None, geometry_st=None):
    """NeuralLumen/model.py:113-131 Model.forward -> render_pixels_lumen."""
    height = height or width
    center, ray = pixel_rays(data["pose"], data["intr"], data["ray_idx"], width, height)
    ray_unit = F.normalize(ray, dim=-1)
    pts_light = light_points(data["pose_light"], height * width)
    bidx = torch.arange(ray.shape[0])[:, None].expand_as(data["ray_idx"])
    pts_light = pts_light[bidx, data["ray_idx"]]
    out = render_rays(weights, cfg, center, ray_unit, pts_light, u, training, progress, dists, geometry,
                      geometry_st)
    vis = getattr(cfg, "light_visibility", None)
    if vis and not training:  # NeuralLumen/model.py:325-336 (flag_light_visibility)
        if cfg.bounding == "box":
            near, far, _ = aabb_bounds(center, F.normalize(ray, dim=-1), cfg.aabb)
        else:
            near, far, _ = sphere_bounds(center, F.normalize(ray, dim=-1))
        out.update(light_visibility(weights, cfg, vis, center, F.normalize(ray, dim=-1), pts_light, near, far,
                                    out))
    return out


# --------------------------------------------------------------------------------------
# stage-b losses (NeuralLumen/trainer.py:133-149, utils.py:142-174, neuralangelo misc.py:74-90)
# --------------------------------------------------------------------------------------
def intrinsic_loss(o_r, o_s, ref, sha, cert, ranges, factors=(1.0, 1.0)):
    def rescale(x, lo, hi):
        return lo + (x - x.min()) / torch.clamp(x.max() - x.min(), min=1e-6) * (hi - lo)
    w_sha = rescale(sha.detach(), *ranges[0])
    w_vis = rescale(cert.detach(), *ranges[1])
    w_ref = torch.minimum(w_vis, w_sha)
    l_ref = (torch.abs(o_r - ref) * w_ref).mean()
    l_sha = (torch.abs(o_s - sha) * w_sha).mean()
    return l_ref * factors[0] + l_sha * factors[1]


def residual_loss(o_re, f_neg, f_pos, e_pos):
    neg = torch.where(o_re < 0.0, o_re, torch.zeros_like(o_re))
    pos = torch.where(o_re >= 0.0, o_re, torch.zeros_like(o_re))
    return torch.abs(neg).mean() * f_neg + torch.pow(pos, e_pos).mean() * f_pos


def stage_b_losses(out, data, cfg):
    mask = (~out["outside"]).float()
    g_err = ((out["gradients"].norm(dim=-1) - 1.0) ** 2).nan_to_num(nan=0.0, posinf=0.0, neginf=0.0)
    lap = out["hessians"].sum(-1).abs().nan_to_num(nan=0.0, posinf=0.0, neginf=0.0)
    losses = dict(
        render=F.l1_loss(out["rgb"], data["image_sampled"]) * 3,
        eikonal=(g_err * mask).mean(),
        curvature=(lap * mask).mean(),
        intrinsic=intrinsic_loss(out["o_r"], out["o_s"], data["pseudo_ref_sampled"],
                                 data["pseudo_sha_sampled"],
                                 data["pseudo_visibility_certainty_sampled"], cfg.intrinsic_ranges),
        regularize_re=residual_loss(out["o_re"], *cfg.re_factors),
    )
    total = sum(losses[k] * cfg.loss_w[k] for k in cfg.loss_w)
    psnr = -10 * torch.log10(F.mse_loss(out["rgb"], data["image_sampled"]))
    return total, losses, psnr


def stage_a_losses(out, data, curvature_weight, eikonal_weight=0.1, render_weight=1.0):
    """Stage-a loss (NeuralLumen/trainer.py:133-141 without the intrinsic terms; weights
    base.yaml:28-31, the curvature weight scheduled by neuralangelo/trainer.py:56-63)."""
    mask = (~out["outside"]).float()
    g_err = ((out["gradients"].norm(dim=-1) - 1.0) ** 2).nan_to_num(nan=0.0, posinf=0.0, neginf=0.0)
    lap = out["hessians"].sum(-1).abs().nan_to_num(nan=0.0, posinf=0.0, neginf=0.0)
    losses = dict(render=F.l1_loss(out["rgb"], data["image_sampled"]) * 3,
                  eikonal=(g_err * mask).mean(), curvature=(lap * mask).mean())
    w = dict(render=render_weight, eikonal=eikonal_weight, curvature=curvature_weight)
    total = sum(losses[k] * w[k] for k in losses)
    psnr = -10 * torch.log10(F.mse_loss(out["rgb"], data["image_sampled"]))
    return total, losses, psnr


def stage_a_param_names(levels=16):
    """Every parameter is trained in stage a (no partial_grad; get_param_groups returns
    self.parameters(), NeuralLumen/model.py:422-438)."""
    names = ["neural_sdf.tcnn_encoding.params"]
    for li in range(2):
        names += ["neural_sdf.mlp.linears.%d.%s" % (li, p) for p in ("weight_g", "weight_v", "bias")]
    names += ["neural_sdf.mlp.linear_sdf.weight", "neural_sdf.mlp.linear_sdf.bias"]
    for li in range(5):
        names += ["neural_rgb.mlp.linears.%d.%s" % (li, p) for p in ("weight_g", "weight_v", "bias")]
    return names + ["s_var"]


def head_param_names():
    """Trainable stage-b parameters (NeuralLumen/trainer.py:44-54 partial_grad neural_rgb)."""
    names = []
    for h in HEAD_NAMES:
        for li in range(5):
            for p in ("weight_g", "weight_v", "bias"):
                names.append("neural_rgb.%s.linears.%d.%s" % (h, li, p))
    return names
