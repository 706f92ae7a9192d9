"""Seeded synthetic inputs and random-init weights of the reference architecture.

There is no network and no dataset / trained checkpoint on the box, so parity tests and
the bench run on seeded synthetic data shaped as SURVEY.md §8(d) specifies:

* cameras: Blender-style look-at poses on a sphere of radius 4 (azimuth uniform,
  elevation 10-60 deg), ``camera_angle_x = 0.6911112`` (f = 711.11 px at 512^2), OpenGL ->
  OpenCV flip as ``projects/neuralangelo/data.py:143-146`` and w2c inversion as
  ``projects/NeuralLumen/data.py`` ``get_camera``;
* lights: ``pose_light`` = w2c of identity-R + translation on a sphere of radius 2.5-5
  (``projects/NeuralLumen/data_blender.py:28-47``);
* rays: ``randperm(H*W)[:R]`` (``projects/NeuralLumen/data.py:120``);
* labels: image / pseudo reflectance ~ U(0,1)^3, pseudo shading / certainty ~ U(0,1);
* weights: SDF MLP geometric init (``projects/neuralangelo/utils/mlp.py:71-84``) with the
  layer-0 encoding columns set to N(0, 1e-2) so the hash grid matters, hash table
  ~ U(-0.1, 0.1); RGB heads default ``nn.Linear`` init with zero last bias
  (``projects/nerf/utils/nerf_util.py:176-183``); weight-norm g = ||v||_row.

All generators are CPU ``torch.Generator`` streams, deterministic across machines.
"""
import math

import numpy as np
import torch

from .hashgrid import level_table, GRID_DEFAULTS

HEAD_SPECS = (("mlp", 294, 3), ("mlp_r", 262, 3), ("mlp_s", 278, 1))   # LumenRGB 'rgb_r_s'
HIDDEN = 256


def _gen(seed):
    g = torch.Generator()
    g.manual_seed(seed)
    return g


def _uniform(shape, lo, hi, g):
    return torch.rand(*shape, generator=g) * (hi - lo) + lo


def _weight_norm_pair(w):
    return w.norm(dim=1, keepdim=True), w.clone()


def make_state_dict(log2T=GRID_DEFAULTS["log2T"], seed=0, s_var=3.0, enc_std=1e-2, table_amp=0.1,
                    heads="rgb_r_s", out_bias=0.5, scale_rule="fp32"):
    """Reference state-dict keys (no DDP ``module.`` prefix) -> fp32 CPU tensors.
    ``heads``: LumenRGB network_mode -- 'rgb_r_s' (stage b, three heads) or 'rgb' (stage a,
    the single 294 -> 3 head, drawn first from the same stream, so it equals stage b's mlp)."""
    sd = {}
    table, total = level_table(log2T=log2T, scale_rule=scale_rule)
    g = _gen(seed * 100 + 5)
    sd["neural_sdf.tcnn_encoding.params"] = _uniform((total * 8,), -table_amp, table_amp, g)
    g = _gen(seed * 100 + 7)
    k_in = 3 + 16 * 8
    w0 = torch.randn(HIDDEN, k_in, generator=g) * math.sqrt(2.0 / HIDDEN)
    w0[:, 3:] = torch.randn(HIDDEN, k_in - 3, generator=g) * enc_std
    w1 = torch.randn(HIDDEN, HIDDEN, generator=g) * math.sqrt(2.0 / HIDDEN)
    for li, w in enumerate((w0, w1)):
        gnorm, v = _weight_norm_pair(w)
        sd["neural_sdf.mlp.linears.%d.weight_g" % li] = gnorm
        sd["neural_sdf.mlp.linears.%d.weight_v" % li] = v
        sd["neural_sdf.mlp.linears.%d.bias" % li] = torch.zeros(HIDDEN)
    sd["neural_sdf.mlp.linear_sdf.weight"] = (torch.randn(1, HIDDEN, generator=g) * 1e-4
                                              + math.sqrt(math.pi / HIDDEN))
    sd["neural_sdf.mlp.linear_sdf.bias"] = torch.full((1,), -float(out_bias))
    g = _gen(seed * 100 + 6)
    for name, k_in, k_out in (HEAD_SPECS[:1] if heads == "rgb" else HEAD_SPECS):
        dims = [k_in] + [HIDDEN] * 4 + [k_out]
        for li in range(5):
            fan_in, fan_out = dims[li], dims[li + 1]
            bound = 1.0 / math.sqrt(fan_in)
            w = _uniform((fan_out, fan_in), -bound, bound, g)
            b = _uniform((fan_out,), -bound, bound, g)
            if li == 4:
                b.zero_()
            gnorm, v = _weight_norm_pair(w)
            pre = "neural_rgb.%s.linears.%d" % (name, li)
            sd[pre + ".weight_g"], sd[pre + ".weight_v"], sd[pre + ".bias"] = gnorm, v, b
    sd["s_var"] = torch.tensor(float(s_var))
    return sd


def look_at_w2c(position):
    """Blender camera at ``position`` looking at the origin, z-up; returns w2c [3,4] in the
    OpenCV convention (projects/neuralangelo/data.py:143-146)."""
    c = np.asarray(position, dtype=np.float64)
    fwd = -c / np.linalg.norm(c)
    z = -fwd
    x = np.cross([0.0, 0.0, 1.0], z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    c2w_gl = np.eye(4)
    c2w_gl[:3, 0], c2w_gl[:3, 1], c2w_gl[:3, 2], c2w_gl[:3, 3] = x, y, z, c
    c2w = torch.tensor(c2w_gl, dtype=torch.float32) * torch.tensor([1.0, -1.0, -1.0, 1.0])
    return invert_pose(c2w[:3])


def invert_pose(pose):
    rot, trans = pose[..., :3], pose[..., 3:]
    rot_t = rot.transpose(-1, -2)
    return torch.cat([rot_t, -(rot_t @ trans)], dim=-1)


def camera_positions(n=100, radius=4.0, seed=0):
    rng = np.random.default_rng(seed)
    az = rng.uniform(0, 2 * np.pi, n)
    el = np.deg2rad(rng.uniform(10, 60, n))
    return np.stack([radius * np.cos(el) * np.cos(az), radius * np.cos(el) * np.sin(az),
                     radius * np.sin(el)], axis=-1)


def light_positions(n=100, seed=1):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    return d * rng.uniform(2.5, 5.0, (n, 1))


def intrinsics(H=512, W=512, camera_angle_x=0.6911112):
    focal = 0.5 * W / np.tan(0.5 * camera_angle_x)
    return torch.tensor([[focal, 0.0, W / 2.0], [0.0, focal, H / 2.0], [0.0, 0.0, 1.0]],
                        dtype=torch.float32)


def make_batch(n_rays, H=512, W=512, frame=0, seed=0, poses=None):
    """One per-rank training sample dict as ``projects/NeuralLumen/data.py:__getitem__``
    returns it, batch dim 1 added (B=1, ``syn_hotdog_b.yaml:38``)."""
    if poses is None:
        cam = camera_positions()[frame % 100]
        pose = look_at_w2c(cam)
        light = light_positions()[frame % 100]
        c2w_l = torch.eye(4) * torch.tensor([1.0, -1.0, -1.0, 1.0])
        c2w_l[:3, 3] = torch.tensor(light, dtype=torch.float32)
        pose_light = invert_pose(c2w_l[:3])
        intr = intrinsics(H, W)
    else:
        pose, pose_light, intr = poses
    g = _gen(seed * 1000 + 2 + 17 * frame)
    ray_idx = torch.randperm(H * W, generator=g)[:n_rays]
    g = _gen(seed * 1000 + 4 + 17 * frame)
    image = torch.rand(n_rays, 3, generator=g)
    ref = torch.rand(n_rays, 3, generator=g)
    sha = torch.rand(n_rays, 1, generator=g)
    cert = torch.rand(n_rays, 1, generator=g)
    return dict(idx=torch.tensor([frame]), pose=pose[None], intr=intr[None],
                pose_light=pose_light[None], ray_idx=ray_idx[None], image_sampled=image[None],
                pseudo_ref_sampled=ref[None], pseudo_sha_sampled=sha[None],
                pseudo_visibility_certainty_sampled=cert[None])


def stratified_uniforms(n_rays, n_coarse, seed=0):
    """The U[0,1) draws ``nerf_util.sample_dists`` makes (nerf_util.py:33), injected."""
    g = _gen(seed * 1000 + 3)
    return torch.rand(1, n_rays, n_coarse, generator=g)
