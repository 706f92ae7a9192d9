"""Ray sharding across ranks for full-frame inference.

The reference renders every frame on one GPU in ``rand_rays_val`` chunks
(NeuralLumen/model.py:86-111, ray_generator.py:6-47).  Here a frame's H·W rays are split
into ``world`` contiguous row-major tiles, one per rank.  Every ray costs the same: each
gets exactly N samples, and outside rays get dummy bounds (neuralangelo/model.py:427-429).
So equal tiles are balanced.  The per-rank outputs (15 fp32 channels per ray) come back
with ONE all_gather (RCCL over xGMI on the node; gloo in the CPU tests).
"""
import math

import torch

# composited per-ray channels gathered for the maps: rgb 3, o_r 3, o_s 1, o_re 3,
# opacity 1, gradient 3, depth 1
CHANNELS = (("rgb", 3), ("o_r", 3), ("o_s", 1), ("o_re", 3), ("opacity", 1), ("gradient", 3), ("depth", 1))
N_CHANNELS = sum(c for _, c in CHANNELS)
# + light visibility (NeuralLumen/model.py:78-83) when enabled
VIS_CHANNELS = (("visibility", 1), ("normal_x_light", 1), ("pseudo_shading", 1), ("inter_dist", 1),
                ("inter_mask", 1))


def _channels(vis):
    return CHANNELS + (VIS_CHANNELS if vis else ())


def n_channels(vis=False):
    return sum(c for _, c in _channels(vis))


def shard_range(n, rank, world):
    """Contiguous tile [lo, hi) of n rays for `rank`; `per` = padded tile length."""
    per = math.ceil(n / world)
    lo = min(n, rank * per)
    return lo, min(n, lo + per), per


def pack(out, vis=False):
    """dict of [R, c] tensors -> [R, n_channels] fp32."""
    return torch.cat([out[k].reshape(out[k].shape[0], c).float() for k, c in _channels(vis)], dim=1)


def unpack(packed, vis=False):
    res, o = {}, 0
    for k, c in _channels(vis):
        res[k] = packed[:, o:o + c]
        o += c
    return res


def gather_tiles(local, n, world, group=None):
    """All ranks' [hi-lo, C] tiles -> the full [n, C] on every rank (one all_gather)."""
    import torch.distributed as dist
    per = math.ceil(n / world)
    buf = local.new_zeros(per, local.shape[1])
    buf[:local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat(parts, 0)[:n]
