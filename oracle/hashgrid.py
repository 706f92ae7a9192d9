"""Oracle restatement of the tiny-cuda-nn ``HashGrid`` encoding (TEST INFRASTRUCTURE ONLY).

Call sites in the reference: ``projects/neuralangelo/utils/modules.py:42-50`` (config:
16 levels x 8 features, log2 T = 22, base resolution 2**5, per-level scale
exp((ln 2**11 - ln 2**5)/15)) and ``:83-86`` (input ``(p + 2) / 4`` in [0,1]).

tiny-cuda-nn is third-party (NVlabs/tiny-cuda-nn, ``bindings/torch``), not vendored
and not version-pinned by the reference: the values here are **parity unpinned**
against real tcnn.  Restated published algorithm (tcnn ``encodings/grid.h``):

* level scale  ``s_l = exp2(l * log2(per_level_scale)) * base - 1``   (float32)
* resolution   ``res_l = ceil(s_l) + 1``
* level size   ``T_l = min(next_multiple(res_l**3, 8), 2**log2T)``; offsets are the
  running sum of ``T_l`` (entries), params flat ``[(offset_l + idx) * 8 + f]``.
* position     ``pos = fmaf(s_l, x, 0.5)``, ``g = floor(pos)`` (as uint32), ``f = pos - g``
* index        dense ``gx + gy*res + gz*res^2`` while the stride stays <= T_l, else the
  coherent prime hash ``gx ^ gy*2654435761 ^ gz*805459861`` (uint32), finally ``% T_l``.
* value        trilinear: corner ``c`` (bit d set -> +1 along d) weight
  ``prod_d (f_d if bit else 1 - f_d)``; output level-major ``[n, L*8]``.

tcnn accumulates the 8 corners in fp16; this oracle keeps everything in fp32 (the fp32
reference the build's tolerance is stated against).
"""
import numpy as np
import torch

PRIMES = (1, 2654435761, 805459861)
MASK32 = 0xFFFFFFFF


def level_table(n_levels=16, log2T=22, base_res=32, per_level_scale=None, scale_rule="fp32"):
    """Return a list of (scale(float32), res, size, offset) per level + total entries.
    ``scale_rule='exact'``: the level scale in float64, rounded to fp32 once (the alternative
    the build accepts for checkpoints whose table size implies a level-5 resolution of 128)."""
    if per_level_scale is None:
        per_level_scale = np.exp((np.log(2.0 ** 11) - np.log(2.0 ** 5)) / (n_levels - 1))
    log2_pls = np.float32(np.log2(np.float32(per_level_scale)))
    table, offset = [], 0
    for lv in range(n_levels):
        if scale_rule == "exact":
            e = lv * np.log2(float(per_level_scale))
            scale = np.float32(base_res * 2.0 ** (round(e) if abs(e - round(e)) < 1e-9 else e) - 1.0)
        else:
            scale = np.float32(np.exp2(np.float32(lv) * log2_pls)) * np.float32(base_res) - np.float32(1.0)
            scale = np.float32(scale)
        res = int(np.ceil(scale)) + 1
        dense = res ** 3
        size = min(((dense + 7) // 8) * 8, 1 << log2T)
        table.append((float(scale), res, size, offset))
        offset += size
    return table, offset


def _mul32(a, b):
    """(a * b) mod 2**32 for int64 tensors a < 2**32 and a python int b < 2**32, without
    relying on int64 overflow wrap-around."""
    b_lo, b_hi = b & 0xFFFF, b >> 16
    return (a * b_lo + (((a * b_hi) & 0xFFFF) << 16)) & MASK32


def _corner_index(gx, gy, gz, res, size):
    """uint32 tcnn grid_index on int64 tensors holding uint32 values."""
    stride, index = 1, torch.zeros_like(gx)
    hashed = False
    for g in (gx, gy, gz):
        if stride > size:
            hashed = True
            break
        index = (index + g * stride) & MASK32
        stride *= res
    if stride > size:
        hashed = True
    if hashed:
        index = _mul32(gx, PRIMES[0]) ^ _mul32(gy, PRIMES[1]) ^ _mul32(gz, PRIMES[2])
    return index % size


_CORNER_BITS = torch.tensor([[(c >> d) & 1 for d in range(3)] for c in range(8)], dtype=torch.int64)


class _Encode(torch.autograd.Function):
    """The encoding with an explicit backward w.r.t. the table (tcnn's kernel_grid_backward:
    every corner receives weight * d output, summed): one dense gradient per call built with
    index_add_, instead of autograd's per-gather dense zero tensors (which make a stage-a
    backward over the 1.46 GB table take minutes per step on the CPU)."""

    @staticmethod
    def forward(ctx, x01, params, table, n_feat):
        out, cache = _encode_fwd(x01, params, table, n_feat)
        ctx.cache, ctx.n_params, ctx.n_feat = cache, params.numel(), n_feat
        return out

    @staticmethod
    def backward(ctx, grad_out):
        grid = torch.zeros(ctx.n_params // ctx.n_feat, ctx.n_feat, dtype=grad_out.dtype)
        f = ctx.n_feat
        for lv, (rows, w) in enumerate(ctx.cache):
            g = grad_out[:, lv * f:(lv + 1) * f]
            for c in range(8):
                grid.index_add_(0, rows[:, c], w[c][:, None] * g)
        ctx.cache = None
        return None, grid.view(-1), None, None


def encode(x01, params, table, n_feat=8):
    """x01 [n,3] float32 in (roughly) [0,1]; params flat float32 -> [n, L*n_feat] float32."""
    if params.requires_grad and torch.is_grad_enabled():
        return _Encode.apply(x01, params, table, n_feat)
    return _encode_fwd(x01, params, table, n_feat)[0]


def _encode_fwd(x01, params, table, n_feat):
    x01 = x01.to(torch.float32)
    n = x01.shape[0]
    grid = params.view(-1, n_feat)
    outs, cache = [], []
    xd = x01.to(torch.float64)
    for scale, res, size, offset in table:
        # fmaf(scale, x, 0.5): exact product+add in float64, one rounding to float32.
        pos = (xd * float(scale) + 0.5).to(torch.float32)
        g = torch.floor(pos)
        frac = pos - g
        gi = g.to(torch.int64) & MASK32  # (uint32_t)(int) conversion
        acc = torch.zeros(n, n_feat, dtype=torch.float32)
        # uint32 corner indices of all 8 corners at once (integer math: order-free); the
        # float weights and the accumulation keep the per-corner order c = 0..7
        gc = (gi[:, None, :] + _CORNER_BITS[None]) & MASK32
        idx8 = _corner_index(gc[..., 0], gc[..., 1], gc[..., 2], res, size)
        ws = []
        for c in range(8):
            bits = [(c >> d) & 1 for d in range(3)]
            w = torch.ones(n, dtype=torch.float32)
            for d in range(3):
                w = w * (frac[:, d] if bits[d] else (1.0 - frac[:, d]))
            acc = acc + w[:, None] * grid[offset + idx8[:, c]]
            ws.append(w)
        outs.append(acc)
        cache.append((offset + idx8, ws))
    return torch.cat(outs, dim=-1), cache


class HashGridStub:
    """Drop-in for ``tinycudann.Encoding(3, cfg)`` used only to import the reference with
    an offline stub (``tests/golden/make_golden.py``).  Owns a flat ``params`` tensor."""

    def __init__(self, n_input_dims, config):
        assert config["otype"] == "HashGrid" and n_input_dims == 3
        self.table, total = level_table(config["n_levels"], config["log2_hashmap_size"],
                                        config["base_resolution"], config["per_level_scale"])
        self.n_feat = config["n_features_per_level"]
        self.n_output_dims = config["n_levels"] * self.n_feat
        self.params = torch.zeros(total * self.n_feat)

    def __call__(self, x):
        return encode(x, self.params, self.table, self.n_feat)
