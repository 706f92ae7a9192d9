"""Multires hash-grid geometry (host side) for the HIP encoder that replaces tiny-cuda-nn.

Reference call site: ``projects/neuralangelo/utils/modules.py:38-55`` builds
``tcnn.Encoding(3, {otype: HashGrid, n_levels: 16, n_features_per_level: 8,
log2_hashmap_size: 22, base_resolution: 32, per_level_scale: 1.3195...})`` and reads
``neural_sdf.tcnn_encoding.params`` (flat fp32) from checkpoints.  The level geometry
below is computed on the host in float32 exactly once and handed to the kernels as a
table, so the device and the CPU oracle use bit-identical per-level scales.
"""
import numpy as np

GRID_DEFAULTS = dict(levels=16, feat=8, log2T=22, min_logres=5, max_logres=11)


def growth_rate(levels=16, min_logres=5, max_logres=11):
    """neuralangelo/utils/modules.py:38-41."""
    r_min, r_max = 2 ** min_logres, 2 ** max_logres
    return np.exp((np.log(r_max) - np.log(r_min)) / (levels - 1))


SCALE_RULES = ("fp32", "exact")


def level_table(levels=16, log2T=22, min_logres=5, max_logres=11, scale_rule="fp32"):
    """Per level (scale fp32, resolution, entries, entry offset) and the total entries.

    tcnn semantics (restated): scale = exp2f(l * log2f(pls)) * base - 1 in fp32,
    res = ceil(scale) + 1, entries = min(next_multiple(res^3, 8), 2^log2T).
    ``scale_rule='exact'``: the scale in exact (float64) arithmetic, rounded to fp32 once.  The
    two rules differ where pls^l is a power of two (levels 5, 10, 15: 127.00002 vs 127 at level
    5), and at level 5 (dense) the resolution -- 129 vs 128 -- changes the table size:
    45,724,048 vs 45,674,504 entries at the default config.  'fp32' is the restatement of tcnn;
    'exact' exists so a checkpoint of the other size loads (Model.load_state_dict)."""
    if scale_rule not in SCALE_RULES:
        raise ValueError("scale_rule must be one of %r" % (SCALE_RULES,))
    pls = np.float32(growth_rate(levels, min_logres, max_logres))
    log2_pls = np.float32(np.log2(pls))
    base = np.float32(2 ** min_logres)
    out, offset = [], 0
    for lv in range(levels):
        if scale_rule == "exact":
            scale = np.float32(2.0 ** min_logres * growth_rate(levels, min_logres, max_logres) ** lv - 1.0)
            # pls^l = 2^(l (max-min)/(levels-1)): snap the float64 rounding of exact powers of two
            e = lv * (max_logres - min_logres) / (levels - 1)
            if abs(e - round(e)) < 1e-12:
                scale = np.float32(2.0 ** (min_logres + round(e)) - 1.0)
        else:
            scale = np.float32(np.float32(np.exp2(np.float32(lv) * log2_pls)) * base - np.float32(1))
        res = int(np.ceil(scale)) + 1
        size = min(-(-res ** 3 // 8) * 8, 1 << log2T)
        out.append((float(scale), res, size, offset))
        offset += size
    return out, offset


def normal_eps(levels=16, min_logres=5, max_logres=11):
    """1 / resolutions[-1] with neuralangelo's own resolution list (modules.py:51-54,102-107)."""
    g = growth_rate(levels, min_logres, max_logres)
    last = np.floor(2 ** min_logres * g ** (levels - 1)).astype(int) + 1
    return 1.0 / float(last)
