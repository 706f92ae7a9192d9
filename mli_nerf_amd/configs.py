"""Built-in stage-b configuration presets (the reference YAML values the hot path reads).

Values restated from projects/neuralangelo/configs/base.yaml and
projects/NeuralLumen/configs/{syn_hotdog_b,NRHints_Pikachu_b,rene_savannah_b}.yaml; the
reference YAMLs themselves load through ``config.load_config`` when available.
"""
import copy

from .config import merge, to_attr

BASE = {
    "max_iter": 500000,                                                     # base.yaml:13
    "max_epoch": 9999999999,                                                # imaginaire/config_base.yaml:22
    "checkpoint": {"save_iter": 20000,                                      # base.yaml:20-21
                   "save_latest_iter": 9999999999, "save_epoch": 9999999999},  # config_base.yaml:44-45
    "trainer": {
        "type": "mli_nerf_amd.trainer",
        "loss_weight": {"render": 1.0, "eikonal": 0.1, "curvature": 5e-4,   # syn_hotdog_b.yaml:4-9
                        "intrinsic": 1.0, "regularize_re": 1.0},
        "para_intrinsic_loss": {"weight_map_range_shading": [0.0, 1.0],
                                "weight_map_range_visibility": [0.0, 1.0],
                                "factor_ref": 1.0, "factor_sha": 1.0},
        "para_regularize_re_loss": {"factor_negative": 10.0, "factor_positive": 1.0,
                                    "exponent_positive": 1.0},
        "partial_grad": ["neural_rgb"],
        "grad_accum_iter": 1,
    },
    "model": {
        "type": "mli_nerf_amd.model",
        "object": {
            "sdf": {"mlp": {"num_layers": 1, "hidden_dim": 256, "inside_out": False,
                            "out_bias": 0.5, "weight_norm": True},
                    "encoding": {"type": "hashgrid", "levels": 16,
                                 "hashgrid": {"min_logres": 5, "max_logres": 11, "dict_size": 22,
                                              "dim": 8, "range": [-2, 2]},
                                 "coarse2fine": {"enabled": False, "init_active_level": 8, "step": 5000}},
                    "gradient": {"mode": "numerical", "taps": 4}},
            "rgb": {"mlp": {"num_layers": 4, "hidden_dim": 256, "weight_norm": True},
                    "encoding_view": {"type": "spherical", "levels": 3},
                    "network_mode": "rgb_r_s", "shading_dim": 1},
            "s_var": {"init_val": 3.0, "anneal_end": 0.1},
        },
        "background": {"enabled": False, "white": True},
        "render": {"rand_rays": 2048, "rand_rays_val": 20000,
                   "num_samples": {"coarse": 64, "fine": 16, "background": 32},
                   "num_sample_hierarchy": 4, "stratified": True},
        "appear_embed": {"enabled": False, "dim": 8},
        "light_visibility": {"enabled": False},
    },
    "optim": {"type": "AdamW", "params": {"lr": 1e-3, "weight_decay": 1e-2},
              "sched": {"type": "two_steps_with_warmup", "warm_up_end": 5000,
                        "two_steps": [300000, 400000], "gamma": 10.0},
              "partial_training": ["neural_rgb"]},
    "data": {"train": {"image_size": [512, 512], "batch_size": 1},
             "val": {"image_size": [512, 512], "batch_size": 1},
             "bounding_type": "unit_sphere", "white_background": True},
}

PRESETS = {
    "syn_hotdog_b": {},
    "NRHints_Pikachu_b": {"model": {"background": {"white": False}},
                          "data": {"white_background": False}},
    # stage a (syn_hotdog_a.yaml): LumenRGB mode 'rgb' (no network_mode), coarse-to-fine from
    # 8 active levels, render/eikonal/curvature losses only, every parameter trained
    "syn_hotdog_a": {"model": {"object": {"sdf": {"encoding": {"coarse2fine": {"enabled": True,
                                                                                "init_active_level": 8}}}}}},
    "rene_savannah_b": {"model": {"background": {"white": False}},
                        "data": {"bounding_type": "box", "white_background": False,
                                 "bounding_box_aabb": [-0.66, -0.516, -0.18, 0.66, 0.42, 0.3],
                                 "train": {"image_size": [270, 360]}, "val": {"image_size": [270, 360]}}},
}


# keys a preset removes from BASE (the stage-b additions the stage-a YAMLs do not have)
DROP = {
    "syn_hotdog_a": ("model.object.rgb.network_mode", "model.object.rgb.shading_dim", "trainer.partial_grad",
                     "optim.partial_training", "trainer.loss_weight.intrinsic",
                     "trainer.loss_weight.regularize_re"),
}


def _drop(cfg, path):
    keys = path.split(".")
    node = cfg
    for k in keys[:-1]:
        node = node[k]
    node.pop(keys[-1], None)


def preset(name="syn_hotdog_b", rays=None, n_coarse=None, n_fine=None, n_hier=None, log2T=None,
           overrides=None):
    cfg = copy.deepcopy(BASE)
    merge(cfg, copy.deepcopy(PRESETS[name]))
    for path in DROP.get(name, ()):
        _drop(cfg, path)
    r = cfg["model"]["render"]
    if rays is not None:
        r["rand_rays"] = rays
    if n_coarse is not None:
        r["num_samples"]["coarse"] = n_coarse
    if n_fine is not None:
        r["num_samples"]["fine"] = n_fine
    if n_hier is not None:
        r["num_sample_hierarchy"] = n_hier
    if log2T is not None:
        cfg["model"]["object"]["sdf"]["encoding"]["hashgrid"]["dict_size"] = log2T
    if overrides:
        merge(cfg, overrides)
    return to_attr(cfg)
