"""The drop-in surface on the reference's own YAMLs (CPU, no kernels): every NeuralLumen config
builds the Model / Trainer with the right stage, bounds, background, coarse-to-fine and loss
set, and the state-dict keys equal the reference's (restated in mli_nerf_amd.synthetic).
Needs the reference checkout for the YAMLs (skipped elsewhere); the built-in presets are
checked against the same expectations without it."""
import os

import pytest

from mli_nerf_amd import synthetic
from mli_nerf_amd.configs import preset
from mli_nerf_amd.model import Model
from mli_nerf_amd.trainer import Trainer

REF = os.environ.get("MLI_REFERENCE", "/root/reference")
CFG_DIR = os.path.join(REF, "projects/NeuralLumen/configs")
SMALL = {"model": {"object": {"sdf": {"encoding": {"hashgrid": {"dict_size": 12}}}}}}

EXPECT = {  # stage, bounding, white background, loss terms
    "syn_hotdog_a": ("a", "sphere", True, {"render", "eikonal", "curvature"}),
    "syn_hotdog_b": ("b", "sphere", True, {"render", "eikonal", "curvature", "intrinsic", "regularize_re"}),
    "NRHints_Pikachu_a": ("a", "sphere", False, {"render", "eikonal", "curvature"}),
    "NRHints_Pikachu_b": ("b", "sphere", False, {"render", "eikonal", "curvature", "intrinsic", "regularize_re"}),
    "rene_savannah_a": ("a", "box", False, {"render", "eikonal", "curvature"}),
    "rene_savannah_b": ("b", "box", False, {"render", "eikonal", "curvature", "intrinsic", "regularize_re"}),
}


def _check(cfg, name):
    stage, bounding, white, losses = EXPECT[name]
    m = Model(cfg.model, cfg.data)
    t = Trainer(cfg, is_inference=False, model=m)
    assert m.stage == stage and m.pcfg.bounding == bounding and m.pcfg.white_bg == white
    assert set(t.weights) == losses
    sd = synthetic.make_state_dict(log2T=12, heads="rgb" if stage == "a" else "rgb_r_s")
    assert set(m.state_dict()) == set(sd)
    assert m.load_state_dict(sd).missing_keys == []
    trainable = {n for n, p in m.named_parameters() if p.requires_grad}
    if stage == "a":  # every parameter (NeuralLumen/model.py:422-438), coarse-to-fine on
        assert trainable == set(sd) and m.neural_sdf.c2f is not None
        t.current_iteration = 20000
        t._start_of_iteration()
        assert (m.neural_sdf.active_levels, m.neural_sdf.anneal_levels) == (8, 3)
        assert abs(m.neural_sdf.normal_eps - 1.0 / m.neural_sdf.resolutions[2]) < 1e-15
    else:             # partial_grad neural_rgb (NeuralLumen/trainer.py:44-54)
        assert trainable == {k for k in sd if k.startswith("neural_rgb")}


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_reference_yaml_builds(name):
    from mli_nerf_amd.config import load_config
    path = os.path.join(CFG_DIR, name + ".yaml")
    if not os.path.exists(path):
        pytest.skip("reference YAMLs not present")
    _check(load_config(path, root=REF, overrides=SMALL), name)


@pytest.mark.parametrize("name", ["syn_hotdog_a", "syn_hotdog_b", "rene_savannah_b"])
def test_builtin_presets(name):
    _check(preset(name, log2T=12), name)
