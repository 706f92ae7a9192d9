"""Pin the CPU oracle against golden vectors produced by the REFERENCE itself
(tests/golden/make_golden.py imports the reference's Python modules with offline stubs).

The hash-grid values inside these fixtures come from the tcnn restatement (parity
unpinned against real tiny-cuda-nn, see oracle/hashgrid.py); every other stage is the
reference's own code.
"""
import pytest
import torch

from mli_nerf_amd import synthetic
from oracle import render as o_render

CASES = ["hotdog_r64_n32_full", "hotdog_r64_n128", "hotdog_r64_n32_eval", "pikachu_r32_n192",
         "savannah_r64_n32_box"]

AABB = {"rene_savannah_b": (-0.66, -0.516, -0.18, 0.66, 0.42, 0.3)}  # rene_savannah_b.yaml:53-60
WHITE = {"syn_hotdog_b": True, "NRHints_Pikachu_b": False, "rene_savannah_b": False, "syn_hotdog_a": True}


def case_cfg(fx):
    box = fx["config"] in AABB
    return o_render.PathCfg(n_coarse=fx["Nc"], n_fine=fx["Nf"], n_hier=fx["H"], log2T=fx["log2T"],
                            white_bg=WHITE[fx["config"]], bounding="box" if box else "sphere",
                            aabb=AABB.get(fx["config"], (-1, -1, -1, 1, 1, 1)))


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_golden(golden, name):
    fx = golden(name)
    cfg = case_cfg(fx)
    sd = synthetic.make_state_dict(log2T=fx["log2T"], seed=0, s_var=fx["s_var"])
    data = synthetic.make_batch(fx["R"], H=fx["H_img"], W=fx["W_img"], frame=3)
    if fx["train"]:
        sd = {k: v.requires_grad_(k.startswith("neural_rgb")) for k, v in sd.items()}
    with torch.set_grad_enabled(fx["train"]):
        out = o_render.forward(sd, cfg, data, u=fx.get("u"), training=fx["train"],
                               progress=fx["progress"], width=fx["W_img"], height=fx["H_img"])
    for key, ref in fx.items():
        if not key.startswith("out.") or key == "out.depth":
            continue
        got = out[key[4:]].detach()
        if ref.dtype == torch.bool:
            assert torch.equal(got, ref), key
        else:
            torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5, msg=key)
    if fx["train"]:
        total, losses, _ = o_render.stage_b_losses(out, data, cfg)
        for k, v in losses.items():
            torch.testing.assert_close(v.detach(), fx["loss." + k], rtol=1e-5, atol=1e-6)
        total.backward()
        for name_p in o_render.head_param_names():
            g = sd[name_p].grad
            if name_p + ":strided" in {k[5:] for k in fx if k.startswith("grad.")}:
                torch.testing.assert_close(g.flatten()[::97], fx["grad." + name_p + ":strided"],
                                           rtol=1e-4, atol=1e-7)
            else:
                torch.testing.assert_close(g, fx["grad." + name_p], rtol=1e-4, atol=1e-7)


def test_level_table_matches_product_side():
    from mli_nerf_amd.hashgrid import level_table as product_table
    from oracle.hashgrid import level_table as oracle_table
    assert product_table()[0] == oracle_table()[0]
    assert product_table()[1] == 45724048  # fp32 tcnn scale arithmetic: level 5 res = 129


STAGE_A_CASES = ["hotdog_a_r64_n32_it20k", "hotdog_a_r32_n128_it80k"]


@pytest.mark.parametrize("name", STAGE_A_CASES)
def test_oracle_stage_a_matches_reference_golden(golden, name):
    """Stage a (syn_hotdog_a): single 'rgb' head, coarse-to-fine mask, tap epsilon of the
    annealed level, gradients of EVERY parameter incl. the hash table and s_var."""
    fx = golden(name)
    cfg = case_cfg({**fx, "config": "syn_hotdog_b"})
    cfg.rgb_mode, cfg.active_levels, cfg.anneal_levels = "rgb", fx["active_levels"], fx["anneal_levels"]
    assert abs(cfg.normal_eps() - fx["normal_eps"]) < 1e-12
    sd = synthetic.make_state_dict(log2T=fx["log2T"], seed=0, s_var=fx["s_var"], heads="rgb")
    sd = {k: v.requires_grad_(True) for k, v in sd.items()}
    out = o_render.forward(sd, cfg, data := synthetic.make_batch(fx["R"], H=fx["H_img"], W=fx["W_img"], frame=3),
                           u=fx["u"], training=True, progress=fx["progress"], width=fx["W_img"], height=fx["H_img"])
    for key, ref in fx.items():
        if not key.startswith("out."):
            continue
        got = out[key[4:]].detach()
        if ref.dtype == torch.bool:
            assert torch.equal(got, ref), key
        else:
            torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5, msg=key)
    total, losses, _ = o_render.stage_a_losses(out, data, fx["curvature_weight"])
    for k, v in losses.items():
        torch.testing.assert_close(v.detach(), fx["loss." + k], rtol=1e-5, atol=1e-6)
    total.backward()
    for name_p in o_render.stage_a_param_names():
        g = sd[name_p].grad
        if "grad." + name_p in fx:
            torch.testing.assert_close(g.reshape(fx["grad." + name_p].shape), fx["grad." + name_p],
                                       rtol=1e-4, atol=1e-7)
        else:
            torch.testing.assert_close(g.flatten()[::97], fx["grad." + name_p + ":strided"], rtol=1e-4, atol=1e-7)
            torch.testing.assert_close(g.double().sum().float(), fx["grad." + name_p + ":sum"],
                                       rtol=1e-4, atol=1e-6)


VIS_CASES = ["hotdog_a_vis_r128_n32", "savannah_b_vis_r128_n32"]


@pytest.mark.parametrize("name", VIS_CASES)
def test_oracle_light_visibility_matches_reference_golden(golden, name):
    """Eval render with light visibility (sphere-traced camera and light rays,
    NeuralLumen/model.py:133-184): visibility / shading / intersection outputs."""
    fx = golden(name)
    cfg = case_cfg(fx)
    if fx["stage_a"]:
        cfg.rgb_mode = "rgb"
    cfg.light_visibility = dict(fx["vis"], aabb=cfg.aabb)
    sd = synthetic.make_state_dict(log2T=fx["log2T"], seed=0, s_var=fx["s_var"],
                                   heads="rgb" if fx["stage_a"] else "rgb_r_s")
    data = synthetic.make_batch(fx["R"], H=fx["H_img"], W=fx["W_img"], frame=fx["frame"])
    with torch.no_grad():
        out = o_render.forward(sd, cfg, data, u=None, training=False, progress=1.0, width=fx["W_img"],
                               height=fx["H_img"])
    for key, ref in fx.items():
        if not key.startswith("out."):
            continue
        got = out[key[4:]].detach()
        if ref.dtype == torch.bool:
            assert torch.equal(got, ref), key
        else:
            torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5, msg=key)


def test_oracle_straight_through_geometry_hook(golden):
    """The conditioning hook of the stage-a decomposition (tests/test_gpu_stage_a_decomp.py leg
    (a)): given the oracle's own SDF-network values as ``geometry_st``, the forward outputs and
    every parameter gradient equal the unhooked oracle's; given shifted values, the outputs move
    with them while the gradients still flow into the SDF network and the hash table."""
    fx = golden(STAGE_A_CASES[0])
    cfg = case_cfg({**fx, "config": "syn_hotdog_b"})
    cfg.rgb_mode, cfg.active_levels, cfg.anneal_levels = "rgb", fx["active_levels"], fx["anneal_levels"]
    data = synthetic.make_batch(fx["R"], H=fx["H_img"], W=fx["W_img"], frame=3)
    runs = []
    for hook in (None, "self", "shift"):
        sd = synthetic.make_state_dict(log2T=fx["log2T"], seed=0, s_var=fx["s_var"], heads="rgb")
        sd = {k: v.requires_grad_(True) for k, v in sd.items()}
        kw = dict(u=fx["u"], training=True, progress=fx["progress"], width=fx["W_img"], height=fx["H_img"])
        geo = None
        if hook is not None:
            with torch.no_grad():
                ref = runs[0][0]
                d = 1e-3 if hook == "shift" else 0.0
                geo = dict(sdfs=ref["sdfs"] + d, grads=ref["gradients"] * (1 + d), hess=ref["hessians"],
                           feats=runs[0][2])
        out = o_render.forward(sd, cfg, data, dists=None if hook is None else runs[0][0]["dists"],
                               geometry_st=geo, **kw)
        total, _, _ = o_render.stage_a_losses(out, data, fx["curvature_weight"])
        total.backward()
        feats = None
        if hook is None:   # the SDF feature at the samples, recomputed for the hook
            with torch.no_grad():
                center, ray = o_render.pixel_rays(data["pose"], data["intr"], data["ray_idx"], fx["W_img"], fx["H_img"])
                p = center[..., None, :] + torch.nn.functional.normalize(ray, dim=-1)[..., None, :] * out["dists"]
                feats = o_render.sdf_net({k: v.detach() for k, v in sd.items()}, cfg, p, with_feat=True)[1]
        runs.append((out, {k: v.grad.clone() for k, v in sd.items() if v.grad is not None}, feats))
    (o0, g0, _), (o1, g1, _), (o2, g2, _) = runs
    torch.testing.assert_close(o1["rgb"], o0["rgb"], rtol=0, atol=1e-6)
    for k in g0:
        torch.testing.assert_close(g1[k], g0[k], rtol=1e-5, atol=1e-9)
    assert not torch.allclose(o2["rgb"], o0["rgb"], rtol=0, atol=1e-7)
    assert float(g2["neural_sdf.tcnn_encoding.params"].abs().sum()) > 0
    assert float(g2["neural_sdf.mlp.linears.0.weight_v"].abs().sum()) > 0
