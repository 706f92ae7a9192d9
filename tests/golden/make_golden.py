#!/usr/bin/env python
"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own Python modules.

Runs only in the survey/build container (needs /root/reference, read-only).  The
reference is imported with offline stubs (SURVEY.md §8c "working oracle recipe"):
``cv2`` -> empty module, ``tinycudann`` -> ``oracle.hashgrid.HashGridStub`` (the tcnn
restatement; hash-grid values are therefore parity-unpinned against real tcnn),
``nerf_util.sample_dists`` default device -> cpu.  For every case the script

  1. builds ``projects.NeuralLumen.model.Model`` from the reference YAMLs,
  2. loads seeded synthetic weights (``mli_nerf_amd.synthetic``),
  3. runs the stage-b forward (train and/or eval), the stage-b losses with the
     reference's own loss functions, and backward through ``neural_rgb`` only,
  4. checks ``oracle.render`` against those outputs, and
  5. saves inputs-that-are-not-regenerable (the stratified uniforms) + outputs as a
     small ``.pt`` fixture (loaded by the tests with ``weights_only=True``).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import sys
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("MLI_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from mli_nerf_amd import synthetic  # noqa: E402
from mli_nerf_amd.config import load_config  # noqa: E402
from oracle import hashgrid as o_hash, render as o_render  # noqa: E402

CASES = {
    # name: (config, R, Nc, Nf, H, log2T, s_var, progress, train, extra overrides)
    "hotdog_r64_n32_full": ("syn_hotdog_b", 64, 16, 4, 4, 22, 3.0, 0.0, True, {}),
    "hotdog_r64_n128": ("syn_hotdog_b", 64, 64, 16, 4, 14, 6.0, 0.05, True, {}),
    "hotdog_r64_n32_eval": ("syn_hotdog_b", 64, 16, 4, 4, 14, 3.0, 1.0, False, {}),
    "pikachu_r32_n192": ("NRHints_Pikachu_b", 32, 64, 32, 4, 14, 3.0, 0.0, True, {}),
    "savannah_r64_n32_box": ("rene_savannah_b", 64, 16, 4, 4, 14, 3.0, 0.0, True, {}),
}

# Stage a (syn_hotdog_a.yaml: LumenRGB mode 'rgb', coarse-to-fine hash grid, every parameter
# trained incl. the hash table and s_var): name -> (config, R, Nc, Nf, H, log2T, s_var, iteration)
STAGE_A_CASES = {
    "hotdog_a_r64_n32_it20k": ("syn_hotdog_a", 64, 16, 4, 4, 14, 3.0, 20000),
    "hotdog_a_r32_n128_it80k": ("syn_hotdog_a", 32, 64, 16, 4, 14, 4.0, 80000),
}
# Light visibility (test.py --inference_mode unpairlights_train --model.light_visibility.enabled=True,
# run_synthetic.sh:13): eval render with the sphere-traced camera / light rays.
# name -> (config, R, Nc, Nf, H, log2T, light_visibility overrides); s_var 6 (sharp weights) and
# frame 5 so a sixth of the surface hits are shadowed (visibility not trivially all-true)
VIS_CASES = {
    "hotdog_a_vis_r128_n32": ("syn_hotdog_a", 128, 16, 4, 4, 14, {"enabled": True}),
    "savannah_b_vis_r128_n32": ("rene_savannah_b", 128, 16, 4, 4, 14,
                                {"enabled": True, "camera_ray_type": "sphere_tracing"}),
}
MAX_ITER = 500000      # neuralangelo/configs/base.yaml:13
WARM_UP_END = 5000     # base.yaml optim.sched.warm_up_end


def install_stubs():
    sys.modules["cv2"] = types.ModuleType("cv2")
    tcnn = types.ModuleType("tinycudann")
    tcnn.Encoding = o_hash.HashGridStub
    sys.modules["tinycudann"] = tcnn
    for name in ("wandb",):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.path.insert(0, REF)


def reference_cfg(config, R, Nc, Nf, H, log2T):
    path = os.path.join(REF, "projects/NeuralLumen/configs/%s.yaml" % config)
    over = {"model": {"render": {"rand_rays": R, "num_samples": {"coarse": Nc, "fine": Nf},
                                 "num_sample_hierarchy": H},
                      "object": {"sdf": {"encoding": {"hashgrid": {"dict_size": log2T}}}}}}
    return load_config(path, root=REF, overrides=over)


def path_cfg(cfg, Nc, Nf, H, log2T):
    box = getattr(cfg.data, "bounding_type", "unit_sphere") == "box"
    return o_render.PathCfg(n_coarse=Nc, n_fine=Nf, n_hier=H, log2T=log2T,
                            white_bg=bool(cfg.model.background.white),
                            bounding="box" if box else "sphere",
                            aabb=tuple(cfg.data.bounding_box_aabb) if box else (-1, -1, -1, 1, 1, 1))


def load_weights(model, sd):
    tgt = model.state_dict()
    missing = [k for k in tgt if k not in sd]
    assert not missing, missing
    with torch.no_grad():
        for k, v in sd.items():
            if k == "neural_sdf.tcnn_encoding.params":
                model.neural_sdf.tcnn_encoding.params = v.clone()
            else:
                tgt[k].copy_(v)


def ref_losses(out, data, cfg):
    from projects.NeuralLumen.utils.utils import intrinsic_loss, regularize_re_loss
    from projects.neuralangelo.utils.misc import eikonal_loss, curvature_loss
    p = cfg.trainer.para_intrinsic_loss
    q = cfg.trainer.para_regularize_re_loss
    losses = dict(
        render=torch.nn.L1Loss()(out["rgb"], data["image_sampled"]) * 3,
        eikonal=eikonal_loss(out["gradients"], outside=out["outside"]),
        curvature=curvature_loss(out["hessians"], outside=out["outside"]),
        intrinsic=intrinsic_loss(out["o_r"], out["o_s"], data["pseudo_ref_sampled"],
                                 data["pseudo_sha_sampled"], data["pseudo_visibility_certainty_sampled"],
                                 weight_map_range_shading=tuple(p["weight_map_range_shading"]),
                                 weight_map_range_visibility=tuple(p["weight_map_range_visibility"]),
                                 factor_ref=p["factor_ref"], factor_sha=p["factor_sha"]),
        regularize_re=regularize_re_loss(out["o_re"], factor_negative=q["factor_negative"],
                                         factor_positive=q["factor_positive"],
                                         exponent_positive=q["exponent_positive"]),
    )
    weights = {k: v for k, v in cfg.trainer.loss_weight.items() if v}
    total = sum(losses[k] * weights[k] for k in weights if k in losses)
    return total, losses


def grad_digest(named_grads):
    """Full grads of biases/weight_g + a fixed strided subset of every weight_v."""
    out = {}
    for k, g in named_grads.items():
        if k.endswith("weight_v"):
            out[k + ":strided"] = g.flatten()[::97].clone()
            out[k + ":sum"] = g.double().sum().float()
        else:
            out[k] = g.clone()
    return out


def run_case(name, spec):
    from projects.nerf.utils import nerf_util
    from projects.NeuralLumen.model import Model
    config, R, Nc, Nf, H, log2T, s_var, progress, train, _ = spec
    nerf_util.sample_dists.__defaults__ = ("cpu",)
    cfg = reference_cfg(config, R, Nc, Nf, H, log2T)
    H_img, W_img = cfg.data.train.image_size
    model = Model(cfg.model, cfg.data)
    sd = synthetic.make_state_dict(log2T=log2T, seed=0, s_var=s_var)
    load_weights(model, sd)
    model.neural_sdf.set_normal_epsilon()
    model.progress = progress
    if hasattr(model, "bounding_box_aabb"):
        model.bounding_box_aabb = model.bounding_box_aabb.float()
    data = synthetic.make_batch(R, H=H_img, W=W_img, frame=3)
    for p_name, p in model.named_parameters():
        p.requires_grad_(p_name.startswith("neural_rgb"))
    torch.manual_seed(1234)
    u = torch.rand(1, R, Nc)  # what sample_dists draws first after this seed
    fix = dict(R=R, Nc=Nc, Nf=Nf, H=H, log2T=log2T, s_var=s_var, progress=progress, train=train,
               config=config, H_img=H_img, W_img=W_img)
    pcfg = path_cfg(cfg, Nc, Nf, H, log2T)
    if train:
        model.train()
        torch.manual_seed(1234)
        out = model(data)
        total, losses = ref_losses(out, data, cfg)
        total.backward()
        grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
        fix["u"] = u
        for k in ("rgb", "o_r", "o_s", "o_re", "dists", "weights", "gradients", "hessians", "outside"):
            fix["out." + k] = out[k].detach().clone()
        fix["loss.total"] = total.detach()
        for k, v in losses.items():
            fix["loss." + k] = v.detach()
        fix.update({"grad." + k: v for k, v in grad_digest(grads).items()})
        # oracle check
        sd_o = {k: v.clone().requires_grad_(k.startswith("neural_rgb")) for k, v in sd.items()}
        o_out = o_render.forward(sd_o, pcfg, data, u=u, training=True, progress=progress, width=W_img,
                                 height=H_img)
        o_total, o_losses, _ = o_render.stage_b_losses(o_out, data, pcfg)
        o_total.backward()
        check(name, fix, o_out, o_losses, o_total, {k: sd_o[k].grad for k in grads})
    else:
        model.eval()
        from projects.nerf.utils import camera
        import torch.nn.functional as F
        from projects.NeuralLumen.utils.utils import get_center
        with torch.no_grad():
            center, ray = camera.get_center_and_ray(data["pose"], data["intr"], (H_img, W_img))
            center = nerf_util.slice_by_ray_idx(center, data["ray_idx"])
            ray = nerf_util.slice_by_ray_idx(ray, data["ray_idx"])
            pts_light = nerf_util.slice_by_ray_idx(get_center(data["pose_light"], (H_img, W_img)),
                                                   data["ray_idx"])
            out = model.render_rays_lumen(center, F.normalize(ray, dim=-1), pts_light, stratified=False)
            out["depth"] = (out["dists"] * out["weights"]).sum(2) / ray.norm(dim=-1, keepdim=True)
        for k in ("rgb", "o_r", "o_s", "o_re", "dists", "weights", "gradients", "opacity",
                  "gradient", "depth", "outside"):
            fix["out." + k] = out[k].detach().clone()
        with torch.no_grad():
            o_out = o_render.forward(sd, pcfg, data, u=None, training=False, progress=progress,
                                     width=W_img, height=H_img)
        check(name, fix, o_out, None, None, None)
    path = os.path.join(HERE, name + ".pt")
    torch.save(fix, path)
    print("wrote %s (%.1f KB)" % (path, os.path.getsize(path) / 1024))


def check(name, fix, o_out, o_losses, o_total, o_grads):
    worst = 0.0
    for k, v in fix.items():
        if not k.startswith("out.") or k[4:] in ("depth",):
            continue
        o = o_out[k[4:]]
        if v.dtype == torch.bool:
            assert torch.equal(v, o), (name, k)
            continue
        err = (v - o.detach()).abs().max().item()
        tol = 1e-4 + 1e-4 * v.abs().max().item()
        if k[4:] == "hessians":
            tol = 1e-2 * max(1.0, v.abs().max().item())
        worst = max(worst, err / tol)
        assert err <= tol, (name, k, err, tol)
    if o_losses is not None:
        for k, v in o_losses.items():
            r = fix["loss." + k].item()
            assert abs(r - v.item()) <= 1e-4 * max(1.0, abs(r)), (name, k, r, v.item())
        for k, g in o_grads.items():
            ref = fix.get("grad." + k)
            if ref is None:
                ref = fix["grad." + k + ":strided"]
                g = g.flatten()[::97]
            if ref.dim() == 0:
                ref, g = ref.reshape(1), g.reshape(1)
            err = (ref - g).abs().max().item()
            assert err <= 1e-5 + 1e-3 * ref.abs().max().item(), (name, k, err)
    print("%s: oracle matches reference (worst err/tol %.3f)" % (name, worst))


def curvature_weight(it, init, growth_rate, anneal_levels):
    """neuralangelo/trainer.py:56-63 get_curvature_weight."""
    if it <= WARM_UP_END:
        return it / WARM_UP_END * init
    return init / growth_rate ** (anneal_levels - 1)


def run_stage_a_case(name, spec):
    """Stage-a train step of the reference model: forward, the stage-a losses with the
    reference's own loss functions, backward into EVERY parameter (hash table included)."""
    from projects.nerf.utils import nerf_util
    from projects.NeuralLumen.model import Model
    from projects.neuralangelo.utils.misc import eikonal_loss, curvature_loss
    config, R, Nc, Nf, H, log2T, s_var, it = spec
    nerf_util.sample_dists.__defaults__ = ("cpu",)
    cfg = reference_cfg(config, R, Nc, Nf, H, log2T)
    H_img, W_img = cfg.data.train.image_size
    model = Model(cfg.model, cfg.data)
    assert model.neural_rgb.network_mode == "rgb"
    sd = synthetic.make_state_dict(log2T=log2T, seed=0, s_var=s_var, heads="rgb")
    load_weights(model, sd)
    table = model.neural_sdf.tcnn_encoding.params.detach().clone().requires_grad_(True)
    model.neural_sdf.tcnn_encoding.params = table
    # neuralangelo/trainer.py:28-34,65-76 (_start_of_iteration)
    model.neural_sdf.warm_up_end = WARM_UP_END
    model.progress = progress = it / MAX_ITER
    model.neural_sdf.set_active_levels(it)
    model.neural_sdf.set_normal_epsilon()
    w_curv = float(curvature_weight(it, float(cfg.trainer.loss_weight.curvature),
                                    float(model.neural_sdf.growth_rate), int(model.neural_sdf.anneal_levels)))
    data = synthetic.make_batch(R, H=H_img, W=W_img, frame=3)
    torch.manual_seed(1234)
    u = torch.rand(1, R, Nc)
    model.train()
    torch.manual_seed(1234)
    out = model(data)
    w = cfg.trainer.loss_weight
    losses = dict(render=torch.nn.L1Loss()(out["rgb"], data["image_sampled"]) * 3,
                  eikonal=eikonal_loss(out["gradients"], outside=out["outside"]),
                  curvature=curvature_loss(out["hessians"], outside=out["outside"]))
    total = losses["render"] * w.render + losses["eikonal"] * w.eikonal + losses["curvature"] * w_curv
    total.backward()
    grads = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    grads["neural_sdf.tcnn_encoding.params"] = table.grad
    fix = dict(R=R, Nc=Nc, Nf=Nf, H=H, log2T=log2T, s_var=s_var, progress=progress, train=True,
               config=config, H_img=H_img, W_img=W_img, iteration=it, u=u,
               active_levels=int(model.neural_sdf.active_levels), anneal_levels=int(model.neural_sdf.anneal_levels),
               normal_eps=float(model.neural_sdf.normal_eps), curvature_weight=w_curv)
    for k in ("rgb", "dists", "weights", "gradients", "hessians", "outside"):
        fix["out." + k] = out[k].detach().clone()
    fix["loss.total"] = total.detach()
    for k, v in losses.items():
        fix["loss." + k] = v.detach()
    dig = grad_digest({k: v for k, v in grads.items() if k != "neural_sdf.tcnn_encoding.params"})
    tg = table.grad.flatten()
    dig["neural_sdf.tcnn_encoding.params:strided"] = tg[::97].clone()
    dig["neural_sdf.tcnn_encoding.params:sum"] = tg.double().sum().float()
    dig["neural_sdf.tcnn_encoding.params:abssum"] = tg.double().abs().sum().float()
    fix.update({"grad." + k: v for k, v in dig.items()})
    # oracle check
    pcfg = path_cfg(cfg, Nc, Nf, H, log2T)
    pcfg.rgb_mode, pcfg.active_levels, pcfg.anneal_levels = "rgb", fix["active_levels"], fix["anneal_levels"]
    sd_o = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    o_out = o_render.forward(sd_o, pcfg, data, u=u, training=True, progress=progress, width=W_img, height=H_img)
    o_total, o_losses, _ = o_render.stage_a_losses(o_out, data, w_curv)
    o_total.backward()
    check(name, fix, o_out, o_losses, o_total, {k: sd_o[k].grad for k in grads})
    path = os.path.join(HERE, name + ".pt")
    torch.save(fix, path)
    print("wrote %s (%.1f KB)" % (path, os.path.getsize(path) / 1024))


def run_vis_case(name, spec):
    """Eval render of the reference model with light visibility on (the test_all_light
    inference: every coarse-to-fine level active, NeuralLumen/trainer.py:224-226)."""
    from projects.nerf.utils import nerf_util, camera
    from projects.NeuralLumen.model import Model
    from projects.NeuralLumen.utils.utils import get_center
    import torch.nn.functional as F
    config, R, Nc, Nf, H, log2T, vis_over = spec
    nerf_util.sample_dists.__defaults__ = ("cpu",)
    cfg = reference_cfg(config, R, Nc, Nf, H, log2T)
    for k, v in vis_over.items():
        cfg.model.light_visibility[k] = v
    H_img, W_img = cfg.data.train.image_size
    model = Model(cfg.model, cfg.data)
    stage_a = model.neural_rgb.network_mode == "rgb"
    sd = synthetic.make_state_dict(log2T=log2T, seed=0, heads="rgb" if stage_a else "rgb_r_s", s_var=6.0)
    load_weights(model, sd)
    if hasattr(model, "bounding_box_aabb"):
        model.bounding_box_aabb = model.bounding_box_aabb.float()
    model.neural_sdf.warm_up_end = WARM_UP_END
    if cfg.model.object.sdf.encoding.coarse2fine.enabled:
        model.neural_sdf.set_active_levels(sys.maxsize)
    model.neural_sdf.set_normal_epsilon()
    model.progress = 1.0
    model.eval()
    data = synthetic.make_batch(R, H=H_img, W=W_img, frame=5)
    with torch.no_grad():
        center, ray = camera.get_center_and_ray(data["pose"], data["intr"], (H_img, W_img))
        center = nerf_util.slice_by_ray_idx(center, data["ray_idx"])
        ray = nerf_util.slice_by_ray_idx(ray, data["ray_idx"])
        pts_light = nerf_util.slice_by_ray_idx(get_center(data["pose_light"], (H_img, W_img)), data["ray_idx"])
        out = model.render_rays_lumen(center, F.normalize(ray, dim=-1), pts_light, stratified=False)
    lv = cfg.model.light_visibility
    fix = dict(R=R, Nc=Nc, Nf=Nf, H=H, log2T=log2T, config=config, H_img=H_img, W_img=W_img, train=False,
               stage_a=stage_a, s_var=6.0, frame=5, vis=dict(camera_ray_type=lv.get("camera_ray_type"), type=lv.type,
                                         bounding=lv.visibility_bounding_type,
                                         radius=float(lv.get("visibility_sphere_radius", 1.0)),
                                         gamma=float(lv.get("gamma_correlation", 0.0))))
    for k in ("rgb", "dists", "weights", "gradient", "visibility", "normal_x_light", "pseudo_shading",
              "inter_dist", "inter_mask", "outside"):
        fix["out." + k] = out[k].detach().clone()
    # oracle check
    pcfg = path_cfg(cfg, Nc, Nf, H, log2T)
    if stage_a:
        pcfg.rgb_mode = "rgb"
    pcfg.light_visibility = dict(fix["vis"], aabb=pcfg.aabb)
    with torch.no_grad():
        o_out = o_render.forward(sd, pcfg, data, u=None, training=False, progress=1.0, width=W_img, height=H_img)
    check(name, fix, o_out, None, None, None)
    path = os.path.join(HERE, name + ".pt")
    torch.save(fix, path)
    print("wrote %s (%.1f KB)" % (path, os.path.getsize(path) / 1024))


def main():
    install_stubs()
    only = sys.argv[1:]
    for name, spec in CASES.items():
        if only and name not in only:
            continue
        run_case(name, spec)
    for name, spec in STAGE_A_CASES.items():
        if only and name not in only:
            continue
        run_stage_a_case(name, spec)
    for name, spec in VIS_CASES.items():
        if only and name not in only:
            continue
        run_vis_case(name, spec)


if __name__ == "__main__":
    main()
