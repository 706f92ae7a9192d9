"""Training parity (SURVEY §8d "PSNR parity"): 500 stage-b steps from identical init on
synthetic data, the HIP trainer (fused forward/backward, fused AdamW) against the CPU
oracle driven by torch.optim.AdamW + LambdaLR(two_steps_with_warmup).  This is the
reference's own optimizer/scheduler pair (imaginaire/trainers/utils/get_trainer.py:106-150,
neuralangelo/utils/misc.py:28-71).

Both sides see the same batches, stratified uniforms, LR schedule and progress.  The
render target is learnable: a smooth function of the view direction, which the view-SH
input of the rgb head can fit, on rays through the object (opaque), so PSNR rises over the run.  Bar: the train-PSNR curves agree
within 0.1 dB, averaged over the last 100 steps, or within 3x the statistic's own noise
floor if that is larger (measured in the test: a second CPU run with 1e-4 gradient noise).
"""
import pytest
import torch
import torch.nn.functional as F

from mli_nerf_amd import synthetic
from mli_nerf_amd.configs import preset
from mli_nerf_amd.trainer import two_steps_with_warmup
from oracle import render as o_render

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
STEPS, R, NC, NF, LOG2T, WARM = 500, 64, 16, 4, 14, 20


def _batches(H, W):
    out = []
    for i in range(STEPS):
        d = synthetic.make_batch(R, H=H, W=W, frame=i % 100, seed=i // 100)
        # rays through the disk the r = 0.5 SDF sphere projects to (radius ~89 px at 512^2,
        # f = 711, distance 4): opaque rays, whose colour the heads control
        g = torch.Generator().manual_seed(5000 + i)
        rad = 70.0 * torch.rand(R, generator=g).sqrt()
        ang = 2 * torch.pi * torch.rand(R, generator=g)
        px = (W / 2 + rad * ang.cos()).long().clamp(0, W - 1)
        py = (H / 2 + rad * ang.sin()).long().clamp(0, H - 1)
        d["ray_idx"] = (py * W + px)[None]
        _, ray = o_render.pixel_rays(d["pose"], d["intr"], d["ray_idx"], W, H)
        d["image_sampled"] = 0.5 + 0.35 * F.normalize(ray, dim=-1)
        u = torch.rand(1, R, NC, generator=torch.Generator().manual_seed(1000 + i))
        out.append((d, u))
    return out


@pytest.mark.timeout(1500)
def test_train_psnr_curve_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    torch.manual_seed(0)
    cfg = preset("syn_hotdog_b", rays=R, n_coarse=NC, n_fine=NF, log2T=LOG2T,
                 overrides={"optim": {"sched": {"warm_up_end": WARM}}})
    H, W = cfg.data.train.image_size
    sd = synthetic.make_state_dict(log2T=LOG2T)
    batches = _batches(H, W)
    # GPU: the product trainer
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(sd)
    model = model.to(DEV)
    trainer = Trainer(cfg, is_inference=False, model=model)
    psnr_gpu = []
    for d, u in batches:
        trainer.train_step({k: v.to(DEV) for k, v in d.items()}, u=u.to(DEV))
        psnr_gpu.append(trainer.metrics["psnr"])
    psnr_gpu = torch.stack(psnr_gpu).cpu()
    # CPU oracle + torch AdamW / LambdaLR (the reference's optimizer and schedule), run twice:
    # nominal, and with a 1e-4 relative perturbation of the gradients (the GPU path's
    # gradient error is ~1e-4: cosine >= 0.9999).  L1 losses train on gradient SIGNS, so
    # runs that differ at the 1e-4 level drift apart chaotically; the spread of the two CPU
    # runs is the noise floor of this statistic (a different CPU thread count alone moves
    # the last-100-step mean by ~0.15 dB at this size).
    torch.set_num_threads(16)
    psnr_cpu = _oracle_run(cfg, sd, batches, H, W, noise=0.0)
    psnr_cpu2 = _oracle_run(cfg, sd, batches, H, W, noise=1e-4)
    last_g, last_c, last_c2 = (x[-100:].mean().item() for x in (psnr_gpu, psnr_cpu, psnr_cpu2))
    first = psnr_cpu[:10].mean().item()
    floor = abs(last_c - last_c2)
    tol = max(0.1, 3.0 * floor)
    print("train PSNR: first10 %.3f  last100 gpu %.4f cpu %.4f cpu(1e-4 grad noise) %.4f  |gpu-cpu| %.4f dB  "
          "noise floor %.4f dB  bar %.4f dB" % (first, last_g, last_c, last_c2, abs(last_g - last_c), floor, tol))
    assert last_c > first + 1.0, "the run should learn the target"
    assert abs(last_g - last_c) < tol


def _oracle_run(cfg, sd, batches, H, W, noise):
    w = dict(sd)
    w["neural_sdf.tcnn_encoding.params"] = w["neural_sdf.tcnn_encoding.params"].half().float()
    heads = [k for k in w if k.startswith("neural_rgb")]
    for k in heads:
        w[k] = w[k].clone().requires_grad_(True)
    o = cfg.optim
    opt = torch.optim.AdamW([w[k] for k in heads], lr=o.params.lr, weight_decay=o.params.weight_decay)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda it: two_steps_with_warmup(it, o.sched.warm_up_end, tuple(o.sched.two_steps), o.sched.gamma))
    pcfg = o_render.PathCfg(n_coarse=NC, n_fine=NF, log2T=LOG2T)
    g = torch.Generator().manual_seed(99)
    out_psnr = []
    for i, (d, u) in enumerate(batches):
        out = o_render.forward(w, pcfg, d, u=u, training=True, progress=i / cfg.max_iter, width=W, height=H)
        total, _, psnr = o_render.stage_b_losses(out, d, pcfg)
        opt.zero_grad()
        total.backward()
        if noise:
            for k in heads:
                w[k].grad.mul_(1 + noise * torch.randn(w[k].grad.shape, generator=g))
        opt.step()
        sched.step()
        out_psnr.append(float(psnr.detach()))
    return torch.tensor(out_psnr)
