#!/usr/bin/env python
"""Benchmark: MLI-NeRF stage-b training step (syn_hotdog_b, 4096 rays x 128 samples per GPU).

One step = one pass of the hot path over one batch: ray generation, hierarchical sampling,
SDF field + 4 taps, the three light-conditioned heads, NeuS compositing, the stage-b losses,
backward through the heads and the fused AdamW update (BASELINE.json configs[1]).
Synthetic seeded inputs / random-init weights of the reference architecture (no dataset
or checkpoint on the box); full-size hash table (log2 T = 22).

Multi-GPU (torchrun): one process per GPU, each rank renders its own image's rays, one
RCCL all-reduce of the 3.2 MB flat gradient per step (DDP semantics); weak scaling.

Prints ONE JSON line (rank 0).  Extra fields: per-kernel live timings (HIP events on the
launch stream), the roofline record of the dominant kernel, the CPU-oracle baseline and
the PSNR agreement GPU vs CPU oracle on the same rays.
"""
import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402

PEAK_F16_TFLOPS = 2516.6   # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
HIDDEN = 256
HEAD_IN = (294, 262, 278)
HEAD_OUT = (3, 3, 1)


def kernel_flops(name, R, N, Nc, Nf, H):
    """Algorithmic MLP FLOPs (2*MAC) per launch of each MFMA kernel."""
    S = R * N
    sdf_point = 2 * ((3 + 128) * HIDDEN + HIDDEN)                  # layer 0 + sdf head
    heads_fwd = sum(k * HIDDEN + 3 * HIDDEN * HIDDEN + HIDDEN * o for k, o in zip(HEAD_IN, HEAD_OUT))
    if name == "mli_rgb_fwd":
        return 2 * S * (HIDDEN * HIDDEN + heads_fwd)               # SDF layer 1 (feat) + heads
    if name == "mli_rgb_bwd":
        return 2 * S * sum(HIDDEN * o + 3 * HIDDEN * HIDDEN for o in HEAD_OUT)
    if name == "mli_wgrad":
        return 2 * S * heads_fwd
    if name == "mli_sdf:field":
        return 5 * S * sdf_point
    return 0


def cpu_baseline(R_cpu, steps, threads):
    """The CPU oracle (fp32 PyTorch restatement of the reference path) timed on the host:
    stage-b forward + losses + backward on R_cpu rays of the same workload."""
    from mli_nerf_amd import synthetic
    from oracle import render as o_render
    torch.set_num_threads(threads)
    sd = synthetic.make_state_dict(log2T=22)
    sd = {k: v.requires_grad_(k.startswith("neural_rgb")) for k, v in sd.items()}
    pcfg = o_render.PathCfg()
    data = synthetic.make_batch(R_cpu, frame=0, seed=7)
    u = synthetic.stratified_uniforms(R_cpu, pcfg.n_coarse, seed=7)
    times = []
    out = psnr = None
    for i in range(steps + 1):
        t0 = time.perf_counter()
        out = o_render.forward(sd, pcfg, data, u=u, training=True, progress=0.0)
        total, _, psnr = o_render.stage_b_losses(out, data, pcfg)
        total.backward()
        for v in sd.values():
            v.grad = None
        if i > 0:
            times.append(time.perf_counter() - t0)
    t = sum(times) / len(times)
    return dict(value=R_cpu / t, unit="rays/s", cores=threads, kind="port",
                sample="oracle fwd+bwd stage-b, %d rays x %d samples, full hash table, %d timed steps "
                       "after 1 warm-up, torch fp32 on %d host threads" % (R_cpu, pcfg.n_samples, steps, threads),
                s_per_step=t), data, u, float(psnr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="syn_hotdog_b")
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--fine", type=int, default=16)
    ap.add_argument("--cpu-rays", type=int, default=256)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from mli_nerf_amd import _lib as L, synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer

    cfg = preset(args.config, rays=args.rays, n_fine=args.fine)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22, seed=0))
    model = model.to(dev)
    trainer = Trainer(cfg, model, world_size=world)
    Hh, W = cfg.data.train.image_size
    batch = {k: v.to(dev) for k, v in synthetic.make_batch(args.rays, H=Hh, W=W, frame=rank).items()}
    R, N = args.rays, model.pcfg.n_samples

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    for _ in range(args.warmup):
        trainer.train_step(batch)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    if not args.no_kernel_timing:
        L.PROFILE = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.train_step(batch)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof, L.PROFILE = L.PROFILE, None
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    psnr = trainer.metrics["psnr"].item()
    loss = trainer.losses["total"].item()

    kernels = {}
    if prof:
        for name, e0, e1 in prof:
            k = kernels.setdefault(name, [0.0, 0])
            k[0] += e0.elapsed_time(e1)
            k[1] += 1
    ktab = {n: {"ms_per_launch": v[0] / v[1], "launches_per_step": v[1] / args.steps,
                "ms_per_step": v[0] / args.steps} for n, v in sorted(kernels.items(), key=lambda kv: -kv[1][0])}
    roof = None
    mfma_kernels = [n for n in ktab if kernel_flops(n, R, N, 64, args.fine, 4) > 0]
    if mfma_kernels:
        dom = max(mfma_kernels, key=lambda n: ktab[n]["ms_per_step"])
        fl = kernel_flops(dom, R, N, 64, args.fine, 4)
        achieved = fl / (ktab[dom]["ms_per_launch"] * 1e-3) / 1e12
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_F16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_F16_TFLOPS, 4), "traffic": None,
                "flops_per_launch": fl}
        for n in ktab:
            f = kernel_flops(n, R, N, 64, args.fine, 4)
            if f:
                ktab[n]["tflops"] = round(f / (ktab[n]["ms_per_launch"] * 1e-3) / 1e12, 2)

    step_ms = elapsed / args.steps * 1e3
    value = R * world * args.steps / elapsed
    result = {
        "metric": "rays/sec + PSNR, syn_hotdog 4096 rays x128 samples, 1/2/4/8 MI355X",
        "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f16 MFMA (fp32 accumulate) / fp32",
        "data": "synthetic (seeded cameras/lights/labels, random-init weights, full 2^22 hash table)",
        "config": {"workload": "%s stage-b train step" % args.config, "rays_per_gpu": R, "samples_per_ray": N,
                   "global_rays": R * world, "image": [Hh, W], "parallelism": "dp%d" % world},
        "psnr": round(psnr, 4), "loss": round(loss, 6),
        "roofline": roof, "kernels": ktab,
        "mfma_tflops_step": round(sum(kernel_flops(n, R, N, 64, args.fine, 4) for n in ktab) /
                                  (step_ms * 1e-3) / 1e12, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = min(16, os.cpu_count() or 1)
        cb, data_cpu, u_cpu, psnr_cpu = cpu_baseline(args.cpu_rays, args.cpu_steps, threads)
        result["cpu_baseline"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in cb.items()}
        result["speedup_vs_cpu"] = round(value / cb["value"], 1)
        # PSNR agreement on the CPU sample's rays (same weights, rays, uniforms)
        cfg2 = preset(args.config, rays=args.cpu_rays, n_fine=args.fine)
        m2 = Model(cfg2.model, cfg2.data)
        m2.load_state_dict(synthetic.make_state_dict(log2T=22, seed=0))
        m2 = m2.to(dev).train()
        from mli_nerf_amd.trainer import stage_b_losses
        out2 = m2({k: v.to(dev) for k, v in data_cpu.items()}, u=u_cpu.to(dev))
        _, _, psnr_gpu = stage_b_losses(out2, {k: v.to(dev) for k, v in data_cpu.items()}, trainer.weights)
        result["psnr_check"] = {"gpu": round(psnr_gpu.item(), 4), "cpu_oracle": round(psnr_cpu, 4),
                                "delta_db": round(abs(psnr_gpu.item() - psnr_cpu), 4),
                                "rays": args.cpu_rays}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
