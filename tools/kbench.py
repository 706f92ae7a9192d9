"""Kernel micro-benchmark: time the individual stage-b kernels at the bench shape.

Usage (on the GPU box): python tools/kbench.py [--rays 4096] [--reps 20]
Prints median ms per launch and TFLOP/s for the MFMA kernels, A/B style in one process
(training-store vs eval variants of the heads forward).
"""
import argparse
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402


def timeit(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--membw", action="store_true", help="also time plain HBM write / copy streams")
    ap.add_argument("--ray-order", default="random", choices=["random", "sorted", "xcd"],
                    help="order of the batch's rays: as drawn, sorted by pixel, or sorted and dealt to "
                         "the 8 XCDs by image band (workgroup b runs on XCD b %% 8)")
    ap.add_argument("--dump", default=None, help="save the sampler's dists and the field's outputs (bit-identity A/B)")
    args = ap.parse_args()
    if args.membw:
        x = torch.empty(2 * 1024 ** 3, dtype=torch.float16, device="cuda")  # 4 GiB
        y = torch.empty_like(x)
        med, _ = timeit(lambda: x.fill_(1.0), 10)
        print("fill 4 GiB            %.3f ms  %.2f TB/s write" % (med, 4 * 1024 ** 3 / med / 1e9))
        med, _ = timeit(lambda: y.copy_(x), 10)
        print("copy 4 GiB            %.3f ms  %.2f TB/s read+write" % (med, 8 * 1024 ** 3 / med / 1e9))
        med, _ = timeit(lambda: x.sum(), 10)
        print("sum 4 GiB             %.3f ms  %.2f TB/s read" % (med, 4 * 1024 ** 3 / med / 1e9))
        del x, y
    from bench import kernel_flops
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    dev = "cuda:0"
    cfg = preset("syn_hotdog_b", rays=args.rays)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22))
    model = model.to(dev)
    tr = Trainer(cfg, is_inference=False, model=model)
    batch = {k: v.to(dev) for k, v in synthetic.make_batch(args.rays, frame=0).items()}
    if args.ray_order != "random":
        idx = batch["ray_idx"].reshape(-1)
        order = torch.argsort(idx)
        if args.ray_order == "xcd":   # band x of the sorted rays -> slots x, x + 8, x + 16, ...
            n = order.numel()
            order = order.reshape(8, n // 8).t().reshape(-1)
        for k, v in list(batch.items()):
            if v.dim() >= 2 and v.shape[1] == idx.numel():
                batch[k] = v[:, order]
        print("ray order", args.ray_order)
    for _ in range(3):
        tr.train_step(batch)
    torch.cuda.synchronize()
    eng = model.engine
    rays, dists, fld, hd, comp = model._last_state
    R, N = args.rays, model.pcfg.n_samples
    if args.dump:
        d0 = eng.sample(rays, None)
        f0 = eng.field(rays, d0, True)
        torch.save({"dists": d0.cpu(), **{k: f0[k].cpu() for k in ("sdf", "grad", "hess", "h0") if k in f0}}, args.dump)
    res = {}
    res["sample (all rounds)"] = timeit(lambda: eng.sample(rays, None), args.reps)
    res["sdf field"] = timeit(lambda: eng.field(rays, dists, True), args.reps)
    res["heads fwd train"] = timeit(lambda: eng.heads(rays, dists, fld, True), args.reps)
    res["heads fwd eval"] = timeit(lambda: eng.heads(rays, dists, fld, False), args.reps)
    hd = eng.heads(rays, dists, fld, True)
    comp = eng.composite(rays, dists, fld, hd, model.s_var.detach(), 0.0, True)
    st = (rays, dists, fld, hd, comp)
    g = torch.zeros_like(model.flat)
    d = torch.full((R, 3), 1e-4, device=dev)
    d1 = torch.full((R, 1), 1e-4, device=dev)
    res["backward (all)"] = timeit(lambda: eng.backward(st, d, d, d1, d, model.flat, model._sdf_l1(), g), args.reps)
    res["pack heads"] = timeit(lambda: eng.pack_heads(model.flat.detach(), model._sdf_l1()), args.reps)
    flops = {"sdf field": kernel_flops("mli_sdf:field", R, N, 64, 16, 4),
             "heads fwd train": kernel_flops("mli_rgb_fwd", R, N, 64, 16, 4),
             "heads fwd eval": kernel_flops("mli_rgb_fwd", R, N, 64, 16, 4)}
    for k, (med, mn) in res.items():
        tf = flops.get(k)
        print("%-22s median %8.3f ms  min %8.3f ms%s" % (k, med, mn, "  %.1f TF/s" % (tf / med / 1e9) if tf else ""))
    # per-kernel split of the backward via the live event profiler
    from mli_nerf_amd import _lib as L
    L.PROFILE = []
    for _ in range(5):
        eng.backward(st, d, d, d1, d, model.flat, model._sdf_l1(), g)
    torch.cuda.synchronize()
    agg = {}
    for name, e0, e1 in L.PROFILE:
        agg.setdefault(name, []).append(e0.elapsed_time(e1))
    L.PROFILE = None
    for k, v in agg.items():
        print("  bwd %-20s %8.3f ms" % (k, statistics.median(v)))


if __name__ == "__main__":
    main()
