"""Heads-forward knockout A/B (rgb_fwd_kernel, train + eval) at the bench shape.

Usage: bash tools/kbench_fwd.sh build   (here), then bash tools/kbench_fwd.sh run (GPU box).
Each variant library removes one ingredient (DMA refills, per-phase barriers, MFMAs,
staging stores); its time says what that ingredient costs.  Results of the knockout
builds are numerically invalid by design -- timing only.
"""
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402


def main():
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    dev = "cuda:0"
    R = 4096
    cfg = preset("syn_hotdog_b", rays=R)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22))
    model = model.to(dev)
    tr = Trainer(cfg, model)
    batch = {k: v.to(dev) for k, v in synthetic.make_batch(R, frame=0).items()}
    for _ in range(2):
        tr.train_step(batch)
    torch.cuda.synchronize()
    eng = model.engine
    rays, dists, fld, hd, comp = model._last_state
    out = []
    for train in (True, False):
        ts = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.heads(rays, dists, fld, train)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out.append("%s %.3f ms" % ("train" if train else "eval", statistics.median(ts[5:])))
    print(os.environ.get("MLI_HIP_LIB", "product"), " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
