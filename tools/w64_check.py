"""EXPERIMENT: eval heads forward, W64 kernel (64 samples per wave) vs the product kernel, in one
process on an experiment library: bit-identical outputs and timing.  python tools/w64_check.py <lib>"""
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
lib_path = os.path.abspath(sys.argv[1])
from mli_nerf_amd import _lib as L, build as B  # noqa: E402

L.LIB_PATH = lib_path
want = B.built_hash(lib_path)
B.source_hash = lambda: want
import torch  # noqa: E402


def timeit(fn, reps=20):
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
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    dev = "cuda:0"
    R = int(os.environ.get("W64_RAYS", "20000"))
    cfg = preset("syn_hotdog_b", rays=4096)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22))
    model = model.to(dev)
    tr = Trainer(cfg, is_inference=False, model=model)
    batch = {k: v.to(dev) for k, v in synthetic.make_batch(4096, frame=0).items()}
    tr.train_step(batch)
    model.eval()
    model.prepare()
    eng = model.engine
    b2 = {k: v.to(dev) for k, v in synthetic.make_batch(R, frame=1).items()}
    rays = eng.rays(b2["pose"], b2["intr"], b2["pose_light"], b2["ray_idx"], 512)
    dists = eng.sample(rays, None)
    fld = eng.field(rays, dists, False)
    torch.cuda.synchronize()
    os.environ.pop("MLI_W64", None)
    y0 = eng.heads(rays, dists, fld, False)["y"].clone()
    for v in ("1", "2"):
        os.environ["MLI_W64"] = v
        y1 = eng.heads(rays, dists, fld, False)["y"].clone()
        torch.cuda.synchronize()
        d = (y0 - y1).abs().max().item()
        print("W64 variant %s vs product: max |dy| = %g, identical %s" % (v, d, torch.equal(y0, y1)))
    S = R * dists.shape[0]
    from bench import kernel_flops
    fl = kernel_flops("mli_rgb_fwd", R, dists.shape[0], 64, 16, 4)
    for arm in ("product", "w64", "w64d", "product", "w64", "w64d"):
        if arm == "product":
            os.environ.pop("MLI_W64", None)
        else:
            os.environ["MLI_W64"] = "1" if arm == "w64" else "2"
        med, mn = timeit(lambda: eng.heads(rays, dists, fld, False))
        print("%-8s eval heads fwd %d rays x %d: median %.3f ms  min %.3f  %.1f TF/s" % (
            arm, R, dists.shape[0], med, mn, fl / med / 1e9))


if __name__ == "__main__":
    main()
