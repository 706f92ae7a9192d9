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
    from bench import kernel_flops
    dev = "cuda:0"
    R = int(os.environ.get("W64_RAYS", "20000"))
    cfg = preset("syn_hotdog_b", rays=4096)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22))
    model = model.to(dev)
    tr = Trainer(cfg, is_inference=False, model=model)
    batch = {k: v.to(dev) for k, v in synthetic.make_batch(4096, frame=0).items()}
    tr.train_step(batch)
    # training (PQ) forward on the 4096-ray batch: every output buffer bit-identical
    model.train()
    eng = model.engine
    rays_t, dists_t, fld_t = model._last_state[0], model._last_state[1], model._last_state[2]
    sv = model.s_var.detach()

    def train_fwd():
        hd = eng.heads(rays_t, dists_t, fld_t, True, sv, 0.0)
        torch.cuda.synchronize()
        return {k: v.clone() for k, v in hd.items() if torch.is_tensor(v)}
    os.environ.pop("MLI_W64", None)
    ref = train_fwd()
    for v in ("1", "2"):
        os.environ["MLI_W64"] = v
        got = train_fwd()
        bad = [k for k in ref if not torch.equal(ref[k], got[k])]
        print("W64 train variant %s vs product: mismatching buffers %s" % (v, bad or "none"))
        for k in bad:
            print("   %s max |d| %g" % (k, (ref[k].float() - got[k].float()).abs().max().item()))
    ft = kernel_flops("mli_rgb_fwd", 4096, dists_t.shape[0], 64, 16, 4)
    for arm in ("product", "w64", "w64d", "product", "w64", "w64d"):
        if arm == "product":
            os.environ.pop("MLI_W64", None)
        else:
            os.environ["MLI_W64"] = "1" if arm == "w64" else "2"
        med, mn = timeit(lambda: eng.heads(rays_t, dists_t, fld_t, True, sv, 0.0))
        print("%-8s train heads fwd (PQ, incl. weights) 4096 x %d: median %.3f ms  min %.3f  %.1f TF/s" % (
            arm, dists_t.shape[0], med, mn, ft / med / 1e9))
    # full deterministic training step (heads fwd + bwd dX chain W64) vs product: flat gradient
    def step_grad(env):
        for k in ("MLI_W64", "MLI_W64B"):
            os.environ.pop(k, None)
        os.environ.update(env)
        m2 = Model(cfg.model, cfg.data)
        m2.load_state_dict(synthetic.make_state_dict(log2T=22))
        m2 = m2.to(dev)
        t2 = Trainer(cfg, is_inference=False, model=m2)
        m2.deterministic = True
        t2.train_step(batch, u=torch.full((1, 4096, 64), 0.5, device=dev))
        torch.cuda.synchronize()
        return t2._grad.clone(), float(t2.losses["total"])
    g_ref, l_ref = step_grad({})
    for env in ({"MLI_W64B": "1"}, {"MLI_W64B": "2"}, {"MLI_W64": "2", "MLI_W64B": "2"}):
        g, l = step_grad(env)
        print("full step %s vs product: grad identical %s, max |dg| %g, loss %r vs %r" % (
            env, torch.equal(g, g_ref), (g - g_ref).abs().max().item(), l, l_ref))
    for k in ("MLI_W64", "MLI_W64B"):
        os.environ.pop(k, None)
    # backward dX chain timing (rgb_bwd alone through the live event profiler)
    for arm in ("product", "b1", "b2", "product", "b1", "b2"):
        os.environ.pop("MLI_W64B", None)
        if arm != "product":
            os.environ["MLI_W64B"] = arm[1]
        L.PROFILE, L.PROFILE_NAMES = [], {"mli_rgb_bwd"}
        for _ in range(10):
            tr.train_step(batch)
        torch.cuda.synchronize()
        ts = [e0.elapsed_time(e1) for n, e0, e1 in L.PROFILE]
        L.PROFILE = None
        print("%-8s rgb_bwd median %.3f ms" % (arm, statistics.median(ts)))
    os.environ.pop("MLI_W64B", None)
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
