"""Stage-a kernel micro-benchmark: one stage-a step at the bench shape, then the geometry
backward kernels timed alone (median of --reps launches).  Run once per library variant:
MLI_HIP_LIB=<experiment .so> python tools/kbench_a.py (experiment builds: mli_nerf_amd.build
with -D flags, see tools/kbench_a.sh)."""
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
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--iteration", type=int, default=100000)
    args = ap.parse_args()
    from mli_nerf_amd import _lib as L, synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    dev = "cuda:0"
    cfg = preset("syn_hotdog_a", rays=args.rays)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22, heads="rgb"))
    model = model.to(dev)
    tr = Trainer(cfg, model)
    tr.current_iteration = args.iteration
    tr._start_of_iteration()
    batch = {k: v.to(dev) for k, v in synthetic.make_batch(args.rays, frame=0).items()}
    st, _ = tr.compute_grads_a(batch)
    torch.cuda.synchronize()
    eng = model.engine
    rays, dists, fld, hd, comp = st
    N, R = dists.shape
    gt = tr._grad_table

    def hash_bwd():
        L.call("mli_hash_bwd", L.HashBwdArgs(R, N, L.ptr(rays["center"]), L.ptr(rays["ray_unit"]), L.ptr(dists),
                                             L.ptr(eng._bufs["d_enc"]), eng.levels, eng.eps,
                                             int(eng.active_levels), L.ptr(gt)))
    print("%s  hash_bwd %.3f ms  zero_table %.3f ms" % (os.environ.get("MLI_HIP_LIB", "default"),
                                                     timeit(hash_bwd, args.reps), timeit(gt.zero_, args.reps)),
          flush=True)


if __name__ == "__main__":
    main()
