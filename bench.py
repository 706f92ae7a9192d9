#!/usr/bin/env python
"""Benchmark: MLI-NeRF stage-b training step (syn_hotdog_b, 4096 rays x 128 samples per GPU).

One step = one pass of the hot path over one batch: ray generation, hierarchical sampling,
SDF field + 4 taps, the three light-conditioned heads, NeuS compositing, the stage-b losses,
backward through the heads and the fused AdamW update (BASELINE.json configs[1]).
Synthetic seeded inputs / random-init weights of the reference architecture (no dataset
or checkpoint on the box); full-size hash table (log2 T = 22).

Multi-GPU: one process per GPU (from torch.distributed.run, or spawned here by ``--gpus N``
when no launcher set WORLD_SIZE); each rank renders its own image's rays, one RCCL all-reduce
of the 3.2 MB flat gradient (with the step's loss terms and PSNR in its tail) per step (DDP
semantics); weak scaling, value = all ranks' rays / the slowest rank's time.

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


def progress(msg):
    """Progress line on stderr (long runs must keep writing: the GPU box kills silent ones)."""
    print("[bench] " + msg, file=sys.stderr, flush=True)


def kernel_flops(name, R, N, Nc, Nf, H, stage="b"):
    """Algorithmic MLP FLOPs (2*MAC) per step (unit) of each MFMA kernel.
    Stage a (LumenRGB mode 'rgb': the single 294 -> 3 head, geometry trained) adds the
    geometry backward: mli_geo_bwd (head dX chain + W0^T to feat/normal + SDF layer 1 dX),
    mli_sdf_bwd (layer 0 recomputed and d enc = W0_enc^T dZ0 for the 5 points) and the two
    dW launches (S samples: head + SDF layer 1; 5S samples: SDF layer 0)."""
    S = R * N
    sdf_point = 2 * ((3 + 128) * HIDDEN + HIDDEN)                  # layer 0 + sdf head
    head_in, head_out = (HEAD_IN[:1], HEAD_OUT[:1]) if stage == "a" else (HEAD_IN, HEAD_OUT)
    heads_fwd = sum(k * HIDDEN + 3 * HIDDEN * HIDDEN + HIDDEN * o for k, o in zip(head_in, head_out))
    if name == "mli_rgb_fwd":
        return 2 * S * (HIDDEN * HIDDEN + heads_fwd)               # SDF layer 1 (feat) + heads
    if name == "mli_sdf:field":
        return 5 * S * sdf_point
    if stage == "a":
        if name == "mli_geo_bwd":  # W4^T..W1^T, W0^T onto feat + normal, W1sdf^T
            return 2 * S * (HIDDEN * 3 + 3 * HIDDEN * HIDDEN + HIDDEN * (HIDDEN + 3) + HIDDEN * HIDDEN)
        if name == "mli_sdf_bwd":  # per point: z0 recompute (131 x 256) + d enc (256 -> 128)
            return 2 * 5 * S * ((3 + 128) * HIDDEN + 128 * HIDDEN)
        if name == "mli_wgrad":    # both launches: head + SDF layer 1 over S, SDF layer 0 over 5S
            return 2 * S * (heads_fwd + HIDDEN * HIDDEN) + 2 * 5 * S * HIDDEN * (3 + 128)
        return 0
    if name == "mli_rgb_bwd":
        return 2 * S * sum(HIDDEN * o + 3 * HIDDEN * HIDDEN for o in HEAD_OUT)
    if name == "mli_dw4":          # algorithmic: the output layers' dW (3 / 3 / 1 rows), contracted
        # in the heads forward (q4) and finished here -- the FLOPs of the THIN class it replaces
        return 2 * S * HIDDEN * sum(HEAD_OUT)
    if name == "mli_wgrad":
        return 2 * S * heads_fwd
    if name == "mli_wgrad:big":    # dW of the 256x256 hidden layers L1..L3 of the 3 heads
        return 2 * S * 3 * 3 * HIDDEN * HIDDEN
    if name == "mli_wgrad:wide":   # dW of layer 0 (294 / 262 / 278 inputs)
        return 2 * S * HIDDEN * sum(HEAD_IN)
    if name == "mli_wgrad:thin":   # dW of the output layers (3 / 3 / 1 rows)
        return 2 * S * HIDDEN * sum(HEAD_OUT)
    return 0


PMC_SUMMARY = os.environ.get("MLI_PMC_SUMMARY") or os.path.join(HERE, "profiles", "r6", "final", "pmc_summary.json")
PMC_SAMPLES = 4096 * 128  # the workload the committed PMC passes ran (tools/pmc.sh: bench.py defaults)


def pmc_traffic(kernel, n_units_check):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary
    (tools/pmc.sh + tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md
    §HBM corrections), when it was collected on this same workload."""
    try:
        with open(PMC_SUMMARY) as f:
            summ = json.load(f)
    except OSError:
        return None
    rec = summ.get(kernel)
    if rec is None or n_units_check != PMC_SAMPLES:
        return None
    return {"traffic": round(rec["hbm_bytes"]), "traffic_read": round(rec["hbm_read_bytes"]),
            "traffic_write": round(rec["hbm_write_bytes"]),
            "traffic_source": os.path.relpath(PMC_SUMMARY, HERE) + " (rocprofv3 --pmc, separate passes)"}


def kernel_table(prof, n_units, R, N, fine, stage="b", per_launch=False):
    """Per-call-name HIP-event timings -> table + roofline record of the dominant MFMA call
    (FLOPs per step / kernel time per step; = per launch for the one-launch kernels).
    per_launch: kernel_flops(R) counts one launch (inference chunks of R rays)."""
    kernels = {}
    for name, e0, e1 in prof or []:
        k = kernels.setdefault(name, [0.0, 0])
        k[0] += e0.elapsed_time(e1)
        k[1] += 1
    ktab = {n: {"ms_per_launch": v[0] / v[1], "launches_per_unit": v[1] / n_units,
                "ms_per_unit": v[0] / n_units} for n, v in sorted(kernels.items(), key=lambda kv: -kv[1][0])}
    def flops(n):
        f = kernel_flops(n, R, N, 64, fine, 4, stage)
        return f * ktab[n]["launches_per_unit"] if per_launch and n in ktab else f
    roof = None
    mfma = [n for n in ktab if flops(n) > 0]
    if mfma:
        dom = max(mfma, key=lambda n: ktab[n]["ms_per_unit"])
        fl = flops(dom)
        achieved = fl / (ktab[dom]["ms_per_unit"] * 1e-3) / 1e12
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_F16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_F16_TFLOPS, 4), "traffic": None,
                "flops_per_launch": int(fl / ktab[dom]["launches_per_unit"])}
        pmc = pmc_traffic(dom, n_units_check=R * N) if stage == "b" else None
        if pmc:
            roof.update(pmc)
        for n in ktab:
            f = flops(n)
            if f:
                ktab[n]["tflops"] = round(f / (ktab[n]["ms_per_unit"] * 1e-3) / 1e12, 2)
    return ktab, roof


def run_infer(args, world, rank, dev):
    """configs[4]: syn_hotdog_b video_train inference, size x size frames rendered in
    `chunk`-ray chunks, tile-sharded over the ranks with one all_gather per frame
    (Model.inference); rays/s = frames * size^2 / wall time (strong scaling)."""
    from mli_nerf_amd import _lib as L, synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    size = args.size
    over = {"data": {"train": {"image_size": [size, size]}, "val": {"image_size": [size, size]}},
            "model": {"render": {"rand_rays_val": args.chunk}}}
    if args.vis:  # the pseudo-label inference (test.py with light_visibility, syn_hotdog_b.yaml:73-78)
        over["model"]["light_visibility"] = {"enabled": True, "camera_ray_type": "blend_z_sphere_tracing",
                                             "type": "sphere_tracing", "visibility_bounding_type": "sphere",
                                             "visibility_sphere_radius": 0.95}
    cfg = preset(args.config, n_fine=args.fine, overrides=over)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=22, seed=0))
    model = model.to(dev)
    N = model.pcfg.n_samples
    frames = [{k: v.to(dev) for k, v in synthetic.make_batch(1, H=size, W=size, frame=f).items()}
              for f in range(args.warmup + args.frames)]

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    for f in range(args.warmup):
        model.inference(frames[f])
    PLATFORM.sync()
    barrier()
    PLATFORM.sync()
    t0 = time.perf_counter()
    out = None
    for f in range(args.warmup, args.warmup + args.frames):
        out = model.inference(frames[f])
    PLATFORM.sync()
    barrier()
    PLATFORM.sync()
    elapsed = time.perf_counter() - t0
    # per-kernel HIP events over one more (untimed) frame rendered with the chunk pipeline off:
    # with two chunks in flight an event pair would also time the other stream's kernels
    n_prof = 0 if args.no_kernel_timing else 1
    if n_prof:
        model.pipeline_chunks = False
        L.PROFILE = []
        model.inference(frames[-1])
        torch.cuda.synchronize()
        model.pipeline_chunks = True
    prof, L.PROFILE = L.PROFILE, None
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    n_pix = size * size
    value = n_pix * args.frames / elapsed
    R_chunk = min(args.chunk, -(-n_pix // world))
    ktab, roof = kernel_table(prof, max(n_prof, 1), R_chunk, N, args.fine, per_launch=True)
    result = {
        "metric": "rays/sec, syn_hotdog_b video_train inference %dx%d full frame (configs[4])%s" % (
            size, size, " + light visibility" if args.vis else ""),
        "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": args.frames,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.frames * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp16",
        "dtype_detail": "fp16 MFMA operands, fp32 accumulate; fp32 sampling / compositing / losses / AdamW",
        "data": "synthetic (seeded cameras/lights, random-init weights, full 2^22 hash table)",
        "config": {"workload": "%s inference, %dx%d frames, %d-ray chunks, tile-sharded" % (args.config, size, size,
                                                                                            args.chunk),
                   "samples_per_ray": N, "frames": args.frames, "parallelism": "tiles%d" % world},
        "roofline": roof, "kernels": ktab,
        "rgb_mean": round(float(out["rgb"].mean()), 5),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        # CPU oracle eval forward on a bounded sample of the same frame's rays
        from oracle import render as o_render
        threads, hc = cpu_threads(args)
        torch.set_num_threads(threads)
        sd = synthetic.make_state_dict(log2T=22, seed=0)
        # the GPU gathers an fp16 shadow of the table (tcnn's precision): same values here
        sd["neural_sdf.tcnn_encoding.params"] = sd["neural_sdf.tcnn_encoding.params"].half().float()
        pcfg = oracle_cfg(cfg)
        data = {k: v.cpu() for k, v in frames[-1].items()}  # the last rendered frame is `out`
        n_cpu = args.cpu_rays * 4
        data["ray_idx"] = torch.arange(n_cpu)[None] * (n_pix // n_cpu)
        # the GPU's own samples of these rays (eval forward: same kernels as the inference chunks)
        model.eval()
        gpu_fwd = model({k: v.to(dev) for k, v in data.items()})
        gpu_dists = gpu_fwd["dists"].detach().cpu()
        with torch.no_grad():
            o_render.forward(sd, pcfg, data, u=None, training=False, width=size, height=size)
            t1 = time.perf_counter()
            ref = o_render.forward(sd, pcfg, data, u=None, training=False, width=size, height=size)
            t_cpu = time.perf_counter() - t1
            ref_cond = o_render.forward(sd, pcfg, data, u=None, training=False, width=size, height=size,
                                        dists=gpu_dists)
        result["cpu_baseline"] = {"value": round(n_cpu / t_cpu, 3), "unit": "rays/s", "cores": threads,
                                  "kind": "port", "sample": "oracle eval forward, %d rays of one %dx%d frame x %d "
                                  "samples, full hash table, torch fp32 on %d host threads" % (n_cpu, size, size, N,
                                                                                             threads),
                                  "host": hc}
        result["speedup_vs_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
        gpu_rgb = out["rgb"][0].cpu()[data["ray_idx"][0]]

        def diff(a, b):
            d = (a - b).abs()
            return {"max_abs": round(float(d.max()), 6),
                    "psnr_of_diff_db": round(-10 * math.log10(max(float((d ** 2).mean()), 1e-20)), 2)}
        # free-running: the hierarchical sampler is chaotic (inv_s up to 512), a 1e-6 sdf
        # difference can move a fine sample; conditioned: the oracle fed the GPU's samples
        result["rgb_check"] = {"rays": n_cpu, "free": diff(gpu_rgb, ref["rgb"][0]),
                               "conditioned_on_gpu_samples": diff(gpu_fwd["rgb"][0].detach().cpu(),
                                                                  ref_cond["rgb"][0]),
                               "inference_vs_forward_max_abs": float((gpu_rgb - gpu_fwd["rgb"][0].cpu()).abs().max())}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def oracle_cfg(cfg):
    """The oracle's PathCfg for a preset (same sampling, background, bounds as the GPU run)."""
    from oracle import render as o_render
    r = cfg.model.render
    return o_render.PathCfg(n_coarse=r.num_samples.coarse, n_fine=r.num_samples.fine,
                            n_hier=r.num_sample_hierarchy, white_bg=bool(cfg.model.background.white),
                            bounding="box" if cfg.data.get("bounding_type") == "box" else "sphere",
                            aabb=tuple(cfg.data.get("bounding_box_aabb", (-1, -1, -1, 1, 1, 1))))


def cpu_baseline(cfg, R_cpu, steps, threads, stage_a=None):
    """The CPU oracle (fp32 PyTorch restatement of the reference path) timed on the host:
    forward + losses + backward on R_cpu rays of the same workload (stage b: into the heads;
    stage a, ``stage_a`` = (active_levels, anneal_levels, curvature weight, progress): into
    every parameter incl. the hash table)."""
    from mli_nerf_amd import synthetic
    from oracle import render as o_render
    torch.set_num_threads(threads)
    pcfg = oracle_cfg(cfg)
    if stage_a is not None:
        sd = synthetic.make_state_dict(log2T=22, heads="rgb")
        sd = {k: v.requires_grad_(True) for k, v in sd.items()}
        pcfg.rgb_mode, pcfg.active_levels, pcfg.anneal_levels = "rgb", stage_a[0], stage_a[1]
    else:
        sd = synthetic.make_state_dict(log2T=22)
        sd = {k: v.requires_grad_(k.startswith("neural_rgb")) for k, v in sd.items()}
    Hh, W = cfg.data.train.image_size
    data = synthetic.make_batch(R_cpu, H=Hh, W=W, frame=0, seed=7)
    u = synthetic.stratified_uniforms(R_cpu, pcfg.n_coarse, seed=7)
    times = []
    out = psnr = None
    for i in range(steps + 2):  # 2 untimed warm-up steps
        t0 = time.perf_counter()
        if stage_a is not None:
            out = o_render.forward(sd, pcfg, data, u=u, training=True, progress=stage_a[3], width=W, height=Hh)
            total, _, psnr = o_render.stage_a_losses(out, data, stage_a[2])
        else:
            out = o_render.forward(sd, pcfg, data, u=u, training=True, progress=0.0, width=W, height=Hh)
            total, _, psnr = o_render.stage_b_losses(out, data, pcfg)
        total.backward()
        for v in sd.values():
            v.grad = None
        if i > 1:
            times.append(time.perf_counter() - t0)
        progress("cpu baseline step %d/%d: %.2f s" % (i + 1, steps + 2, time.perf_counter() - t0))
    t = sum(times) / len(times)
    return dict(value=R_cpu / t, unit="rays/s", cores=threads, kind="port", per_thread=R_cpu / t / threads,
                sample="oracle fwd+bwd stage-%s, %d rays x %d samples, full hash table, %d timed steps "
                       "after 2 warm-up, torch fp32 on %d host threads" % ("a" if stage_a else "b", R_cpu,
                                                                          pcfg.n_samples, steps, threads),
                s_per_step=t), data, u, float(psnr)


def host_cpu():
    """The host CPU for the cpu_baseline record (lscpu model, sockets, cores,
    threads) and the threads the baseline uses: the physical cores this process may run on
    (its affinity mask, SMT siblings counted once), capped by the job's CPU share
    (OMP_NUM_THREADS: the GPU box allots 16 CPUs per one-GPU job; nproc / os.cpu_count() there
    show the whole machine) unless ``--cpu-threads`` says otherwise."""
    info = {"model": None, "sockets": None, "cores_per_socket": None, "threads_per_core": None,
            "logical_cpus": os.cpu_count()}
    try:
        blocks = open("/proc/cpuinfo").read().strip().split("\n\n")
        recs = [dict((k.strip(), v.strip()) for k, _, v in (ln.partition(":") for ln in b.splitlines())) for b in blocks]
        info["model"] = recs[0].get("model name")
        sockets = {r.get("physical id") for r in recs}
        info["sockets"] = len(sockets)
        cores = int(recs[0].get("cpu cores", 0)) or None
        info["cores_per_socket"] = cores
        if cores:
            info["threads_per_core"] = int(recs[0].get("siblings", cores)) // cores
    except (OSError, ValueError, IndexError):
        pass
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    phys = set()
    for c in cpus:
        try:
            with open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c) as f:
                phys.add(f.read().strip().split(",")[0].split("-")[0])
        except OSError:
            phys.add(str(c))
    info["affinity_cpus"] = len(cpus)
    info["affinity_physical_cores"] = len(phys)
    share = os.environ.get("OMP_NUM_THREADS")
    info["job_cpu_share"] = int(share) if share and share.isdigit() else None
    return info


def cpu_threads(args):
    """(threads, host info); host["threads_rule"] says which count was taken and why (VERDICT r5
    item 8): SURVEY §8(d) asks for the physical cores, and the affinity mask's physical cores are
    that count; on the GPU box a one-GPU job is allotted a share of the host (OMP_NUM_THREADS, 16)
    and the rest of the cores run other jobs, so the baseline takes the smaller of the two and the
    record says so (the per-thread rate is reported beside it)."""
    hc = host_cpu()
    if args.cpu_threads:
        hc["threads_rule"] = "--cpu-threads %d (explicit)" % args.cpu_threads
        return args.cpu_threads, hc
    n = hc["affinity_physical_cores"] or 1
    rule = "affinity physical cores (%d)" % n
    if hc["job_cpu_share"] and hc["job_cpu_share"] < n:
        rule = ("job CPU share OMP_NUM_THREADS=%d < affinity physical cores %d (SURVEY 8d's count): the box "
                "allots %d CPUs to this one-GPU job, the other cores belong to other jobs" % (
                    hc["job_cpu_share"], n, hc["job_cpu_share"]))
        n = hc["job_cpu_share"]
    hc["threads_rule"] = rule
    return n, hc


def count_gpus():
    """GPUs this process may use, counted WITHOUT initialising HIP: the KFD topology nodes that
    have SIMDs (sysfs), narrowed by ROCR/HIP/CUDA_VISIBLE_DEVICES.  The parent of ``--gpus N``
    spawns the ranks and must never open the GPU itself (a process that initialised HIP must not
    start others by fork / exec)."""
    import re
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    for d in (sorted(os.listdir(base)) if os.path.isdir(base) else []):
        try:
            with open(os.path.join(base, d, "properties")) as f:
                props = f.read()
        except OSError:
            continue
        m = re.search(r"^simd_count\s+(\d+)", props, re.M)
        if m and int(m.group(1)) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def gpu_handles():
    """This process's open GPU device files (/dev/kfd, /dev/dri/*): empty while HIP is untouched."""
    out = []
    fd_dir = "/proc/self/fd"
    for fd in (os.listdir(fd_dir) if os.path.isdir(fd_dir) else []):
        try:
            tgt = os.readlink(os.path.join(fd_dir, fd))
        except OSError:
            continue
        if tgt == "/dev/kfd" or tgt.startswith("/dev/dri/"):
            out.append(tgt)
    return out


class HipPlatform:
    """A rank's device plumbing: its GPU, stream sync, the collective backend.
    tests/test_bench_launch.py swaps in a CPU stand-in (with tests/stub_engine.py) to rehearse the
    --gpus N process flow end to end on CPU; the bench itself always runs this one."""
    name = "hip"

    def device(self, local):
        torch.cuda.set_device(local)
        return torch.device("cuda", local)

    def sync(self):
        torch.cuda.synchronize()

    def priority_range(self):
        return torch.cuda.Stream.priority_range()

    def backend(self, rehearse):
        return "gloo" if rehearse else "nccl"


PLATFORM = HipPlatform()


def cu_mask_stream(dev, spec):
    """Experiment: a stream whose kernels run only on a CU subset (hipExtStreamCreateWithCUMask),
    wrapped as a torch ExternalStream.  spec: every:K (CU ids i % K == 0), skip:K (the rest),
    first:K (ids 0..K-1)."""
    import ctypes
    kind, k = spec.split(":")
    k = int(k)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    sel = {"every": lambda i: i % k == 0, "skip": lambda i: i % k != 0, "first": lambda i: i < k}[kind]
    words = [0] * ((ncu + 31) // 32)
    for i in range(ncu):
        if sel(i):
            words[i // 32] |= 1 << (i % 32)
    hip = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError("hipExtStreamCreateWithCUMask: %d" % rc)
    progress("stream %s: %d of %d CUs" % (spec, sum(bin(w).count("1") for w in words), ncu))
    return torch.cuda.ExternalStream(s.value, device=dev)
WORKER_SCRIPT = None   # the rank program --gpus N spawns (default: this file)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_workers(n, argv, script=None, poll_s=0.2):
    """``--gpus N`` without a launcher: start N processes, one per GPU, with the environment
    torch.distributed.run gives its workers (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
    MASTER_ADDR=127.0.0.1, MASTER_PORT), and wait for them.  This process never touches the GPU.
    The workers inherit stdout / stderr (rank 0 prints the JSON line); if one fails the others
    are stopped (they would wait in a collective forever).  Returns the first non-zero exit
    code, else 0."""
    import subprocess
    script = script or os.path.abspath(__file__)
    held = gpu_handles()
    if held:
        raise RuntimeError("launch_workers: this process holds GPU device files %s; the ranks must be "
                           "started by a process that never initialised HIP" % held)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]   # poll every process (no short-circuit)
            if all(c is not None for c in codes):
                break
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc or next((p.returncode for p in procs if p.returncode), 0)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; without a launcher's WORLD_SIZE, one process per GPU is spawned")
    ap.add_argument("--steps", type=int, default=200, help="timed steps (200 x ~5 ms: a >= 1 s timed region)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="syn_hotdog_b")
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--fine", type=int, default=16)
    ap.add_argument("--cpu-rays", type=int, default=512)
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="cpu_baseline threads (default: the physical cores of this process's affinity mask, "
                         "capped by the job's CPU share OMP_NUM_THREADS)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--time-all-kernels", action="store_true",
                    help="train: HIP events around every launch (default: the MFMA kernels only; "
                         "each event pair costs GPU time between launches)")
    ap.add_argument("--pipeline", choices=("off", "call", "heads", "wgrad"), default="heads",
                    help="train: prefetch the next batch's geometry (sampling/FIELD) on a side stream, "
                         "gated as Trainer.prefetch_gate (heads: after the heads forward of the step in "
                         "flight); measured 4.77 vs 5.07 ms/step off (profiles/r2/s7)")
    ap.add_argument("--priority", choices=("none", "main", "side"), default="none",
                    help="pipeline: run the step on a high-priority stream (main) or give the prefetch "
                         "stream the high priority (side)")
    ap.add_argument("--prefetch-depth", type=int, default=2, choices=(1, 2),
                    help="pipeline: batches prefetched ahead of the trained one (2: the geometry of step "
                         "k+2 runs beside step k and never holds up step k+1)")
    ap.add_argument("--side-cus", default=None,
                    help="pipeline experiment: restrict the prefetch stream to a CU subset "
                         "(hipExtStreamCreateWithCUMask): every:K = CUs i %% K == 0, first:K, skip:K = the complement of every:K")
    ap.add_argument("--main-cus", default=None, help="pipeline experiment: the same for the step's stream")
    ap.add_argument("--tail", choices=("fused", "three"), default="fused",
                    help="stage-b training tail: fused (mli_composite_loss, one launch) or the three calls "
                         "mli_composite_fwd / mli_stage_b_loss / mli_composite_bwd")
    ap.add_argument("--pq", choices=("on", "off"), default="on",
                    help="stage-b output-layer dW: on = per-tile partials formed in the heads forward "
                         "(mli_rgb_fwd PQ mode + mli_dw4; X3 never written), off = X3 through HBM and the "
                         "THIN split-K class")
    ap.add_argument("--mode", choices=("train", "infer"), default="train",
                    help="train: BASELINE configs[1] step; infer: configs[4] full-frame render")
    ap.add_argument("--frames", type=int, default=4, help="infer: frames timed (after --warmup frames)")
    ap.add_argument("--vis", action="store_true", help="infer: light visibility on (sphere-traced camera/light rays)")
    ap.add_argument("--size", type=int, default=800, help="infer: frame is size x size")
    ap.add_argument("--chunk", type=int, default=20000, help="infer: rand_rays_val")
    ap.add_argument("--iteration", type=int, default=100000,
                    help="stage a (--config syn_hotdog_a): training iteration (sets the coarse-to-fine "
                         "levels, tap epsilon and curvature weight; >= 80000: all 16 levels active)")
    args = ap.parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        n_dev = count_gpus()  # sysfs: HIP stays uninitialised in this process
        if n_dev < args.gpus:
            raise SystemExit("--gpus %d: only %d GPU(s) visible" % (args.gpus, n_dev))
        sys.exit(launch_workers(args.gpus, argv, script=WORKER_SCRIPT))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MLI_BENCH_REHEARSE=1: rehearse the N-rank path on a one-GPU box -- every rank on cuda:0 and
    # the collectives on gloo (RCCL refuses two ranks on one device); the line says so
    rehearse = os.environ.get("MLI_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    dev = PLATFORM.device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = PLATFORM.backend(rehearse)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from mli_nerf_amd import _lib as L, synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    if args.mode == "infer":
        return run_infer(args, world, rank, dev)

    cfg = preset(args.config, rays=args.rays, n_fine=args.fine)
    model = Model(cfg.model, cfg.data)
    stage_a = model.stage == "a"
    model.load_state_dict(synthetic.make_state_dict(log2T=22, seed=0, heads="rgb" if stage_a else "rgb_r_s"))
    model = model.to(dev)
    trainer = Trainer(cfg, is_inference=False, model=model, world_size=world)
    trainer.fused_tail = args.tail == "fused"
    model.pq = args.pq == "on"
    if stage_a:
        # steady state of stage a: past the coarse-to-fine ramp (all 16 levels active)
        trainer.current_iteration = args.iteration
    Hh, W = cfg.data.train.image_size
    R, N = args.rays, model.pcfg.n_samples
    # training frames resident in HBM; every step draws its R rays on the device
    # (mli_ray_batch: distinct pixels + image / pseudo-label gather) inside the timed region
    from mli_nerf_amd.data import DeviceFeed
    n_frames = 8
    g = torch.Generator().manual_seed(1000 + rank)
    cams = []
    real_cams = args.config == "rene_savannah_b"
    if real_cams:
        # configs[3]: the reference's real ReNe savannah camera + light poses, rank r -> frame r
        # (dataset_rene/savannah/train_transforms.json, package data mli_nerf_amd/assets/rene_savannah_train16.json)
        from mli_nerf_amd.data import rene_savannah_cameras
        cams = [rene_savannah_cameras(Hh, W, frames=[rank % 16])[0]] * n_frames
    for f in range(0 if real_cams else n_frames):
        fb = synthetic.make_batch(1, H=Hh, W=W, frame=rank * n_frames + f)
        cams.append((fb["intr"][0], fb["pose"][0], fb["pose_light"][0]))
    feed = DeviceFeed(device=dev, images=torch.rand(n_frames, 3, Hh * W, generator=g),
                      pseudo=(torch.rand(n_frames, 3, Hh * W, generator=g), torch.rand(n_frames, Hh * W, generator=g),
                              torch.rand(n_frames, Hh * W, generator=g)), cameras=cams)
    draws = iter(range(1 << 62))

    def next_batch():
        i = next(draws)
        return feed.batch(i % n_frames, (rank << 40) + i, R)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    # --pipeline: step k draws batch k+1 and issues its geometry (rays, sampling rounds, FIELD:
    # frozen SDF) on a side stream (Trainer.prefetch), and trains on batch k.  Every timed step
    # still draws, samples, renders and trains one full batch.  On by default (gate heads).
    # stream priorities (experiment): torch range (lowest, highest)
    lo, hi = PLATFORM.priority_range()
    if args.priority == "side":
        trainer.side_priority = hi
    main_stream = torch.cuda.Stream(device=dev, priority=hi) if args.priority == "main" else None
    if args.side_cus:
        trainer._side = cu_mask_stream(dev, args.side_cus)
    if args.main_cus:
        main_stream = cu_mask_stream(dev, args.main_cus)
    if main_stream is not None:
        torch.cuda.synchronize()
        torch.cuda.set_stream(main_stream)
    pipe = args.pipeline != "off" and model.stage == "b"
    depth = args.prefetch_depth if pipe else 1
    trainer.prefetch_depth = depth
    ahead = [next_batch() for _ in range(depth)]   # drawn (and prefetched) ahead of training
    if pipe:
        for b in ahead:
            trainer.prefetch(b)

    trainer.prefetch_gate = args.pipeline if pipe else "call"

    def step():
        nxt = next_batch()
        cur = ahead.pop(0)
        ahead.append(nxt)
        if pipe and args.pipeline == "call":
            trainer.prefetch(nxt)
        trainer.train_step(cur)
        if pipe and args.pipeline != "call":
            trainer.prefetch(nxt)

    for _ in range(args.warmup):
        step()
    PLATFORM.sync()
    progress("warm-up done (%d steps)" % args.warmup)
    barrier()
    PLATFORM.sync()
    names = None if args.time_all_kernels else {"mli_rgb_fwd", "mli_rgb_bwd", "mli_dw4", "mli_wgrad", "mli_sdf"}
    if not args.no_kernel_timing and not pipe:
        L.PROFILE = []  # per-kernel HIP events on the launch stream, over the timed region
        L.PROFILE_NAMES = names
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    PLATFORM.sync()
    barrier()
    PLATFORM.sync()
    elapsed = time.perf_counter() - t0
    progress("timed steps done: %.3f ms/step" % (elapsed / args.steps * 1e3))
    prof, L.PROFILE = L.PROFILE, None
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    psnr = trainer.metrics["psnr"].item()
    loss = trainer.losses["total"].item()
    k_steps = args.steps
    if pipe and not args.no_kernel_timing:
        # with the prefetch on, an event pair on one stream also times the other stream's
        # kernels: the per-kernel table comes from extra (untimed) steps with the pipeline off
        for b in ahead:                  # retire the prefetched batches
            trainer.train_step(b)
        k_steps = 200  # >= 1 s of GPU work whatever --steps is (per-kernel averages; a busy GPU for samplers)
        L.PROFILE, L.PROFILE_NAMES = [], names
        for _ in range(k_steps):
            trainer.train_step(next_batch())
        torch.cuda.synchronize()
        prof, L.PROFILE = L.PROFILE, None

    ktab, roof = kernel_table(prof, k_steps, R, N, args.fine, model.stage)

    step_ms = elapsed / args.steps * 1e3
    value = R * world * args.steps / elapsed
    result = {
        "metric": "rays/sec + PSNR, syn_hotdog 4096 rays x128 samples, 1/2/4/8 MI355X",
        "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp16",
        "dtype_detail": "fp16 MFMA operands, fp32 accumulate; fp32 sampling / compositing / losses / AdamW",
        "data": ("real ReNe savannah cameras/lights (frame = rank), synthetic images/labels, random-init "
                 "weights, full 2^22 hash table" if real_cams else
                 "synthetic (seeded cameras/lights/labels, random-init weights, full 2^22 hash table)"),
        "config": {"workload": "%s stage-%s train step" % (args.config, model.stage), "rays_per_gpu": R,
                   "samples_per_ray": N, "global_rays": R * world, "image": [Hh, W], "parallelism": "dp%d" % world,
                   "pipeline": ("geometry prefetch on a side stream, gate %s, %d batch(es) ahead" % (args.pipeline, depth)) if pipe else "off",
                   "output_layer_dw": "forward partials (pq)" if args.pq == "on" else "THIN split-K",
                   "tail": args.tail},
        "kernel_timing": ("HIP events on the launch stream over %d extra steps with the prefetch off" % k_steps)
        if pipe else "HIP events on the launch stream over the timed steps",
        "psnr": round(psnr, 4), "loss": round(loss, 6),
        "roofline": roof, "kernels": ktab,
        "mfma_tflops_step": round(sum(kernel_flops(n, R, N, 64, args.fine, 4, model.stage) for n in ktab) /
                                  (step_ms * 1e-3) / 1e12, 2),
        # peak HBM held by torch's allocator: the prefetch lanes each hold a full set of step buffers
        "hbm_peak_gib": (round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2)
                         if torch.device(dev).type == "cuda" else None),
    }
    if rehearse:  # every rank shared ONE GPU over gloo: a process-flow check, not a scaling number
        result["config"]["rehearsal"] = "%d ranks on one GPU, gloo collectives" % world
    if stage_a:
        sdf = model.neural_sdf
        result["config"].update(iteration=trainer.current_iteration - 1, active_levels=int(sdf.active_levels),
                                curvature_weight=trainer.weights["curvature"])
    if rank == 0 and world == 1 and not args.no_cpu and stage_a:
        threads, hc = cpu_threads(args)
        sdf = model.neural_sdf
        sa = (int(sdf.active_levels), int(sdf.anneal_levels), trainer.weights["curvature"], model.progress)
        cb, data_cpu, u_cpu, psnr_cpu = cpu_baseline(cfg, args.cpu_rays, args.cpu_steps, threads, stage_a=sa)
        result["cpu_baseline"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in cb.items()}
        result["cpu_baseline"]["host"] = hc
        result["speedup_vs_cpu"] = round(value / cb["value"], 1)
    elif rank == 0 and world == 1 and not args.no_cpu:
        threads, hc = cpu_threads(args)
        cb, data_cpu, u_cpu, psnr_cpu = cpu_baseline(cfg, args.cpu_rays, args.cpu_steps, threads)
        result["cpu_baseline"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in cb.items()}
        result["cpu_baseline"]["host"] = hc
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
