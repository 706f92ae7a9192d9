"""Stage-b trainer surface (drop-in for projects.NeuralLumen.trainer on the hot path).

Mirrors NeuralLumen/trainer.py:20-214 + neuralangelo/trainer.py:23-112 +
imaginaire/trainers/base.py (train_step, _get_total_loss, checkpoint layout):

* losses: 3 x L1 render, PSNR, eikonal, curvature, intrinsic (global min/max weight maps),
  residual regulariser (NeuralLumen/trainer.py:133-149, utils.py:142-174,
  neuralangelo/utils/misc.py:74-90), total = sum weight_k * loss_k (base.py:534-544);
* optimiser: AdamW (lr 1e-3, wd 1e-2) on the trainable neural_rgb parameters only, run as
  ONE fused HIP kernel over the flat parameter buffer; LR schedule two_steps_with_warmup
  (neuralangelo/utils/misc.py:28-54);
* multi-GPU: one process per GPU, gradients averaged with ONE all-reduce of the flat
  gradient buffer (3.2 MB) over RCCL (DDP semantics, get_trainer.py:80-88), the step's loss
  terms and PSNR riding in the same collective;
* checkpoints: {"model", "optim", "sched", "epoch", "iteration"} with ``module.``-prefixed
  model keys and ``latest_checkpoint.txt`` (imaginaire/trainers/base.py:570-607); ``optim`` /
  ``sched`` are torch ``AdamW`` / ``LambdaLR`` state dicts over the reference's parameter order,
  so either side resumes the other's checkpoints.

Construction follows the plugin call ``trainer_lib.Trainer(cfg, is_inference=..., seed=...)``
(imaginaire/trainers/utils/get_trainer.py:31-32): the model is built from ``cfg.model.type``
(imaginaire/trainers/base.py:103-131), ``cfg.model.use_pre_trained`` is loaded and
``cfg.trainer.partial_grad`` sets the requires_grad flags (NeuralLumen/trainer.py:22-54).
"""
import importlib
import math
import os

import torch
import torch.nn.functional as F

from . import _lib as L


def intrinsic_loss(o_r, o_s, ref, sha, cert, ranges, factors=(1.0, 1.0)):
    """NeuralLumen/utils/utils.py:142-162."""
    def rescale(x, lo, hi):
        return lo + (x - x.min()) / torch.clamp(x.max() - x.min(), min=1e-6) * (hi - lo)
    w_sha = rescale(sha.detach(), *ranges[0])
    w_vis = rescale(cert.detach(), *ranges[1])
    w_ref = torch.minimum(w_vis, w_sha)
    return (torch.abs(o_r - ref) * w_ref).mean() * factors[0] + (torch.abs(o_s - sha) * w_sha).mean() * factors[1]


def regularize_re_loss(o_re, f_neg=10.0, f_pos=1.0, e_pos=1.0):
    """NeuralLumen/utils/utils.py:165-174."""
    zero = torch.zeros_like(o_re)
    neg = torch.where(o_re < 0.0, o_re, zero)
    pos = torch.where(o_re >= 0.0, o_re, zero)
    return torch.abs(neg).mean() * f_neg + torch.pow(pos, e_pos).mean() * f_pos


def eikonal_loss(gradients, outside):
    """neuralangelo/utils/misc.py:74-81."""
    err = ((gradients.norm(dim=-1) - 1.0) ** 2).nan_to_num(nan=0.0, posinf=0.0, neginf=0.0)
    return (err * (~outside).float()).mean()


def curvature_loss(hessians, outside):
    """neuralangelo/utils/misc.py:83-90."""
    lap = hessians.sum(dim=-1).abs().nan_to_num(nan=0.0, posinf=0.0, neginf=0.0)
    return (lap * (~outside).float()).mean()


FUSED_LOSSES = {"render", "eikonal", "curvature", "intrinsic", "regularize_re"}
FUSED_LOSSES_A = {"render", "eikonal", "curvature"}
LOSS_NAMES = ("render", "eikonal", "curvature", "intrinsic", "regularize_re")


def _c(t):
    return None if t is None else t.contiguous()


def _strip_module(sd):
    """Model keys of an imaginaire checkpoint (saved from the DDP / WrappedModel wrapper)."""
    return {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}


def stage_b_losses(out, data, weights, ranges=((0.0, 1.0), (0.0, 1.0)), re_factors=(10.0, 1.0, 1.0),
                   intr_factors=(1.0, 1.0)):
    losses = {}
    if "render" in weights:
        losses["render"] = F.l1_loss(out["rgb"], data["image_sampled"]) * 3
    if "eikonal" in weights:
        losses["eikonal"] = eikonal_loss(out["gradients"], out["outside"])
    if "curvature" in weights and out.get("hessians") is not None:
        losses["curvature"] = curvature_loss(out["hessians"], out["outside"])
    if "intrinsic" in weights:
        losses["intrinsic"] = intrinsic_loss(out["o_r"], out["o_s"], data["pseudo_ref_sampled"],
                                             data["pseudo_sha_sampled"],
                                             data["pseudo_visibility_certainty_sampled"], ranges, intr_factors)
    if "regularize_re" in weights:
        losses["regularize_re"] = regularize_re_loss(out["o_re"], *re_factors)
    total = sum(losses[k] * weights[k] for k in weights if k in losses)
    psnr = -10 * torch.log10(F.mse_loss(out["rgb"].detach(), data["image_sampled"]))
    return total, losses, psnr


def two_steps_with_warmup(it, warm_up_end=5000, two_steps=(300000, 400000), gamma=10.0):
    """neuralangelo/utils/misc.py:43-52."""
    if it < warm_up_end:
        return it / warm_up_end
    if it > two_steps[1]:
        return 1.0 / gamma ** 2
    if it > two_steps[0]:
        return 1.0 / gamma
    return 1.0


class FusedAdamW:
    """torch.optim.AdamW semantics over the model's flat trainable buffer, one HIP launch."""

    def __init__(self, flat, lr=1e-3, weight_decay=1e-2, betas=(0.9, 0.999), eps=1e-8):
        self.flat = flat
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.m = torch.zeros_like(flat.detach())
        self.v = torch.zeros_like(flat.detach())
        self.step_count = 0

    def step(self, grad, lr, p16=None, ranges=None, before=None, zero_grad=False):
        """``p16``: fp16 tensor to receive a copy of the updated parameters (the hash table's
        gather shadow), or None.  ``ranges``: [(offset, n)] of the trainable elements when only
        part of the buffer trains (the rest -- frozen by partial_grad / partial_training -- gets
        no update, no weight decay and keeps its moments, as torch AdamW skips a parameter whose
        grad is None); None: the whole buffer.  ``before(i)`` runs before range i is issued (the
        chunked table reduction waits there for chunk i's all-reduce); one step either way, the
        update is element-wise, so a split into ranges changes no result.  ``zero_grad``: the kernel
        leaves ``grad`` all zero (storing 0 only where it was not), so a sparse scatter can add
        into it next step without a dense fill (ABI 17; the stage-a table gradient)."""
        self.step_count += 1
        p = self.flat.detach()
        for i, (off, n) in enumerate([(0, p.numel())] if ranges is None else ranges):
            if before is not None:
                before(i)
            L.call("mli_adamw", L.AdamwArgs(L.ptr(p[off:]), L.ptr(grad[off:]), L.ptr(self.m[off:]),
                                            L.ptr(self.v[off:]), n, float(lr), self.betas[0], self.betas[1],
                                            self.eps, self.wd, self.step_count,
                                            L.ptr(None if p16 is None else p16[off:]), 1 if zero_grad else 0))

    def resize(self, numel):
        """Moments for a parameter whose size changed (a table-size rule switch on load)."""
        if self.m.numel() != numel:
            self.m = torch.zeros(numel, device=self.m.device)
            self.v = torch.zeros(numel, device=self.v.device)


N_METRICS = 8  # loss terms (LOSS_NAMES), total, PSNR, spare -- the tail of the gradient buffer


def reduce_gradients(grad, world_size, group=None):
    """Data-parallel gradient average = DDP's bucketed all-reduce (imaginaire wraps the model
    in DistributedDataParallel, imaginaire/trainers/utils/get_trainer.py:81): the whole trainable state
    is ONE flat fp32 buffer (3.2 MB), so it goes as ONE all-reduce (RCCL over xGMI on the
    MI355X node, gloo in the CPU tests), then / world_size."""
    if world_size > 1:
        import torch.distributed as dist
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
        grad.div_(world_size)
    return grad


def grad_class_ranges(items):
    """{dW class: [(offset, length)]} of the stage-b flat gradient (engine.GRAD_CLASSES: the
    output layers, the hidden layers, layer 0 of each head), adjacent parameters merged.
    ``items``: Model._trainable_items()."""
    from .engine import GRAD_CLASS_LAYERS
    cls_of = {li: c for c, lis in GRAD_CLASS_LAYERS.items() for li in lis}
    out = {c: [] for c in GRAD_CLASS_LAYERS}
    for name, _, off, n in items:
        parts = name.split(".")
        c = cls_of[int(parts[parts.index("linears") + 1])]
        r = out[c]
        if r and r[-1][0] + r[-1][1] == off:
            r[-1] = (r[-1][0], r[-1][1] + n)
        else:
            r.append((off, n))
    return out


class OverlappedGradReduce:
    """DDP-style overlap of the stage-b gradient average with the backward (DDP's buckets,
    imaginaire/trainers/utils/get_trainer.py:81-88, static_graph=True config_base.yaml:58-60):
    as each dW class of the backward completes its layers' gradient (RenderEngine.backward
    ``on_class``), that class's ranges of the flat buffer go out as async all-reduces (RCCL on
    its own stream, behind the compute stream's work so far) while the next class's dW runs;
    ``finish`` adds the metric slots, waits once and divides by the world size.  Every element
    sees the serial form's operations (its rank sum, / world); a two-rank sum is exact in any
    order, so at world size 2 the result is bit-identical to reduce_gradients (tested)."""

    def __init__(self, grad_full, ranges, world_size, group=None):
        self.grad, self.ranges, self.world, self.group = grad_full, ranges, world_size, group
        self.works = []

    def __call__(self, cls):
        import torch.distributed as dist
        for o, k in self.ranges[cls]:
            self.works.append(dist.all_reduce(self.grad[o:o + k], op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True))

    def finish(self, tail_off):
        import torch.distributed as dist
        self.works.append(dist.all_reduce(self.grad[tail_off:], op=dist.ReduceOp.SUM, group=self.group,
                                          async_op=True))
        for w in self.works:
            w.wait()   # NCCL: the compute stream waits; gloo: the host does
        self.works = []
        self.grad.div_(self.world)
        return self.grad


def table_chunks(n, chunk):
    """[(offset, length)] cutting n elements into pieces of ``chunk`` (the last one ragged)."""
    chunk = max(1, int(chunk))
    return [(o, min(chunk, n - o)) for o in range(0, n, chunk)]


def reduce_and_step_table(optim, grad, lr, p16, world_size, chunk, overlap=True, group=None, zero_grad=False):
    """Stage a: average the hash-table gradient over the ranks (DDP wraps the table with every
    other parameter, imaginaire/trainers/utils/get_trainer.py:80-88) and take the table's AdamW
    step.  At 2^22 entries per level the gradient is 1.46 GB, so the serial form -- ONE all-reduce,
    then the 11 GB AdamW pass -- leaves the collective and the update back to back.  Overlapped:
    the table goes as ``chunk``-element all-reduces issued together (async; RCCL runs them in
    order on its stream), and the AdamW of chunk i is issued behind chunk i's completion only, so
    it runs on the compute stream while chunk i+1 reduces.  Every element sees the same ops as
    in the serial form (its sum, / world_size, the element-wise update); a two-rank sum is
    exact in either order, so at world size 2 the two forms are bit-identical (tested), and
    ``overlap=False`` (the deterministic mode) keeps the single collective for more ranks, whose
    ring order depends on the message split."""
    if world_size == 1:
        optim.step(grad, lr, p16=p16, zero_grad=zero_grad)
        return
    import torch.distributed as dist
    if not overlap:
        reduce_gradients(grad, world_size, group)
        optim.step(grad, lr, p16=p16, zero_grad=zero_grad)
        return
    chunks = table_chunks(grad.numel(), chunk)
    works = [dist.all_reduce(grad[o:o + k], op=dist.ReduceOp.SUM, group=group, async_op=True) for o, k in chunks]

    def ready(i):
        works[i].wait()   # NCCL: the current stream waits for chunk i; gloo: the host does
        o, k = chunks[i]
        grad[o:o + k].div_(world_size)
    optim.step(grad, lr, p16=p16, ranges=chunks, before=ready, zero_grad=zero_grad)


class ZeroTableAdamW:
    """Stage a over several ranks, ZeRO-style: the hash table's AdamW state is
    sharded.  Rank r owns table elements [lo, hi) = [r * per, (r + 1) * per) (per = ceil(n / world);
    the gradient and fp16-shadow buffers are padded to world * per):

      reduce-scatter of the table gradient -> this rank's shard of the sum, / world
      -> AdamW on the shard (fp32 master slice, shard-sized moments, the fp16 shadow slice)
      -> all-gather of the fp16 gather shadow only (what every rank's kernels read).

    Per rank that moves (w-1)/w x (4 B + 2 B) per element instead of the all-reduce's
    2 (w-1)/w x 4 B, and runs 1/w of the 11 GB AdamW pass.  The fp32 master outside [lo, hi) and
    the moments are only gathered for a checkpoint (sync(), a collective every rank calls: the
    file layout is that of the unsharded run).  Every element sees the serial path's operations
    (its rank sum, / world, the element-wise update); at world size 2 the sums are exact in any
    order, so the sharded and serial steps are bit-identical (tests/test_distributed.py)."""

    def __init__(self, table, world_size, rank, lr=1e-3, weight_decay=1e-2, group=None):
        self.table, self.world, self.rank, self.group = table, world_size, rank, group
        self.lr, self.wd = lr, weight_decay
        self._shard(table.numel())
        self.p16_pad = None     # [world * per] fp16; the engine's table16 is its [:n] view

    def _shard(self, n):
        self.n = n
        self.per = -(-n // self.world)
        self.lo = min(n, self.rank * self.per)
        self.hi = min(n, self.lo + self.per)
        self.optim = FusedAdamW(self.table.detach()[self.lo:self.hi], lr=self.lr, weight_decay=self.wd)
        self.gshard = torch.zeros(self.per, device=self.table.device)

    @property
    def step_count(self):
        return self.optim.step_count

    @step_count.setter
    def step_count(self, k):
        self.optim.step_count = k

    @property
    def m(self):
        return self.optim.m

    @property
    def v(self):
        return self.optim.v

    def resize(self, numel):
        """A table of another size rule (Model.load_state_dict): new shards, zero moments."""
        if numel != self.n:
            k = self.optim.step_count
            self._shard(numel)
            self.optim.step_count = k
            self.p16_pad = None

    def padded_grad(self, cur=None):
        """A [world * per] gradient buffer; the engine writes its [:n] view."""
        if cur is None or cur.numel() != self.world * self.per or cur.device != self.table.device:
            cur = torch.zeros(self.world * self.per, device=self.table.device)
        return cur

    def bind_shadow(self, engine):
        """Make the engine's fp16 gather shadow a view of the padded all-gather target."""
        t16 = engine.table16
        if self.p16_pad is not None and t16 is not None and t16.data_ptr() == self.p16_pad.data_ptr() \
                and t16.numel() == self.n:
            return
        pad = torch.zeros(self.world * self.per, dtype=torch.float16, device=self.table.device)
        if t16 is not None and t16.numel() == self.n:
            pad[:self.n].copy_(t16)
        self.p16_pad = pad
        engine.table16 = pad[:self.n]

    def step(self, grad_pad, lr):
        import torch.distributed as dist
        dist.reduce_scatter_tensor(self.gshard, grad_pad, op=dist.ReduceOp.SUM, group=self.group)
        k = self.hi - self.lo
        g = self.gshard[:k]
        g.div_(self.world)
        self.optim.step(g, lr, p16=self.p16_pad[self.lo:self.hi])
        mine = self.p16_pad[self.rank * self.per:(self.rank + 1) * self.per]
        dist.all_gather_into_tensor(self.p16_pad, mine, group=self.group)

    def _gather(self, shard):
        import torch.distributed as dist
        buf = torch.zeros(self.per, dtype=shard.dtype, device=shard.device)
        buf[:shard.numel()] = shard
        full = torch.empty(self.world * self.per, dtype=shard.dtype, device=shard.device)
        dist.all_gather_into_tensor(full, buf, group=self.group)
        return full[:self.n]

    def sync(self):
        """Collective (every rank): the fp32 master gathered into the table parameter; returns the
        full moments (exp_avg, exp_avg_sq) for the optimizer state dict."""
        t = self.table.detach()
        t.copy_(self._gather(t[self.lo:self.hi].clone()))
        return self._gather(self.optim.m), self._gather(self.optim.v)

    def load_full(self, m_full, v_full):
        """Moments of the unsharded layout (a checkpoint): this rank's slice."""
        self.optim.m.copy_(m_full.reshape(-1)[self.lo:self.hi])
        self.optim.v.copy_(v_full.reshape(-1)[self.lo:self.hi])


class Checkpointer:
    """imaginaire/trainers/base.py:557-687 surface over the Trainer's checkpoint layout:
    ``trainer.checkpointer.load(path, resume, load_opt=..., load_sch=...)`` as test.py:93 calls
    it, ``save(epoch, iteration, latest)``, the ``latest_checkpoint.txt`` pointer in cfg.logdir."""

    def __init__(self, cfg, trainer):
        self.trainer = trainer
        self.logdir = cfg.get("logdir", None)
        ck = cfg.get("checkpoint", None) or {}
        self.strict_resume = bool(ck.get("strict_resume", True))
        self.resume = False
        self.resume_epoch = self.resume_iteration = None
        self.eval_epoch = self.eval_iteration = None
        self.checkpoint_path = None

    def _get_full_path(self, name):
        return os.path.join(self.logdir or ".", name)

    def read_latest_checkpoint_file(self):
        """base.py:663-671 (incl. the old 'latest_checkpoint: <file>' form)."""
        path = self._get_full_path("latest_checkpoint.txt")
        if not os.path.exists(path):
            return None
        name = open(path).read().strip()
        return name.split(" ")[-1] if name.startswith("latest_checkpoint:") else name

    def load(self, checkpoint_path=None, resume=False, load_opt=True, load_sch=True, **kwargs):
        """base.py:609-652: priority (1) checkpoint_path, (2) with ``resume`` the latest checkpoint of
        cfg.logdir, (3) nothing (train from scratch).  Model weights with cfg.checkpoint.strict_resume;
        with ``resume`` also epoch / iteration and (optionally) the optimizer / scheduler."""
        self.resume = resume
        if resume and checkpoint_path is None:
            latest = self.read_latest_checkpoint_file()
            if latest is not None:
                checkpoint_path = self._get_full_path(latest)
        if checkpoint_path is None:
            return None
        if not os.path.exists(checkpoint_path):
            raise FileNotFoundError("File not found (local): %s" % checkpoint_path)
        self.checkpoint_path = checkpoint_path
        tr = self.trainer
        res = tr.load_checkpoint(checkpoint_path, resume=resume, strict=self.strict_resume,
                                 load_opt=load_opt and tr.optim is not None, load_sch=load_sch)
        meta = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        self.eval_epoch, self.eval_iteration = meta.get("epoch"), meta.get("iteration")
        if resume:
            self.resume_epoch, self.resume_iteration = self.eval_epoch, self.eval_iteration
        return res

    def save(self, current_epoch, current_iteration, latest=False):
        """base.py:569-589 (synchronously; master only under a process group)."""
        import torch.distributed as dist
        tr = self.trainer
        tr.current_epoch, tr.current_iteration = current_epoch, current_iteration
        tr.sync_table()   # ZeRO table (stage a, several ranks): a collective every rank takes part in
        if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
            name = "latest_checkpoint.pt" if latest else \
                "epoch_{:05}_iteration_{:09}_checkpoint.pt".format(current_epoch, current_iteration)
            return self._get_full_path(name)
        return tr.save_checkpoint(self.logdir or ".", latest=latest)


class Trainer:
    """Stage-b / stage-a trainer: ``train_step(data)`` = forward + loss + backward + AdamW."""

    # stage b: composite + losses + composite backward as ONE launch (mli_composite_loss);
    # False: the three calls mli_composite_fwd / mli_stage_b_loss / mli_composite_bwd
    fused_tail = True

    def __init__(self, cfg, is_inference=True, seed=0, model=None, world_size=None):
        self.cfg = cfg
        self.is_inference = is_inference
        built = model is None
        if built:
            model = self.setup_model(cfg, seed)
        self.model = self.model_module = model
        if world_size is None:
            import torch.distributed as dist
            world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.world_size = world_size
        if built:  # an injected model is already set up by its caller
            self._load_pre_trained(cfg)
        # cfg.trainer.deterministic: fixed-order reductions instead of fp32 atomics in the
        # split-K weight gradients and the hash-grid scatter (bit-reproducible steps)
        model.deterministic = bool(cfg.trainer.get("deterministic", False))
        self.partial_grad_keywords = list(cfg.trainer.get("partial_grad", None) or [])
        self._set_requires_grad()
        self.weights = {k: v for k, v in cfg.trainer.loss_weight.items() if v}
        # stage-a configs have no intrinsic / residual losses (and no parameters for them)
        p = cfg.trainer.get("para_intrinsic_loss", None) or {}
        self.ranges = (tuple(p.get("weight_map_range_shading", (0.0, 1.0))),
                       tuple(p.get("weight_map_range_visibility", (0.0, 1.0))))
        self.intr_factors = (float(p.get("factor_ref", 1.0)), float(p.get("factor_sha", 1.0)))
        q = cfg.trainer.get("para_regularize_re_loss", None) or {}
        self.re_factors = (q.get("factor_negative", 10.0), q.get("factor_positive", 1.0),
                           q.get("exponent_positive", 1.0))
        self._scratch = self._grad = None
        o = cfg.optim
        self.stage = getattr(model, "stage", "b")
        self.optim = self.optim_table = None
        if not is_inference:
            self.optim = FusedAdamW(model.flat, lr=o.params.lr, weight_decay=o.params.weight_decay)
            if self.stage == "a":
                # stage a trains the hash table too (one AdamW group, NeuralLumen/model.py:422-438);
                # over several ranks cfg.trainer.zero_table: True shards its optimizer state
                # (ZeroTableAdamW).  Opt-in: the sharded form is gloo-tested only, no
                # multi-GPU RCCL run has checked it against the replicated default on hardware
                zero = bool(cfg.trainer.get("zero_table", False)) and not model.deterministic
                if zero and world_size > 1:
                    import torch.distributed as dist
                    self.optim_table = ZeroTableAdamW(model.neural_sdf.tcnn_encoding.params, world_size,
                                                      dist.get_rank(), lr=o.params.lr,
                                                      weight_decay=o.params.weight_decay)
                else:
                    self.optim_table = FusedAdamW(model.neural_sdf.tcnn_encoding.params, lr=o.params.lr,
                                                  weight_decay=o.params.weight_decay)
        self._table_full_moments = None   # ZeRO: the gathered moments of the last sync_table()
        if self.stage == "a":
            self.init_curvature = float(cfg.trainer.loss_weight.get("curvature", 0.0))
            if model.neural_sdf.c2f is not None:   # neuralangelo/trainer.py:30-32
                model.neural_sdf.warm_up_end = o.sched.warm_up_end
        self._grad_table = None
        # stage a: the table AdamW leaves the consumed table gradient zero for the next scatter
        # (mli_adamw zero_grad: only the touched entries rewritten, no 1.46 GB fill per step);
        # False keeps the averaged gradient readable after the step (tests)
        self.table_grad_consume = True
        # stage b over several ranks: the gradient all-reduce per dW class, overlapped with the
        # next class's dW (OverlappedGradReduce); False: one collective after the backward
        self.grad_overlap = None
        # stage a over several ranks: the table gradient's all-reduce in chunks, each chunk's
        # AdamW issued behind its own reduction (reduce_and_step_table); 2^25 elements = 128 MiB.
        # None: overlapped unless the deterministic mode is on; True / False force it
        self.table_overlap = None
        self.table_chunk = 1 << 25
        self._side = None      # prefetch stream (stage-b geometry of the next batch)
        self._pending = []     # prefetched geometries not yet consumed by train_step
        self._pf_lane = 0
        # where the side stream may start the prefetched geometry: "call" (when prefetch is
        # called: draw, prefetch, then train_step the previous batch), "heads" (after the
        # heads forward of the last train_step) or "wgrad" (after its heads backward); with
        # the last two, prefetch is called after train_step
        self.prefetch_gate = "call"
        self.side_priority = 0  # torch stream priority of the prefetch stream (lower = higher)
        # batches prefetched ahead of the one being trained (each in its own buffer lane): with 2
        # the geometry of batch k+2 runs beside step k and may run on into step k+1 without
        # holding it up (step k+1 trains on batch k+1, prefetched a step earlier)
        self._prefetch_depth = 1
        self._gate_ev = None
        self.sched = o.sched
        self.current_iteration = 0
        self.current_epoch = 0
        self.losses, self.metrics = {}, {}
        self.checkpointer = Checkpointer(cfg, self)

    @property
    def prefetch_depth(self):
        return self._prefetch_depth

    @prefetch_depth.setter
    def prefetch_depth(self, d):
        """The lanes rotate modulo depth + 1: a change while prefetched batches are pending could
        point the next prefetch at a lane still in use, so it is refused then.

        Memory: a prefetch lane holds only the geometry of its batch (rays, the sampling rounds,
        the FIELD pass: sdf / grad / hess, the h0 and encoding images); the step's buffers
        (activations, dZ images, masks, dW slabs) are one set shared by the lanes
        (engine._GeometryLane), since the steps themselves run one after another on the main
        stream.  bench.py reports the allocator's peak as ``hbm_peak_gib``."""
        d = int(d)
        if d < 1:
            raise ValueError("prefetch_depth must be >= 1")
        if d != self._prefetch_depth:
            if self._pending:
                raise RuntimeError("prefetch_depth cannot change while %d prefetched batches are pending"
                                   % len(self._pending))
            self._pf_lane = 0
        self._prefetch_depth = d

    # ------------------------------------------------------------ construction (reference)
    @staticmethod
    def setup_model(cfg, seed=0):
        """imaginaire/trainers/base.py:103-131: seeded, built from cfg.model.type, moved to this
        rank's GPU (LOCAL_RANK / cfg.local_rank) when one is present."""
        torch.manual_seed(seed)
        lib = importlib.import_module(cfg.model.type)
        model = lib.Model(cfg.model, cfg.data)
        model.init_weights(seed)
        if torch.cuda.is_available():
            rank = int(os.environ.get("LOCAL_RANK", cfg.get("local_rank", 0) or 0))
            model = model.to("cuda:%d" % rank)
        return model

    def _load_pre_trained(self, cfg):
        """NeuralLumen/trainer.py:27-42: cfg.model.use_pre_trained.pt_filename (a checkpoint or a
        latest_checkpoint.txt pointer), model weights only, strict=False."""
        pre = cfg.model.get("use_pre_trained", None)
        if not pre:
            return None
        path = pre["pt_filename"]
        if path.endswith(".txt"):
            with open(path) as f:
                name = f.readline().strip()
            if not name:
                raise FileNotFoundError(path)
            path = os.path.join(os.path.dirname(path), name)
        sd = torch.load(path, map_location="cpu", weights_only=True)
        return self.model.load_state_dict(_strip_module(sd["model"]), strict=False)

    def _set_requires_grad(self):
        """NeuralLumen/trainer.py:44-54 (partial_grad keywords); without keywords every
        parameter of the stage trains (stage a) / the colour heads do (stage b default)."""
        kw = self.partial_grad_keywords
        for name, p in self.model.named_parameters():
            if kw:
                p.requires_grad_(any(k in name for k in kw))

    def adam_ranges(self):
        """[(offset, n)] of the flat buffer the optimizer steps: the Parameters of
        model.get_param_groups(cfg.optim) whose requires_grad is on (NeuralLumen/trainer.py:44-54
        partial_grad, NeuralLumen/model.py:422-438 partial_training), adjacent ones merged; None when
        that is the whole buffer (one launch).  Recomputed only when a requires_grad flag of the
        optimized Parameters changed (the key), not every step."""
        opt = self._optimized_cached()
        key = tuple(p.requires_grad for _, p in opt)
        if getattr(self, "_ranges_key", None) == key:
            return self._ranges
        live = {n for n, p in opt if p.requires_grad}
        items = self.model._trainable_items()
        ranges = []
        for name, _, off, n in items:
            if name in live:
                if ranges and ranges[-1][0] + ranges[-1][1] == off:
                    ranges[-1] = (ranges[-1][0], ranges[-1][1] + n)
                else:
                    ranges.append((off, n))
        full = ranges == [(0, self.model.flat.numel())]
        self._ranges_key, self._ranges = key, None if full else ranges
        return self._ranges

    def _step_flat(self, grad, lr):
        """The fused AdamW over adam_ranges(); the optimized Parameters it stepped are recorded
        (``stepped``), so a parameter stepped earlier and frozen later keeps its moments in the
        optimizer state dict, as torch AdamW keeps them."""
        self.optim.step(grad, lr, ranges=self.adam_ranges())
        key = getattr(self, "_ranges_key", None)
        if getattr(self, "_stepped_key", None) != key:
            self._stepped_key = key
            self.stepped.update(n for n, p in self._optimized_cached() if p.requires_grad)

    @property
    def stepped(self):
        """Names of the optimized Parameters an optimizer step has updated (or whose moments a
        loaded optimizer state holds)."""
        if getattr(self, "_stepped", None) is None:
            self._stepped = set()
        return self._stepped

    def _step_table(self, grad, lr, consume=False):
        """The table's averaged-gradient AdamW step: sharded (ZeroTableAdamW) or replicated
        (reduce_and_step_table: one all-reduce, or chunks overlapped with their AdamW).
        ``consume`` (the fused step's own gradient buffer, replicated form): the AdamW leaves the
        buffer zeroed for the next hash-grid scatter (RenderEngine.backward_a then skips its fill)."""
        eng = self.model.engine
        if isinstance(self.optim_table, ZeroTableAdamW):
            z = self.optim_table
            z.bind_shadow(eng)
            pad = getattr(self, "_grad_table_pad", None)
            if pad is None or grad.data_ptr() != pad.data_ptr():   # (the autograd path's table.grad)
                pad = self._grad_table_pad = z.padded_grad(pad)
                pad[:grad.numel()].copy_(grad.reshape(-1))
            z.step(pad, lr)
            self._table_synced = False
            self.model.table_sharded_stale = True
            self._shadow_current()
            return
        consume = consume and not self.model.deterministic
        reduce_and_step_table(self.optim_table, grad, lr, eng.table16, self.world_size, self.table_chunk,
                              overlap=self._table_overlap(), zero_grad=consume)
        if consume:
            eng.table_grad_clean = grad.data_ptr()

    def sync_table(self):
        """ZeRO table: gather the fp32 master and the moments (a collective: every rank calls it,
        Checkpointer.save does) so that state_dict / the optimizer state are the unsharded ones.
        A no-op otherwise."""
        if isinstance(self.optim_table, ZeroTableAdamW) and not getattr(self, "_table_synced", True):
            self._table_full_moments = self.optim_table.sync()
            self._table_synced = True
            self.model.table_sharded_stale = False
            self._shadow_current()

    def _shadow_current(self):
        """ZeRO table: the all-gathered fp16 shadow is the table the kernels read; mark it current
        for the table's present version, so that Model.prepare does not re-cast it from the fp32
        master (stale outside this rank's shard between syncs, and equal to it after one)."""
        m = self.model
        if m.engine is not None and m._sdf_version is not None:
            t = m.neural_sdf.tcnn_encoding.params
            m._sdf_version = (t._version, t.data_ptr())

    def _table_overlap(self):
        return (not self.model.deterministic) if self.table_overlap is None else bool(self.table_overlap)

    def table_trains(self):
        """Stage a: whether the hash table is among the optimized, requires_grad parameters."""
        t = self.model.neural_sdf.tcnn_encoding.params
        return any(p is t and p.requires_grad for _, p in self._optimized_cached())

    def _optimized_cached(self):
        """optimized_parameters(), computed once (the Parameter objects never change: load and
        .to() replace their data only)."""
        if getattr(self, "_opt_params", None) is None:
            self._opt_params = self.optimized_parameters()
        return self._opt_params

    def optimized_parameters(self):
        """[(name, Parameter)] of the reference optimizer, in its order:
        model.get_param_groups(cfg.optim) (get_trainer.py:106-118)."""
        groups = self.model.get_param_groups(self.cfg.optim)
        ids = {id(p) for p in groups}
        return [(n, p) for n, p in self.model.named_parameters() if id(p) in ids]

    def lr(self):
        s = self.sched
        return self.optim.lr * two_steps_with_warmup(self.current_iteration, s.warm_up_end,
                                                     tuple(s.two_steps), s.gamma)

    def _start_of_iteration(self):
        """neuralangelo/trainer.py:65-76: progress = iteration / max_iter (restarting at 0 in
        stage b: no resume); coarse-to-fine active levels, tap epsilon and the curvature weight
        schedule (get_curvature_weight, :56-63) when coarse-to-fine is on (stage a)."""
        m = self.model
        m.progress = self.current_iteration / self.cfg.max_iter
        sdf = m.neural_sdf
        if getattr(sdf, "c2f", None) is not None:
            sdf.set_active_levels(self.current_iteration)
            sdf.set_normal_epsilon()
            if "curvature" in self.weights:
                it, wue = self.current_iteration, self.sched.warm_up_end
                self.weights["curvature"] = (it / wue * self.init_curvature if it <= wue else
                                             self.init_curvature / sdf.growth_rate ** (sdf.anneal_levels - 1))
        else:
            sdf.set_normal_epsilon()

    def prefetch(self, data, u=None):
        """Stage-b software pipeline: issue ``data``'s geometry (rays, the hierarchical sampling
        rounds and the FIELD pass) on a side stream, into a spare engine buffer lane, so that it
        runs under the heads / backward of the step issued next.  In stage b the geometry reads
        only the frozen SDF and hash table (NeuralLumen/model.py:422-438 trains neural_rgb
        alone), so it does not depend on the optimiser step in flight.  ``train_step(data)``
        with the same dict then runs the heads onward on the prefetched geometry; its results
        equal the unpipelined step's on the same ``u`` (tests/test_gpu_parity.py).

        Call order: draw the batch, ``prefetch`` it, then ``train_step`` the batch
        ``prefetch_depth`` draws earlier (with the gates ``heads`` / ``wgrad``: train, then
        prefetch).  The side stream waits for an event recorded on the current stream (the
        gate), i.e. after the step that last read the lane it rewrites: ``prefetch_depth + 1``
        lanes rotate, so that step is at least the one issued before the gate's.  A no-op
        outside the fused stage-b path."""
        m = self.model
        if self.stage != "b" or not set(self.weights) <= FUSED_LOSSES:
            return
        # gate "call": prefetch, then train the batch depth draws earlier (depth + 1 may be
        # pending); gates "heads" / "wgrad": train, then prefetch, so at most depth may be -- one
        # more would land in the lane of the step just issued, whose tail (composite, backward)
        # still reads it after the gate event
        limit = self.prefetch_depth + (1 if self.prefetch_gate == "call" else 0)
        if len(self._pending) >= limit:
            raise RuntimeError("prefetch: %d batches already prefetched and not yet trained on (gate %s, depth %d)"
                               % (len(self._pending), self.prefetch_gate, self.prefetch_depth))
        m.train()
        if m.engine is None:
            m.prepare()
        eng = m.engine
        dev = m.flat.device
        main = torch.cuda.current_stream(dev)
        if self._side is None or self._side.device != dev:
            self._side = torch.cuda.Stream(device=dev, priority=self.side_priority)
        ready = self._gate_ev if self.prefetch_gate != "call" else None
        if ready is None:
            ready = torch.cuda.Event()
            ready.record(main)
        self._gate_ev = None
        side = self._side
        side.wait_event(ready)
        lane = ("pf", self._pf_lane)
        self._pf_lane = (self._pf_lane + 1) % (self.prefetch_depth + 1)
        prev = eng._bufs
        try:
            with torch.cuda.stream(side):
                for k in ("ray_idx", "pose", "intr", "pose_light"):
                    data[k].record_stream(side)
                eng.use_lane(lane, geometry_only=True)
                rays = eng.rays(data["pose"], data["intr"], data["pose_light"], data["ray_idx"],
                                m.image_size_train[1])
                dists = eng.sample(rays, m.stratified_uniforms(data, u))
                fld = eng.field(rays, dists, True)
        finally:
            eng._bufs = prev
        done = torch.cuda.Event()
        done.record(side)
        self._pending.append((data, lane, rays, dists, fld, done))

    def _take_prefetched(self, data):
        for i, pf in enumerate(self._pending):
            if pf[0] is data:
                del self._pending[: i + 1]  # older unconsumed prefetches are dropped
                return pf[1:]
        return None

    def start_of_iteration(self, data, current_iteration):
        """imaginaire/trainers/base.py:284-296 for a reference-style outer loop: the iteration
        number and the per-iteration schedules; the batch moved to the model's device."""
        self.current_iteration = current_iteration
        dev = self.model.device()
        return {k: v.to(dev) if torch.is_tensor(v) else v for k, v in data.items()}

    def train_step(self, data, u=None, return_outputs=False, last_iter_in_epoch=False):
        """One iteration.  Hot path (stage b): render -> fused losses + output gradients
        (mli_stage_b_loss) -> heads backward -> all-reduce -> fused AdamW, no torch autograd.
        Loss configurations the fused kernel does not cover take the autograd path (the
        reference's loss code on Model.forward's outputs).  A batch handed to ``prefetch``
        earlier reuses its prefetched geometry (``u`` is then the one given to prefetch).
        ``last_iter_in_epoch`` is accepted for the reference loop (grad_accum_iter is 1)."""
        if self.is_inference:
            raise RuntimeError("Trainer(is_inference=True) has no optimizer")
        self._start_of_iteration()
        self.model.train()
        if self.stage == "a":
            if not set(self.weights) <= FUSED_LOSSES_A:
                raise NotImplementedError("stage a (LumenRGB mode 'rgb') has no outputs for the loss terms %s"
                                          % sorted(set(self.weights) - FUSED_LOSSES_A))
            return self.train_step_a(data, u, return_outputs)
        if not set(self.weights) <= FUSED_LOSSES:
            return self._train_step_autograd(data, u)
        m = self.model
        pf = self._take_prefetched(data)
        prev = m.engine._bufs if m.engine is not None else None
        try:
            return self._train_step_b(data, u, return_outputs, pf)
        finally:
            if prev is not None:
                m.engine._bufs = prev

    def _grad_buffer(self):
        """The flat gradient + N_METRICS metric slots: the loss kernel writes the step's loss
        terms / PSNR into the tail, so ONE all-reduce averages gradients and metrics."""
        m = self.model
        n = m.flat.numel()
        if self._grad is None or self._grad.device != m.flat.device or self._grad.numel() != n + N_METRICS:
            self._grad = torch.empty(n + N_METRICS, device=m.flat.device)
        return self._grad[:n], self._grad[n:]

    def _grad_reducer(self, m):
        """Several ranks: the per-class overlapped all-reduce (``grad_overlap`` None / True), or
        None for the single collective after the backward (``grad_overlap`` False, one rank)."""
        if self.world_size <= 1 or self.grad_overlap is False:
            return None
        key = (id(self._grad), self._grad.numel())
        if getattr(self, "_class_ranges_key", None) != key:
            self._class_ranges_key, self._class_ranges = key, grad_class_ranges(m._trainable_items())
        return OverlappedGradReduce(self._grad, self._class_ranges, self.world_size)

    def _publish(self, lv):
        """Step losses / PSNR as tensors of their own (the buffer tail is rewritten next step)."""
        lv = lv.clone()
        self.losses = {k: lv[i] for i, k in enumerate(LOSS_NAMES) if k in self.weights}
        self.losses["total"] = lv[5]
        self.metrics["psnr"] = lv[6]

    def _train_step_b(self, data, u, return_outputs, pf):
        m = self.model
        m.prepare()
        m.image_width = m.image_size_train[1]
        eng = m.engine
        fused = self.fused_tail
        if pf is None:
            st = eng.render(data, m.s_var.detach(), m.progress, True, u=m.stratified_uniforms(data, u),
                            W=m.image_width, **({"composite": False} if fused else {}))
        else:
            lane, rays, dists, fld, done = pf
            torch.cuda.current_stream(m.flat.device).wait_event(done)
            eng.use_lane(lane, geometry_only=True)
            hd = eng.heads(rays, dists, fld, True, m.s_var.detach(), m.progress)
            comp = None if fused else eng.composite(rays, dists, fld, hd, m.s_var.detach(), m.progress, True)
            st = (rays, dists, fld, hd, comp)
        if self.prefetch_gate == "heads":
            self._gate_ev = torch.cuda.Event()
            self._gate_ev.record()
        eng.gate_wgrad = self.prefetch_gate == "wgrad"
        grad, lv = self._grad_buffer()  # every element is written by the backward / the loss kernel
        red = self._grad_reducer(m)
        if fused:
            # composite + losses + composite backward in one launch (mli_composite_loss)
            rays, dists, fld, hd, _ = st
            # (the loss values only after the backward is issued: the finalize then runs at the
            # step's tail, where the prefetch stream is idle, not beside the sampling rounds)
            comp, dz4 = eng.composite_loss(rays, dists, fld, hd, m.s_var.detach(), m.progress,
                                           self._loss_args(rays, fld, None, data, lv), defer=True)
            st = (rays, dists, fld, hd, comp)
            try:
                eng.backward(st, None, None, None, None, m.flat, m._sdf_l1(), grad, dz4=dz4,
                             **({} if red is None else {"on_class": red}))
            except BaseException:
                eng.drop_deferred()
                raise
            eng.finish_losses()
        else:
            d_rgb, d_o_r, d_o_s, d_o_re = self._fused_losses(st, data, lv)
            eng.backward(st, d_rgb, d_o_r, d_o_s, d_o_re, m.flat, m._sdf_l1(), grad,
                         **({} if red is None else {"on_class": red}))
        m._last_state = st
        if eng.gate_wgrad:
            self._gate_ev, eng.gate_event = eng.gate_event, None
        if red is None:
            reduce_gradients(self._grad, self.world_size)   # gradients + metrics, one collective
        else:
            red.finish(grad.numel())   # the metric slots (loss values: after finish_losses), wait, / world
        m.set_flat_grad(grad)
        self._step_flat(grad, self.lr())
        self.current_iteration += 1
        self._publish(lv)
        return m.outputs(st) if return_outputs else None

    def _loss_args(self, rays, fld, comp, data, lv, d=(None, None, None, None), scratch=None):
        """mli_loss_args of this step: the loss inputs, weights and factors (trainer.py:133-149
        of the reference), the composited outputs (``comp``; None for mli_composite_loss, which
        keeps them in registers), the gradient outputs ``d`` and the losses[8] slot ``lv``."""
        R, N = rays["outside"].shape[0], fld["sdf"].shape[0]
        w = self.weights
        intr = "intrinsic" in w
        cp = (lambda k: None) if comp is None else (lambda k: L.ptr(comp[k]))  # noqa: E731
        self._keep = [_c(data["image_sampled"])] + [_c(data.get(k)) if intr else None for k in (
            "pseudo_ref_sampled", "pseudo_sha_sampled", "pseudo_visibility_certainty_sampled")]
        gt, ref, sha, cert = self._keep
        return L.LossArgs(
            R, N, cp("rgb"), cp("o_r"), cp("o_s"), cp("o_re"), L.ptr(gt), L.ptr(ref), L.ptr(sha), L.ptr(cert),
            L.ptr(rays["outside"]), L.ptr(fld["grad"]) if "eikonal" in w else None,
            L.ptr(fld["hess"]) if "curvature" in w else None,
            w.get("render", 0.0), w.get("eikonal", 0.0), w.get("curvature", 0.0), w.get("intrinsic", 0.0),
            w.get("regularize_re", 0.0), self.ranges[0][0], self.ranges[0][1], self.ranges[1][0],
            self.ranges[1][1], self.intr_factors[0], self.intr_factors[1], *self.re_factors,
            *[L.ptr(t) for t in d], L.ptr(lv), L.ptr(scratch))

    def _fused_losses(self, st, data, lv):
        """mli_stage_b_loss: loss values + d total / d (rgb, o_r, o_s, o_re) (the three-call tail,
        ``fused_tail = False``, and stage a)."""
        m, eng = self.model, self.model.engine
        rays, dists, fld, hd, comp = st
        N, R = dists.shape
        d_rgb, d_o_r = eng._buf("d_rgb", (R, 3)), eng._buf("d_o_r", (R, 3))
        d_o_s, d_o_re = eng._buf("d_o_s", (R, 1)), eng._buf("d_o_re", (R, 3))
        n = L.workspace("mli_stage_b_loss", L.LossArgs(R, N))[0] // 4
        if self._scratch is None or self._scratch.device != m.flat.device or self._scratch.numel() < n:
            self._scratch = torch.empty(n, device=m.flat.device)
        L.call("mli_stage_b_loss", self._loss_args(rays, fld, comp, data, lv, (d_rgb, d_o_r, d_o_s, d_o_re),
                                                   self._scratch))
        return d_rgb, d_o_r, d_o_s, d_o_re

    def compute_grads_a(self, data, u=None):
        """Stage-a forward + fused losses + backward (no optimizer step): fills the flat
        gradient (MLP buffer incl. s_var, metrics in its tail) and self._grad_table; returns
        (render state, loss values)."""
        m = self.model
        m.prepare()
        m.image_width = m.image_size_train[1]
        table = m.neural_sdf.tcnn_encoding.params
        if isinstance(self.optim_table, ZeroTableAdamW):
            self._grad_table_pad = self.optim_table.padded_grad(getattr(self, "_grad_table_pad", None))
            self._grad_table = self._grad_table_pad[:table.numel()]
        elif self._grad_table is None or self._grad_table.device != table.device or \
                self._grad_table.numel() != table.numel():
            self._grad_table = torch.empty_like(table.detach())
        st = m.engine.render(data, m.s_var.detach(), m.progress, True, u=m.stratified_uniforms(data, u),
                             W=m.image_width)
        m._last_state = st
        grad, lv = self._grad_buffer()
        d_rgb = self._fused_losses(st, data, lv)[0]
        m.engine.backward_a(st, d_rgb, m.flat.detach(), grad, self._grad_table,
                            self.weights.get("eikonal", 0.0), self.weights.get("curvature", 0.0), m.progress)
        return st, lv

    def train_step_a(self, data, u=None, return_outputs=False):
        """One stage-a iteration (syn_hotdog_a): render -> fused losses (render, eikonal,
        curvature) -> geometry backward (composite, head, SDF MLP of the 5 points, hash-grid
        scatter) -> all-reduce -> fused AdamW on the flat MLP buffer and on the hash table
        (which also refreshes the fp16 gather shadow)."""
        m = self.model
        st, lv = self.compute_grads_a(data, u)
        eng = m.engine
        grad = self._grad[:m.flat.numel()]
        reduce_gradients(self._grad, self.world_size)
        m.set_flat_grad(grad)
        lr = self.lr()
        self._step_flat(grad, lr)
        if self.table_trains():
            # (a frozen table needs no averaged gradient: no collective for it)
            self._step_table(self._grad_table, lr, consume=self.table_grad_consume)
        self.current_iteration += 1
        self._publish(lv)
        return m.outputs(st) if return_outputs else None

    def train_step_autograd(self, data, u=None):
        """Reference semantics through torch autograd on Model.forward's outputs (one iteration,
        schedules included)."""
        self._start_of_iteration()
        return self._train_step_autograd(data, u)

    def _train_step_autograd(self, data, u=None):
        m = self.model
        m.train()
        for p in list(m.trainable_parameters()) + [m.neural_sdf.tcnn_encoding.params]:
            p.grad = None
        out = m(data, u=u)
        total, losses, psnr = stage_b_losses(out, data, self.weights, self.ranges, self.re_factors,
                                             self.intr_factors)
        total.backward()
        grad, lv = self._grad_buffer()
        g = m.flat_grad_from_params()
        grad.copy_(g) if g is not None else grad.zero_()
        lv.zero_()
        for i, k in enumerate(LOSS_NAMES):
            if k in losses:
                lv[i] = losses[k].detach()
        lv[5], lv[6] = total.detach(), psnr.detach()
        reduce_gradients(self._grad, self.world_size)
        m.set_flat_grad(grad)
        self._step_flat(grad, self.lr())
        if self.stage == "a" and self.table_trains():
            self._step_table(m.neural_sdf.tcnn_encoding.params.grad, self.lr())
        self.current_iteration += 1
        self._publish(lv)
        return out

    # ------------------------------------------------------------ checkpoint layout
    def _lr_lambda(self, it):
        s = self.sched
        return two_steps_with_warmup(it, s.warm_up_end, tuple(s.two_steps), s.gamma)

    def _moment_views(self):
        """[(name, Parameter, exp_avg view, exp_avg_sq view)] over the reference optimizer's
        parameters: flat-buffer Parameters map to slices of the fused AdamW's moments, the hash
        table (stage a) to the table AdamW's."""
        offs = {n: (off, shape, k) for n, shape, off, k in self.model._trainable_items()}
        out = []
        for name, p in self.optimized_parameters():
            if name in offs:
                off, shape, k = offs[name]
                out.append((name, p, self.optim.m[off:off + k].view(shape), self.optim.v[off:off + k].view(shape)))
            elif self.optim_table is not None and p is self.model.neural_sdf.tcnn_encoding.params:
                if isinstance(self.optim_table, ZeroTableAdamW):
                    # the full moments exist only as sync_table() gathered them (None: never stepped);
                    # after a later step they are stale: refuse rather than return them
                    if not getattr(self, "_table_synced", True):
                        raise RuntimeError("the ZeRO-sharded table moments are not gathered since the last "
                                           "step: call trainer.sync_table() on every rank first")
                    mv = self._table_full_moments
                    out.append((name, p, None if mv is None else mv[0], None if mv is None else mv[1]))
                else:
                    out.append((name, p, self.optim_table.m, self.optim_table.v))
            else:
                raise RuntimeError("optimized parameter %s is not trained by this build's optimizer" % name)
        return out

    def optim_state_dict(self):
        """torch.optim.AdamW.state_dict() of the reference optimizer (get_trainer.py:106-150,
        imaginaire/trainers/base.py:601-607): per-parameter state indexed in
        model.get_param_groups(cfg.optim) order, one param group with the LambdaLR
        initial_lr; the group keys come from this torch version's own AdamW."""
        views = self._moment_views()
        lr0 = float(self.cfg.optim.params.lr)
        probe = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=lr0, betas=self.optim.betas,
                                  eps=self.optim.eps, weight_decay=self.optim.wd)
        group = dict(probe.state_dict()["param_groups"][0])
        group.update(lr=lr0 * self._lr_lambda(self.current_iteration), initial_lr=lr0,
                     params=list(range(len(views))))
        state = {}
        if self.optim.step_count > 0:
            stepped = self.stepped | ({"neural_sdf.tcnn_encoding.params"} if self.optim_table is not None and
                                      self.optim_table.step_count > 0 else set())
            for i, (name, p, m, v) in enumerate(views):
                # torch AdamW keeps no state for a parameter it never stepped (grad None: frozen by
                # partial_grad / partial_training): no entry, so no resume applies a bias
                # correction to moments that were never accumulated.  A parameter stepped earlier
                # and frozen since keeps its entry (torch keeps its state).
                if name not in stepped and not p.requires_grad:
                    continue
                if m is None:   # ZeRO table never stepped or not gathered (sync_table)
                    if self.optim_table.step_count > 0:
                        raise RuntimeError("the sharded table's moments were not gathered: save through "
                                           "trainer.checkpointer.save (or call sync_table on every rank)")
                    continue
                state[i] = {"step": torch.tensor(float(self.optim.step_count)),
                            "exp_avg": m.detach().cpu().clone(), "exp_avg_sq": v.detach().cpu().clone()}
        return {"state": state, "param_groups": [group]}

    def sched_state_dict(self):
        """torch.optim.lr_scheduler.LambdaLR.state_dict() in iteration mode
        (neuralangelo/utils/misc.py:28-54 two_steps_with_warmup; last_epoch = iteration)."""
        from torch.optim.lr_scheduler import LambdaLR
        lr0 = float(self.cfg.optim.params.lr)
        probe = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=lr0)
        sched = LambdaLR(probe, self._lr_lambda)
        sched.last_epoch = self.current_iteration
        sched._step_count = self.current_iteration + 1
        sched._last_lr = [lr0 * self._lr_lambda(self.current_iteration)]
        return sched.state_dict()

    def load_optim_state_dict(self, osd):
        """Accepts torch AdamW state dicts (this build's or the reference's) and the round-1
        layout {"step", "exp_avg", "exp_avg_sq"} of the flat buffer; anything else raises."""
        if "state" in osd and "param_groups" in osd:
            views = self._moment_views()
            idx = [i for g in osd["param_groups"] for i in g["params"]]
            if len(idx) != len(views):
                raise ValueError("optimizer state covers %d parameters, the model trains %d"
                                 % (len(idx), len(views)))
            step = 0
            for i, (name, p, m, v) in zip(idx, views):
                st = osd["state"].get(i)
                zt = isinstance(self.optim_table, ZeroTableAdamW) and p is self.model.neural_sdf.tcnn_encoding.params
                if zt:   # this rank's slice of the unsharded moments
                    z = self.optim_table
                    if st:
                        z.load_full(st["exp_avg"], st["exp_avg_sq"])
                        step = int(float(st["step"]))
                        self.stepped.add(name)
                    else:
                        z.m.zero_()
                        z.v.zero_()
                    self._table_full_moments, self._table_synced = None, True
                    self.model.table_sharded_stale = False
                    continue
                if not st:
                    m.zero_()
                    v.zero_()
                    continue
                if tuple(st["exp_avg"].shape) != tuple(m.shape):
                    raise ValueError("optimizer state of %s has shape %s, expected %s"
                                     % (name, tuple(st["exp_avg"].shape), tuple(m.shape)))
                m.copy_(st["exp_avg"])
                v.copy_(st["exp_avg_sq"])
                step = int(float(st["step"]))
                self.stepped.add(name)
            self.optim.step_count = step
            if self.optim_table is not None:
                self.optim_table.step_count = step
        elif "exp_avg" in osd:
            self.optim.step_count = int(osd["step"])
            self.optim.m.copy_(osd["exp_avg"])
            self.optim.v.copy_(osd["exp_avg_sq"])
        else:
            raise ValueError("unknown optimizer state layout (keys %s)" % sorted(osd))

    def save_checkpoint(self, logdir, latest=False):
        """imaginaire/trainers/base.py:570-607: file naming (or latest_checkpoint.pt),
        latest_checkpoint.txt, {model, optim, sched, epoch, iteration} with ``module.`` keys."""
        os.makedirs(logdir, exist_ok=True)
        name = "latest_checkpoint.pt" if latest else \
            "epoch_{:05}_iteration_{:09}_checkpoint.pt".format(self.current_epoch, self.current_iteration)
        if not getattr(self, "_table_synced", True):
            raise RuntimeError("save_checkpoint: the ZeRO-sharded table is not gathered; save through "
                               "trainer.checkpointer.save (every rank) or call sync_table() on every rank")
        sd = {"module." + k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        ck = dict(model=sd, epoch=self.current_epoch, iteration=self.current_iteration)
        if self.optim is not None:
            ck.update(optim=self.optim_state_dict(), sched=self.sched_state_dict())
        torch.save(ck, os.path.join(logdir, name))
        with open(os.path.join(logdir, "latest_checkpoint.txt"), "w") as f:
            f.write(name + "\n")
        return os.path.join(logdir, name)

    def load_checkpoint(self, path, resume=True, strict=None, load_opt=True, load_sch=True):
        """imaginaire Checkpointer.load (base.py:609-652): the model with
        cfg.checkpoint.strict_resume; with ``resume`` also epoch / iteration (always, when
        present), the optimizer and the scheduler.  A hash table of the other size rule
        re-sizes the table optimizer's moments (Model.load_state_dict)."""
        if path.endswith(".txt"):
            with open(path) as f:
                path = os.path.join(os.path.dirname(path), f.readline().strip())
        if strict is None:
            strict = bool(self.cfg.get("checkpoint", {}).get("strict_resume", True))
        sd = torch.load(path, map_location="cpu", weights_only=True)
        res = self.model.load_state_dict(_strip_module(sd["model"]), strict=strict)
        if self.optim_table is not None:
            self.optim_table.resize(self.model.neural_sdf.tcnn_encoding.params.numel())
        if resume:
            self.current_epoch = int(sd.get("epoch", 0))
            self.current_iteration = int(sd.get("iteration", 0))
            if load_opt and self.optim is not None and "optim" in sd:
                self.load_optim_state_dict(sd["optim"])
            if load_sch and "sched" in sd and "last_epoch" in sd["sched"]:
                # iteration mode: the LambdaLR step count is the iteration (base.py:637)
                self.current_iteration = int(sd["sched"]["last_epoch"])
        return res

    def load_pre_trained(self, path):
        """NeuralLumen/trainer.py:27-42 warm start (model weights only, strict=False)."""
        sd = torch.load(path, map_location="cpu", weights_only=True)
        res = self.model.load_state_dict(_strip_module(sd["model"]), strict=False)
        if self.optim_table is not None:
            self.optim_table.resize(self.model.neural_sdf.tcnn_encoding.params.numel())
        return res

    # ------------------------------------------------------------ train.py / test.py surface
    # (mli_nerf_amd.loop: the imaginaire loop reduced to the hot path; W&B is out of scope)
    train_data_loader = eval_data_loader = None

    def set_data_loader(self, cfg, split, shuffle=True, drop_last=True, seed=0, subset_indices=None):
        """imaginaire/trainers/base.py:87-101 (train.py:81-82, test.py:104-116)."""
        from . import loop
        loop.set_data_loader(self, cfg, split, shuffle, drop_last, seed, subset_indices)

    def init_wandb(self, cfg, wandb_id=None, project="", run_name=None, mode="online", resume="allow",
                   use_group=False):
        """base.py:231-272 (train.py:86-90): W&B is not part of this build: recorded only."""
        self.wandb_args = dict(project=project, run_name=run_name, mode=mode, resume=resume)

    def train(self, cfg, data_loader, single_gpu=False, profile=False, show_pbar=False):
        """base.py:474-527 + neuralangelo/trainer.py:110-112 (train.py:94-98)."""
        from . import loop
        loop.train(self, cfg, data_loader, single_gpu, profile, show_pbar)

    def finalize(self, cfg):
        """base.py:551-554 (train.py:101): closes the W&B run in the reference; nothing to close here."""
        return None

    def test_save(self, data_loader, output_dir=None, inference_args=None, mode="test", show_pbar=False):
        """projects/nerf/trainers/base.py:176-216 (test.py:119-121)."""
        from . import loop
        return loop.test_save(self, data_loader, output_dir, inference_args, mode, show_pbar)

    def test_images(self, data_loader, output_dir=None, setting_list=None, mode="test", show_pbar=False):
        """projects/nerf/trainers/base.py:218-260 (test.py:122-126)."""
        from . import loop
        return loop.test_images(self, data_loader, output_dir, setting_list, mode, show_pbar)

    def test_video(self, data_loader, setting1, setting2, output_dir, mode="test",
                   video_content=("rgb", "gt", "o_r", "o_s"), show_pbar=False):
        """projects/nerf/trainers/base.py:264-346 (see mli_nerf_amd.video); ``data_loader`` as
        test.py:142 passes it (its ``.dataset`` is used) or the Dataset itself."""
        from . import video
        dataset = getattr(data_loader, "dataset", data_loader)
        return video.render_video(self.model, dataset, setting1, setting2, output_dir, trainer=self, mode=mode,
                                  video_content=video_content, show_pbar=show_pbar)

    def test_all_light(self, data_loader, output_dir=None, mode="test", dataset_type="pair", sample_num=4,
                       seed=999):
        """NeuralLumen/trainer.py:216-316: every (camera, light) pair of the enumeration
        (pair / unpair / limitedlights) rendered with the light-visibility pass, the maps saved as
        PNGs and ``results_all.pt`` for scripts/pseudo_label.py (see mli_nerf_amd.relight)."""
        from . import relight
        return relight.test_all_light(self, data_loader, output_dir, mode, dataset_type, sample_num, seed)
