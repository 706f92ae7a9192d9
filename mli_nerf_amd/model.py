"""Drop-in ``Model`` for the NeuralLumen stage-b render path on MI355X.

Mirrors the reference plugin surface (``cfg.model.type`` -> ``Model(cfg_model, cfg_data)``,
imaginaire/trainers/base.py:118-119; NeuralLumen/model.py:17-131):

* module / parameter names and shapes match the reference state dict, so checkpoints
  load with ``load_state_dict`` (keys ``neural_sdf.tcnn_encoding.params``,
  ``neural_sdf.mlp.linears.{0,1}.{weight_g,weight_v,bias}``, ``neural_sdf.mlp.linear_sdf.*``,
  ``neural_rgb.{mlp,mlp_r,mlp_s}.linears.{0..4}.*``, ``s_var``);
* ``forward(data)`` returns the reference output dict (rgb, o_r, o_s, o_re, opacity, outside,
  dists, weights, gradient, gradients, hessians) with rgb/o_r/o_s/o_re differentiable w.r.t.
  the trainable ``neural_rgb`` parameters (stage b, NeuralLumen/trainer.py:44-54);
* ``inference(data)`` renders the full image in ``rand_rays_val`` chunks (:60-111).

All compute runs in libmli_hip.so; the trainable parameters live in ONE flat fp32 buffer
(``self.flat``), the named ``nn.Parameter``s are views into it.  Under autograd the backward
hands each named Parameter its gradient as a view of one flat gradient buffer, so the
reference trainer's ``AdamW(model.get_param_groups(cfg.optim))``, DDP's gradient hooks and
``requires_grad`` flags work as on the reference Model (imaginaire/trainers/base.py:118-119,
450-457; get_trainer.py:70-118), while the fused Trainer steps the flat buffer in one launch.
Parameters are registered in the reference's order (tests/golden/param_order.json), so a
torch optimizer state dict indexes the same tensors in both.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import layout
from .engine import PathConfig, RenderEngine
from .hashgrid import GRID_DEFAULTS, level_table


def _cfg_get(node, path, default=None):
    cur = node
    for key in path.split("."):
        if cur is None or not hasattr(cur, key) and not (isinstance(cur, dict) and key in cur):
            return default
        cur = cur[key] if isinstance(cur, dict) else getattr(cur, key)
    return cur


def path_config_from(cfg_model, cfg_data):
    ns = cfg_model.render.num_samples
    hg = cfg_model.object.sdf.encoding.hashgrid
    box = _cfg_get(cfg_data, "bounding_type", "unit_sphere") == "box"
    inside_out = bool(_cfg_get(cfg_model, "object.sdf.mlp.inside_out", False))
    lv = _cfg_get(cfg_model, "light_visibility", None)
    vis = None
    if lv is not None and _cfg_get(lv, "enabled", False):  # NeuralLumen/model.py:25-35
        vis = dict(camera_ray_type=_cfg_get(lv, "camera_ray_type", None), type=_cfg_get(lv, "type", None),
                   bounding=_cfg_get(lv, "visibility_bounding_type", "sphere"),
                   radius=float(_cfg_get(lv, "visibility_sphere_radius", 1.0)),
                   gamma=float(_cfg_get(lv, "gamma_correlation", 0.0) or 0.0))
    return PathConfig(light_visibility=vis, n_coarse=ns.coarse, n_fine=ns.fine, n_hier=cfg_model.render.num_sample_hierarchy,
                      white_bg=bool(cfg_model.background.white), bounding="box" if box else "sphere",
                      aabb=tuple(_cfg_get(cfg_data, "bounding_box_aabb", (-1, -1, -1, 1, 1, 1))),
                      outside_val=1000.0 * (-1 if inside_out else 1),
                      anneal_end=float(cfg_model.object.s_var.anneal_end),
                      log2T=int(hg.dict_size), levels=int(cfg_model.object.sdf.encoding.levels),
                      min_logres=int(hg.min_logres), max_logres=int(hg.max_logres),
                      scale_rule=str(_cfg_get(hg, "scale_rule", "fp32")))


class WNLinear(torch.nn.Module):
    """Parameter holder with torch weight_norm names (nerf_util.py:176-178), registered in the
    order weight_norm leaves them on an nn.Linear: bias, weight_g, weight_v."""

    def __init__(self, v, g, b):
        super().__init__()
        self.bias = v_param(b)
        self.weight_g = v_param(g)
        self.weight_v = v_param(v)


class PlainLinear(torch.nn.Module):
    def __init__(self, w, b):
        super().__init__()
        self.weight, self.bias = v_param(w), v_param(b)


def v_param(t, requires_grad=False):
    return torch.nn.Parameter(t, requires_grad=requires_grad)


class _MLP(torch.nn.Module):
    def __init__(self, linears):
        super().__init__()
        self.linears = torch.nn.ModuleList(linears)


class _Encoding(torch.nn.Module):
    def __init__(self, n_params):
        super().__init__()
        self.params = torch.nn.Parameter(torch.zeros(n_params), requires_grad=False)


class NeuralSDF(torch.nn.Module):
    """Parameter-compatible stand-in for neuralangelo/utils/modules.py:NeuralSDF.  Stage b:
    frozen standalone tensors.  Stage a (``view`` given): the MLP parameters are views of the
    model's flat trainable buffer and the hash table is trainable.  Attributes the trainers
    poke are kept (normal_eps, resolutions, active_levels, anneal_levels, warm_up_end, ...)."""

    def __init__(self, pcfg, c2f=None, view=None):
        super().__init__()
        _, total = level_table(pcfg.levels, pcfg.log2T, pcfg.min_logres, pcfg.max_logres, pcfg.scale_rule)
        self.tcnn_encoding = _Encoding(total * 8)
        k0 = 3 + pcfg.levels * 8
        if view is None:
            mlp = _MLP([WNLinear(torch.zeros(256, k0), torch.ones(256, 1), torch.zeros(256)),
                        WNLinear(torch.zeros(256, 256), torch.ones(256, 1), torch.zeros(256))])
            mlp.linear_sdf = PlainLinear(torch.zeros(1, 256), torch.zeros(1))
        else:
            pre = "neural_sdf.mlp."
            mlp = _MLP([WNLinear(*(view(pre + "linears.%d.%s" % (li, n)) for n in ("weight_v", "weight_g", "bias")))
                        for li in range(2)])
            mlp.linear_sdf = PlainLinear(view(pre + "linear_sdf.weight"), view(pre + "linear_sdf.bias"))
            for p in list(mlp.parameters()) + [self.tcnn_encoding.params]:
                p.requires_grad_(True)
        self.mlp = mlp
        self.levels = pcfg.levels
        g = np.exp((np.log(2 ** pcfg.max_logres) - np.log(2 ** pcfg.min_logres)) / (pcfg.levels - 1))
        self.growth_rate = g
        self.resolutions = [int(np.floor(2 ** pcfg.min_logres * g ** lv)) + 1 for lv in range(pcfg.levels)]
        self.normal_eps = 1.0 / self.resolutions[-1]
        self.active_levels = self.anneal_levels = pcfg.levels
        self.warm_up_end = 0
        # coarse-to-fine (neuralangelo/configs/base.yaml:64-67; enabled in stage a)
        self.c2f = c2f if c2f is not None and c2f.get("enabled", False) else None

    def set_normal_epsilon(self):
        """modules.py:102-107: tap epsilon = 1 / resolution of level anneal_levels - 1 under
        coarse-to-fine, else of the finest level."""
        res = self.resolutions[self.anneal_levels - 1] if self.c2f else self.resolutions[-1]
        self.normal_eps = 1.0 / res

    def set_active_levels(self, current_iter=None):
        """modules.py:97-100."""
        if self.c2f is None or current_iter is None:
            self.active_levels = self.anneal_levels = len(self.resolutions)
            return
        anneal = max((current_iter - self.warm_up_end) // self.c2f["step"], 1)
        self.anneal_levels = min(self.levels, anneal)
        self.active_levels = max(self.c2f["init_active_level"], self.anneal_levels)


class LumenRGB(torch.nn.Module):
    """Parameter layout of NeuralLumen/utils/modules.py:LumenRGB -- mode 'rgb_r_s' (three
    heads, stage b) or 'rgb' (the single ``mlp`` head, stage a); the tensors are views of the
    model's flat trainable buffer."""

    def __init__(self, view, heads=layout.HEADS):
        super().__init__()
        self.network_mode = "rgb" if len(heads) == 1 else "rgb_r_s"
        for head, _, _ in heads:
            lins = []
            for li in range(5):
                pre = layout.param_prefix(head, li)
                lins.append(WNLinear(view(pre + ".weight_v"), view(pre + ".weight_g"), view(pre + ".bias")))
                for p in lins[-1].parameters():
                    p.requires_grad_(True)
            setattr(self, head, _MLP(lins))


class _RenderHeads(torch.autograd.Function):
    """Forward: the whole render on the GPU.  Backward (stage b): composite -> heads dX chain
    -> dW GEMMs -> weight-norm backward into one flat fp32 gradient buffer, handed out as
    per-Parameter views (``params`` = the model's trainable Parameters in flat-layout order).
    Stage a: the gradients / hessians are differentiable outputs too and the backward runs the
    geometry chain (Engine.backward_a) into the flat buffer and the hash table.  Inputs whose
    ``requires_grad`` is off get no gradient (the reference's partial_grad)."""

    @staticmethod
    def forward(ctx, table, model, data, u, progress, training, *params):
        eng = model.engine
        st = eng.render(data, model.s_var.detach(), progress, training, u=u, W=model.image_width)
        ctx.state = st
        ctx.stamp = eng.stamp()
        ctx.model = model
        ctx.progress = progress
        model._last_state = st
        comp, fld = st[4], st[2]
        if model.stage != "a":
            return comp["rgb"], comp["o_r"], comp["o_s"], comp["o_re"]
        hess = fld["hess"].clone() if fld["hess"] is not None else torch.zeros_like(fld["grad"])
        return comp["rgb"], comp["o_r"], comp["o_s"], comp["o_re"], fld["grad"].clone(), hess

    @staticmethod
    def backward(ctx, d_rgb, d_o_r, d_o_s, d_o_re, d_grads=None, d_hess=None):
        model = ctx.model
        if ctx.state is None:
            raise RuntimeError("_RenderHeads: backward through the same render twice")
        model.engine.check_stamp(ctx.stamp)
        grad = torch.zeros_like(model.flat)
        gt = None
        if model.stage == "a":
            st = ctx.state
            N, R = st[1].shape
            d_rgb = torch.zeros(R, 3, device=grad.device) if d_rgb is None else d_rgb.contiguous()
            gt = torch.empty_like(model.neural_sdf.tcnn_encoding.params)
            c = lambda t: None if t is None else t.contiguous()  # noqa: E731
            model.engine.backward_a(st, d_rgb, model.flat.detach(), grad, gt, 0.0, 0.0, ctx.progress,
                                    d_grad_ext=c(d_grads), d_hess_ext=c(d_hess))
        else:
            model.engine.backward(ctx.state, d_rgb, d_o_r, d_o_s, d_o_re, model.flat, model._sdf_l1(), grad)
        ctx.state = None
        views = [grad[off:off + n].view(shape) if need else None
                 for (_, shape, off, n), need in zip(model._trainable_items(), ctx.needs_input_grad[6:])]
        return (gt if ctx.needs_input_grad[0] else None, None, None, None, None, None, *views)


class Model(torch.nn.Module):
    def __init__(self, cfg_model, cfg_data):
        super().__init__()
        self.cfg_model, self.cfg_data = cfg_model, cfg_data
        self.pcfg = path_config_from(cfg_model, cfg_data)
        self.image_size_train = list(cfg_data.train.image_size)
        self.image_size_val = list(cfg_data.val.image_size)
        self.rand_rays_val = int(_cfg_get(cfg_model, "render.rand_rays_val", cfg_model.render.rand_rays))
        self.white_background = self.pcfg.white_bg
        self.outside_val = self.pcfg.outside_val
        self.anneal_end = self.pcfg.anneal_end
        self.progress = 0.0
        self.stratified = bool(cfg_model.render.stratified)
        mode = _cfg_get(cfg_model, "object.rgb.network_mode", None)
        if mode not in (None, "rgb", "rgb_r_s"):
            raise NotImplementedError("LumenRGB network_mode %r is outside the built hot path" % mode)
        # 'rgb' (no network_mode, NeuralLumen/utils/modules.py:50-55): stage a -- every parameter
        # trains (no partial_grad); 'rgb_r_s': stage b -- the heads train on frozen geometry
        self.stage = "b" if mode == "rgb_r_s" else "a"
        self._layout = {name: (shape, off) for name, shape, off in layout.trainable_layout(self.stage)[0]}
        n_train = layout.trainable_layout(self.stage)[1]
        self.register_buffer("flat", torch.zeros(n_train), persistent=False)
        c2f = _cfg_get(cfg_model, "object.sdf.encoding.coarse2fine", None)
        c2f = None if c2f is None else {k: c2f[k] for k in ("enabled", "init_active_level", "step") if k in c2f}
        if self.stage == "a":
            self.neural_sdf = NeuralSDF(self.pcfg, c2f, view=self._view)
            self.neural_rgb = LumenRGB(self._view, layout.HEADS_A)
            self.s_var = torch.nn.Parameter(self._view("s_var"), requires_grad=True)
            with torch.no_grad():
                self.s_var.fill_(float(cfg_model.object.s_var.init_val))
        else:
            self.neural_sdf = NeuralSDF(self.pcfg, c2f)
            self.neural_rgb = LumenRGB(self._view)
            self.s_var = torch.nn.Parameter(torch.tensor(float(cfg_model.object.s_var.init_val)),
                                            requires_grad=False)
        if self.pcfg.bounding == "box":
            self.bounding_box_aabb = torch.tensor(self.pcfg.aabb)
        self.engine = None
        self._streams = None  # inference chunk-pipeline streams
        self.pipeline_chunks = True  # two inference chunks in flight (False: one stream)
        self._sdf_version = None
        self.image_width = self.image_size_train[1]
        self.deterministic = False  # fixed-order gradient reductions (RenderEngine.deterministic)
        self.pq = True              # stage-b output-layer dW from the forward's partials (RenderEngine.pq)

    # -------------------------------------------------------------- parameter plumbing
    def _view(self, name, flat=None):
        shape, off = self._layout[name]
        flat = self.flat if flat is None else flat
        return flat.data[off:off + int(np.prod(shape))].view(shape)

    def _layout_items(self):
        """[(name, shape, offset)] of the flat trainable buffer."""
        return layout.trainable_layout(self.stage)[0]

    def _trainable_items(self):
        """[(name, shape, offset, numel)] in flat-layout order (the autograd inputs)."""
        return [(n, shape, off, int(np.prod(shape))) for n, shape, off in layout.trainable_layout(self.stage)[0]]

    def trainable_parameters(self):
        """The named Parameters that are views of the flat buffer, in flat-layout order."""
        named = dict(self.named_parameters())
        return [named[n] for n, _, _, _ in self._trainable_items()]

    def device(self):
        return self.flat.device

    def set_flat_grad(self, grad):
        """Publish a flat gradient (the fused Trainer's) as flat.grad and as per-Parameter views,
        as the autograd backward does."""
        self.flat.grad = grad
        for p, (_, shape, off, n) in zip(self.trainable_parameters(), self._trainable_items()):
            p.grad = grad[off:off + n].view(shape)

    def flat_grad_from_params(self):
        """The flat gradient behind the named Parameters' .grad (a view of one buffer after the
        autograd backward; gathered into one otherwise).  None where no Parameter has a grad."""
        ps = self.trainable_parameters()
        if all(p.grad is None for p in ps):
            return None
        out = torch.zeros_like(self.flat)
        for p, (_, _, off, n) in zip(ps, self._trainable_items()):
            if p.grad is not None:
                out[off:off + n].copy_(p.grad.reshape(-1))
        return out

    @torch.no_grad()
    def init_weights(self, seed=0):
        """The reference's initial weights (imaginaire trainer.init.type 'none': module inits
        only): SDF MLP geometric init (neuralangelo/utils/mlp.py:71-84, out_bias from the config),
        tcnn table U(-1e-4, 1e-4), colour heads nn.Linear default init with zero last bias
        (nerf_util.py:176-183), s_var = init_val; drawn from seeded CPU generators."""
        from . import synthetic
        pc = self.pcfg
        sd = synthetic.make_state_dict(
            log2T=pc.log2T, seed=seed, s_var=float(self.cfg_model.object.s_var.init_val), enc_std=0.0,
            table_amp=1e-4, heads="rgb" if self.stage == "a" else "rgb_r_s",
            out_bias=float(_cfg_get(self.cfg_model, "object.sdf.mlp.out_bias", 0.5)), scale_rule=pc.scale_rule)
        self.load_state_dict(sd)

    # -------------------------------------------------------------- checkpoints
    TABLE_KEY = "neural_sdf.tcnn_encoding.params"

    def load_state_dict(self, state_dict, strict=True, assign=False):
        """nn.Module.load_state_dict, plus the hash-table size rule: the table size depends on
        the level-5 resolution tcnn derives from its fp32 scale arithmetic (129 here, 45,724,048
        entries at the default config) or from exact arithmetic (128, 45,674,504); a checkpoint
        of the other size switches the level table to that rule instead of failing on shape
        (neuralangelo/utils/modules.py:42-50; SURVEY.md §8c: the tcnn rule is unpinned)."""
        src = state_dict.get(self.TABLE_KEY)
        if src is not None and src.numel() != self.neural_sdf.tcnn_encoding.params.numel():
            self._adopt_table_size(src.numel())
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        if src is not None:
            self.table_sharded_stale = False   # the whole fp32 table was just written
        return res

    def _adopt_table_size(self, numel):
        from .hashgrid import SCALE_RULES
        pc = self.pcfg
        sizes = {}
        for rule in SCALE_RULES:
            table, total = level_table(pc.levels, pc.log2T, pc.min_logres, pc.max_logres, rule)
            sizes[rule] = (total * 8, [r for _, r, _, _ in table])
        match = [r for r, (n, _) in sizes.items() if n == numel]
        if not match:
            raise ValueError(
                "%s has %d elements; this hash-grid config expects %s" % (
                    self.TABLE_KEY, numel, ", ".join("%d (%d entries x 8; %s scale rule, level resolutions %s)"
                                                     % (n, n // 8, r, res[:7]) for r, (n, res) in sizes.items())))
        rule = match[0]
        import warnings
        warnings.warn("checkpoint hash table has %d elements: level-5 resolution %d (%s scale rule); the level "
                      "table follows it" % (numel, sizes[rule][1][5], rule))
        pc.scale_rule = rule
        p = self.neural_sdf.tcnn_encoding.params
        p.data = torch.zeros(numel, dtype=p.dtype, device=p.device)
        self.engine = None
        self._sdf_version = None

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        # re-point the parameter views at the (possibly moved) flat buffer
        flat = self.flat.detach()
        self._buffers["flat"] = flat
        for name, p in self.named_parameters():
            if name in self._layout:
                p.data = self._view(name, flat)
        self.engine = None
        self._sdf_version = None
        return self

    def _sdf_l1(self):
        if self.stage == "a":
            return None  # packed from the flat buffer with the heads
        l1 = self.neural_sdf.mlp.linears[1]
        return (l1.weight_v.detach(), l1.weight_g.detach().reshape(-1), l1.bias.detach())

    def prepare(self):
        """(Re)build the device weight images.  Stage b: SDF once (frozen) + heads every step.
        Stage a: the fp16 table shadow when the table changed outside the fused AdamW (which
        keeps it in sync), the SDF blocks and the heads every step; tap epsilon and the
        coarse-to-fine level count from neural_sdf."""
        if self.engine is None:
            self.engine = RenderEngine(self.pcfg, self.flat.device, self.stage)
        sdf = self.neural_sdf
        eng = self.engine
        eng.deterministic = self.deterministic
        eng.pq = self.pq
        eng.set_normal_eps(sdf.normal_eps)
        eng.active_levels = int(sdf.active_levels)
        l0 = sdf.mlp.linears[0]
        pack_args = (l0.weight_v.detach(), l0.weight_g.detach().reshape(-1), l0.bias.detach(),
                     sdf.mlp.linear_sdf.weight.detach().reshape(-1), sdf.mlp.linear_sdf.bias.detach())
        if self.stage == "a":
            table = sdf.tcnn_encoding.params
            ver = (table._version, table.data_ptr())
            if ver != self._sdf_version:
                if getattr(self, "table_sharded_stale", False):
                    # ZeRO (trainer.ZeroTableAdamW): outside this rank's shard the fp32 master is
                    # older than the fp16 shadow the kernels read; re-casting it would revert the
                    # other ranks' updates
                    raise RuntimeError("the hash table is ZeRO-sharded and not gathered: call "
                                       "trainer.sync_table() on every rank before rebuilding the engine")
                eng.load_table(table.detach())
                self._sdf_version = ver
            eng.pack_sdf(*pack_args)
        else:
            ver = tuple(p._version for p in sdf.parameters()) + tuple(p.data_ptr() for p in sdf.parameters())
            if ver != self._sdf_version:
                eng.load_sdf(sdf.tcnn_encoding.params.detach(), *pack_args)
                self._sdf_version = ver
        eng.pack_heads(self.flat.detach(), self._sdf_l1())

    # -------------------------------------------------------------- reference API
    def get_param_groups(self, cfg_optim):
        """NeuralLumen/model.py:422-438 (partial_training keywords)."""
        keywords = _cfg_get(cfg_optim, "partial_training", None)
        if keywords is None:
            return self.parameters()
        return [p for n, p in self.named_parameters() if any(k in n for k in keywords)]

    def forward(self, data, u=None):
        """NeuralLumen/model.py:113-118 -> render_pixels_lumen; ``u`` injects the stratified
        uniforms (nerf_util.py:33) for parity runs."""
        self.prepare()
        u = self.stratified_uniforms(data, u)
        self.image_width = self.image_size_train[1]
        table = self.neural_sdf.tcnn_encoding.params
        res = _RenderHeads.apply(table, self, data, u, self.progress, self.training, *self.trainable_parameters())
        return self.outputs(self._last_state, res)

    def stratified_uniforms(self, data, u=None):
        """nerf_util.py:33: U[0,1) per coarse bin in training, midpoints (None) in eval."""
        if not (self.stratified and self.training):
            return None
        if u is None:
            u = torch.rand(1, data["ray_idx"].shape[-1], self.pcfg.n_coarse, device=self.flat.device)
        return u

    def outputs(self, st, heads=None):
        """The reference output dict (NeuralLumen/model.py:312-323) of a render state; ``heads``
        = differentiable (rgb, o_r, o_s, o_re) when called under autograd."""
        rays, dists, fld, hd, comp = st
        heads = heads if heads is not None else (comp["rgb"], comp["o_r"], comp["o_s"], comp["o_re"])
        rgb, o_r, o_s, o_re = heads[:4]
        grads, hess = (heads[4], heads[5]) if len(heads) == 6 else (fld["grad"], fld["hess"])
        if len(heads) == 6 and fld["hess"] is None:
            hess = None
        N, R = dists.shape
        out = dict(rgb=rgb[None], o_r=o_r[None], o_s=o_s[None], o_re=o_re[None],
                   outside=rays["outside"].bool().view(1, R, 1),
                   dists=dists.t().reshape(1, R, N, 1),
                   weights=comp["weights"].t().reshape(1, R, N, 1),
                   gradients=grads.permute(1, 0, 2).reshape(1, R, N, 3),
                   hessians=None if hess is None else hess.permute(1, 0, 2).reshape(1, R, N, 3),
                   opacity=None, gradient=None)
        if self.stage == "a":  # mode 'rgb' has no intrinsic outputs (NeuralLumen/model.py:300-303)
            for k in ("o_r", "o_s", "o_re"):
                out.pop(k)
        if not self.training:
            out["opacity"] = comp["opacity"][None]
            out["gradient"] = comp["gradient"][None]
            out["depth"] = comp["depth"][None]
            if "visibility" in comp:  # NeuralLumen/model.py:325-336
                for k in ("visibility", "normal_x_light", "pseudo_shading", "inter_dist", "inter_mask"):
                    out[k] = comp[k][None]
        return out

    @torch.no_grad()
    def inference(self, data, shard=True):
        """NeuralLumen/model.py:60-111: full image in rand_rays_val chunks, eval branch.

        Under an initialised process group with world > 1 (and shard=True) each rank renders
        one contiguous tile of the frame and ONE all_gather assembles it, so
        every rank returns the full maps."""
        from . import shard as sh
        self.eval()
        self.prepare()
        H, W = self.image_size_val
        n_pix = H * W
        self.image_width = W
        world, rank, group = 1, 0, None
        if shard:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                world, rank = dist.get_world_size(), dist.get_rank()
        lo, hi, _ = sh.shard_range(n_pix, rank, world)
        # mli_rgb_fwd takes whole 256-sample workgroups: pad each chunk's ray count so
        # R * N % 256 == 0 (repeating the last pixel), drop the padding afterwards
        N = self.pcfg.n_samples
        vis = self.pcfg.light_visibility is not None
        step = 256 // math.gcd(N, 256)
        dev = self.flat.device
        parts = []
        # Two chunks in flight on two streams, each with its own engine buffer lane: one
        # chunk's gather-bound sampling / FIELD kernels overlap the other's MFMA-bound heads.
        main = torch.cuda.current_stream(dev)
        if self._streams is None or self._streams[0].device != dev:
            self._streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
        for s in self._streams:
            s.wait_stream(main)
        try:
            for i, start in enumerate(range(lo, hi, self.rand_rays_val)):
                R = min(self.rand_rays_val, hi - start)
                Rp = -(-R // step) * step
                lane = i % 2 if self.pipeline_chunks else 0
                with torch.cuda.stream(self._streams[lane]):
                    self.engine.use_lane(lane)
                    ridx = torch.arange(start, start + Rp, device=dev).clamp_(max=start + R - 1)[None]
                    d = dict(pose=data["pose"], intr=data["intr"], pose_light=data["pose_light"], ray_idx=ridx)
                    st = self.engine.render(d, self.s_var.detach(), self.progress, False, u=None, W=W)
                    parts.append(sh.pack(st[4], vis)[:R])
        finally:
            self.engine.use_lane(0)
            for s in self._streams:
                main.wait_stream(s)
        for p in parts:
            p.record_stream(main)
        local = torch.cat(parts, 0) if parts else torch.zeros(0, sh.n_channels(vis), device=dev)
        packed = sh.gather_tiles(local, n_pix, world, group) if world > 1 else local
        out = {k: v.contiguous()[None] for k, v in sh.unpack(packed, vis).items()}
        rot = data["pose"][..., :3, :3]
        normal_cam = -out["gradient"] @ rot.transpose(-1, -2)

        def full(x):
            return x.unflatten(1, (H, W)).moveaxis(-1, 1)
        out.update(rgb_map=full(out["rgb"]), opacity_map=full(out["opacity"]), depth_map=full(out["depth"]),
                   normal_map=full(normal_cam))
        for k in ("o_r", "o_s", "o_re"):
            out[k + "_map"] = full(out[k])
        if vis:  # NeuralLumen/model.py:78-83
            for k in ("visibility", "normal_x_light", "pseudo_shading", "inter_dist", "inter_mask"):
                out[k + "_map"] = full(out[k]).float()
            out["visibility"] = out["visibility"] > 0.5
            out["inter_mask"] = out["inter_mask"] > 0.5
        return out
