"""CPU stand-in for ``mli_nerf_amd.engine.RenderEngine`` (TEST INFRASTRUCTURE ONLY).

The render kernels need the MI355X.  The multi-process tests exercise what sits around them --
Trainer's step plumbing (gradient + metric all-reduce, fused-AdamW bookkeeping, gradient views),
Model.inference's tile sharding and gather -- on CPU with gloo, so the engine is replaced by this
stub: the same call surface, with outputs that are cheap, deterministic functions of the ray
indices and of three trainable parameters.  ``install(monkeypatch)`` swaps it in together with
torch versions of the two kernel calls the Trainer issues itself (loss, AdamW).  Nothing here is
product code; the product path raises without a GPU (RenderEngine.__init__).
"""
import math

import torch


class StubEngine:
    def __init__(self, cfg, device, stage="b"):
        self.cfg, self.device, self.stage = cfg, torch.device(device), stage
        self.active_levels = cfg.levels
        self.table16 = None
        self.gate_wgrad, self.gate_event = False, None
        self._lanes = {0: {}}
        self._bufs = self._lanes[0]
        self.flat = None

    # parameter plumbing (RenderEngine keeps device weight images; the stub keeps the buffer)
    def set_normal_eps(self, eps):
        pass

    def load_sdf(self, *a):
        pass

    def load_table(self, *a):
        pass

    def pack_sdf(self, *a):
        pass

    def pack_heads(self, flat, sdf_l1):
        self.flat = flat

    def use_lane(self, lane):
        self._bufs = self._lanes.setdefault(lane, {})

    def _buf(self, name, shape, dtype=torch.float32):
        t = self._bufs.get(name)
        n = math.prod(shape)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t[:n].view(*shape)

    def stamp(self):
        return (id(self._bufs), self._bufs.get("__gen", 0))

    def check_stamp(self, stamp):
        pass

    @staticmethod
    def features(ray_idx):
        return (ray_idx.reshape(-1).double() % 97 / 97.0).float()

    def render(self, data, s_var, progress, training, u=None, W=512):
        """rgb[r, c] = x_r * flat[c] (x_r a function of the pixel index); the other outputs are
        fixed functions of x_r (no parameters)."""
        x = self.features(data["ray_idx"])
        R, N = x.shape[0], self.cfg.n_samples
        rgb = x[:, None] * self.flat[:3][None]
        comp = dict(rgb=rgb, o_r=x[:, None].expand(R, 3) * 0.5, o_s=x[:, None] * 0.25,
                    o_re=x[:, None].expand(R, 3) * 0.1, weights=torch.zeros(N, R),
                    opacity=x[:, None], gradient=torch.stack([x, -x, 2 * x], -1), depth=x[:, None] * 3)
        rays = dict(outside=torch.zeros(R, dtype=torch.uint8), x=x)
        fld = dict(grad=torch.zeros(N, R, 3), hess=torch.zeros(N, R, 3))
        return rays, torch.zeros(N, R), fld, {}, comp

    def backward(self, st, d_rgb, d_o_r, d_o_s, d_o_re, flat, sdf_l1, grad_out, dz4=None, on_class=None):
        x = st[0]["x"]
        grad_out.zero_()
        grad_out[:3] = (d_rgb * x[:, None]).sum(0)
        # every element rank-specific, so that each class range's reduction is exercised
        k = torch.arange(3, grad_out.numel(), dtype=torch.float64)
        grad_out[3:] = (torch.sin(k * 1e-3) * float(x.double().sum()) + torch.cos(k * 7e-4) * float(
            (d_rgb.double() * x.double()[:, None]).sum())).float()
        if on_class is not None:   # RenderEngine.backward's per-class completion, in launch order
            for c in ("out", "big", "wide"):
                on_class(c)
        return grad_out

    def load_table(self, params_flat):
        self.table16 = params_flat.detach().half()

    def backward_a(self, st, d_rgb, flat, grad_flat, grad_table, w_eikonal, w_curvature, progress,
                   d_grad_ext=None, d_hess_ext=None):
        """Stage a: the flat gradient as in ``backward``, and a dense rank-specific table gradient
        (every element a function of the rays' pixel features and d rgb: the ranks' rays differ)."""
        x = st[0]["x"]
        self.backward(st, d_rgb, None, None, None, flat, None, grad_flat)
        n = grad_table.numel()
        k = torch.arange(n, dtype=torch.float64)
        s = d_rgb.double().sum(1) * x.double()                  # one value per ray
        grad_table.copy_(torch.sin(k * 1e-3) * float(s.sum()) + torch.cos(k * 7e-4) * float((s * s).sum()))
        return grad_flat, grad_table


def stub_losses(trainer, st, data, lv):
    """render L1 x3 and PSNR (NeuralLumen/trainer.py:135-136) in torch, into lv like the kernel."""
    rgb = st[4]["rgb"]
    gt = data["image_sampled"].reshape(rgb.shape)
    diff = rgb - gt
    lv.zero_()
    lv[0] = diff.abs().mean() * 3
    lv[5] = lv[0] * trainer.weights.get("render", 1.0)
    lv[6] = -10 * torch.log10(diff.square().mean())
    d_rgb = torch.sign(diff) * (3 * trainer.weights.get("render", 1.0) / diff.numel())
    z = torch.zeros_like(rgb)
    return d_rgb, z, z[:, :1], z


def stub_adamw_step(self, grad, lr, p16=None, ranges=None, before=None, zero_grad=False):
    """torch.optim.AdamW's update on the flat buffer (FusedAdamW.step's semantics, incl. ranges,
    the per-range hook, the fp16 copy and the consumed gradient left zero)."""
    self.step_count += 1
    b1, b2 = self.betas
    for i, (off, n) in enumerate([(0, self.flat.numel())] if ranges is None else ranges):
        if before is not None:
            before(i)
        p, g = self.flat.detach()[off:off + n], grad[off:off + n]
        m, v = self.m[off:off + n], self.v[off:off + n]
        p.mul_(1 - lr * self.wd)
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v / (1 - b2 ** self.step_count)).sqrt_().add_(self.eps)
        p.addcdiv_(m, denom, value=-lr / (1 - b1 ** self.step_count))
        if p16 is not None:
            p16[off:off + n].copy_(p)
        if zero_grad:
            g.zero_()


def install(monkeypatch=None):
    """Swap the stub in (monkeypatch fixture, or plain setattr in a spawned worker)."""
    from mli_nerf_amd import model as model_mod, trainer as trainer_mod
    pairs = [(model_mod, "RenderEngine", StubEngine),
             (trainer_mod.Trainer, "_fused_losses", lambda self, st, data, lv: stub_losses(self, st, data, lv)),
             (trainer_mod.FusedAdamW, "step", stub_adamw_step),
             (trainer_mod.Trainer, "fused_tail", False)]  # the stub stands in for the three-call tail
    for obj, name, val in pairs:
        if monkeypatch is not None:
            monkeypatch.setattr(obj, name, val)
        else:
            setattr(obj, name, val)


class _NullStream:
    def __init__(self, *a, **k):
        self.device = torch.device("cpu")

    def wait_stream(self, *a):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def install_cpu_streams():
    """Model.inference pipelines chunks over two HIP streams; on CPU those are no-ops."""
    torch.cuda.current_stream = lambda device=None: _NullStream()
    torch.cuda.Stream = _NullStream
    torch.cuda.stream = lambda s: _NullStream()
    torch.Tensor.record_stream = lambda self, s: None
