"""Device-side orchestration of the stage-b render path on libmli_hip.so.

One ``RenderEngine`` per device/rank.  It owns every buffer the kernels use (allocated by
PyTorch, handed to the C ABI as raw pointers on the current stream) and runs:

  rays -> coarse samples -> sdf -> 4 x (section pdf -> fine samples -> sdf) -> merge
       -> field (sdf + 4 taps + h0) -> heads (feat + rgb/o_r/o_s) -> NeuS composite
and, in training, the backward of the composite into the heads, the dX chain, the weight
gradients and the weight-norm backward into one flat fp32 gradient buffer.

Reference call stack mirrored: NeuralLumen/model.py:113-131 (forward),
:232-336 (render_rays_lumen), :338-403 (render_rays_object_lumen),
neuralangelo/model.py:449-515 (sampling, NeuS alphas).
"""
import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib as L
from . import layout
from .hashgrid import level_table, normal_eps


class PathConfig:
    """Hot-path knobs, filled from the reference config tree (see model.py)."""

    def __init__(self, n_coarse=64, n_fine=16, n_hier=4, white_bg=True, bounding="sphere",
                 aabb=(-1, -1, -1, 1, 1, 1), outside_val=1000.0, anneal_end=0.1, log2T=22,
                 levels=16, min_logres=5, max_logres=11, light_visibility=None, scale_rule="fp32"):
        self.n_coarse, self.n_fine, self.n_hier = n_coarse, n_fine, n_hier
        self.scale_rule = scale_rule  # hash-grid level scale rule (hashgrid.level_table)
        self.white_bg, self.bounding, self.aabb = white_bg, bounding, tuple(float(x) for x in aabb)
        self.outside_val, self.anneal_end = outside_val, anneal_end
        self.log2T, self.levels, self.min_logres, self.max_logres = log2T, levels, min_logres, max_logres
        # model.light_visibility when enabled (NeuralLumen/model.py:25-35): dict(camera_ray_type,
        # type, bounding, radius, gamma) -- None: off
        self.light_visibility = light_visibility

    @property
    def n_samples(self):
        return self.n_coarse + self.n_fine * self.n_hier


def _grid_levels(cfg):
    table, total = level_table(cfg.levels, cfg.log2T, cfg.min_logres, cfg.max_logres, cfg.scale_rule)
    g = L.GridLevels()
    for i, (scale, res, size, off) in enumerate(table):
        g.scale[i], g.res[i], g.size[i], g.offset[i] = scale, res, size, off
        g.modmagic[i] = layout.fastmod_magic(size)
    return g, total


# The scratch buffers a render's geometry writes (rays, the sampling rounds, the FIELD pass):
# the only ones a training prefetch lane needs of its own (RenderEngine.use_lane(geometry_only)).
GEOMETRY_BUFS = frozenset(["center", "ray_unit", "ray_norm", "pts_light", "near", "far", "outside",
                           "d_coarse", "s_coarse", "d_m0", "d_m1", "s_m0", "s_m1", "d_f0", "d_f1", "s_f0",
                           "s_f1", "dists", "sdf", "grad", "hess", "h0", "enc5"])


class _GeometryLane(dict):
    """A lane's buffer set whose geometry buffers (GEOMETRY_BUFS) are its own and every other
    buffer (the heads' activations, the backward's dZ images and dW slabs, the loss scratch, the
    render generation) lives in one set shared by all such lanes.  The training prefetch renders
    only the geometry of batch k+1 / k+2 into its lane while step k runs, and the steps run one
    after another on the main stream, so one set of step buffers serves every lane (VERDICT r4
    item 7: ~7.5 GiB per lane at 4096 x 128 otherwise)."""

    def __init__(self, shared):
        super().__init__()
        self.shared = shared

    def _d(self, k):
        return self if k in GEOMETRY_BUFS else self.shared

    def __getitem__(self, k):
        d = self._d(k)
        return dict.__getitem__(d, k) if d is self else d[k]

    def __setitem__(self, k, v):
        d = self._d(k)
        if d is self:
            dict.__setitem__(self, k, v)
        else:
            d[k] = v

    def __contains__(self, k):
        d = self._d(k)
        return dict.__contains__(d, k) if d is self else k in d

    def get(self, k, default=None):
        d = self._d(k)
        return dict.get(d, k, default) if d is self else d.get(k, default)

    def pop(self, k, *default):
        d = self._d(k)
        return dict.pop(d, k, *default) if d is self else d.pop(k, *default)


# stage-b weight-gradient classes in launch order and the head layers each one completes
# (mli_dw4 / THIN: the output layers; BIG: the hidden 256 x 256 layers; WIDE: layer 0)
GRAD_CLASSES = ("out", "big", "wide")
GRAD_CLASS_LAYERS = {"out": (4,), "big": (1, 2, 3), "wide": (0,)}


def _to_device_structs(structs, device):
    raw = b"".join(bytes(s) for s in structs)
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)


class RenderEngine:
    """``stage`` 'b': LumenRGB 'rgb_r_s' (three heads, frozen geometry); 'a': mode 'rgb' (one
    head) with the geometry trained -- hash table, SDF MLP and s_var (backward_a)."""

    def __init__(self, cfg, device, stage="b"):
        if torch.device(device).type != "cuda":
            raise RuntimeError("RenderEngine runs on the MI355X (libmli_hip.so); the model is on %s" % device)
        self.cfg = cfg
        self.stage = stage
        self.head_specs = layout.HEADS_A if stage == "a" else layout.HEADS
        self.device = torch.device(device)
        self.levels, self.table_entries = _grid_levels(cfg)
        self.set_normal_eps(normal_eps(cfg.levels, cfg.min_logres, cfg.max_logres))
        self.active_levels = cfg.levels
        self.table16 = None
        # data_ptr of a table-gradient buffer the last table AdamW left all zero (mli_adamw zero_grad),
        # of the split-K dW buffer the last assemble left zero (zero_dw), of the zeroed head outputs
        self.table_grad_clean = None
        self._dw_zero = None
        self._y_zeroed = None
        self.wsdf = torch.empty(65536 + 5 * 1024 + 16, dtype=torch.uint8, device=self.device)
        self.fplan, fbytes = layout.fwd_plan(self.head_specs)
        self.bplan, bbytes = layout.geo_plan() if stage == "a" else layout.bwd_plan()
        # both weight images in one allocation, so one mli_pack call (2 launches) fills them
        self._bwd_off = (fbytes + 255) // 256 * 256
        self._wimg = torch.empty(self._bwd_off + bbytes, dtype=torch.uint8, device=self.device)
        self.wfwd = self._wimg[:fbytes]
        self.wbwd = self._wimg[self._bwd_off:]
        self.wsdf_t = torch.empty(65536, dtype=torch.uint8, device=self.device) if stage == "a" else None
        self._kmaps = []  # keep host kmap tensors alive
        self.tlayout, self.n_train = layout.trainable_layout(stage)
        self.toff = {name: (off, shape) for name, shape, off in self.tlayout}
        self._lanes = {0: {}}
        self._bufs = self._lanes[0]  # the current lane's scratch buffers (see use_lane)
        self._shared_step = None     # the step buffers shared by the geometry-only lanes
        self.gate_wgrad, self.gate_event = False, None  # event before the dW launches (Trainer.prefetch)
        self.u_fine = (C.c_float * 64)(*(layout.u_fine(cfg.n_fine) + [2.0] * (64 - cfg.n_fine)))
        self._pack_descs = None
        self.trace = None  # set to a list to record per-round sampler outputs (debug/tests)
        # fixed-order reductions instead of fp32 atomics in mli_wgrad / mli_hash_bwd:
        # bit-reproducible gradients at the cost of partial-slab traffic
        self.deterministic = False
        # mli_wgrad classes (bit mask) whose k-slices are reduced through partial slabs + an
        # ordered sum (the deterministic mode's) instead of fp32 atomics outside that mode too:
        # WIDE (its 80 k-slices x 3 x 256 x 304 atomic adds burst at the end of the launch).
        # Measured (profiles/r5/slabs, same box): WIDE 0.299 -> 0.265 ms; BIG 0.831 -> 0.840 and
        # THIN 0.143 -> 0.204 ms the other way, stage a slower with its 5S job on slabs.
        self.wgrad_slab_classes = int(os.environ.get("MLI_WGRAD_SLABS", "2"))
        # stage-b training: the output layers' dW from per-tile partials the heads forward forms
        # while X3 is in registers (mli_rgb_fwd PQ mode + mli_dw4) instead of X3 through HBM and
        # the THIN split-K GEMM; needs N % 32 == 0 (a 32-sample tile within one ray)
        self.pq = True
        self._wplans = {}   # wgrad plans per buffer set (the prefetch lanes alternate)
        # reference column -> packed k maps of the head layers (constant; uploaded once)
        self._kinv = {(name, li): torch.from_numpy((layout.head_kinv(name, k_in) if li == 0 else
                                                    np.arange(256)).astype(np.int16)).to(self.device)
                      for name, k_in, _ in layout.HEADS for li in range(5)}

    # ------------------------------------------------------------------ parameters
    def set_normal_eps(self, normal_eps_value):
        """Tap epsilon normal_eps / sqrt(3) (modules.py:102-107,159) and the fp32 denominators
        of the gradient / hessian stencils (:167,172)."""
        eps64 = float(normal_eps_value) / np.sqrt(3)
        self.eps = float(np.float32(eps64))
        self.grad_den = float(np.float32(4.0 * eps64))
        self.hess_den = float(np.float32(eps64 ** 2))

    def load_table(self, params_flat):
        """fp16 gather shadow of the hash table (tcnn precision)."""
        assert params_flat.numel() == self.table_entries * 8, (params_flat.numel(), self.table_entries)
        if self.table16 is None or self.table16.numel() != params_flat.numel():
            self.table16 = torch.empty(params_flat.numel(), dtype=torch.float16, device=self.device)
        L.call("mli_cast_f16", L.CastArgs(L.ptr(params_flat), L.ptr(self.table16), params_flat.numel()))

    def pack_sdf(self, v0, g0, b0, w_sdf, b_sdf):
        """SDF layer 0 + sdf head block (and, in stage a, W0_enc^T for the backward)."""
        L.call("mli_pack_sdf", L.PackSdfArgs(L.ptr(v0), L.ptr(g0), L.ptr(b0), L.ptr(w_sdf), L.ptr(b_sdf),
                                             L.ptr(self.wsdf)))
        if self.wsdf_t is not None:
            L.call("mli_pack_sdf_t", L.PackSdfTArgs(L.ptr(v0), L.ptr(g0), L.ptr(self.wsdf_t)))

    def load_sdf(self, params_flat, v0, g0, b0, w_sdf, b_sdf):
        """Frozen geometry (stage b): fp16 shadow of the hash table + packed layer 0."""
        self.load_table(params_flat)
        self.pack_sdf(v0, g0, b0, w_sdf, b_sdf)

    def _descs(self, plan, tensors, base=0):
        descs = []
        for p in plan:
            km = torch.from_numpy(p["kmap"].astype(np.int16)).to(self.device)
            kmode = torch.from_numpy(p["kmode"].astype(np.uint8)).to(self.device)
            nm = None
            if p.get("nmap") is not None:
                nm = torch.from_numpy(p["nmap"].astype(np.int16)).to(self.device)
            self._kmaps += [km, kmode, nm]
            v, g, b = tensors(p["prefix"])
            descs.append(L.PackLayer(L.ptr(v), L.ptr(g), L.ptr(b), p["n_out"], p["k_ref"], p["transpose"],
                                     p["n_tiles"], p["k_steps"], L.ptr(km), L.ptr(kmode), base + p["dst_offset"],
                                     p["chunk_stride"], L.ptr(nm)))
        return descs

    def pack_heads(self, flat, sdf_l1):
        """Weight-norm fold + fp16 fragment packing of SDF layer 1 and the heads (forward
        image) and of the transposed layers of the backward (stage b: the heads' dX chain;
        stage a: the geometry chain, layout.geo_plan)."""
        def tensors(prefix):
            if prefix == "neural_sdf.mlp.linears.1" and sdf_l1 is not None:
                return sdf_l1
            return tuple(self.param_view(flat, prefix + s) for s in (".weight_v", ".weight_g", ".bias"))
        key = (flat.data_ptr(), None if sdf_l1 is None else sdf_l1[0].data_ptr())
        if self._pack_descs is None or self._pack_descs[0] != key:
            self._kmaps = []
            descs = self._descs(self.fplan, tensors) + self._descs(self.bplan, tensors, self._bwd_off)
            self._pack_descs = (key, _to_device_structs(descs, self.device), len(descs))
        _, d, n = self._pack_descs
        L.call("mli_pack", L.PackArgs(n, L.ptr(d), L.ptr(self._wimg), L.ptr(self._buf("pack_scale", (n, 256)))))

    def param_view(self, flat, name):
        off, shape = self.toff[name]
        n = int(np.prod(shape))
        return flat[off:off + n].reshape(shape)

    # ------------------------------------------------------------------ buffers
    def use_lane(self, lane, geometry_only=False):
        """Switch to scratch-buffer set ``lane``: renders in flight on different streams (the
        pipelined inference chunks, Model.inference) each own a buffer set; a lane is reused
        only on its own stream, so stream order protects it.  ``geometry_only`` (the training
        prefetch lanes, Trainer.prefetch): the lane owns only the geometry buffers and shares the
        rest with the other such lanes (_GeometryLane)."""
        if lane not in self._lanes:
            if geometry_only:
                if self._shared_step is None:
                    self._shared_step = {}
                self._lanes[lane] = _GeometryLane(self._shared_step)
            else:
                self._lanes[lane] = {}
        self._bufs = self._lanes[lane]
        if geometry_only != isinstance(self._bufs, _GeometryLane):
            raise RuntimeError("engine lane %r was created with geometry_only=%s" % (lane, not geometry_only))

    def _buf(self, name, shape, dtype=torch.float32):
        t = self._bufs.get(name)
        n = int(np.prod(shape))
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t[:n].view(*shape)

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def rays(self, pose, intr, pose_light, ray_idx, W, R=None, first_pixel=0):
        """pose/intr/pose_light [1,3,4]/[1,3,3]/[1,3,4] (inverted in-kernel); ray_idx [1,R] int64 or None."""
        w2c, w2l, K = pose[0].contiguous(), pose_light[0].contiguous(), intr[0].contiguous()
        R = R if ray_idx is None else ray_idx.shape[-1]
        ridx = None if ray_idx is None else ray_idx.reshape(-1).to(torch.int64).contiguous()
        out = dict(center=self._buf("center", (R, 3)), ray_unit=self._buf("ray_unit", (R, 3)),
                   ray_norm=self._buf("ray_norm", (R,)), pts_light=self._buf("pts_light", (R, 3)),
                   near=self._buf("near", (R,)), far=self._buf("far", (R,)),
                   outside=self._buf("outside", (R,), torch.uint8))
        aabb = (C.c_float * 6)(*self.cfg.aabb)
        L.call("mli_rays", L.RaysArgs(L.ptr(K), L.ptr(w2c), L.ptr(w2l), L.ptr(ridx), first_pixel, R, W,
                                      1 if self.cfg.bounding == "box" else 0, aabb,
                                      L.ptr(out["center"]), L.ptr(out["ray_unit"]), L.ptr(out["ray_norm"]),
                                      L.ptr(out["pts_light"]), L.ptr(out["near"]), L.ptr(out["far"]),
                                      L.ptr(out["outside"])))
        out["_keep"] = (w2c, w2l, K, ridx)
        return out

    def _sdf(self, rays, dists, n_per_ray, out, mode=0, grad=None, hess=None, h0=None):
        R = rays["center"].shape[0]
        enc = None
        if mode == 1:
            # the FIELD encoding image (stage a's backward re-reads it)
            tiles = (R * n_per_ray + 31) // 32
            enc = self._buf("enc5", (tiles * 32 * 640,), torch.float16)
        L.call("mli_sdf", L.SdfArgs(mode, R, n_per_ray, L.ptr(rays["center"]), L.ptr(rays["ray_unit"]),
                                    L.ptr(dists), L.ptr(rays["outside"]), L.ptr(self.table16), self.levels,
                                    L.ptr(self.wsdf), self.eps, self.grad_den, self.hess_den,
                                    self.cfg.outside_val, 1 if hess is not None else 0, L.ptr(out),
                                    L.ptr(grad), L.ptr(hess), L.ptr(h0), L.ptr(enc), int(self.active_levels)))
        return enc

    @torch.no_grad()
    def sample(self, rays, u=None):
        """sample_dists_all (neuralangelo/model.py:449-465) -> dists [N][R]."""
        cfg = self.cfg
        R = rays["center"].shape[0]
        Nc, Nf, H = cfg.n_coarse, cfg.n_fine, cfg.n_hier
        N = cfg.n_samples
        d0 = self._buf("d_coarse", (Nc, R))
        uu = None if u is None else u.reshape(R, Nc).contiguous()
        L.call("mli_sample_coarse", L.SampleCoarseArgs(L.ptr(rays["near"]), L.ptr(rays["far"]), L.ptr(uu),
                                                       R, Nc, L.ptr(d0)))
        s0 = self._buf("s_coarse", (Nc, R))
        self._sdf(rays, d0, Nc, s0)
        da, sa, na = d0, s0, Nc
        db = sb = None
        nb = 0
        for h in range(H):
            dm = self._buf("d_m%d" % (h & 1), (na + nb, R))
            sm = self._buf("s_m%d" % (h & 1), (na + nb, R))
            f = self._buf("d_f%d" % (h & 1), (Nf, R))
            L.call("mli_sample_fine", L.SampleFineArgs(R, L.ptr(da), L.ptr(sa), na, L.ptr(db), L.ptr(sb), nb,
                                                       L.ptr(dm), L.ptr(sm), Nf, float(64 * 2 ** h),
                                                       C.cast(self.u_fine, C.c_void_p), L.ptr(f)))
            sf = None
            if h < H - 1:
                sf = self._buf("s_f%d" % (h & 1), (Nf, R))
                self._sdf(rays, f, Nf, sf)
            if self.trace is not None:
                self.trace.append(dict(merged=dm.clone(), merged_sdf=sm.clone(), fine=f.clone(),
                                       fine_sdf=None if sf is None else sf.clone()))
            da, sa, na, db, sb, nb = dm, sm, na + nb, f, sf, Nf
        dists = self._buf("dists", (N, R))
        L.call("mli_sample_fine", L.SampleFineArgs(R, L.ptr(da), None, na, L.ptr(db), None, nb, L.ptr(dists),
                                                   None, 0, 0.0, None, None))
        return dists

    @torch.no_grad()
    def field(self, rays, dists, training):
        N, R = dists.shape
        S = N * R
        sdf = self._buf("sdf", (N, R))
        grad = self._buf("grad", (N, R, 3))
        hess = self._buf("hess", (N, R, 3)) if training else None
        h0 = self._buf("h0", (S * 256,), torch.float16)
        enc = self._sdf(rays, dists, N, sdf, mode=1, grad=grad, hess=hess, h0=h0)
        return dict(sdf=sdf, grad=grad, hess=hess, h0=h0, enc=enc)

    def pq_mode(self, N, training):
        """The heads run in PQ mode (mli_rgb_fwd weights / q4, mli_dw4) for this render."""
        return bool(self.pq and training and self.stage == "b" and N % 32 == 0)

    @torch.no_grad()
    def weights(self, rays, dists, fld, s_var, progress):
        """The composite weights alone (mli_composite_fwd with y = NULL): the PQ heads forward
        needs them before the heads run (compute_neus_alphas + alpha_compositing_weights,
        neuralangelo/model.py:492-515, render.py:87-99)."""
        N, R = dists.shape
        w = self._buf("weights", (N, R))
        out = dict(weights=w, rgb=None, o_r=None, o_s=None, o_re=None)
        L.call("mli_composite_fwd", self._composite_args(rays, dists, fld, dict(y=None), s_var, progress, out))
        return w

    @torch.no_grad()
    def heads(self, rays, dists, fld, training, s_var=None, progress=0.0):
        """Heads forward; stage-b training with ``s_var`` given (and N % 32 == 0) runs the PQ
        mode: the composite weights first, then the heads with the output-layer partials."""
        N, R = dists.shape
        S = N * R
        if S % 256:
            raise ValueError("heads: rays x samples = %d x %d is not a whole number of 256-sample tiles (the "
                             "reference configs' batches are: 4096 / 8192 rays x 128 / 192 samples)" % (R, N))
        nh = len(self.head_specs)
        y = self._buf("y", (N, R, 8))
        if nh == 1 and self._y_zeroed != y.data_ptr():
            # o_r / o_s slots the single head never writes (composite reads them): zeroed once per
            # allocation (rows of 8 at any shape, so they stay zero)
            y.zero_()
            self._y_zeroed = y.data_ptr()
        # the x0 image: SDF feature (k-steps 0..15 of each 32-sample tile) + in training the extras
        # (16..18); the WIDE dW operand (ABI 15)
        feat = self._buf("feat", (S * layout.K0,), torch.float16)
        xT = masks = w = q4 = None
        pq = s_var is not None and self.pq_mode(N, training)
        if training and self.stage == "b" and not self.deterministic:
            # the split-K dW accumulators of this lane's backward: left zero by the last
            # mli_grad_assemble (zero_dw, ABI 17), else zeroed here at the start of the step, where
            # the GPU is not shared with the prefetched geometry (before the heads backward the
            # fill competed with the sampling rounds: 5 -> 19 us)
            self._zero_once(self._buf("dw", (self._dw_total(),)))
        if training:
            xT = self._buf("xT", (nh, 3 if pq else 4, S * 256), torch.float16)  # ACC frag images
            masks = self._buf("masks", (nh, 4, S // 32, 64, 4), torch.int32)
        if pq:
            w = self.weights(rays, dists, fld, s_var, progress)
            q4 = self._buf("q4", (S // 256, layout.q4_segs(N), nh, 257, 4))
        L.call("mli_rgb_fwd", L.RgbFwdArgs(R, N, L.ptr(rays["center"]), L.ptr(rays["ray_unit"]),
                                           L.ptr(rays["pts_light"]), L.ptr(dists), L.ptr(fld["grad"]),
                                           L.ptr(fld["h0"]), L.ptr(self.wfwd), L.ptr(y), L.ptr(feat),
                                           L.ptr(xT), L.ptr(masks), nh, L.ptr(w), L.ptr(q4)))
        return dict(y=y, x0T=feat if training else None, xT=xT, masks=masks, feat=feat, q4=q4)

    @torch.no_grad()
    def composite(self, rays, dists, fld, hd, s_var, progress, training):
        N, R = dists.shape
        out = dict(weights=self._buf("weights", (N, R)),
                   rgb=torch.empty(R, 3, device=self.device), o_r=torch.empty(R, 3, device=self.device),
                   o_s=torch.empty(R, 1, device=self.device), o_re=torch.empty(R, 3, device=self.device))
        if not training:
            out.update(opacity=torch.empty(R, 1, device=self.device),
                       gradient=torch.empty(R, 3, device=self.device),
                       depth=torch.empty(R, 1, device=self.device))
            if self.cfg.light_visibility:
                out["blend_dist"] = torch.empty(R, 1, device=self.device)
        L.call("mli_composite_fwd", self._composite_args(rays, dists, fld, hd, s_var, progress, out))
        return out

    def _composite_args(self, rays, dists, fld, hd, s_var, progress, out):
        N, R = dists.shape
        anneal = min(progress / self.cfg.anneal_end, 1.0)
        return L.CompositeArgs(R, N, L.ptr(dists), L.ptr(rays["far"]), L.ptr(rays["ray_unit"]),
                               L.ptr(rays["ray_norm"]), L.ptr(fld["sdf"]), L.ptr(fld["grad"]), L.ptr(hd["y"]),
                               L.ptr(s_var), float(anneal), 1 if self.cfg.white_bg else 0, L.ptr(out["weights"]),
                               L.ptr(out["rgb"]), L.ptr(out["o_r"]), L.ptr(out["o_s"]), L.ptr(out["o_re"]),
                               L.ptr(out.get("opacity")), L.ptr(out.get("gradient")), L.ptr(out.get("depth")),
                               L.ptr(out.get("blend_dist")))

    @staticmethod
    def grad_scale(R):
        """Power-of-two loss scale of the fp16 backward images (undone in mli_grad_assemble)."""
        return float(2.0 ** round(math.log2(max(R, 1)) + 2))

    @torch.no_grad()
    def composite_loss(self, rays, dists, fld, hd, s_var, progress, loss, defer=False):
        """Fused training tail (mli_composite_loss): composite + stage-b losses + composite
        backward in one launch.  ``loss``: an L.LossArgs carrying the loss inputs, weights and the
        losses[8] output (its rgb / o_r / o_s / o_re / d_* fields are not read).  Returns the
        composite dict and dz4 for backward()."""
        N, R = dists.shape
        out = dict(weights=self._buf("weights", (N, R)),
                   rgb=torch.empty(R, 3, device=self.device), o_r=torch.empty(R, 3, device=self.device),
                   o_s=torch.empty(R, 1, device=self.device), o_re=torch.empty(R, 3, device=self.device))
        dz4 = self._buf("dz4", (N, R, 8))
        dray = self._buf("dray", (R, 8)) if hd.get("q4") is not None else None
        args = L.CompositeLossArgs(self._composite_args(rays, dists, fld, hd, s_var, progress, out), loss,
                                   self.grad_scale(R), L.ptr(dz4), 1 if defer else 0, L.ptr(dray))
        n = L.workspace("mli_composite_loss", args)[0] // 4
        args.loss.scratch = L.ptr(self._buf("cl_scratch", (n,)))
        L.call("mli_composite_loss", args)
        if defer:  # the loss values: finish_losses(), once the gradients are issued
            if self._bufs.get("cl_deferred") is not None:
                raise RuntimeError("composite_loss(defer=True): the previous deferred loss values on this "
                                   "lane were never finished (finish_losses)")
            self._bufs["cl_deferred"] = args
        return out, dz4

    def finish_losses(self):
        """The loss values of a deferred composite_loss on this lane (mli_composite_loss_finalize)."""
        args = self._bufs.pop("cl_deferred", None)
        if args is not None:
            L.call("mli_composite_loss_finalize", args)

    def drop_deferred(self):
        """Forget a deferred composite_loss whose step failed (its loss slot is not valid)."""
        self._bufs.pop("cl_deferred", None)

    @torch.no_grad()
    def light_visibility(self, rays, comp, iters=20):
        """get_light_visibility (NeuralLumen/model.py:133-184): adds visibility, normal_x_light,
        pseudo_shading, inter_dist, inter_mask ([R,1]) to the composite dict."""
        vis = self.cfg.light_visibility
        if vis.get("type", "sphere_tracing") != "sphere_tracing":
            raise NotImplementedError("light visibility type %r (only 'sphere_tracing', the configs' choice, "
                                      "is built)" % vis.get("type"))
        kind = {"blend_z_sphere_tracing": 0, "blend_z": 1, "sphere_tracing": 2}[vis["camera_ray_type"]]
        R = rays["center"].shape[0]
        f = lambda *shape: torch.empty(*shape, device=self.device)  # noqa: E731
        u8 = lambda n: torch.empty(n, 1, dtype=torch.uint8, device=self.device)  # noqa: E731
        o = dict(inter_dist=f(R, 1), inter_mask=u8(R), visibility=u8(R), normal_x_light=f(R, 1),
                 pseudo_shading=f(R, 1))
        scratch = dict(light_unit=f(R, 3), near_l=f(R), far_t=f(R), inside=u8(R), inter_pts=f(R, 3))
        box = vis.get("bounding", "sphere") == "box"
        r2 = float(np.float32(float(vis.get("radius", 1.0)) ** 2))
        L.call("mli_light_visibility", L.LightVisibilityArgs(
            R, L.ptr(rays["center"]), L.ptr(rays["ray_unit"]), L.ptr(rays["pts_light"]), L.ptr(rays["near"]),
            L.ptr(rays["far"]), L.ptr(comp["blend_dist"]), L.ptr(comp["gradient"]), kind, iters, 1 if box else 0,
            r2, (C.c_float * 6)(*self.cfg.aabb), float(vis.get("gamma") or 0.0), L.ptr(self.table16), self.levels,
            int(self.active_levels), L.ptr(self.wsdf), L.ptr(scratch["light_unit"]), L.ptr(scratch["near_l"]),
            L.ptr(scratch["far_t"]), L.ptr(scratch["inside"]), L.ptr(o["inter_dist"]), L.ptr(o["inter_mask"]),
            L.ptr(scratch["inter_pts"]), L.ptr(o["visibility"]), L.ptr(o["normal_x_light"]),
            L.ptr(o["pseudo_shading"])))
        o["visibility"] = o["visibility"].bool()
        o["inter_mask"] = o["inter_mask"].bool()
        comp.update(o)
        return comp

    def stamp(self):
        """Identifies the current lane's last render: the render state handed out aliases the
        lane's scratch buffers, so a later render on the same lane overwrites it."""
        return (id(self._bufs), self._bufs.get("__gen", 0))

    def check_stamp(self, stamp):
        for bufs in self._lanes.values():
            if id(bufs) == stamp[0]:
                if bufs.get("__gen", 0) != stamp[1]:
                    raise RuntimeError("render state overwritten: another render ran on the same engine lane "
                                       "between this forward and its backward")
                return
        raise RuntimeError("render state of an unknown engine lane")

    def render(self, data, s_var, progress, training, u=None, W=512, composite=True):
        """rays -> sampling -> FIELD -> heads -> composite; ``composite=False`` stops after the
        heads (comp None: the fused training tail, composite_loss, composites)."""
        self._bufs["__gen"] = self._bufs.get("__gen", 0) + 1
        rays = self.rays(data["pose"], data["intr"], data["pose_light"], data["ray_idx"], W)
        dists = self.sample(rays, u)
        fld = self.field(rays, dists, training)
        hd = self.heads(rays, dists, fld, training, s_var, progress)
        if not composite:
            return rays, dists, fld, hd, None
        comp = self.composite(rays, dists, fld, hd, s_var, progress, training)
        if self.cfg.light_visibility and not training:
            self.light_visibility(rays, comp)
        return rays, dists, fld, hd, comp

    # ------------------------------------------------------------------ backward
    @staticmethod
    def _dw_sizes():
        sizes = []
        for name, k_in, k_out in layout.HEADS:
            sizes += [(256, layout.K0), (256, 256), (256, 256), (256, 256), (k_out, 256)]
        return sizes

    def _dw_total(self):
        return sum(m * k + m for m, k in self._dw_sizes())

    def _wgrad_plan(self, dzT, dz4T, hd, dwbuf, flat, grad_out, S):
        """Split-K jobs (host array) + device assemble descriptors + (PQ mode) the mli_dw4
        output pointers of the layer-4 dW / db; cached per buffer set (a few: Trainer.prefetch
        alternates two engine lanes, each with its own buffers)."""
        pq = hd.get("q4") is not None
        key = (dzT.data_ptr(), None if dz4T is None else dz4T.data_ptr(), hd["x0T"].data_ptr(),
               hd["xT"].data_ptr(), dwbuf.data_ptr(), flat.data_ptr(), grad_out.data_ptr(), S, pq)
        hit = self._wplans.get(key)
        if hit is not None:
            return hit
        if len(self._wplans) >= 8:
            self._wplans.clear()
        sizes = self._dw_sizes()
        jobs, assemble, off = [], [], 0
        dw4, db4, k4 = [None] * 3, [None] * 3, [0] * 3
        for hdx, (name, k_in, k_out) in enumerate(layout.HEADS):
            for li in range(5):
                m, k = sizes[hdx * 5 + li]
                dw = dwbuf[off:off + m * k]
                db = dwbuf[off + m * k:off + m * k + m]
                off += m * k + m
                # every operand is a fragment image (ABI 15): 16 k-steps per 32-sample tile, the
                # x0 image 19, dZ4 1
                if li == 0:
                    jobs.append(L.frag_job(L.ptr(dzT[hdx, 0]), L.ptr(hd["x0T"]), m, k, L.ptr(dw), L.ptr(db), k, 16,
                                           layout.K0 // 16))
                elif li < 4:
                    jobs.append(L.frag_job(L.ptr(dzT[hdx, li]), L.ptr(hd["xT"][hdx, li - 1]), m, k, L.ptr(dw),
                                           L.ptr(db), k, 16, 16))
                elif pq:
                    dw4[hdx], db4[hdx], k4[hdx] = L.ptr(dw), L.ptr(db), m
                else:
                    jobs.append(L.frag_job(L.ptr(dz4T[hdx]), L.ptr(hd["xT"][hdx, 3]), m, k, L.ptr(dw), L.ptr(db), k,
                                           1, 16))
                pre = layout.param_prefix(name, li)
                v = self.param_view(flat, pre + ".weight_v")
                g = self.param_view(flat, pre + ".weight_g")
                k_ref = v.shape[1]
                kinv_t = self._kinv[(name, li)]
                assemble.append(L.AssembleLayer(L.ptr(dw), L.ptr(db), L.ptr(v), L.ptr(g), m, k_ref, k,
                                                L.ptr(kinv_t), L.ptr(self.param_view(grad_out, pre + ".weight_v")),
                                                L.ptr(self.param_view(grad_out, pre + ".weight_g")),
                                                L.ptr(self.param_view(grad_out, pre + ".bias")), None))
        job_arr = (L.WgradJob * len(jobs))(*jobs)
        # descriptors in dW-class order (one block row per layer, independent): the output layers
        # (mli_dw4 / THIN), the hidden layers (BIG), the layer-0 ones (WIDE), so that a class's
        # layers can be assembled -- and their gradient all-reduced -- as soon as its dW is done
        order = [h * 5 + li for cls in GRAD_CLASSES for li in GRAD_CLASS_LAYERS[cls] for h in range(len(layout.HEADS))]
        ad = _to_device_structs([assemble[i] for i in order], self.device)
        plan = (job_arr, ad, (dw4, db4, k4))
        self._wplans[key] = plan
        return plan

    def _wgrad(self, S, jobs, classes):
        """mli_wgrad over `classes` (separate launches, timed separately); deterministic mode:
        partial slabs in a workspace sized by mli_wgrad_workspace, else fp32 atomics into the
        zeroed outputs (the caller zeroes them)."""
        slab = 7 if self.deterministic else self.wgrad_slab_classes
        need = sum(classes) & slab
        ws = None
        if need:
            q = L.WgradArgs(S, len(jobs), C.cast(jobs, C.c_void_p), need, 1, None)
            nbytes = L.workspace("mli_wgrad", q)[0]
            ws = self._buf("wgrad_ws", (max(nbytes, 4) // 4,))
        for cls in classes:   # (a mask of several classes: its slab and atomic classes apart)
            for part, det in ((cls & ~slab, 0), (cls & slab, 1)):
                if part:
                    L.call("mli_wgrad", L.WgradArgs(S, len(jobs), C.cast(jobs, C.c_void_p), part, det, L.ptr(ws)))

    @torch.no_grad()
    def backward(self, st, d_rgb, d_o_r, d_o_s, d_o_re, flat, sdf_l1, grad_out, dz4=None, on_class=None):
        """Gradient of the loss w.r.t. the trainable head parameters into grad_out (flat), from
        d loss / d (rgb, o_r, o_s, o_re) -- or from ``dz4`` when composite_loss already ran the
        composite backward (the d_* are then unused; in PQ mode it also wrote the per-ray D).
        ``on_class(name)``: called (host side, in stream order) once the gradient of the layers
        of dW class ``name`` (GRAD_CLASSES) is complete in grad_out."""
        rays, dists, fld, hd, comp = st
        N, R = dists.shape
        S = N * R
        scale = self.grad_scale(R)
        pq = hd.get("q4") is not None
        if dz4 is None:
            dz4 = self._buf("dz4", (N, R, 8))
            c = lambda t: None if t is None else t.contiguous()  # noqa: E731
            L.call("mli_composite_bwd", L.CompositeBwdArgs(R, N, L.ptr(comp["weights"]), L.ptr(hd["y"]),
                                                           L.ptr(comp["o_r"]), L.ptr(comp["o_s"]), L.ptr(c(d_rgb)),
                                                           L.ptr(c(d_o_r)), L.ptr(c(d_o_s)), L.ptr(c(d_o_re)),
                                                           scale, L.ptr(dz4),
                                                           L.ptr(self._buf("dray", (R, 8)) if pq else None)))
        dz4T = None if pq else self._buf("dz4T", (3, S * 16), torch.float16)  # one-k-step frag images
        dwbuf = self._buf("dw", (self._dw_total(),))
        zero_dw = 0 if self.deterministic else 1
        if zero_dw:
            self._zero_once(dwbuf)   # split-K partials add into it (fp32 atomics)
            self._dw_zero = None     # (accumulating from here on, until the assemble zeroes it)
        dzT = self._buf("dzT", (3, 4, S * 256), torch.float16)  # ACC frag images
        L.call("mli_rgb_bwd", L.RgbBwdArgs(R, N, L.ptr(dz4), L.ptr(self.wbwd), L.ptr(hd["masks"]), L.ptr(dzT),
                                           L.ptr(dz4T)))
        jobs, ad, (dw4, db4, k4) = self._wgrad_plan(dzT, dz4T, hd, dwbuf, flat, grad_out, S)
        if self.gate_wgrad:  # Trainer.prefetch(gate="wgrad"): next geometry may start here
            self.gate_event = torch.cuda.Event()
            self.gate_event.record()
        if on_class is None:   # one assemble launch once every dW class is done
            if pq:
                self._dw4(R, N, hd, scale, dw4, db4, k4)
                self._wgrad(S, jobs, (1, 2))  # BIG, WIDE
            else:
                self._wgrad(S, jobs, (1, 2, 4))  # BIG, WIDE, THIN launch classes
            L.call("mli_grad_assemble", L.AssembleArgs(15, L.ptr(ad), 1.0 / scale, zero_dw))
            self._dw_zero = dwbuf.data_ptr() if zero_dw else None
            return grad_out
        # per class (the DDP bucket order of the overlapped all-reduce): dW, its layers'
        # assemble, then on_class(name) -- the caller issues that class's reduction while the
        # next class's dW runs
        nh, sz = len(layout.HEADS), C.sizeof(L.AssembleLayer)
        first = 0
        for cls in GRAD_CLASSES:
            if cls == "out":
                if pq:
                    self._dw4(R, N, hd, scale, dw4, db4, k4)
                else:
                    self._wgrad(S, jobs, (4,))
            else:
                self._wgrad(S, jobs, (1,) if cls == "big" else (2,))
            n = nh * len(GRAD_CLASS_LAYERS[cls])
            L.call("mli_grad_assemble", L.AssembleArgs(n, L.ptr(ad) + first * sz, 1.0 / scale, zero_dw))
            first += n
            on_class(cls)
        self._dw_zero = dwbuf.data_ptr() if zero_dw else None
        return grad_out

    def _zero_once(self, buf):
        """Zero a split-K dW accumulator unless the last mli_grad_assemble left it zero."""
        if self._dw_zero != buf.data_ptr():
            buf.zero_()
            self._dw_zero = buf.data_ptr()

    def _dw4(self, R, N, hd, scale, dw4, db4, k4):
        """PQ mode: the output layers' dW / db from the forward's q4 and the per-ray D."""
        args = L.Dw4Args(R, N, 3, L.ptr(hd["q4"]), L.ptr(self._bufs["dray"]), scale / L.Q4_SCALE,
                         (C.c_void_p * 3)(*dw4), (C.c_void_p * 3)(*db4), (C.c_int * 3)(*k4), None)
        args.workspace = L.ptr(self._buf("dw4_ws", (L.workspace("mli_dw4", args)[0] // 4,)))
        L.call("mli_dw4", args)


    # ------------------------------------------------------------------ stage a backward
    def _assemble_desc(self, dw, db, v, g, n_out, k_ref, k_pack, kinv, gv, gg, gb, plain=0):
        kinv_t = torch.from_numpy(np.asarray(kinv).astype(np.int16)).to(self.device)
        return L.AssembleLayer(L.ptr(dw), L.ptr(db), L.ptr(v), L.ptr(g), n_out, k_ref, k_pack, L.ptr(kinv_t),
                               L.ptr(gv), L.ptr(gg), L.ptr(gb), None, plain), kinv_t

    def _plan_a(self, bufs, flat, grad_flat, S):
        """wgrad jobs (two launches: S samples, 5S samples) + assemble descriptors, cached."""
        key = tuple(t.data_ptr() for t in bufs.values()) + (flat.data_ptr(), grad_flat.data_ptr(), S)
        if getattr(self, "_aplan", None) is not None and self._aplan[0] == key:
            return self._aplan[1:]
        head = layout.HEADS_A[0][0]
        sizes = [(256, layout.K0), (256, 256), (256, 256), (256, 256), (3, 256)]
        dw, off = bufs["dw"], 0
        jobs_s, jobs_5s, descs, keep = [], [], [], []

        def take(m, k):
            nonlocal off
            w, b = dw[off:off + m * k], dw[off + m * k:off + m * k + m]
            off += m * k + m
            return w, b
        pv = lambda n: self.param_view(flat, n)  # noqa: E731
        gv = lambda n: self.param_view(grad_flat, n)  # noqa: E731
        for li, (m, k) in enumerate(sizes):
            w, b = take(m, k)
            a_rows = bufs["dzT"][li] if li < 4 else bufs["dz4T"]
            b_rows = bufs["x0T"] if li == 0 else bufs["xT"][0, li - 1]
            # fragment images (ABI 15): dZ0..dZ3 / X 16 k-steps per tile, x0 19, dZ4 1
            jobs_s.append(L.frag_job(L.ptr(a_rows), L.ptr(b_rows), m, k, L.ptr(w), L.ptr(b), k, 16 if li < 4 else 1,
                                     layout.K0 // 16 if li == 0 else 16))
            pre = layout.param_prefix(head, li)
            k_ref = pv(pre + ".weight_v").shape[1]
            kinv = layout.head_kinv(head, k_ref) if li == 0 else np.arange(k_ref)
            d, kt = self._assemble_desc(w, b, pv(pre + ".weight_v"), pv(pre + ".weight_g"), m, k_ref, k, kinv,
                                        gv(pre + ".weight_v"), gv(pre + ".weight_g"), gv(pre + ".bias"))
            descs.append(d)
            keep.append(kt)
        # neural_sdf.mlp.linears.1: dZ1sdf x h0 (S samples)
        w, b = take(256, 256)
        # dZ1sdf and the FIELD's h0 image (ACC order, as the heads read it): both fragment images
        jobs_s.append(L.frag_job(L.ptr(bufs["dz1T"]), L.ptr(bufs["h0"]), 256, 256, L.ptr(w), L.ptr(b), 256, 16, 16))
        pre = "neural_sdf.mlp.linears.1"
        d, kt = self._assemble_desc(w, b, pv(pre + ".weight_v"), pv(pre + ".weight_g"), 256, 256, 256,
                                    np.arange(256), gv(pre + ".weight_v"), gv(pre + ".weight_g"), gv(pre + ".bias"))
        descs.append(d)
        keep.append(kt)
        # neural_sdf.mlp.linears.0: dZ0 x [enc, p] of the 5 points (5S samples, ABI 16): the dZ0
        # image of mli_sdf_bwd (ACC) against the FIELD's enc image (NAT, 8 k-steps per tile) with
        # p as a ninth k-step from the p image; packed column c < 128 is enc feature c
        # (reference column 3 + c), 128 + i is p_i (reference column i)
        w, b = take(256, layout.SDF_K0)
        jobs_5s.append(L.frag_job(L.ptr(bufs["dz0_frag"]), L.ptr(bufs["enc"]), 256, layout.SDF_K0, L.ptr(w), L.ptr(b),
                                  layout.SDF_K0, 16, 8, order=L.FRAG_ACC, b_order=L.FRAG_NAT,
                                  b2=L.ptr(bufs["p_frag"]), b2_q=8, b2_kst=1))
        pre = "neural_sdf.mlp.linears.0"
        kinv0 = np.concatenate([128 + np.arange(3), np.arange(128)])   # reference column -> packed column
        d, kt = self._assemble_desc(w, b, pv(pre + ".weight_v"), pv(pre + ".weight_g"), 256, layout.SDF_K0,
                                    layout.SDF_K0, kinv0, gv(pre + ".weight_v"),
                                    gv(pre + ".weight_g"), gv(pre + ".bias"))
        descs.append(d)
        keep.append(kt)
        # linear_sdf (plain Linear): in-kernel reductions of mli_sdf_bwd
        dws = bufs["dws"]
        d, kt = self._assemble_desc(dws[:256], dws[256:257], None, None, 1, 256, 256, np.arange(256),
                                    gv("neural_sdf.mlp.linear_sdf.weight"), None,
                                    gv("neural_sdf.mlp.linear_sdf.bias"), plain=1)
        descs.append(d)
        keep.append(kt)
        js = (L.WgradJob * len(jobs_s))(*jobs_s)
        j5 = (L.WgradJob * len(jobs_5s))(*jobs_5s)
        ad = _to_device_structs(descs, self.device)
        self._aplan = (key, js, j5, ad, len(descs), keep, off)
        return self._aplan[1:]

    def _table_grad_target(self, grad_table):
        """The buffer mli_hash_bwd accumulates into: the int64 fixed-point workspace in
        deterministic mode (mli_hash_bwd_workspace; 8 B per table element, 2.9 GB at 2^22, freed
        outside that mode), else the fp32 table gradient itself."""
        if self.deterministic:
            return self._buf("hash_ws", (grad_table.numel(),), torch.int64)
        self._bufs.pop("hash_ws", None)
        return grad_table

    @torch.no_grad()
    def backward_a(self, st, d_rgb, flat, grad_flat, grad_table, w_eikonal, w_curvature, progress,
                   d_grad_ext=None, d_hess_ext=None):
        """Stage-a gradient of the loss w.r.t. every parameter: the flat buffer (SDF MLP, head,
        s_var) into grad_flat and the hash table into grad_table (both fully overwritten).
        The eikonal / curvature terms are computed in-kernel from their weights (fused path)
        and/or arrive as d loss / d gradients, hessians ([N][R][3], autograd path)."""
        rays, dists, fld, hd, comp = st
        N, R = dists.shape
        S = N * R
        scale = self.grad_scale(R)   # (x8 / x64 measured: leg (a) of test_gpu_stage_a_decomp unchanged)
        f16 = torch.float16
        dz4, d_sdf, d_grad = self._buf("dz4", (N, R, 8)), self._buf("d_sdf", (N, R)), self._buf("d_grad", (N, R, 3))
        dinv = self._buf("d_inv_s_part", (R,))
        anneal = min(progress / self.cfg.anneal_end, 1.0)
        s_var = self.param_view(flat, "s_var")
        L.call("mli_composite_bwd_geo", L.CompositeBwdGeoArgs(
            R, N, L.ptr(dists), L.ptr(rays["far"]), L.ptr(rays["ray_unit"]), L.ptr(fld["sdf"]), L.ptr(fld["grad"]),
            L.ptr(hd["y"]), L.ptr(s_var), float(anneal), 1 if self.cfg.white_bg else 0, L.ptr(d_rgb.contiguous()),
            scale, L.ptr(dz4), L.ptr(d_sdf), L.ptr(d_grad), L.ptr(dinv), L.ptr(self.param_view(grad_flat, "s_var"))))
        b = dict(dzT=self._buf("dzT", (4, 256 * S), f16), dz4T=self._buf("dz4T", (16 * S,), f16),
                 x0T=hd["x0T"], xT=hd["xT"], dz1T=self._buf("dz1T", (256 * S,), f16),
                 h0=fld["h0"], enc=fld["enc"], dz0_frag=self._buf("dz0_frag", (5 * S * 256,), f16),
                 p_frag=self._buf("p_frag", (5 * S * 16,), f16), dws=self._buf("dws", (257,)))
        d_nrm = self._buf("d_nrm", (N, R, 4))
        dh0 = self._buf("dh0", (S * 256,), f16)
        L.call("mli_geo_bwd", L.GeoBwdArgs(R, N, L.ptr(dz4), L.ptr(self.wbwd), L.ptr(hd["masks"]), L.ptr(hd["feat"]),
                                           L.ptr(b["dzT"]), L.ptr(b["dz4T"]), L.ptr(d_nrm), L.ptr(b["dz1T"]),
                                           L.ptr(dh0)))
        d_enc = self._buf("d_enc", (S * 640,))
        part = self._buf("sdf_bwd_part", (L.workspace("mli_sdf_bwd", L.SdfBwdArgs(R, N))[3] // 4,))
        L.call("mli_sdf_bwd", L.SdfBwdArgs(
            R, N, L.ptr(rays["center"]), L.ptr(rays["ray_unit"]), L.ptr(dists), L.ptr(rays["outside"]),
            L.ptr(fld["grad"]), L.ptr(fld["hess"]), L.ptr(d_sdf), L.ptr(d_grad), L.ptr(d_nrm), L.ptr(dh0),
            L.ptr(fld["enc"]), L.ptr(self.wsdf), L.ptr(self.wsdf_t), self.eps, self.grad_den, self.hess_den,
            float(w_eikonal), float(w_curvature), scale, L.ptr(d_enc), L.ptr(b["dz0_frag"]), L.ptr(b["p_frag"]),
            L.ptr(b["dws"][:256]), L.ptr(b["dws"][256:]), L.ptr(d_grad_ext), L.ptr(d_hess_ext), L.ptr(part)))
        det = 1 if self.deterministic else 0
        # (zeroed here: on a side stream beside the forward it measured 0.5-1 % slower,
        # DESIGN.md §9.6)
        target = self._table_grad_target(grad_table)
        hws = target if det else None   # det: a fixed-point accumulator, zeroed; d_table is overwritten
        # the fp32 gradient is accumulated into: zeroed here, unless the last table AdamW consumed
        # this very buffer and left it zero (mli_adamw zero_grad, ABI 17: only the touched entries
        # are rewritten, not a 1.46 GB fill per step)
        if det or self.table_grad_clean != grad_table.data_ptr():
            target.zero_()
        self.table_grad_clean = None
        L.call("mli_hash_bwd", L.HashBwdArgs(R, N, L.ptr(rays["center"]), L.ptr(rays["ray_unit"]), L.ptr(dists),
                                             L.ptr(d_enc), self.levels, self.eps, int(self.active_levels),
                                             L.ptr(grad_table), det, L.ptr(hws), grad_table.numel()))
        dw_total = sum(m * k + m for m, k in [(256, layout.K0), (256, 256), (256, 256), (256, 256), (3, 256),
                                              (256, 256), (256, layout.SDF_K0)])
        b["dw"] = self._buf("dw_a", (dw_total,))
        js, j5, ad, n_desc, _, _ = self._plan_a(b, flat, grad_flat, S)
        zero_dw = 0 if self.deterministic else 1
        if zero_dw:   # left zero by the last assemble (ABI 17), else one fill
            self._zero_once(b["dw"])
            self._dw_zero = None
        self._wgrad(S, js, (7,))
        self._wgrad(5 * S, j5, (7,))
        L.call("mli_grad_assemble", L.AssembleArgs(n_desc, L.ptr(ad), 1.0 / scale, zero_dw))
        self._dw_zero = b["dw"].data_ptr() if zero_dw else None
        return grad_flat, grad_table
