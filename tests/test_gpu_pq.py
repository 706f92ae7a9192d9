"""Output-layer weight gradients from the heads forward's partials (PQ mode, ABI 12; GPU).

In stage b the composite weights do not depend on the heads, so the output layer's pre-sigmoid
gradient factors per ray: dz4[c, s] = D[r, c] * w_s * y_sc (1 - y_sc).  mli_rgb_fwd (PQ) forms
q4[tile, c, :] = sum_s w_s y_sc (1 - y_sc) X3[:, s] while X3 is in registers, and mli_dw4 contracts
it with the per-ray D written by the fused tail (or mli_composite_bwd): X3 never goes to HBM and
the THIN split-K GEMM is gone.  Checked here, deterministic mode (fixed-order sums in both paths):

* every parameter gradient except the output layers' is bit-identical between PQ and the THIN
  path (the forward activations, dz4 and the dX chain do not change);
* the output layers' dW / db of both paths agree with a float64 contraction of the THIN path's
  own operands (fp32 dz4, the fp16 X3 rows the forward wrote), PQ within 2e-3 relative;
* N not a multiple of 32 (a tile straddles two rays) falls back to the THIN path;
* the autograd path (Model.forward + backward through mli_composite_bwd's D) equals the fused one.
"""
import pytest
import torch

from mli_nerf_amd import layout, synthetic
from mli_nerf_amd.configs import preset
from mli_nerf_amd.model import Model
from mli_nerf_amd.trainer import Trainer

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _trainer(pq, R, Nc, Nf, log2T=16):
    cfg = preset("syn_hotdog_b", rays=R, n_coarse=Nc, n_fine=Nf, log2T=log2T)
    cfg.trainer["deterministic"] = True
    m = Model(cfg.model, cfg.data)
    m.load_state_dict(synthetic.make_state_dict(log2T=log2T))
    m.pq = pq
    tr = Trainer(cfg, is_inference=False, model=m.to(DEV))
    tr.current_iteration = 10000
    return tr


def _step(tr, R, Nc, seed=1):
    d = {k: v.to(DEV) for k, v in synthetic.make_batch(R, frame=seed).items()}
    u = synthetic.stratified_uniforms(R, Nc, seed=seed).to(DEV)
    tr.train_step(d, u=u)
    torch.cuda.synchronize()
    return tr.model.flat.grad.clone()


def _out_layer_slices(model):
    """flat-buffer slices of the three output layers (weight_v, weight_g, bias of linears.4)."""
    out = []
    for name, shape, off, n in model._trainable_items():
        if ".linears.4." in name:
            out.append((name, slice(off, off + n)))
    return out


@pytest.mark.parametrize("R,Nc,Nf", [(512, 32, 8), (512, 32, 16), (256, 64, 32)])
def test_pq_matches_thin_path(R, Nc, Nf):
    ta, tb = _trainer(True, R, Nc, Nf), _trainer(False, R, Nc, Nf)
    ga, gb = _step(ta, R, Nc), _step(tb, R, Nc)
    assert ta.model.engine._bufs.get("q4") is not None        # PQ ran
    outs = _out_layer_slices(ta.model)
    mask = torch.ones_like(ga, dtype=torch.bool)
    for _, sl in outs:
        mask[sl] = False
    assert torch.equal(ga[mask], gb[mask])                     # every other layer bit-identical
    for name, sl in outs:
        a, b = ga[sl], gb[sl]
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < 2e-3, (name, rel)


def test_pq_output_dw_against_float64():
    """dW4 / db4 (scaled, packed order; the mli_wgrad / mli_dw4 outputs before the weight-norm
    backward) of both paths against sum_s dz4[c, s] X3[f, s] in float64 from the THIN run's own
    operands: the X3 the PQ forward contracts in registers is the same fp16 activation."""
    R, Nc, Nf = 512, 32, 8
    ta, tb = _trainer(True, R, Nc, Nf), _trainer(False, R, Nc, Nf)
    _step(ta, R, Nc)
    _step(tb, R, Nc)
    ea, eb = ta.model.engine, tb.model.engine
    N = Nc + 4 * Nf
    S = R * N
    dz4 = eb._bufs["dz4"].view(N, R, 8).permute(1, 0, 2).reshape(S, 8).double()   # tile order m = r*N + k
    xT = eb._bufs["xT"].view(3, 4, 256 * S)  # ACC fragment images [S/32][16][64][8] per matrix
    sizes = eb._dw_sizes()
    offs, off = [], 0
    for m_, k_ in sizes:
        offs.append(off)
        off += m_ * k_ + m_
    for hdx, (_, _, k_out) in enumerate(layout.HEADS):
        o = offs[hdx * 5 + 4]
        x3 = layout.unfrag(xT[hdx, 3], 256).double()             # [256][S]
        z = dz4[:, 3 * hdx:3 * hdx + k_out]                      # [S][k_out] (scaled)
        ref_w = (z.t() @ x3.t())                                 # [k_out][256]
        ref_b = z.sum(0)
        for eng, tol in ((ea, 2e-3), (eb, 2e-3)):
            dw = eng._bufs["dw"][o:o + k_out * 256].view(k_out, 256).double()
            db = eng._bufs["dw"][o + k_out * 256:o + k_out * 256 + k_out].double()
            assert float((dw - ref_w).norm() / ref_w.norm()) < tol
            assert float((db - ref_b).norm() / ref_b.norm()) < tol


def test_pq_falls_back_when_tiles_straddle_rays():
    R, Nc, Nf = 512, 24, 4    # N = 40: a 32-sample tile holds parts of two rays
    ta = _trainer(True, R, Nc, Nf)
    g = _step(ta, R, Nc)
    assert ta.model.engine._bufs.get("q4") is None and torch.isfinite(g).all() and g.abs().sum() > 0
    gb = _step(_trainer(False, R, Nc, Nf), R, Nc)
    assert torch.equal(g, gb)


def test_pq_autograd_path_matches_fused():
    """Model.forward + loss.backward (mli_composite_bwd writes D) against the fused train step
    (mli_composite_loss writes D): the same flat gradient, both in PQ mode."""
    R, Nc, Nf = 512, 32, 8
    ta = _trainer(True, R, Nc, Nf)
    ga = _step(ta, R, Nc)
    tb = _trainer(True, R, Nc, Nf)
    d = {k: v.to(DEV) for k, v in synthetic.make_batch(R, frame=1).items()}
    u = synthetic.stratified_uniforms(R, Nc, seed=1).to(DEV)
    tb.train_step_autograd(d, u=u)
    torch.cuda.synchronize()
    assert tb.model.engine._bufs.get("q4") is not None
    gb = tb.model.flat.grad
    rel = float((ga - gb).norm() / gb.norm())
    assert rel < 1e-5, rel


class _ClassHook:
    """Stands in for trainer.OverlappedGradReduce on one rank: records the class order."""

    def __init__(self):
        self.calls = []

    def __call__(self, cls):
        self.calls.append(cls)

    def finish(self, off):
        self.calls.append("finish")


@pytest.mark.parametrize("pq", [True, False])
def test_per_class_backward_matches_single_assemble(pq):
    """VERDICT r5 item 7 (GPU leg): the backward issued per dW class -- each class's dW launch, then
    its layers' weight-norm assemble, then the caller's hook (where several ranks issue that
    class's all-reduce) -- writes the same flat gradient, bit for bit (deterministic mode), as the
    single assemble after every class; the hook sees the classes in launch order."""
    R, Nc, Nf = 512, 32, 8
    ta, tb = _trainer(pq, R, Nc, Nf), _trainer(pq, R, Nc, Nf)
    hook = _ClassHook()
    ta._grad_reducer = lambda model: hook
    ga, gb = _step(ta, R, Nc), _step(tb, R, Nc)
    assert hook.calls == ["out", "big", "wide", "finish"]
    assert torch.equal(ga, gb)
    assert float(ga.abs().sum()) > 0
