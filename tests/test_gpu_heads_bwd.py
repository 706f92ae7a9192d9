"""The fused heads backward (mli_heads_bwd, GPU) against the split path it replaces and a
float64 reference.

mli_heads_bwd recomputes the dX chain of the three heads inside the workgroups that own the
256 x 256 weight gradients (layers 1..3), so dZ_1..dZ_3 never reach HBM.  Checked, on the
split path's own operands (mli_rgb_bwd's dZ rows, mli_rgb_fwd's X rows):

* dZ_0 rows and dz4 rows (the operands it hands to the layer-0 / layer-4 dW) are BIT-identical
  to mli_rgb_bwd's: same packed weights, same MFMA order, same masks and fp16 roundings;
* every fused dW_l / db_l equals the float64 product dZ_l^T X_l / sum_s dZ_l to 1e-5 of the
  matrix's largest element (fp32 accumulation over S samples), and the split path's to 1e-5;
* the whole parameter gradient equals the split path's (cosine >= 0.9999999);
* the k-slicing is irrelevant: custom splits, and more slices than 128-sample tiles (empty
  slices), give the same result; deterministic mode is bit-reproducible.
"""
import pytest
import torch

from test_gpu_parity import build, to_dev

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _backward(mode, R=512, Nc=32, Nf=8, det=False, split=(0, 0, 0), seed=5):
    model, sd, data, pcfg, hw = build(R=R, Nc=Nc, Nf=Nf, H=4)
    model.heads_bwd = mode
    model.heads_split = split
    model.deterministic = det
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(1, R, Nc, generator=g).to(DEV)
    model.train()
    out = model(to_dev(data), u=u)
    coef = {k: torch.randn(out[k].shape, generator=g).to(DEV) for k in ("rgb", "o_r", "o_s", "o_re")}
    loss = sum((out[k] * coef[k]).sum() for k in coef)
    loss.backward()
    torch.cuda.synchronize()
    b = model.engine._bufs   # flat scratch tensors (RenderEngine._buf views them)
    S = out["dists"].shape[1] * out["dists"].shape[2]

    def v(name, *shape):
        n = 1
        for d in shape:
            n *= d
        return b[name][:n].view(*shape).clone()
    keep = {"dw": v("dw", model.engine._dw_total()), "dz4T": v("dz4T", 3, 4, S),
            "grad": model.flat_grad_from_params().clone(), "S": S}
    if mode == "fused":
        keep["dz0"] = v("dz0T", 3, 256, S)
    else:
        keep["dzT"] = v("dzT", 3, 4, 256, S)
        keep["dz0"] = keep["dzT"][:, 0].clone()
        keep["xT"] = v("xT", 3, 4, 256, S)
    return model, keep


def _dw_views(model, dw):
    """(head, layer 1..3) -> (dW [256][256], db [256]) views of the engine's dW buffer."""
    sizes = model.engine._dw_sizes()
    out, off = {}, 0
    for i, (m, k) in enumerate(sizes):
        hd, li = divmod(i, 5)
        if 1 <= li <= 3:
            out[(hd, li)] = (dw[off:off + m * k].view(m, k), dw[off + m * k:off + m * k + m])
        off += m * k + m
    return out


def test_fused_matches_split_and_float64():
    model, fu = _backward("fused")
    _, sp = _backward("split")
    S = sp["S"]
    ok_dz0 = torch.equal(fu["dz0"], sp["dz0"])
    print("dz0 bit-identical:", ok_dz0)
    no = (3, 3, 1)
    for hd in range(3):
        a, b = fu["dz4T"][hd, :no[hd]], sp["dz4T"][hd, :no[hd]]
        bad = (a != b).nonzero()
        if bad.numel():
            print("dz4T head %d: %d mismatches, first %s: %s vs %s" % (
                hd, bad.shape[0], bad[:8].tolist(), a[tuple(bad[:8].T)].tolist(), b[tuple(bad[:8].T)].tolist()))
        assert bad.numel() == 0, hd
    vf, vs = _dw_views(model, fu["dw"]), _dw_views(model, sp["dw"])
    errs = []
    for (hd, li), (dw, db) in vf.items():
        a = sp["dzT"][hd, li].view(256, S).double()
        x = sp["xT"][hd, li - 1].view(256, S).double()
        ref_w, ref_b = a @ x.T, a.sum(1)
        scale_w, scale_b = ref_w.abs().max().item(), ref_b.abs().max().item()
        assert scale_w > 0 and scale_b > 0, (hd, li)
        ew = (dw.double() - ref_w).abs().max().item() / scale_w
        eb = (db.double() - ref_b).abs().max().item() / scale_b
        es = (dw - vs[(hd, li)][0]).abs().max().item() / scale_w
        print("head %d layer %d: dW err %.2e (split %.2e)  db err %.2e" % (hd, li, ew, es, eb))
        errs.append((hd, li, ew, eb, es))
    assert ok_dz0
    for hd, li, ew, eb, es in errs:
        assert ew < 1e-5 and eb < 1e-5 and es < 1e-5, (hd, li, ew, eb, es)
    cos = torch.nn.functional.cosine_similarity(fu["grad"], sp["grad"], dim=0).item()
    print("parameter gradient cosine fused vs split %.9f" % cos)
    assert cos > 0.9999999


@pytest.mark.parametrize("R,Nc,split", [(512, 32, (5, 3, 2)), (64, 16, (0, 0, 0)), (64, 16, (40, 17, 9))])
def test_k_slicing_is_irrelevant(R, Nc, split):
    """Custom workgroup splits; at 64 rays x 32 samples there are 16 tiles for 48 / 40
    slices of layer 1 (empty slices)."""
    model, fu = _backward("fused", R=R, Nc=Nc, Nf=Nc // 4, split=split)
    _, sp = _backward("split", R=R, Nc=Nc, Nf=Nc // 4)
    assert torch.equal(fu["dz0"], sp["dz0"])
    vf, vs = _dw_views(model, fu["dw"]), _dw_views(model, sp["dw"])
    for key, (dw, db) in vf.items():
        scale = vs[key][0].abs().max().item()
        assert (dw - vs[key][0]).abs().max().item() <= 1e-5 * scale, key
        assert (db - vs[key][1]).abs().max().item() <= 1e-5 * vs[key][1].abs().max().item(), key


def test_deterministic_fused_is_bit_reproducible():
    _, d1 = _backward("fused", det=True)
    _, d2 = _backward("fused", det=True)
    _, a1 = _backward("fused", det=False)
    assert torch.equal(d1["dw"], d2["dw"]) and torch.equal(d1["grad"], d2["grad"])
    cos = torch.nn.functional.cosine_similarity(d1["grad"], a1["grad"], dim=0).item()
    assert cos > 0.9999999, cos
