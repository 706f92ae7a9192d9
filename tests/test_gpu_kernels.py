"""GPU unit tests of individual kernels against torch fp32 references (same op)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("S", [8192, 8384, 65536])
def test_wgrad_matches_torch(S):
    """dW = A B^T (fp32 accumulate), db = row sums of A: jobs of all three launch classes
    (BIG 256x256, WIDE 256x320, THIN 32x256), a ragged sample count (8384 = 131 x 64) and a
    job writing a column sub-range of a wider dW (ldw > K)."""
    _need_gpu()
    from mli_nerf_amd import _lib as L
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(256, 304), (256, 256), (3, 256), (1, 256), (256, 256), (3, 256), (256, 48)]
    jobs, refs = [], []
    keep = []
    for M, K in shapes:
        a = (torch.randn(M, S, generator=g) * 0.5).half().to(DEV)
        b = (torch.randn(K, S, generator=g) * 0.5).half().to(DEV)
        ldw = K + 40 if K == 48 else K
        full = torch.zeros(M, ldw, device=DEV)
        dw = full[:, 40:] if K == 48 else full
        db = torch.zeros(M, device=DEV)
        keep += [a, b, full, db]
        jobs.append(L.WgradJob(L.ptr(a), L.ptr(b), M, K, L.ptr(dw), L.ptr(db), ldw))
        refs.append((a.float() @ b.float().t(), a.float().sum(1), dw, db))
        if K == 48:
            refs.append((torch.zeros(M, 40, device=DEV), torch.zeros(1, device=DEV), full[:, :40], None))
    arr = (L.WgradJob * len(jobs))(*jobs)
    for cls in (1, 2, 4):
        L.call("mli_wgrad", L.WgradArgs(S, len(jobs), C.cast(arr, C.c_void_p), cls))
    torch.cuda.synchronize()
    for i, (rw, rb, dw, db) in enumerate(refs):
        if db is None:  # columns outside the job's range stay untouched
            assert torch.equal(dw, rw)
            continue
        err_w = ((dw - rw).abs().max() / rw.abs().max()).item()
        err_b = ((db - rb).abs().max() / rb.abs().max()).item()
        print("job %d %s: rel err dW %.2e db %.2e" % (i, tuple(rw.shape), err_w, err_b))
        assert err_w < 1e-4 and err_b < 1e-4, (i, err_w, err_b)


@pytest.mark.parametrize("S", [65536, 8384])
def test_wgrad_wide_jobs_sharing_b(S):
    """The layer-0 weight gradients of the three heads as the engine issues them: three WIDE
    jobs (M = 256, K = 304) streaming the SAME feature-major input x0T (ragged S too)."""
    _need_gpu()
    from mli_nerf_amd import _lib as L
    g = torch.Generator(device="cpu").manual_seed(5)
    b = (torch.randn(304, S, generator=g) * 0.5).half().to(DEV)
    jobs, refs, keep = [], [], [b]
    for _ in range(3):
        a = (torch.randn(256, S, generator=g) * 0.5).half().to(DEV)
        dw = torch.zeros(256, 304, device=DEV)
        db = torch.zeros(256, device=DEV)
        keep += [a, dw, db]
        jobs.append(L.WgradJob(L.ptr(a), L.ptr(b), 256, 304, L.ptr(dw), L.ptr(db), 304))
        refs.append((a.float() @ b.float().t(), a.float().sum(1), dw, db))
    arr = (L.WgradJob * 3)(*jobs)
    L.call("mli_wgrad", L.WgradArgs(S, 3, C.cast(arr, C.c_void_p), 2))
    torch.cuda.synchronize()
    for i, (rw, rb, dw, db) in enumerate(refs):
        err_w = ((dw - rw).abs().max() / rw.abs().max()).item()
        err_b = ((db - rb).abs().max() / rb.abs().max()).item()
        print("wide job %d: rel err dW %.2e db %.2e" % (i, err_w, err_b))
        assert err_w < 1e-4 and err_b < 1e-4


@pytest.mark.parametrize("S", [8448, 65536])
def test_wgrad_operand_layouts_bitwise(S):
    """Every operand layout mli_wgrad takes (include/mli_hip.h MLI_WGRAD_LAYOUT_*) gives the weight
    gradient of the feature-major rows call, bit for bit (deterministic mode: fixed-order slice
    sums), in every launch class: BIG (256 x 256), WIDE (three jobs sharing the 304-row B operand,
    its last 32-row tile half past the image's 19 k-steps) and THIN (M = 3, a one-k-step A image)
    -- the tile-blocked images of ABI 14 (the three combinations the engine used) and the fragment
    images of ABI 15, ACC and NAT order, with a tile stride above rows / 16, and (ABI 16) an ACC
    A against a NAT B split over two images at k-step 8 (the SDF layer-0 job: the FIELD's 8-k-step
    enc image + the p image; K = 131 is in the set).  The bias of the
    fragment kernel is summed from the MFMA A fragments (another fp32 order): within 2e-6 of the
    rows call, and both within 1e-4 of float64."""
    _need_gpu()
    from mli_nerf_amd import _lib as L
    from mli_nerf_amd import layout
    g = torch.Generator(device="cpu").manual_seed(11)
    shared = (torch.randn(304, S, generator=g) * 0.5).half()
    shapes = [(256, 256, None), (256, 304, shared), (256, 304, shared), (256, 304, shared), (3, 256, None),
              (256, 131, None)]
    ops = []
    for M, K, b in shapes:
        a = (torch.randn(M, S, generator=g) * 0.5).half()
        b = (torch.randn(K, S, generator=g) * 0.5).half() if b is None else b
        ops.append((a, b))

    def run(kind):
        keep, jobs, outs = [], [], []
        dev_b = {}   # one device image per distinct B (the WIDE jobs share one: SHARE_B)
        dev_b2 = {}
        for (a, b), (M, K, _) in zip(ops, shapes):
            dw = torch.zeros(M, K, device=DEV)
            db = torch.zeros(M, device=DEV)
            if kind == "rows":
                A, B, la, lb, ka, kb = a, b, 0, 0, 0, 0
            elif kind.startswith("tiled"):
                la, lb = {"tiled11": (1, 1), "tiled01": (0, 1), "tiled10": (1, 0)}[kind]
                A = layout.to_tiled(a) if la else a
                B = layout.to_tiled(b) if lb else b
                ka = kb = 0
            elif kind == "fragsplit":
                ka, kb, k2 = (M + 15) // 16, 8, (K - 128 + 15) // 16
                A, B = layout.to_frag(a, ka, "acc"), layout.to_frag(b[:128], kb, "nat")
                la, lb = L.FRAG_ACC, L.FRAG_NAT
            else:
                order = kind[5:]
                ka, kb = (M + 15) // 16 + 1, (K + 15) // 16 + 2   # tile strides above rows / 16
                A, B = layout.to_frag(a, ka, order), layout.to_frag(b, kb, order)
                la = lb = L.FRAG_ACC if order == "acc" else L.FRAG_NAT
            A = A.to(DEV)
            B = dev_b.setdefault(id(b), B.to(DEV))
            keep += [A, B, dw, db]
            if kind == "fragsplit":
                B2 = dev_b2.setdefault(id(b), layout.to_frag(b[128:], k2, "nat").to(DEV))
                keep.append(B2)
                jobs.append(L.WgradJob(L.ptr(A), L.ptr(B), M, K, L.ptr(dw), L.ptr(db), K, la, lb, ka, kb,
                                       L.ptr(B2), 8, k2))
            else:
                jobs.append(L.WgradJob(L.ptr(A), L.ptr(B), M, K, L.ptr(dw), L.ptr(db), K, la, lb, ka, kb))
            outs.append((dw, db))
        arr = (L.WgradJob * len(jobs))(*jobs)
        q = L.WgradArgs(S, len(jobs), C.cast(arr, C.c_void_p), 7, 1, None)
        ws = torch.empty(max(L.workspace("mli_wgrad", q)[0], 4) // 4, device=DEV)
        q.workspace = L.ptr(ws)
        for cls in (1, 2, 4):
            q.classes = cls
            L.call("mli_wgrad", q)
        torch.cuda.synchronize()
        return [(dw.cpu(), db.cpu()) for dw, db in outs]

    base = run("rows")
    for i, ((a, b), (dw, db)) in enumerate(zip(ops, base)):
        rw, rb = a.double() @ b.double().t(), a.double().sum(1)
        assert ((dw.double() - rw).abs().max() / rw.abs().max()).item() < 1e-4, i
        assert ((db.double() - rb).abs().max() / rb.abs().max()).item() < 1e-4, i
    for kind in ("tiled11", "tiled01", "tiled10", "fragacc", "fragnat", "fragsplit"):
        if kind.startswith("tiled") and S % 256:
            continue
        for i, ((dw, db), (bw, bb)) in enumerate(zip(run(kind), base)):
            assert torch.equal(dw, bw), (kind, i, (dw - bw).abs().max().item())
            if kind.startswith("tiled"):
                assert torch.equal(db, bb), (kind, i)
            else:
                assert ((db - bb).abs().max() / bb.abs().max()).item() < 2e-6, (kind, i)


def test_abi_rejects_bad_shapes_and_accepts_empty():
    """Error convention of the C ABI (include/mli_hip.h): shapes a kernel's grid cannot take
    are refused before any launch (non-zero hipError_t -> RuntimeError on the Python side,
    no CPU fallback), and an empty batch is a no-op that returns 0."""
    _need_gpu()
    from mli_nerf_amd import _lib as L
    from mli_nerf_amd.engine import _grid_levels, PathConfig
    # heads forward: R * N must be whole 256-sample workgroups; 1 or 3 heads
    with pytest.raises(RuntimeError, match="mli_rgb_fwd"):
        L.call("mli_rgb_fwd", L.RgbFwdArgs(3, 32, *([None] * 11), 3))
    with pytest.raises(RuntimeError, match="mli_rgb_fwd"):
        L.call("mli_rgb_fwd", L.RgbFwdArgs(8, 32, *([None] * 11), 2))
    # weight gradients: the sample count must be whole 64-sample k-steps
    with pytest.raises(RuntimeError, match="mli_wgrad"):
        L.call("mli_wgrad", L.WgradArgs(100, 0, None, 7))
    # SDF on an empty batch: nothing to launch, success
    levels, _ = _grid_levels(PathConfig(log2T=14))
    L.call("mli_sdf", L.SdfArgs(0, 0, 32, None, None, None, None, None, levels, None, 0.0, 1.0, 1.0,
                                1000.0, 0, None, None, None, None, None, 16))
    torch.cuda.synchronize()


@pytest.mark.parametrize("n,offset", [(1 << 20, 0), (1000003, 0), (4099, 1), (3, 0)])
def test_adamw_matches_torch(n, offset):
    """mli_adamw (one parameter per lane; sizes cover whole and ragged blocks and an unaligned
    view) against torch.optim.AdamW (the reference's optimizer,
    the configs' optim: AdamW lr 1e-3, wd 1e-2) over three steps, with the fp16
    shadow of the updated parameters.  fp32 elementwise: 3e-8 + 1e-6 |p|; shadow exact."""
    _need_gpu()
    from mli_nerf_amd.trainer import FusedAdamW
    g0 = torch.Generator().manual_seed(n)
    base = torch.randn(n + offset, generator=g0).to(DEV)
    p = base[offset:]  # offset 1: a view that is only 4 B aligned
    ref = p.detach().clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-2)
    fused = FusedAdamW(p, lr=1e-3, weight_decay=1e-2)
    p16 = torch.empty(n + offset, dtype=torch.float16, device=DEV)[offset:]
    for step in range(3):
        grad = torch.randn(n, generator=g0).to(DEV)
        ref.grad = grad.clone()
        opt.step()
        fused.step(grad, 1e-3, p16=p16)
    torch.cuda.synchronize()
    # the per-step update is lr * m / denom ~ 1e-3: a few fp32 ulps of it (sqrt / divide order
    # against torch's addcdiv) plus 1e-6 of |p|
    err = ((p - ref.detach()).abs() - 1e-6 * ref.detach().abs()).max().item()
    assert err < 3e-8, err
    assert torch.equal(p16, p.half())
    # moments: 1-2 fp32 ulps (fused multiply-add against torch's lerp / addcmul rounding)
    dm = (fused.m - opt.state[ref]["exp_avg"]).abs().max().item()
    v_ref = opt.state[ref]["exp_avg_sq"]
    dv = ((fused.v - v_ref).abs() / v_ref.clamp(min=1e-12)).max().item()
    assert dm < 2e-7 and dv < 2.5e-7, (dm, dv)
