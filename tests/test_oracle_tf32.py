"""The oracle's TF32 GEMM mode (the reference's own arithmetic, imaginaire/trainers/base.py:172-178),
used by tests/test_gpu_stage_a_decomp.py leg (a) as the precision yardstick."""
import torch

from oracle import render as o_render


def test_tf32_round_nearest_even():
    one = 1.0
    x = torch.tensor([one + 2 ** -11, one + 3 * 2 ** -11, one + 2 ** -10, -one - 3 * 2 ** -11, 0.0, 65504.0 * 4])
    want = torch.tensor([one, one + 2 ** -9, one + 2 ** -10, -one - 2 ** -9, 0.0, 65504.0 * 4])
    assert torch.equal(o_render.tf32_round(x), want)


def test_tf32_linear_matches_rounded_operands():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 6, 40, generator=g, requires_grad=True)
    w = torch.randn(12, 40, generator=g, requires_grad=True)
    b = torch.randn(12, generator=g, requires_grad=True)
    o_render.MATMUL_OPERANDS = "tf32"
    try:
        y = o_render.linear(x, w, b)
        gy = torch.randn(y.shape, generator=g)
        y.backward(gy)
    finally:
        o_render.MATMUL_OPERANDS = None
    r = o_render.tf32_round
    xd, wd, gd = r(x).double().reshape(-1, 40), r(w).double(), r(gy).double().reshape(-1, 12)
    torch.testing.assert_close(y.double(), (xd @ wd.t() + b.double()).reshape(4, 6, 12), rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(x.grad.double(), (gd @ wd).reshape(4, 6, 40), rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(w.grad.double(), gd.t() @ xd, rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(b.grad.double(), gy.double().reshape(-1, 12).sum(0), rtol=1e-6, atol=1e-5)
    # fp32 mode is plain F.linear
    assert torch.equal(o_render.linear(x, w, b), torch.nn.functional.linear(x, w, b))
