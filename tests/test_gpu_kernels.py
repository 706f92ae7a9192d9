"""GPU unit tests of individual kernels against torch fp32 references (same op)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("S", [8192, 65536])
def test_wgrad_matches_torch(S):
    """dW = A B^T (fp32 accumulate), db = row sums of A, several jobs in one launch incl. thin."""
    _need_gpu()
    from mli_nerf_amd import _lib as L
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(256, 304), (256, 256), (3, 256), (1, 256), (256, 256), (3, 256)]
    jobs, refs = [], []
    keep = []
    for M, K in shapes:
        a = (torch.randn(M, S, generator=g) * 0.5).half().to(DEV)
        b = (torch.randn(K, S, generator=g) * 0.5).half().to(DEV)
        dw = torch.zeros(M, K, device=DEV)
        db = torch.zeros(M, device=DEV)
        keep += [a, b, dw, db]
        jobs.append(L.WgradJob(L.ptr(a), L.ptr(b), M, K, L.ptr(dw), L.ptr(db)))
        refs.append((a.float() @ b.float().t(), a.float().sum(1), dw, db))
    arr = (L.WgradJob * len(jobs))(*jobs)
    L.call("mli_wgrad", L.WgradArgs(S, len(jobs), C.cast(arr, C.c_void_p), 2048))
    torch.cuda.synchronize()
    for i, (rw, rb, dw, db) in enumerate(refs):
        err_w = ((dw - rw).abs().max() / rw.abs().max()).item()
        err_b = ((db - rb).abs().max() / rb.abs().max()).item()
        print("job %d %s: rel err dW %.2e db %.2e" % (i, tuple(rw.shape), err_w, err_b))
        assert err_w < 1e-4 and err_b < 1e-4, (i, err_w, err_b)
