"""Which engine buffers differ between two deterministic stage-b steps (GPU diagnostic)."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_determinism as T


def run(pq):
    tr = T._trainer("b", True)
    tr.model.pq = pq
    d, u = T._batch(512, 0)
    tr.train_step(d, u=u)
    torch.cuda.synchronize()
    bufs = {k: v.clone() for k, v in tr.model.engine._bufs.items() if torch.is_tensor(v)}
    bufs["__grad"] = tr.model.flat.grad.clone()
    return bufs


for pq in (False, True):
    a = run(pq)
    b = run(pq)
    for k in a:
        x, y = a[k], b.get(k)
        if y is None or x.shape != y.shape:
            continue
        if not torch.equal(x, y):
            xf, yf = x.float(), y.float()
            bad = (xf != yf) & ~(torch.isnan(xf) & torch.isnan(yf))
            print("pq", pq, k, tuple(x.shape), x.dtype, "n_diff", int(bad.sum()),
                  "first", bad.flatten().nonzero()[:4].flatten().tolist(), flush=True)
    print("pq", pq, "done", sorted(a), flush=True)
