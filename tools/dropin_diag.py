"""Diagnostic: fused Trainer.train_step vs autograd + torch AdamW, per-parameter gradient and
parameter differences (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import test_gpu_dropin as T

cfg, ma = T._model(deterministic=True)
tra = T.Trainer(cfg, is_inference=False, model=ma)
tra.current_iteration = 10000
cfg_b, mb = T._model(deterministic=True)
trb = T.Trainer(cfg_b, is_inference=False, model=mb)
opt = torch.optim.AdamW(mb.get_param_groups(cfg_b.optim), lr=1e-3, weight_decay=1e-2)
p0 = mb.flat.detach().clone()
for step in range(5):
    data, u = T._batch(step)
    tra.train_step(data, u=u)
    trb.current_iteration = 10000 + step
    trb._start_of_iteration()
    mb.train()
    out = mb(data, u=u)
    total, losses, _ = T._losses(trb, out, data)
    total.backward()
    ga = ma.flat.grad[:ma.flat.numel()].clone()
    gb = mb.flat_grad_from_params()
    print("step", step, "loss fused", float(tra.losses["total"]), "autograd", float(total))
    print("  grads: bitwise equal %s, rel %.3e, maxabs %.3e" % (bool(torch.equal(ga, gb)), float((ga - gb).norm() / gb.norm()), float((ga - gb).abs().max())))
    opt.step()
    opt.zero_grad(set_to_none=True)
    d = (ma.flat - mb.flat).abs()
    i = int(d.argmax())
    name = [n for n, s, off, k in ma._trainable_items() if off <= i < off + k][0]
    upd = (mb.flat - p0).norm()
    print("  param maxdiff %.3e at %d (%s) ga %.3e gb %.3e; |diff|/|update| %.3e; #elems > 1e-6: %d" % (float(d.max()), i, name, float(ga[i]), float(gb[i]), float(d.norm() / upd), int((d > 1e-6).sum())))
