"""Stage-a gradients of one seeded batch in deterministic mode (bit-identity A/B of experiment
libraries): python tools/r6/grad_a_dump.py out.pt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from mli_nerf_amd import synthetic  # noqa: E402
from mli_nerf_amd.configs import preset  # noqa: E402
from mli_nerf_amd.model import Model  # noqa: E402
from mli_nerf_amd.trainer import Trainer  # noqa: E402

DEV = "cuda:0"
cfg = preset("syn_hotdog_a", rays=512, n_coarse=32, n_fine=8, log2T=16)
cfg.trainer["deterministic"] = True
m = Model(cfg.model, cfg.data)
m.load_state_dict(synthetic.make_state_dict(log2T=16, heads="rgb"))
tr = Trainer(cfg, is_inference=False, model=m.to(DEV))
tr.current_iteration = 90000
d = {k: v.to(DEV) for k, v in synthetic.make_batch(512, frame=5).items()}
u = synthetic.stratified_uniforms(512, 32, seed=5).to(DEV)
tr.table_grad_consume = False
tr.compute_grads_a(d, u=u)
torch.cuda.synchronize()
torch.save({"flat": tr._grad[:m.flat.numel()].cpu(), "table": tr._grad_table.cpu()}, sys.argv[1])
