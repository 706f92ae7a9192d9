"""Debug helper: run the GPU sampler with per-round tracing and dump the rounds."""
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))
import torch  # noqa: E402
from test_gpu_parity import build, to_dev, DEV  # noqa: E402
model, sd, data, pcfg, (Hh, W) = build()
model.train()
model.prepare()
eng = model.engine
d = to_dev(data)
rays = eng.rays(d["pose"], d["intr"], d["pose_light"], d["ray_idx"], W)
torch.manual_seed(0)
u = torch.rand(1, 64, 16)
eng.trace = []
dists = eng.sample(rays, u.to(DEV))
torch.cuda.synchronize()
out = {"u": u, "dists": dists.cpu(), "trace": [{k: (None if v is None else v.cpu()) for k, v in t.items()}
                                               for t in eng.trace]}
out.update({"r_" + k: v.cpu() for k, v in rays.items() if torch.is_tensor(v)})
torch.save(out, "gpurun_out/sampler_dump.pt")
print("dumped")
