"""FIELD encoding image (``encode5_kernel``: center + 4 taps, level-outer, the taps' own gathers
run as compacted job rounds) against the oracle hash grid (``oracle/hashgrid.py``) evaluated
at the same 5 points of every sample, element by element.

The image holds fp16 values of fp32 trilinear sums: it must equal the oracle's fp32 encoding
rounded to fp16 up to one fp16 ulp (|e| <= 2^-10 |v| + 2^-24; the oracle sums the corners in
another order).  At the finest levels most taps leave the center's cell (the job path); the
coarse levels reuse the center's corners -- both are covered, and the stage-a case masks the
levels >= active_levels (coarse-to-fine) to zero.  The FIELD outputs built on this image (sdf,
normals, hessian, h0) are checked against the oracle in tests/test_gpu_parity.py."""
import pytest
import torch

from mli_nerf_amd import synthetic
from mli_nerf_amd.configs import preset
from oracle import hashgrid as o_hash

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("config,R,Nc,Nf,H,active", [("syn_hotdog_b", 512, 32, 16, 2, 16),
                                                      ("syn_hotdog_b", 100, 16, 5, 1, 16),   # ragged tile
                                                      ("syn_hotdog_a", 256, 32, 16, 2, 11)])
def test_encoding_image_matches_oracle(config, R, Nc, Nf, H, active):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from mli_nerf_amd.model import Model
    log2T = 19
    cfg = preset(config, rays=R, n_coarse=Nc, n_fine=Nf, n_hier=H, log2T=log2T)
    model = Model(cfg.model, cfg.data)
    sd = synthetic.make_state_dict(log2T=log2T, heads="rgb" if config.endswith("_a") else "rgb_r_s")
    model.load_state_dict(sd)
    model = model.to(DEV)
    model.train()
    model.prepare()
    eng = model.engine
    eng.active_levels = active
    data = {k: v.to(DEV) for k, v in synthetic.make_batch(R, H=cfg.data.train.image_size[0],
                                                          W=cfg.data.train.image_size[1], frame=3).items()}
    rays = eng.rays(data["pose"], data["intr"], data["pose_light"], data["ray_idx"], cfg.data.train.image_size[1])
    dists = eng.sample(rays)
    fld = eng.field(rays, dists, True)
    torch.cuda.synchronize()
    N = dists.shape[0]
    S = R * N
    tiles = (S + 31) // 32
    enc = fld["enc"][:tiles * 32 * 640].view(tiles, 5, 8, 2, 32, 8).float().cpu()  # tile, p, qq, h, c, f
    enc = enc.permute(0, 4, 1, 2, 3, 5).reshape(tiles * 32, 5, 128)[:S]            # sample m, p, level*8+f
    # the 5 points of sample m = r*N + k, as the kernels form them (fp32, no fma)
    m = torch.arange(S)
    r, k = m // N, m % N
    c, v = rays["center"].cpu()[r], rays["ray_unit"].cpu()[r]
    d = dists.cpu()[k, r]
    p = c + v * d[:, None]
    e = float(eng.eps)
    offs = torch.tensor([[0, 0, 0], [1, -1, -1], [-1, -1, 1], [-1, 1, -1], [1, 1, 1]], dtype=torch.float32) * e
    pts = p[:, None, :] + offs[None]
    pts[:, 0] = p
    x01 = (pts + 2.0) * 0.25
    table, _ = o_hash.level_table(log2T=log2T)
    params16 = model.neural_sdf.tcnn_encoding.params.detach().cpu().half().float()
    ref = o_hash.encode(x01.reshape(-1, 3), params16, table).reshape(S, 5, 128)
    ref[:, :, active * 8:] = 0.0
    err = (enc - ref).abs()
    tol = ref.abs() * 2.0 ** -10 + 2.0 ** -24
    bad = err > tol
    assert not bad.any(), (int(bad.sum()), float(err.max()))

