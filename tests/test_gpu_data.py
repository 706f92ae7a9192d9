"""GPU parity of the on-device training-ray draw (mli_ray_batch).

The drawn indices are integer work: bit-exact against oracle/raybatch.py (the kernel's Feistel
bijection + cycle walking restated in numpy), which in turn is checked for distinctness /
permutation-prefix / uniformity in tests/test_data.py.  The gathers are exact copies:
compared with the reference's ``image.flatten(1, 2)[:, ray_idx].t()``.
"""
import numpy as np
import pytest
import torch

from oracle import raybatch as RB

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("H,W,R,seed", [(1, 1, 1, 0), (8, 8, 64, 3), (12, 16, 40, 2 ** 63 + 11),
                                        (270, 360, 512, 77), (800, 800, 4096, 123456789)])
def test_ray_batch_matches_oracle(H, W, R, seed):
    _need_gpu()
    from mli_nerf_amd.data import DeviceFeed
    g = torch.Generator().manual_seed(H * W)
    F = 3
    images = torch.rand(F, 3, H * W, generator=g)
    pseudo = (torch.rand(F, 3, H * W, generator=g), torch.rand(F, H * W, generator=g),
              torch.rand(F, H * W, generator=g))
    feed = DeviceFeed(device=DEV, images=images, pseudo=pseudo)
    d = feed.batch(F - 1, seed, R)
    torch.cuda.synchronize()
    idx = d["ray_idx"][0].cpu().numpy()
    assert np.array_equal(idx, RB.ray_indices(seed, H * W, R))
    assert len(np.unique(idx)) == R
    ti = torch.from_numpy(idx)
    assert torch.equal(d["image_sampled"][0].cpu(), images[F - 1][:, ti].t())
    assert torch.equal(d["pseudo_ref_sampled"][0].cpu(), pseudo[0][F - 1][:, ti].t())
    assert torch.equal(d["pseudo_sha_sampled"][0, :, 0].cpu(), pseudo[1][F - 1][ti])
    assert torch.equal(d["pseudo_visibility_certainty_sampled"][0, :, 0].cpu(), pseudo[2][F - 1][ti])


def test_ray_batch_without_labels_and_errors():
    _need_gpu()
    from mli_nerf_amd import _lib as L
    from mli_nerf_amd.data import DeviceFeed
    feed = DeviceFeed(device=DEV, images=torch.rand(1, 3, 100))
    a, b = feed.sample(0, 5, 100)[0], feed.sample(0, 6, 100)[0]
    assert torch.equal(a.sort().values.cpu(), torch.arange(100))
    assert not torch.equal(a, b)
    ridx = torch.empty(8, dtype=torch.int64, device=DEV)
    with pytest.raises(RuntimeError):  # R > n_pixels
        L.call("mli_ray_batch", L.RayBatchArgs(seed=1, n_pixels=4, R=8, ray_idx=L.ptr(ridx)))
    with pytest.raises(RuntimeError):  # no output buffer
        L.call("mli_ray_batch", L.RayBatchArgs(seed=1, n_pixels=64, R=8))


def test_feed_drives_stage_b_training():
    """Trainer.train_step on DeviceFeed batches (no host sampling per step) moves the loss."""
    _need_gpu()
    from mli_nerf_amd import synthetic
    from mli_nerf_amd.configs import preset
    from mli_nerf_amd.data import DeviceFeed
    from mli_nerf_amd.model import Model
    from mli_nerf_amd.trainer import Trainer
    R = 256
    cfg = preset("syn_hotdog_b", rays=R, n_coarse=16, n_fine=4, log2T=14)
    model = Model(cfg.model, cfg.data)
    model.load_state_dict(synthetic.make_state_dict(log2T=14, s_var=3.0))
    model = model.to(DEV)
    trainer = Trainer(cfg, is_inference=False, model=model)
    H, W = cfg.data.train.image_size
    frames = [synthetic.make_batch(8, frame=f) for f in range(2)]
    g = torch.Generator().manual_seed(0)
    # a learnable target: a constant colour per frame + small noise
    images = torch.tensor([0.8, 0.5, 0.2])[None, :, None] + 0.05 * torch.rand(2, 3, H * W, generator=g)
    pseudo = (torch.rand(2, 3, H * W, generator=g), torch.rand(2, H * W, generator=g),
              torch.rand(2, H * W, generator=g))
    cams = [(f["intr"][0], f["pose"][0], f["pose_light"][0]) for f in frames]
    feed = DeviceFeed(device=DEV, images=images, pseudo=pseudo, cameras=cams)
    losses = []
    for it in range(20):
        batch = feed.batch(it % 2, 1000 + it, R)
        trainer.train_step(batch)
        trainer.current_iteration += 1
        losses.append(trainer.losses["total"].item())
    assert all(l == l for l in losses)
    assert sum(losses[-4:]) < sum(losses[:4]), losses
