"""Data formats and the ray-draw oracle (CPU).

* oracle/raybatch.py (the bit-exact restatement of mli_ray_batch): R distinct in-range
  pixels for every (n_pixels, R) shape incl. R = n_pixels, deterministic per seed.
* mli_nerf_amd.data.Dataset on synthetic files in both reference layouts:
  Blender (data_blender.py: camera_angle_x, pl_pos, RGBA + white background, Ref/Sha/Res)
  and ReNe / NeuralLumen data.py (fl_x..., transform_matrix_light, camera/light index,
  pseudo_label_all.pt).  Expected values are written out from the reference's formulas
  (cited per assertion); the reference Dataset itself needs torchvision, absent here.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from mli_nerf_amd import data as D
from mli_nerf_amd.config import to_attr
from oracle import raybatch as RB


# ----------------------------------------------------------------------------- ray draw
@pytest.mark.parametrize("n,R", [(1, 1), (7, 7), (64, 5), (1000, 1000), (800 * 800, 4096),
                                 (270 * 360, 512), ((1 << 20) + 3, 8192)])
def test_ray_indices_distinct_in_range(n, R):
    idx = RB.ray_indices(12345, n, R)
    assert idx.dtype == np.int64 and idx.shape == (R,)
    assert idx.min() >= 0 and idx.max() < n
    assert len(np.unique(idx)) == R
    assert np.array_equal(idx, RB.ray_indices(12345, n, R))


def test_ray_indices_full_permutation_and_seeds():
    n = 3001
    perm = RB.ray_indices(7, n, n)
    assert np.array_equal(np.sort(perm), np.arange(n))
    other = RB.ray_indices(8, n, n)
    assert not np.array_equal(perm, other)
    # prefix property: the R-draw is the prefix of the full permutation (like randperm[:R])
    assert np.array_equal(RB.ray_indices(7, n, 100), perm[:100])


def test_ray_indices_roughly_uniform():
    n, R, trials = 4096, 256, 64
    counts = np.zeros(n)
    for s in range(trials):
        counts[RB.ray_indices(s * 7919 + 1, n, R)] += 1
    # each pixel expected R*trials/n = 4 times; a uniform draw's max over 4096 pixels stays < 16
    assert counts.max() < 16 and abs(counts.mean() - R * trials / n) < 1e-9
    # spatial spread: all 16 row bands of a 64x64 image are hit in one draw
    bands = np.unique(RB.ray_indices(99, n, R) // (64 * 4))
    assert len(bands) == 16


def test_feistel_is_bijection():
    for bits in (1, 2, 5, 12, 17):
        x = np.arange(1 << bits, dtype=np.uint64)
        y = RB.feistel(x, bits, 0xDEADBEEFCAFEF00D)
        assert np.array_equal(np.sort(y), x)


# ----------------------------------------------------------------------------- files
def _write_png(path, arr):
    from PIL import Image
    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.fromarray(arr).save(path)


def _c2w(i):
    ang = 0.3 * i
    c, s = math.cos(ang), math.sin(ang)
    return [[c, 0.0, s, 2.0 * s], [0.0, 1.0, 0.0, 0.1 * i], [-s, 0.0, c, 2.0 * c], [0, 0, 0, 1]]


def _ref_w2c(c2w_gl, center=(0, 0, 0), scale=1.0):
    """neuralangelo/data.py:122-133 + camera.Pose.invert, written out in numpy."""
    m = np.array(c2w_gl, dtype=np.float32) * np.array([1, -1, -1, 1], dtype=np.float32)
    m[:3, 3] = (m[:3, 3] - np.array(center, dtype=np.float32)) / np.float32(scale)
    R, t = m[:3, :3], m[:3, 3:]
    return np.concatenate([R.T, -R.T @ t], 1)


def _cfg(root, blender, train_size=(12, 16), val_size=(6, 8), pseudo=None, white=True, readjust=None):
    d = {"root": str(root), "type": "projects.NeuralLumen.data_blender" if blender else "projects.NeuralLumen.data",
         "white_background": white, "preload": False,
         "train": {"image_size": list(train_size), "load_iid": blender, "subset": None},
         "val": {"image_size": list(val_size), "load_iid": False, "subset": 2}}
    if pseudo:
        d["train"]["pseudo_label"] = {"enabled": True, "pt_file": str(pseudo)}
    if readjust:
        d["readjust"] = readjust
    return to_attr({"data": d, "model": {"render": {"rand_rays": 40}}})


@pytest.fixture
def blender_dir(tmp_path):
    rng = np.random.default_rng(0)
    H, W = 24, 32
    frames = []
    for i in range(3):
        fp = f"./train/r_{i}_"
        rgba = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
        _write_png(str(tmp_path / f"train/r_{i}_Img.png"), rgba)
        for key in ("Ref", "Sha", "Res"):
            a = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
            a[..., 3] = 255
            _write_png(str(tmp_path / f"train/r_{i}_{key}.png"), a)
        frames.append({"file_path": fp, "transform_matrix": _c2w(i), "pl_pos": [0.5 * i, 1.0, -2.0]})
    meta = {"camera_angle_x": 0.69, "frames": frames, "sphere_center": [5.0, 5.0, 5.0], "sphere_radius": 3.0}
    for split in ("train", "val"):
        (tmp_path / f"{split}_transforms.json").write_text(json.dumps(meta))
    return tmp_path, H, W


def test_blender_dataset_train_sample(blender_dir):
    from PIL import Image
    root, H, W = blender_dir
    ds = D.Dataset(_cfg(root, True))
    assert len(ds) == 3 and (ds.raw_W, ds.raw_H) == (W, H)
    s = ds[1]
    # intrinsics: focal from camera_angle_x on the raw size, rescaled to 16x12 (data_blender.py:58-69,
    # neuralangelo/data.py:135-141)
    f = 0.5 * W / np.tan(0.5 * 0.69)
    ref_intr = np.array([[f * 16 / W, 0, W / 2 * 16 / W], [0, f * 12 / H, H / 2 * 12 / H], [0, 0, 1]], np.float32)
    assert np.allclose(s["intr"].numpy(), ref_intr, rtol=1e-6)
    # the JSON's sphere_center / sphere_radius are ignored (neuralangelo/data.py:39-42 hasattr quirk)
    assert np.allclose(s["pose"].numpy(), _ref_w2c(_c2w(1)), atol=1e-6)
    light = np.eye(4, dtype=np.float32)
    light[:3, 3] = [0.5, 1.0, -2.0]
    assert np.allclose(s["pose_light"].numpy(), _ref_w2c(light), atol=1e-6)
    # image: resized RGBA composited on white (data_blender.py:107-142)
    im = np.asarray(Image.open(root / "train/r_1_Img.png").resize((16, 12))).astype(np.float32) / 255
    rgb = im[..., :3] * im[..., 3:] + (1 - im[..., 3:])
    flat = rgb.reshape(-1, 3)
    ri = s["ray_idx"].numpy()
    assert ri.shape == (40,) and len(np.unique(ri)) == 40
    assert np.allclose(s["image_sampled"].numpy(), flat[ri], atol=1e-6)
    ref = np.asarray(Image.open(root / "train/r_1_Ref.png").resize((16, 12))).astype(np.float32)[..., :3] / 255
    ref = ref * im[..., 3:] + (1 - im[..., 3:])
    assert np.allclose(s["Ref_sampled"].numpy(), ref.reshape(-1, 3)[ri], atol=1e-6)


def test_blender_dataset_val_and_readjust(blender_dir):
    root, H, W = blender_dir
    ds = D.Dataset(_cfg(root, True, readjust={"center": [0.1, 0.2, 0.3], "scale": 2.0}), is_inference=True)
    assert len(ds) == 2  # subset 2 -> frames linspace(0, 3, 3)[:-1] = 0, 1
    s = ds[1]
    assert s["image"].shape == (3, 6, 8) and "ray_idx" not in s
    assert np.allclose(s["pose"].numpy(), _ref_w2c(_c2w(1), (0.1, 0.2, 0.3), 2.0), atol=1e-6)


@pytest.fixture
def rene_dir(tmp_path):
    rng = np.random.default_rng(1)
    H, W = 18, 24
    frames = []
    for cam in range(2):
        for light in range(2):
            name = f"c{cam:02d}l{light:02d}.png"
            _write_png(str(tmp_path / "img" / name), rng.integers(0, 256, (H, W, 3), dtype=np.uint8))
            frames.append({"file_path": f"img/{name}", "transform_matrix": _c2w(cam),
                           "transform_matrix_light": _c2w(3 + 2 * light), "camera_index": cam, "light_index": light})
    meta = {"fl_x": 20.0, "fl_y": 21.0, "cx": 12.0, "cy": 9.0, "sk_x": 0.0, "sk_y": 0.0, "frames": frames}
    for split in ("train", "val"):
        (tmp_path / f"{split}_transforms.json").write_text(json.dumps(meta))
    labels = {}
    for cam in range(2):
        labels[str(cam)] = {"pseudo_reflectance": torch.rand(3, 9, 12)}
        for light in range(2):
            labels[str(cam)][str(light)] = {"pseudo_shading_gamma": torch.rand(1, 9, 12),
                                            "visibility_certainty": torch.rand(1, 9, 12)}
    D.save_pseudo_labels(labels, str(tmp_path / "pseudo_label_all.pt"))
    return tmp_path, H, W, labels


def test_rene_dataset_pseudo_labels(rene_dir):
    root, H, W, labels = rene_dir
    ds = D.Dataset(_cfg(root, False, train_size=(9, 12), pseudo=root / "pseudo_label_all.pt"))
    assert ds.has_pseudo_label and len(ds) == 4
    s = ds[3]  # camera 1, light 1 (data.py:104-112 keys)
    ri = s["ray_idx"].numpy()
    assert np.allclose(s["intr"].numpy(), [[20 * 12 / 24, 0, 12 * 12 / 24], [0, 21 * 9 / 18, 9 * 9 / 18], [0, 0, 1]])
    assert np.allclose(s["pose_light"].numpy(), _ref_w2c(_c2w(5)), atol=1e-6)
    lab = labels["1"]
    assert torch.equal(s["pseudo_ref_sampled"], lab["pseudo_reflectance"].flatten(1, 2)[:, ri].t())
    assert torch.equal(s["pseudo_sha_sampled"], lab["1"]["pseudo_shading_gamma"].flatten(1, 2)[:, ri].t())
    assert torch.equal(s["pseudo_visibility_certainty_sampled"],
                       lab["1"]["visibility_certainty"].flatten(1, 2)[:, ri].t())
    assert ds.find_idx_cam_light("c01l00") == 2 and ds.find_idx_cam_light("c05l00") is None
    for i in range(4):  # a frame's own camera + light is its closest frame
        assert ds.find_closest_idx(ds.get_camera(i)[1], ds.get_light(i)) == i


def test_pseudo_label_file_loads_weights_only(rene_dir):
    root, _, _, labels = rene_dir
    got = D.load_pseudo_labels(str(root / "pseudo_label_all.pt"))
    assert set(got) == {"0", "1"} and torch.equal(got["0"]["1"]["visibility_certainty"],
                                                   labels["0"]["1"]["visibility_certainty"])


def test_device_feed_validates_shapes():
    with pytest.raises(ValueError):
        D.DeviceFeed(device="cpu", images=torch.zeros(2, 4, 10))
    with pytest.raises(ValueError):
        D.DeviceFeed(device="cpu", images=torch.zeros(2, 3, 10),
                     pseudo=(torch.zeros(2, 3, 10), torch.zeros(2, 9), torch.zeros(2, 10)))
    f = D.DeviceFeed(device="cpu", images=torch.zeros(2, 3, 10))
    with pytest.raises(ValueError):
        f.sample(0, 1, 11)
    with pytest.raises(IndexError):
        f.sample(2, 1, 4)


def test_rene_savannah_cameras_match_dataset(tmp_path):
    """The savannah bench / full-size test cameras (data.rene_savannah_cameras, from the committed
    frames of dataset_rene/savannah/train_transforms.json) equal what data.Dataset builds from the
    same JSON with images of the scene's raw size, at rene_savannah_b's 270 x 360."""
    import json as _json
    from PIL import Image
    from mli_nerf_amd import data as D
    from mli_nerf_amd.configs import preset
    meta = _json.load(open(D.RENE_SAVANNAH))
    assert meta["w"] == 1440 and meta["h"] == 1080 and len(meta["frames"]) == 16
    root = tmp_path / "savannah"
    for fr in meta["frames"][:3]:
        p = root / fr["file_path"]
        p.parent.mkdir(parents=True, exist_ok=True)
        Image.new("RGB", (meta["w"], meta["h"]), (255, 255, 255)).save(p)
    ann = tmp_path / "train_transforms.json"
    ann.write_text(_json.dumps(dict(meta, frames=meta["frames"][:3])))
    cfg = preset("rene_savannah_b")
    cfg.data["root"] = str(root)
    cfg.data.train["annotation"] = str(ann)
    ds = D.Dataset(cfg)
    cams = D.rene_savannah_cameras(270, 360, frames=[0, 1, 2])
    for i in range(3):
        intr, pose = ds.preprocess_camera(*ds.get_camera(i), (meta["w"], meta["h"]))
        assert torch.equal(intr, cams[i][0]) and torch.equal(pose, cams[i][1]) and torch.equal(ds.get_light(i), cams[i][2])
    # the AABB the fixture's scene declares is the preset's (rene_savannah_b.yaml:53-60)
    assert meta["bounding_box_aabb"] == list(cfg.data.bounding_box_aabb)
