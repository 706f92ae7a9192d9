"""NeuralLumen data: the on-disk formats and the on-device training-ray feed.

The reference's Dataset (``projects/NeuralLumen/data.py:12-140``, ``data_blender.py:12-206``,
on top of ``projects/neuralangelo/data.py:25-146``) reads ``{split}_transforms.json`` plus
one PNG per frame and, for training, pre-samples ``rand_rays`` pixel indices with
``torch.randperm(H*W)[:R]`` on the host, gathering the image (and the pseudo labels of
``scripts/pseudo_label.py``) at those indices.

Here the file formats are read the same way (``Dataset``: cameras, lights, images, the
``pseudo_label_all.pt`` nested dict), but the per-step sampling lives on the GPU:
``DeviceFeed`` keeps every frame's image and pseudo labels resident in HBM and draws R
distinct pixels with ``mli_ray_batch`` (a seeded Feistel bijection of the pixel range with
cycle walking: R distinct indices, a scrambled prefix of a permutation like randperm's) and
gathers image / pseudo-reflectance / pseudo-shading / certainty in the same launch.  No host
round trip per step.
"""
import json
import os
import re

import numpy as np
import torch

from . import _lib as L


# --------------------------------------------------------------------------- poses
def gl_to_cv(gl):
    """neuralangelo/data.py:143-146: flip the y and z camera axes."""
    return gl * torch.tensor([1.0, -1.0, -1.0, 1.0], dtype=gl.dtype)


def invert_pose(pose):
    """nerf/utils/camera.py Pose.invert: [R|t] -> [R^T | -R^T t]."""
    R, t = pose[..., :3, :3], pose[..., :3, 3:]
    Rt = R.transpose(-1, -2)
    return torch.cat([Rt, -Rt @ t], dim=-1)


def _center_scale(readjust):
    """neuralangelo/data.py:37-42 + :124-131.

    ``hasattr(dict, key)`` is always False, so the reference ALWAYS resets
    ``sphere_center`` to 0 and ``sphere_radius`` to 1, whatever the JSON holds; only
    ``cfg.data.readjust`` moves the scene.  Kept as is: a user switching frameworks gets
    the same cameras."""
    center = np.zeros(3)
    scale = 1.0
    if readjust:
        center = center + np.array(readjust.get("center", [0]))
        scale = scale * readjust.get("scale", 1.0)
    return center, scale


def world_to_camera(c2w_gl, readjust=None):
    c2w = gl_to_cv(torch.as_tensor(c2w_gl, dtype=torch.float32).clone())
    center, scale = _center_scale(readjust)
    c2w[:3, -1] -= torch.as_tensor(center, dtype=torch.float32)
    c2w[:3, -1] /= float(scale)
    return invert_pose(c2w[:3])


def transforms_cameras(meta, H, W, readjust=None, frames=None):
    """[(intr [3,3], pose [3,4], pose_light [3,4])] of a ReNe-style transforms dict at image size
    H x W, as Dataset.get_camera + preprocess_camera + get_light give them (neuralangelo
    data.py:116-141, NeuralLumen/data.py:30-43): intrinsics from fl_x / sk_x / cx / sk_y / fl_y / cy
    rescaled from the raw ``w`` x ``h`` (the size of the scene's images), GL->CV world-to-camera poses
    of ``transform_matrix`` / ``transform_matrix_light``."""
    intr0 = torch.tensor([[meta["fl_x"], meta["sk_x"], meta["cx"]], [meta["sk_y"], meta["fl_y"], meta["cy"]],
                          [0, 0, 1]]).float()
    intr0[0] *= W / meta["w"]
    intr0[1] *= H / meta["h"]
    out = []
    for fr in (meta["frames"] if frames is None else [meta["frames"][i] for i in frames]):
        out.append((intr0.clone(), world_to_camera(fr["transform_matrix"], readjust),
                    world_to_camera(fr["transform_matrix_light"], readjust)))
    return out


# the real cameras of BASELINE.json configs[3] (rene_savannah_b): the reference's first 16
# savannah training frames, package data (tools/make_rene_savannah.py extracts them)
RENE_SAVANNAH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "rene_savannah_train16.json")


def rene_savannah_cameras(H=270, W=360, frames=None):
    with open(RENE_SAVANNAH) as f:
        meta = json.load(f)
    return transforms_cameras(meta, H, W, frames=frames)


# --------------------------------------------------------------------------- images
def to_tensor(img):
    """torchvision to_tensor on a PIL image: [C,H,W] float in [0,1] (8-bit) or as stored."""
    a = np.asarray(img)
    if a.ndim == 2:
        a = a[:, :, None]
    t = torch.from_numpy(a.copy()).permute(2, 0, 1)
    return t.float() / 255.0 if a.dtype == np.uint8 else t.float()


def _resize(img, W, H):
    return img.resize((W, H))


def _cfg_get(c, key, default=None):
    if c is None:
        return default
    if isinstance(c, dict):
        return c.get(key, default)
    return getattr(c, key, default)


class Dataset:
    """NeuralLumen Dataset: data.py:12-140 (ReNe-style JSON with ``transform_matrix_light``,
    ``camera_index`` / ``light_index``) and data_blender.py:12-206 (synthetic Blender sets with
    ``pl_pos`` and the optional Ref/Sha/Res intrinsic images).

    ``__getitem__`` returns the reference's dict.  In training it also pre-samples rays on
    the host exactly as the reference does (``torch.randperm``), for callers that want the
    reference's sampler; the GPU trainer uses ``DeviceFeed`` instead."""

    def __init__(self, cfg, is_inference=False, is_test=False):
        cfg_data = cfg.data
        self.split = "test" if is_test else ("val" if is_inference else "train")
        split_cfg = cfg_data[self.split]
        self.root = cfg_data.root
        self.H, self.W = (cfg_data.val.image_size if is_inference else cfg_data.train.image_size)
        self.blender = "blender" in str(_cfg_get(cfg_data, "type", "")).lower()
        self.data_source = _cfg_get(cfg_data, "data_source")
        self.white_background = bool(_cfg_get(cfg_data, "white_background", False))
        ann = _cfg_get(split_cfg, "annotation")
        meta_fname = ann if ann else f"{self.root}/{self.split}_transforms.json"
        with open(meta_fname) as f:
            self.meta = json.load(f)
        use_light = _cfg_get(split_cfg, "use_light_index")
        if use_light is not None:
            self.meta["frames"] = [x for x in self.meta["frames"] if x["light_index"] in use_light]
        self.list = self.meta["frames"]
        _, (self.raw_W, self.raw_H) = self.get_image(0)
        subset = _cfg_get(split_cfg, "subset")
        if subset:
            keep = np.linspace(0, len(self.list), subset + 1)[:-1].astype(int)
            self.list = [self.list[i] for i in keep]
        self.num_rays = cfg.model.render.rand_rays
        ra = _cfg_get(cfg_data, "readjust")
        self.readjust = dict(ra) if ra else None
        self.load_iid = self.blender and bool(_cfg_get(split_cfg, "load_iid", False))
        pl = _cfg_get(split_cfg, "pseudo_label")
        self.has_pseudo_label = self.split == "train" and bool(_cfg_get(pl, "enabled", False))
        self.pseudo_label = load_pseudo_labels(_cfg_get(pl, "pt_file")) if self.has_pseudo_label else None
        self.sample_train_rays = self.split == "train"
        self._centers = None

    def __len__(self):
        return len(self.list)

    # --- files
    def image_path(self, idx, suffix=None):
        fr = self.list[idx]
        if suffix is not None:  # data_blender.py:97-105
            return os.path.normpath(os.path.join(self.root, fr["file_path"] + suffix + ".png"))
        if self.blender:  # data_blender.py:86-95
            if self.data_source == "NRHints":
                return os.path.normpath(os.path.join(self.root, fr["file_path"] + fr["file_ext"]))
            return os.path.normpath(os.path.join(self.root, fr["file_path"] + "Img.png"))
        return f"{self.root}/{fr['file_path']}"  # neuralangelo/data.py:101-107

    def get_image(self, idx):
        from PIL import Image
        im = Image.open(self.image_path(idx))
        im.load()
        return im, im.size

    def get_iid(self, idx):
        from PIL import Image
        out = {}
        for key in ("Ref", "Sha", "Res"):
            im = Image.open(self.image_path(idx, key))
            im.load()
            out[key] = im
        return out

    def get_camera(self, idx):
        """data_blender.py:49-84 (camera_intrinsics, else camera_angle_x) / neuralangelo
        data.py:116-133 (fl_x, sk_x, cx, ...)."""
        m = self.meta
        if not self.blender:
            intr = torch.tensor([[m["fl_x"], m["sk_x"], m["cx"]], [m["sk_y"], m["fl_y"], m["cy"]],
                                 [0, 0, 1]]).float()
        elif "camera_intrinsics" in m:
            cx, cy, fx, fy = m["camera_intrinsics"][:4]
            intr = torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0, 0, 1]]).float()
        else:
            focal = float(0.5 * self.raw_W / np.tan(0.5 * float(m["camera_angle_x"])))
            intr = torch.tensor([[focal, 0.0, self.raw_W / 2.0], [0.0, focal, self.raw_H / 2.0],
                                 [0, 0, 1]]).float()
        return intr, world_to_camera(self.list[idx]["transform_matrix"], self.readjust)

    def get_light(self, idx):
        """data.py:30-43 (transform_matrix_light) / data_blender.py:28-47 (pl_pos, identity R)."""
        fr = self.list[idx]
        if not self.blender:
            c2w = fr["transform_matrix_light"]
        else:
            c2w = torch.eye(4)
            c2w[:3, 3] = torch.tensor(fr["pl_pos"], dtype=torch.float32)
        return world_to_camera(c2w, self.readjust)

    def preprocess_camera(self, intr, pose, size_raw):
        """neuralangelo/data.py:135-141: rescale the intrinsics to the resized image."""
        intr = intr.clone()
        intr[0] *= self.W / size_raw[0]
        intr[1] *= self.H / size_raw[1]
        return intr, pose

    def preprocess_image(self, image, iid=None):
        """data_blender.py:107-142 / neuralangelo/data.py:109-114: resize, then RGB (white
        background composited on alpha for Blender sets with white_background)."""
        t = to_tensor(_resize(image, self.W, self.H))
        iid_t = None
        if iid is not None:
            iid_t = {k: to_tensor(_resize(v, self.W, self.H))[:3] for k, v in iid.items()}
        if self.blender and self.white_background:
            a = t[3:]
            if iid_t is not None:
                iid_t = {k: v * a + (1.0 - a) for k, v in iid_t.items()}
            t = t[:3] * a + (1.0 - a)
        else:
            t = t[:3]
        return t, iid_t

    def pseudo_elements(self, idx):
        """data.py:104-112 (camera/light index keys) / data_blender.py:165-171 (frame index,
        light '0')."""
        fr = self.list[idx]
        if self.blender:
            cam, light = str(idx), "0"
        else:
            cam, light = str(fr["camera_index"]), str(fr["light_index"])
        e = self.pseudo_label
        return dict(pseudo_ref=e[cam]["pseudo_reflectance"], pseudo_sha=e[cam][light]["pseudo_shading_gamma"],
                    pseudo_visibility_certainty=e[cam][light]["visibility_certainty"])

    def __getitem__(self, idx):
        sample = dict(idx=idx)
        image, size_raw = self.get_image(idx)
        image, iid = self.preprocess_image(image, self.get_iid(idx) if self.load_iid else None)
        intr, pose = self.preprocess_camera(*self.get_camera(idx), size_raw)
        pose_light = self.get_light(idx)
        sample.update(intr=intr, pose=pose, pose_light=pose_light)
        if self.sample_train_rays:
            ray_idx = torch.randperm(self.H * self.W)[:self.num_rays]
            sample.update(ray_idx=ray_idx, image_sampled=image.flatten(1, 2)[:, ray_idx].t())
            if iid is not None:
                for k, v in iid.items():
                    sample[k + "_sampled"] = v.flatten(1, 2)[:, ray_idx].t()
            if self.has_pseudo_label:
                for k, v in self.pseudo_elements(idx).items():
                    sample[k + "_sampled"] = chw(v).flatten(1, 2)[:, ray_idx].t()
        else:
            sample["image"] = image
            if iid is not None:
                sample.update(iid)
        return sample

    # --- frame lookup for the video writer
    def find_idx_cam_light(self, s="c00l00"):
        """data.py:76-85: frame index of camera/light index pair 'cXXlYY'."""
        digits = re.findall(r"\d+", s)
        cam = int(digits[0]) if digits else None
        light = int(digits[-1]) if digits else None
        for i, fr in enumerate(self.list):
            if fr.get("camera_index") == cam and fr.get("light_index") == light:
                return i
        return None

    def find_closest_idx(self, pose_cam, pose_light):
        """data.py:45-74: argmin over frames of |camera center - c| + (1 - cos(view dir)) +
        |light center - l| (all in world space)."""
        if self._centers is None:
            cams = torch.stack([self.get_camera(i)[1] for i in range(len(self))])
            lights = torch.stack([self.get_light(i) for i in range(len(self))])
            self._centers = (_center(cams), _axis(cams), _center(lights))
        cc, cr, lc = self._centers
        pose_cam, pose_light = pose_cam.reshape(-1, 3, 4)[:1], pose_light.reshape(-1, 3, 4)[:1]
        d = (_center(pose_cam) - cc).abs().norm(dim=-1)
        d = d + (1.0 - torch.nn.functional.cosine_similarity(_axis(pose_cam), cr, dim=-1))
        d = d + (_center(pose_light) - lc).abs().norm(dim=-1)
        return int(torch.argmin(d))


def _center(w2c):
    """cam2world of the camera-space origin: -R^T t."""
    return invert_pose(w2c)[..., :3, 3]


def _axis(w2c):
    """cam2world([0,0,1]) - cam2world(0): the optical axis R^T e_z."""
    return w2c[..., 2, :3]


def chw(t):
    t = torch.as_tensor(t).float()
    return t if t.dim() == 3 else t.reshape(-1, *t.shape[-2:])


# --------------------------------------------------------------------------- pseudo labels
def load_pseudo_labels(path):
    """data.py:21: the ``pseudo_label_all.pt`` written by scripts/pseudo_label.py:418
    ({cam: {'pseudo_reflectance': [3,H,W], light: {'pseudo_shading_gamma': [1,H,W],
    'visibility_certainty': [1,H,W]}}}).  Tensors and string keys only: loaded with
    weights_only=True (nothing in the file is executed)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def save_pseudo_labels(labels, path):
    """The same nested-dict layout, written with torch.save."""
    clean = {}
    for cam, d in labels.items():
        clean[str(cam)] = {}
        for k, v in d.items():
            if isinstance(v, dict):
                clean[str(cam)][str(k)] = {kk: torch.as_tensor(vv).float().cpu() for kk, vv in v.items()}
            else:
                clean[str(cam)][str(k)] = torch.as_tensor(v).float().cpu()
    torch.save(clean, path)


# --------------------------------------------------------------------------- on-device feed
class DeviceFeed:
    """All training frames resident in HBM; one ``mli_ray_batch`` launch per step draws R
    distinct pixels of a frame and gathers its supervision at them.

    Layout: ``images`` [F,3,H·W] fp32 (channel-planar, as ``image.flatten(1,2)``), optional
    pseudo labels ``ref`` [F,3,H·W], ``sha`` / ``cert`` [F,H·W].  ``batch(idx, seed, R)``
    returns the reference's training dict (``ray_idx`` [1,R] int64, ``image_sampled``
    [1,R,3], ``pseudo_*_sampled``, cameras)."""

    def __init__(self, dataset=None, device="cuda", images=None, pseudo=None, cameras=None):
        self.device = torch.device(device)
        if dataset is not None:
            imgs, refs, shas, certs, cams = [], [], [], [], []
            for i in range(len(dataset)):
                im, size_raw = dataset.get_image(i)
                t, _ = dataset.preprocess_image(im)
                imgs.append(t.flatten(1, 2))
                intr, pose = dataset.preprocess_camera(*dataset.get_camera(i), size_raw)
                cams.append((intr, pose, dataset.get_light(i)))
                if dataset.has_pseudo_label:
                    e = dataset.pseudo_elements(i)
                    refs.append(chw(e["pseudo_ref"]).flatten(1, 2))
                    shas.append(chw(e["pseudo_sha"])[0].flatten())
                    certs.append(chw(e["pseudo_visibility_certainty"])[0].flatten())
            images = torch.stack(imgs)
            pseudo = (torch.stack(refs), torch.stack(shas), torch.stack(certs)) if refs else None
            cameras = cams
        self.images = images.to(self.device, torch.float32).contiguous()
        if self.images.dim() != 3 or self.images.shape[1] != 3:
            raise ValueError("images must be [F,3,H*W]")
        self.n_pixels = self.images.shape[-1]
        self.ref = self.sha = self.cert = None
        if pseudo is not None:
            self.ref, self.sha, self.cert = (p.to(self.device, torch.float32).contiguous() for p in pseudo)
            if (self.ref.shape != self.images.shape or self.sha.shape != self.images.shape[::2]
                    or self.cert.shape != self.sha.shape):
                raise ValueError("pseudo labels must be [F,3,H*W], [F,H*W], [F,H*W]")
        # cameras resident on the device too: a step makes no host -> device copy
        self.cameras = None if cameras is None else [
            tuple(torch.as_tensor(c).float().to(self.device)[None] for c in cam) for cam in cameras]

    def __len__(self):
        return self.images.shape[0]

    def sample(self, idx, seed, R, stream=None):
        """ray_idx [R] int64 + the gathered [R,3] / [R] device tensors, one launch."""
        if not 0 <= idx < len(self):
            raise IndexError(idx)
        if not 0 < R <= self.n_pixels:
            raise ValueError(f"R={R} outside (0, {self.n_pixels}]")
        dev = self.device
        ray_idx = torch.empty(R, dtype=torch.int64, device=dev)
        img_s = torch.empty(R, 3, device=dev)
        have = self.ref is not None
        ref_s = torch.empty(R, 3, device=dev) if have else None
        sha_s = torch.empty(R, device=dev) if have else None
        cert_s = torch.empty(R, device=dev) if have else None
        a = L.RayBatchArgs(seed=int(seed) & (2 ** 64 - 1), n_pixels=self.n_pixels, R=R,
                           image=L.ptr(self.images[idx]), ref=L.ptr(self.ref[idx]) if have else None,
                           sha=L.ptr(self.sha[idx]) if have else None, cert=L.ptr(self.cert[idx]) if have else None,
                           ray_idx=L.ptr(ray_idx), image_sampled=L.ptr(img_s), ref_sampled=L.ptr(ref_s),
                           sha_sampled=L.ptr(sha_s), cert_sampled=L.ptr(cert_s))
        L.call("mli_ray_batch", a, stream)
        return ray_idx, img_s, ref_s, sha_s, cert_s

    def batch(self, idx, seed, R, stream=None):
        """The reference's training sample for frame ``idx`` (data.py:120-132), batched [1,...]."""
        ray_idx, img_s, ref_s, sha_s, cert_s = self.sample(idx, seed, R, stream)
        d = dict(idx=torch.tensor([idx]), ray_idx=ray_idx[None], image_sampled=img_s[None])
        if self.cameras is not None:
            intr, pose, light = self.cameras[idx]
            d.update(intr=intr, pose=pose, pose_light=light)
        if ref_s is not None:
            d.update(pseudo_ref_sampled=ref_s[None], pseudo_sha_sampled=sha_s[None, :, None],
                     pseudo_visibility_certainty_sampled=cert_s[None, :, None])
        return d
