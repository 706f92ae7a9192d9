"""Novel-view / relighting video between two frames.

Reference: ``projects/nerf/trainers/base.py:264-346`` (``test_video``) with the helpers of
``projects/NeuralLumen/utils/utils.py`` (``interpolate_pose`` :12-33, ``img_to_np`` :36-58,
``create_collage`` :177-199) and the closest-GT lookup of ``NeuralLumen/data.py:45-74``.

60 frames with ratio ``sin((i/60 - 0.5) pi) / 2 + 1/2`` interpolate the camera AND the light
pose (rotation by quaternion slerp, translation linearly), each frame is one
``Model.inference`` call (the GPU renderer, tile-sharded over ranks when a process group is
up), the selected maps are labelled and tiled into a collage, and the sequence is played
forward then mirrored.  The reference writes an mp4 (OpenCV ``mp4v`` at 30 fps); OpenCV is
optional here: with ``cv2`` importable the same mp4 is written, otherwise an animated GIF at
30 fps plus the PNG frames (the labels are then drawn with PIL's default font instead of
OpenCV's Hershey font, the only visual difference).
"""
import math
import os
import sys

import numpy as np
import torch

N_FRAMES = 60

_LABELS = {"rgb": ("rgb_map", "Image (render)"), "o_r": ("o_r_map", "Reflectance"),
           "o_s": ("o_s_map", "Shading"), "o_re": ("o_re_map", "Residual")}


def frame_ratio(i, n_frames=N_FRAMES):
    """base.py:297, in the reference's float32 arithmetic."""
    return torch.sin(torch.tensor([((i / n_frames) - 0.5) * math.pi], dtype=torch.float32)) * 0.5 + 0.5


def interpolate_pose(pose1, pose2, ratio):
    """utils.py:12-33: slerp of the two w2c rotations, lerp of the translations -> [3,4] float32."""
    from scipy.spatial.transform import Rotation, Slerp
    is_t = torch.is_tensor(pose1)
    p1 = pose1.detach().cpu().numpy() if is_t else np.asarray(pose1)
    p2 = pose2.detach().cpu().numpy() if is_t else np.asarray(pose2)
    r = np.float32(ratio.item() if torch.is_tensor(ratio) else ratio)
    rot = Slerp([0, 1], Rotation.from_matrix(np.stack([p1[:3, :3], p2[:3, :3]])))([float(r)])
    pose = np.eye(4, dtype=np.float32)
    pose[:3, :3] = rot.as_matrix()[0]
    pose[:3, 3] = ((np.float32(1.0) - r) * p1.astype(np.float32) + r * p2.astype(np.float32))[:3, 3]
    pose = pose[:3]
    return torch.from_numpy(pose) if is_t else pose


def _label(img, text):
    """A white band of height H/10 under the image with the label at its bottom left."""
    band = np.full((int(img.shape[0] / 10), img.shape[1], 3), 255, np.uint8)
    out = np.vstack((img, band))
    try:
        import cv2
        cv2.putText(out, text, (10, out.shape[0] - 10), cv2.FONT_HERSHEY_SIMPLEX, 0.5, (0, 0, 0), 1, cv2.LINE_AA)
        return out
    except ImportError:
        from PIL import Image, ImageDraw
        im = Image.fromarray(out)
        d = ImageDraw.Draw(im)
        d.text((10, out.shape[0] - 10), text, fill=(0, 0, 0), anchor="ls")  # baseline, as cv2
        return np.asarray(im).copy()


def img_to_np(t, add_text=True, text=" "):
    """utils.py:36-58: [C,H,W] in [0,1] -> uint8 [H,W,3] RGB (x256, clipped; 1 channel
    repeated), optionally labelled.  Kept RGB: the BGR swap of the reference is OpenCV's
    writer convention and is applied in ``write_video``."""
    a = (t.detach().float().cpu().numpy().transpose(1, 2, 0) * 256).clip(0, 255).astype(np.uint8)
    if a.shape[2] == 1:
        a = np.repeat(a, 3, axis=2)
    return _label(a, text) if add_text else a


def create_collage(imgs, padding=5):
    """utils.py:177-199: rows = floor(sqrt(n)), cols = ceil(n / rows), white padding between
    columns."""
    h, w, _ = imgs[0].shape
    rows = int(np.sqrt(len(imgs)))
    cols = int(np.ceil(len(imgs) / rows))
    out = np.full((h * rows, w * cols + padding * (cols - 1), 3), 255, np.uint8)
    for i, im in enumerate(imgs):
        y, x = (i // cols) * h, (i % cols) * (w + padding)
        out[y:y + h, x:x + w] = im
    return out


def write_video(frames, path_noext, fps=30):
    """mp4 (mp4v) through OpenCV when present (base.py:335-346), else GIF + PNG frames.
    Returns the path written."""
    try:
        import cv2
        h, w, _ = frames[0].shape
        path = path_noext + ".mp4"
        wr = cv2.VideoWriter(path, cv2.VideoWriter_fourcc(*"mp4v"), fps, (w, h))
        for f in frames:
            wr.write(cv2.cvtColor(f, cv2.COLOR_RGB2BGR))
        wr.release()
        return path
    except ImportError:
        from PIL import Image
        fdir = path_noext + "_frames"
        os.makedirs(fdir, exist_ok=True)
        ims = [Image.fromarray(f) for f in frames]
        for i, im in enumerate(ims):
            im.save(os.path.join(fdir, f"{i:04d}.png"))
        path = path_noext + ".gif"
        ims[0].save(path, save_all=True, append_images=ims[1:], duration=int(round(1000 / fps)), loop=0)
        return path


@torch.no_grad()
def render_video(model, dataset, setting1, setting2, output_dir, trainer=None, mode="test",
                 video_content=("rgb", "gt", "o_r", "o_s"), n_frames=N_FRAMES, show_pbar=False):
    """base.py:264-346.  ``dataset``: a ``mli_nerf_amd.data.Dataset`` (its __getitem__ in
    eval mode gives full images and poses).  ``trainer``: sets the model's progress /
    coarse-to-fine state for the iteration (sys.maxsize in 'test' mode, as the reference)."""
    model.eval()
    dataset.sample_train_rays = False   # full images (base.py:282-283)
    dataset.has_pseudo_label = False
    s1, s2 = dataset[int(setting1)], dataset[int(setting2)]
    dev = model.flat.device
    if trainer is not None:
        saved = trainer.current_iteration
        trainer.current_iteration = sys.maxsize if mode == "test" else saved
        trainer._start_of_iteration()
        trainer.current_iteration = saved
    frames = []
    for i in range(n_frames):
        if show_pbar:
            print(i, file=sys.stderr)
        r = frame_ratio(i, n_frames)
        data = dict(idx=None, intr=s1["intr"][None].to(dev),
                    pose=interpolate_pose(s1["pose"], s2["pose"], r)[None].to(dev),
                    pose_light=interpolate_pose(s1["pose_light"], s2["pose_light"], r)[None].to(dev))
        out = model.inference(data)
        tiles = []
        for key in video_content:
            if key == "gt":
                j = dataset.find_closest_idx(data["pose"].cpu(), data["pose_light"].cpu())
                tiles.append(img_to_np(dataset[j]["image"], True, "Image (the closest GT)"))
            elif key in _LABELS and _LABELS[key][0] in out:
                mk, label = _LABELS[key]
                tiles.append(img_to_np(out[mk][0], True, label))
        frames.append(create_collage(tiles))
    frames = frames + frames[::-1]
    vdir = os.path.join(output_dir, "render")
    os.makedirs(vdir, exist_ok=True)
    return write_video(frames, os.path.join(vdir, f"{setting1}_{setting2}"))
