"""Camera x light enumeration for the pseudo labels: ``Trainer.test_all_light``.

Reference: ``projects/NeuralLumen/trainer.py:216-316`` (``test_all_light``), called by
``test.py:146-172`` for the inference modes ``lights`` (pair), ``unpairlights`` (unpair, 4 lights
per camera, seed 999), ``limitedlights`` and ``singlelight`` (limitedlights with 4 / 1 lights);
``get_random_other_index`` of ``projects/NeuralLumen/utils/utils.py:230-252``; the image writer
``preprocess_image`` of ``imaginaire/utils/visualization.py:29-41``.

For every (camera, light) pair one ``Model.inference`` renders the full frame with the light
visibility pass on (the GPU renderer: sampling, FIELD, heads, composite, sphere-traced camera and
light rays, tile-sharded over ranks when a process group is up) at iteration ``sys.maxsize``
(mode 'test': the NeuS anneal finished).  The maps go to ``<output_dir>/<camera>/<light>_*.png``
and ``results_all.pt`` holds ``{camera: {light: {normal, normal_x_light, rgb_render, visibility,
inter_mask[, rgb_target]}}}`` (string keys, CPU tensors [1,C,H,W]) -- the file
``scripts/pseudo_label.py:294-410`` reads.
"""
import copy
import os
import random
import sys

import numpy as np
import torch


def get_random_other_index(num_indexes, length_selected, seed=0):
    """utils.py:230-252: for camera i, [i] + ``length_selected - 1`` other frame indices drawn by
    Python's ``random.sample`` from a ``random.seed(seed)`` stream (the same draws as the
    reference under the same Python)."""
    rng = random.Random(seed)
    out = []
    for i in range(num_indexes):
        others = list(range(num_indexes))
        others.remove(i)
        out.append([i] + rng.sample(others, length_selected - 1))
    return out


def index_info(dataset, dataset_type="pair", sample_num=4, seed=999):
    """The {camera: {light: frame index}} enumeration of trainer.py:231-264."""
    if dataset_type == "pair":
        info = {}
        for fi, fr in enumerate(dataset.list):
            info.setdefault(fr["camera_index"], {})[fr["light_index"]] = fi
        return info
    if dataset_type == "unpair":
        lists = get_random_other_index(len(dataset), sample_num, seed)
        return {cam: {li: fi for li, fi in enumerate(lst)} for cam, lst in enumerate(lists)}
    if dataset_type == "limitedlights":
        frames = dataset.list
        pl_frame = {}
        for fi in range(sample_num):   # the frame of each of the first sample_num pl_index values
            pl_frame[frames[fi]["pl_index"]] = fi
        info = {}
        for cam in range(len(frames)):
            info[cam] = {0: cam}
            rest = list(pl_frame.keys())
            rest.remove(frames[cam]["pl_index"])
            for k, pl in enumerate(rest):
                info[cam][k + 1] = pl_frame[pl]
        return info
    raise NotImplementedError(dataset_type)


def preprocess_image(images, from_range=(0, 1)):
    """visualization.py:29-41: rescale to [0,1], clamp; one channel -> the 'gray' colormap's RGB
    (matplotlib, as the reference; a plain channel repeat when matplotlib is absent)."""
    lo, hi = (float(v) for v in from_range)
    images = ((images - lo) / (hi - lo)).detach().cpu().float().clamp_(min=0, max=1)
    if images.shape[1] == 1:
        try:
            from matplotlib import pyplot as plt
            color = plt.get_cmap("gray")(images[:, 0].numpy())
            images = torch.from_numpy(color[..., :3]).permute(0, 3, 1, 2).float()
        except ImportError:
            images = images.repeat(1, 3, 1, 1)
    return images


def save_image(image, path, from_range=(0, 1)):
    """trainer.py:270-274: the [1,C,H,W] map squeezed to [C,H,W] BEFORE preprocess_image, so its
    one-channel test looks at H and the maps keep their channel count (no colormap); then
    torchvision's to_pil_image: x255 truncated to uint8 (``mul(255).byte()``), one channel -> an
    'L' PNG, three -> 'RGB'."""
    from PIL import Image
    im = preprocess_image(image.squeeze(0), from_range)
    a = im.mul(255).byte().permute(1, 2, 0).numpy()
    Image.fromarray(a[:, :, 0] if a.shape[2] == 1 else a, mode="L" if a.shape[2] == 1 else "RGB").save(path)


@torch.no_grad()
def test_all_light(trainer, data_loader, output_dir=None, mode="test", dataset_type="pair", sample_num=4, seed=999,
                   save_images=True):
    """trainer.py:216-316.  ``data_loader``: a DataLoader (its ``.dataset``) or the Dataset."""
    model = trainer.model
    if model.pcfg.light_visibility is None:
        raise ValueError("test_all_light needs model.light_visibility.enabled (its maps: visibility, "
                         "normal_x_light, inter_mask)")
    model.eval()
    dataset = getattr(data_loader, "dataset", data_loader)
    dataset.sample_train_rays = False    # full images (trainer.py:228)
    c_iter = sys.maxsize if mode == "test" else trainer.current_iteration
    info = index_info(dataset, dataset_type, sample_num, seed)
    saved = trainer.current_iteration
    results_cam = {}
    try:
        for cam in info:
            cam_dir = os.path.join(output_dir, str(cam))
            os.makedirs(cam_dir, exist_ok=True)
            results_light = {}
            data_input = None
            for light in info[cam]:
                if dataset_type == "pair":
                    data = dataset[info[cam][light]]
                else:
                    if light == 0:
                        data_input = dataset[cam]
                    else:
                        data_input["pose_light"] = dataset.get_light(light)
                    data = copy.deepcopy(data_input)
                data = {k: v[None] if torch.is_tensor(v) else v for k, v in data.items()}
                data = trainer.start_of_iteration(data, current_iteration=c_iter)
                trainer._start_of_iteration()
                out = model.inference(data)
                pre = str(light) + "_"

                def save(img, name, from_range=(0, 1)):
                    if save_images:
                        save_image(img, os.path.join(cam_dir, pre + name + ".png"), from_range)
                if dataset_type == "pair" or light == 0:
                    save(data["image"], "rgb_target")
                save(out["rgb_map"], "rgb_render")
                save(out["normal_map"], "normal", (-1, 1))
                save(out["visibility_map"], "visibility")
                save(out["inter_dist_map"], "inter_dist", (out["inter_dist_map"].min(), out["inter_dist_map"].max()))
                save(out["inter_mask_map"], "inter_mask")
                save(out["normal_x_light_map"], "normal_x_light")
                save(out["visibility_map"].float() * out["normal_x_light_map"], "pseudo_shading")
                res = {"normal": out["normal_map"].detach().cpu(),
                       "normal_x_light": out["normal_x_light_map"].detach().cpu(),
                       "rgb_render": out["rgb_map"].detach().cpu(),
                       "visibility": out["visibility_map"].detach().cpu(),
                       "inter_mask": out["inter_mask_map"].detach().cpu()}
                if dataset_type == "pair":
                    res["rgb_target"] = data["image"].detach().cpu()
                results_light[str(light)] = res
            results_cam[str(cam)] = results_light
    finally:
        trainer.current_iteration = saved
    if output_dir is not None:
        torch.save(results_cam, os.path.join(output_dir, "results_all.pt"))
    return results_cam
