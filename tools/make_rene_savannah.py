#!/usr/bin/env python
"""Package data: the first 16 training frames of the reference's ReNe savannah scene
(``dataset_rene/savannah/train_transforms.json``: camera + light poses, camera / light indices)
with the scene header (intrinsics, raw image size, AABB) -- the real cameras of BASELINE.json
configs[3] (rene_savannah_b, rank r -> frame r).  Data only (no images ship with the reference).

Runs only in the build container (needs /root/reference, read-only).
Usage:  python tools/make_rene_savannah.py   (writes mli_nerf_amd/assets/rene_savannah_train16.json)
"""
import json
import os

HERE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mli_nerf_amd", "assets")
REF = os.environ.get("MLI_REFERENCE", "/root/reference")
HEADER = ("fl_x", "fl_y", "cx", "cy", "sk_x", "sk_y", "w", "h", "camera_angle_x", "camera_angle_y",
          "sphere_center", "sphere_radius", "bounding_box_aabb", "aabb_scale")
FRAME = ("index", "file_path", "camera_index", "light_index", "transform_matrix", "transform_matrix_light")


def main(n=16):
    with open(os.path.join(REF, "dataset_rene", "savannah", "train_transforms.json")) as f:
        meta = json.load(f)
    out = {k: meta[k] for k in HEADER}
    out["frames"] = [{k: fr[k] for k in FRAME} for fr in meta["frames"][:n]]
    out["source"] = "dataset_rene/savannah/train_transforms.json, frames 0..%d of %d" % (n - 1, len(meta["frames"]))
    path = os.path.join(HERE, "rene_savannah_train16.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
