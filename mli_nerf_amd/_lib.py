"""ctypes binding of libmli_hip.so (include/mli_hip.h).  Fails loudly if the library is
missing -- there is no CPU fallback on the product path."""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MLI_HIP_LIB selects an experiment build (tools/kbench.py A/B runs); default: the in-tree lib
LIB_PATH = os.environ.get("MLI_HIP_LIB") or os.path.join(HERE, "libmli_hip.so")

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
F32 = C.c_float
F64 = C.c_double


class GridLevels(C.Structure):
    _fields_ = [("scale", F32 * 16), ("res", C.c_uint32 * 16), ("size", C.c_uint32 * 16),
                ("offset", C.c_uint32 * 16), ("modmagic", C.c_uint64 * 16)]


class RaysArgs(C.Structure):
    _fields_ = [("intr", P), ("pose", P), ("pose_light", P), ("ray_idx", P), ("first_pixel", I64),
                ("R", I32), ("W", I32), ("bounding", I32), ("aabb", F32 * 6),
                ("center", P), ("ray_unit", P), ("ray_norm", P), ("pts_light", P),
                ("near_", P), ("far_", P), ("outside", P)]


class HashgridArgs(C.Structure):
    _fields_ = [("x01", P), ("table", P), ("levels", GridLevels), ("n", I32), ("out", P)]


class SdfArgs(C.Structure):
    _fields_ = [("mode", I32), ("R", I32), ("n_per_ray", I32), ("center", P), ("ray_unit", P),
                ("dists", P), ("outside", P), ("table", P), ("levels", GridLevels), ("wsdf", P),
                ("eps", F32), ("grad_den", F32), ("hess_den", F32), ("outside_val", F32),
                ("with_hessian", I32), ("sdf", P), ("grad", P), ("hess", P), ("h0", P),
                ("enc", P), ("active_levels", I32)]


class SampleCoarseArgs(C.Structure):
    _fields_ = [("near_", P), ("far_", P), ("u", P), ("R", I32), ("Nc", I32), ("dists", P)]


class SampleFineArgs(C.Structure):
    _fields_ = [("R", I32), ("dists_a", P), ("sdf_a", P), ("Na", I32), ("dists_b", P), ("sdf_b", P),
                ("Nb", I32), ("dists_out", P), ("sdf_out", P), ("Nf", I32), ("inv_s", F32),
                ("u_fine", P), ("fine_out", P)]


class RgbFwdArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("center", P), ("ray_unit", P), ("pts_light", P),
                ("dists", P), ("grad", P), ("h0", P), ("wfwd", P), ("y", P), ("feat_frag", P),
                ("xT", P), ("masks", P), ("n_heads", I32), ("weights", P), ("q4", P)]


class CompositeArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("dists", P), ("far_", P), ("ray_unit", P), ("ray_norm", P),
                ("sdf", P), ("grad", P), ("y", P), ("s_var", P), ("anneal", F32), ("white_bg", I32),
                ("weights", P), ("rgb", P), ("o_r", P), ("o_s", P), ("o_re", P), ("opacity", P),
                ("gradient", P), ("depth", P), ("blend_dist", P)]


class CompositeBwdArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("weights", P), ("y", P), ("o_r", P), ("o_s", P),
                ("d_rgb", P), ("d_o_r", P), ("d_o_s", P), ("d_o_re", P), ("grad_scale", F32),
                ("dz4", P), ("dray", P)]


class RgbBwdArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("dz4", P), ("wbwd", P), ("masks", P), ("dzT", P),
                ("dz4T", P)]


class WgradJob(C.Structure):
    _fields_ = [("a_rows", P), ("b_rows", P), ("M", I32), ("K", I32), ("dw", P), ("db", P), ("ldw", I32),
                ("a_tiled", I32), ("b_tiled", I32), ("a_kst", I32), ("b_kst", I32), ("b2_rows", P),
                ("b2_q", I32), ("b2_kst", I32)]


# mli_wgrad_job operand layouts (MLI_WGRAD_LAYOUT_*)
ROWS, TILED, FRAG_ACC, FRAG_NAT = 0, 1, 2, 3


def frag_job(a, b, M, K, dw, db, ldw, a_kst, b_kst, order=FRAG_ACC, b_order=None, b2=None, b2_q=0, b2_kst=0):
    """A mli_wgrad job over two fragment images (ABI 15) with a_kst / b_kst k-steps per tile;
    b2: B's k-steps from b2_q on come from a second image with b2_kst k-steps per tile (ABI 16)."""
    return WgradJob(a, b, M, K, dw, db, ldw, order, order if b_order is None else b_order, a_kst, b_kst,
                    b2, b2_q, b2_kst)


class WgradArgs(C.Structure):
    _fields_ = [("S", I32), ("n_jobs", I32), ("jobs", P), ("classes", I32), ("deterministic", I32),
                ("workspace", P)]


class Dw4Args(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("n_heads", I32), ("q4", P), ("dray", P), ("scale", F32),
                ("dw", P * 3), ("db", P * 3), ("k_out", I32 * 3), ("workspace", P)]


Q4_SCALE = 65536.0  # include/mli_hip.h MLI_Q4_SCALE


class LossArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("rgb", P), ("o_r", P), ("o_s", P), ("o_re", P), ("gt", P),
                ("ref", P), ("sha", P), ("cert", P), ("outside", P), ("grad", P), ("hess", P),
                ("w_render", F32), ("w_eikonal", F32), ("w_curvature", F32), ("w_intrinsic", F32),
                ("w_re", F32), ("range_sha_lo", F32), ("range_sha_hi", F32), ("range_vis_lo", F32),
                ("range_vis_hi", F32), ("f_ref", F32), ("f_sha", F32), ("f_neg", F32), ("f_pos", F32),
                ("e_pos", F32), ("d_rgb", P), ("d_o_r", P), ("d_o_s", P), ("d_o_re", P), ("losses", P),
                ("scratch", P)]



class CompositeLossArgs(C.Structure):
    _fields_ = [("comp", CompositeArgs), ("loss", LossArgs), ("grad_scale", F32), ("dz4", P),
                ("defer_finalize", I32), ("dray", P)]

class PackLayer(C.Structure):
    _fields_ = [("v", P), ("g", P), ("bias", P), ("n_out", I32), ("k_ref", I32), ("transpose", I32),
                ("n_tiles", I32), ("k_steps", I32), ("kmap", P), ("kmode", P), ("dst_offset", I64),
                ("chunk_stride", I32), ("nmap", P)]


class PackArgs(C.Structure):
    _fields_ = [("n_layers", I32), ("layers", P), ("dst", P), ("row_scale", P)]


class PackSdfArgs(C.Structure):
    _fields_ = [("v0", P), ("g0", P), ("b0", P), ("w_sdf", P), ("b_sdf", P), ("dst", P)]


class AssembleLayer(C.Structure):
    _fields_ = [("dw", P), ("db", P), ("v", P), ("g", P), ("n_out", I32), ("k_ref", I32),
                ("k_pack", I32), ("kinv", P), ("grad_v", P), ("grad_g", P), ("grad_b", P),
                ("extra_db", P), ("plain", I32)]


class AssembleArgs(C.Structure):
    _fields_ = [("n_layers", I32), ("layers", P), ("inv_scale", F32), ("zero_dw", I32)]


class AdamwArgs(C.Structure):
    _fields_ = [("p", P), ("g", P), ("m", P), ("v", P), ("n", I64), ("lr", F64), ("beta1", F64),
                ("beta2", F64), ("eps", F64), ("weight_decay", F64), ("step", I32), ("p16", P),
                ("zero_grad", I32)]


class CastArgs(C.Structure):
    _fields_ = [("src", P), ("dst", P), ("n", I64)]


class CompositeBwdGeoArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("dists", P), ("far_", P), ("ray_unit", P), ("sdf", P), ("grad", P),
                ("y", P), ("s_var", P), ("anneal", F32), ("white_bg", I32), ("d_rgb", P), ("grad_scale", F32),
                ("dz4", P), ("d_sdf", P), ("d_grad", P), ("d_inv_s_part", P), ("d_s_var", P)]


class GeoBwdArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("dz4", P), ("wgeo", P), ("masks", P), ("feat_frag", P), ("dzT", P),
                ("dz4T", P), ("d_nrm", P), ("dz1T", P), ("dh0_frag", P)]


class SdfBwdArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("center", P), ("ray_unit", P), ("dists", P), ("outside", P),
                ("grad", P), ("hess", P), ("d_sdf", P), ("d_grad", P), ("d_nrm", P), ("dh0_frag", P), ("enc", P),
                ("wsdf", P), ("wsdf_t", P), ("eps", F32), ("grad_den", F32), ("hess_den", F32),
                ("w_eikonal", F32), ("w_curvature", F32), ("grad_scale", F32), ("d_enc", P), ("dz0_frag", P),
                ("p_frag", P), ("dw_sdf", P), ("db_sdf", P), ("d_grad_ext", P), ("d_hess_ext", P),
                ("partials", P)]


class PackSdfTArgs(C.Structure):
    _fields_ = [("v0", P), ("g0", P), ("dst", P)]


class HashBwdArgs(C.Structure):
    _fields_ = [("R", I32), ("N", I32), ("center", P), ("ray_unit", P), ("dists", P), ("d_enc", P),
                ("levels", GridLevels), ("eps", F32), ("active_levels", I32), ("d_table", P),
                ("deterministic", I32), ("workspace", P), ("n_params", I64)]


class LightVisibilityArgs(C.Structure):
    _fields_ = [("R", I32), ("center", P), ("ray_unit", P), ("pts_light", P), ("near_", P), ("far_", P),
                ("blend_dist", P), ("gradient", P), ("camera_ray_type", I32), ("iters", I32), ("vis_box", I32),
                ("vis_r2", F32), ("aabb", F32 * 6), ("gamma", F32), ("table", P), ("levels", GridLevels),
                ("active_levels", I32), ("wsdf", P), ("light_unit", P), ("near_l", P), ("far_t", P),
                ("inside", P), ("inter_dist", P), ("inter_mask", P), ("inter_pts", P), ("visibility", P),
                ("normal_x_light", P), ("pseudo_shading", P)]


class RayBatchArgs(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_pixels", I64), ("R", I32), ("image", P), ("ref", P), ("sha", P),
                ("cert", P), ("ray_idx", P), ("image_sampled", P), ("ref_sampled", P), ("sha_sampled", P),
                ("cert_sampled", P)]


class FragRowsArgs(C.Structure):
    _fields_ = [("src", P), ("tile_stride", I64), ("tiles", I32), ("k_steps", I32), ("order", I32), ("dst", P),
                ("ld", I64), ("col0", I64), ("row0", I32)]


ABI_VERSION = 17  # include/mli_hip.h MLI_ABI_VERSION

ENTRY_POINTS = {
    "mli_rays": RaysArgs, "mli_hashgrid_fwd": HashgridArgs, "mli_sdf": SdfArgs,
    "mli_sample_coarse": SampleCoarseArgs, "mli_sample_fine": SampleFineArgs,
    "mli_rgb_fwd": RgbFwdArgs, "mli_composite_fwd": CompositeArgs,
    "mli_composite_bwd": CompositeBwdArgs, "mli_rgb_bwd": RgbBwdArgs,
    "mli_wgrad": WgradArgs, "mli_dw4": Dw4Args,
    "mli_pack": PackArgs, "mli_pack_sdf": PackSdfArgs, "mli_grad_assemble": AssembleArgs,
    "mli_adamw": AdamwArgs, "mli_cast_f16": CastArgs, "mli_stage_b_loss": LossArgs,
    "mli_composite_bwd_geo": CompositeBwdGeoArgs, "mli_geo_bwd": GeoBwdArgs, "mli_sdf_bwd": SdfBwdArgs,
    "mli_pack_sdf_t": PackSdfTArgs, "mli_hash_bwd": HashBwdArgs, "mli_frag_rows": FragRowsArgs,
    "mli_light_visibility": LightVisibilityArgs, "mli_ray_batch": RayBatchArgs,
    "mli_composite_loss": CompositeLossArgs, "mli_composite_loss_finalize": CompositeLossArgs,
}

# host-only scratch-size queries: int mli_<op>_workspace(const args*, int64_t* bytes) -> how many
# sizes each writes (include/mli_hip.h lists their order)
WORKSPACE = {
    "mli_sdf": 1, "mli_rgb_fwd": 6, "mli_rgb_bwd": 2, "mli_wgrad": 1, "mli_composite_bwd_geo": 4,
    "mli_geo_bwd": 6, "mli_sdf_bwd": 4, "mli_hash_bwd": 1, "mli_light_visibility": 5, "mli_stage_b_loss": 5,
    "mli_pack": 1, "mli_dw4": 1, "mli_composite_loss": 2,
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libmli_hip.so is not built (%s); run mli_nerf_amd.build.build() -- "
                              "there is no CPU fallback for the hot path" % LIB_PATH)
        _lib = C.CDLL(LIB_PATH)
        for name, st in ENTRY_POINTS.items():
            fn = getattr(_lib, name)
            fn.argtypes = [C.POINTER(st), P]
            fn.restype = I32
        for name in WORKSPACE:
            fn = getattr(_lib, name + "_workspace")
            fn.argtypes = [C.POINTER(ENTRY_POINTS[name]), C.POINTER(I64)]
            fn.restype = I32
        _lib.mli_abi_version.restype = I32
        _lib.mli_error_string.restype = C.c_char_p
        _lib.mli_error_string.argtypes = [I32]
        _lib.mli_source_hash.restype = C.c_char_p
        if _lib.mli_abi_version() != ABI_VERSION:
            raise ImportError("libmli_hip.so ABI mismatch")
        from . import build as _build
        # in-tree sources: the in-tree library must match them.  Only a library OUTSIDE the in-tree
        # build output (an experiment build named by MLI_HIP_LIB, built from a modified tree on
        # purpose) is exempt, and it is reported when its sources differ from the tree's.
        if all(os.path.exists(d) for d in _build._deps()):
            want, got = _build.source_hash(), _lib.mli_source_hash().decode()
            in_tree = os.path.realpath(LIB_PATH) == os.path.realpath(_build.OUT)
            if got != want and in_tree:
                raise ImportError("libmli_hip.so is stale (built from sources %s, the tree is %s); rebuild with "
                                  "mli_nerf_amd.build.build()" % (got, want))
            if got != want:
                import warnings
                warnings.warn("MLI_HIP_LIB=%s was built from sources %s, not this tree's %s (experiment build)"
                              % (LIB_PATH, got, want))
    return _lib


def _variant(name, args):
    if name == "mli_sdf":
        return ":field" if args.mode == 1 else ":sdf"
    if name == "mli_wgrad":
        return {1: ":big", 2: ":wide", 4: ":thin"}.get(args.classes, "")
    return ""


def workspace(name, args):
    """Byte sizes of op ``name``'s scratch buffers for ``args`` (host-only, no GPU call)."""
    out = (I64 * 8)()
    rc = getattr(lib(), name + "_workspace")(C.byref(args), out)
    if rc != 0:
        raise RuntimeError("%s_workspace failed: %s (%d)" % (name, lib().mli_error_string(rc).decode(), rc))
    return [int(out[i]) for i in range(WORKSPACE[name])]


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


# Optional per-launch timing: set to a list to record (name, start_event, end_event) for every
# C-ABI call on the current stream (used by bench.py for the live roofline measurement).
PROFILE = None
PROFILE_NAMES = None  # with PROFILE on: the call names to time (None = every call)


def call(name, args, stream=None):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    if PROFILE is not None and (PROFILE_NAMES is None or name in PROFILE_NAMES):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib(), name)(C.byref(args), stream)
        e1.record()
        PROFILE.append((name + _variant(name, args), e0, e1))
    else:
        rc = getattr(lib(), name)(C.byref(args), stream)
    if rc != 0:
        raise RuntimeError("%s failed: %s (%d)" % (name, lib().mli_error_string(rc).decode(), rc))
