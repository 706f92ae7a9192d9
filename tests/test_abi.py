"""C-ABI boundary checks that need no GPU: the ctypes mirrors in mli_nerf_amd/_lib.py have
the same size and field offsets as the structs gcc lays out from include/mli_hip.h, and the
built libmli_hip.so loads and exports every entry point the header declares (no compute
calls are made)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from mli_nerf_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mli_hip.h")

STRUCTS = {
    "mli_grid_levels": L.GridLevels, "mli_rays_args": L.RaysArgs, "mli_hashgrid_args": L.HashgridArgs,
    "mli_sdf_args": L.SdfArgs, "mli_sample_coarse_args": L.SampleCoarseArgs,
    "mli_sample_fine_args": L.SampleFineArgs, "mli_rgb_fwd_args": L.RgbFwdArgs,
    "mli_composite_args": L.CompositeArgs, "mli_composite_bwd_args": L.CompositeBwdArgs,
    "mli_rgb_bwd_args": L.RgbBwdArgs, "mli_wgrad_job": L.WgradJob, "mli_wgrad_args": L.WgradArgs,
    "mli_pack_layer": L.PackLayer, "mli_pack_args": L.PackArgs, "mli_pack_sdf_args": L.PackSdfArgs,
    "mli_assemble_layer": L.AssembleLayer, "mli_assemble_args": L.AssembleArgs,
    "mli_adamw_args": L.AdamwArgs, "mli_cast_args": L.CastArgs, "mli_loss_args": L.LossArgs,
    "mli_composite_bwd_geo_args": L.CompositeBwdGeoArgs, "mli_geo_bwd_args": L.GeoBwdArgs,
    "mli_sdf_bwd_args": L.SdfBwdArgs, "mli_pack_sdf_t_args": L.PackSdfTArgs, "mli_hash_bwd_args": L.HashBwdArgs,
    "mli_frag_rows_args": L.FragRowsArgs, "mli_light_visibility_args": L.LightVisibilityArgs,
    "mli_ray_batch_args": L.RayBatchArgs, "mli_dw4_args": L.Dw4Args,
    "mli_composite_loss_args": L.CompositeLossArgs,
}


def _declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(mli_\w+)\s*\(", src, re.M)))


def test_struct_layout_matches_gcc(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mli_hip.h"', "int main(void) {"]
    for cname, st in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in st._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    lines += ["return 0; }"]
    c = tmp_path / "abi.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "abi"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(c), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                  text=True).stdout.splitlines())
    for cname, st in STRUCTS.items():
        assert int(got[cname]) == C.sizeof(st), cname
        for f in st._fields_:
            assert int(got["%s.%s" % (cname, f[0])]) == getattr(st, f[0]).offset, (cname, f[0])


def test_every_header_struct_is_mirrored():
    src = open(HEADER).read()
    declared = set(re.findall(r"}\s*(mli_\w+)\s*;", src))
    assert declared == set(STRUCTS), declared ^ set(STRUCTS)


def test_library_exports_header_entry_points():
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libmli_hip.so not built (run __graft_entry__.build())")
    lib = L.lib()  # loads, binds argtypes and checks the ABI version
    assert lib.mli_abi_version() == L.ABI_VERSION
    fns = _declared_functions()
    queries = {n + "_workspace" for n in L.WORKSPACE}
    assert set(L.ENTRY_POINTS) | {"mli_abi_version", "mli_error_string", "mli_source_hash"} | queries == set(fns)
    for name in fns:
        assert hasattr(lib, name), name
    assert lib.mli_error_string(0)
    from mli_nerf_amd import build as B
    assert lib.mli_source_hash().decode() == B.source_hash() == B.built_hash(L.LIB_PATH)


def test_product_path_does_not_import_oracle():
    pkg = os.path.join(ROOT, "mli_nerf_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith(".py"):
                txt = open(os.path.join(dirpath, fn)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", txt, re.M), fn


def test_workspace_queries_match_engine_buffers():
    """The host-only mli_<op>_workspace queries (no GPU call) give the byte sizes the engine
    allocates for each op's scratch (mli_nerf_amd/engine.py), at the bench size."""
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libmli_hip.so not built")
    from mli_nerf_amd import layout
    R, N = 4096, 128
    S = R * N
    f16, f32 = 2, 4
    assert L.workspace("mli_sdf", L.SdfArgs(1, R, N)) == [(S // 32) * 32 * 640 * f16]
    assert L.workspace("mli_sdf", L.SdfArgs(0, R, 64)) == [0]
    assert L.workspace("mli_rgb_fwd", L.RgbFwdArgs(R, N, n_heads=3)) == [
        N * R * 8 * f32, layout.K0 * S * f16, 0, 3 * 4 * 256 * S * f16, 3 * 4 * (S // 32) * 64 * 4 * 4, 0]
    # PQ mode (weights set): X3 not stored, the output-layer partials q4 instead
    pq = L.RgbFwdArgs(R, N, n_heads=3)
    pq.weights = 1
    assert L.workspace("mli_rgb_fwd", pq)[3:] == [3 * 3 * 256 * S * f16, 3 * 4 * (S // 32) * 64 * 4 * 4,
                                                  (S // 256) * 2 * 3 * 257 * 4 * f32]   # 2 rays per workgroup
    assert [layout.q4_segs(n) for n in (32, 64, 96, 128, 192, 256, 384, 512)] == [8, 4, 4, 2, 3, 1, 2, 1]
    pq.N = 96 + 8   # a 32-sample tile would straddle two rays
    pq.R = 256
    with pytest.raises(RuntimeError):
        L.workspace("mli_rgb_fwd", pq)
    d4 = L.Dw4Args(R, N, 3)
    d4.k_out = (C.c_int * 3)(3, 3, 1)
    assert L.workspace("mli_dw4", d4) == [256 * 3 * 257 * 4 * f32]
    d4.k_out = (C.c_int * 3)(3, 3, 4)   # head 2 has one output slot left in dray
    with pytest.raises(RuntimeError):
        L.workspace("mli_dw4", d4)
    assert L.workspace("mli_rgb_bwd", L.RgbBwdArgs(R, N)) == [3 * 4 * 256 * S * f16, 3 * 16 * S * f16]
    assert L.workspace("mli_geo_bwd", L.GeoBwdArgs(R, N)) == [
        4 * 256 * S * f16, 16 * S * f16, N * R * 4 * f32, 256 * S * f16, S * 256 * f16, 0]
    assert L.workspace("mli_composite_bwd_geo", L.CompositeBwdGeoArgs(R, N)) == [
        N * R * 8 * f32, N * R * f32, N * R * 3 * f32, R * f32]
    assert L.workspace("mli_sdf_bwd", L.SdfBwdArgs(R, N)) == [
        S * 640 * f32, 5 * S * 256 * f16, 5 * S * 16 * f16, 1024 * 257 * f32]
    loss = L.workspace("mli_stage_b_loss", L.LossArgs(R, N))
    assert loss[0] == (4 + 8 * (R // 256 + 256)) * f32 and loss[1:] == [R * 3 * f32, R * 3 * f32, R * f32, R * 3 * f32]
    assert L.workspace("mli_light_visibility", L.LightVisibilityArgs(R)) == [R * 12, R * 4, R * 4, R, R * 12]
    assert L.workspace("mli_pack", L.PackArgs(7)) == [7 * 256 * f32]
    n_params = 45724048 * 8
    assert L.workspace("mli_hash_bwd", L.HashBwdArgs(R, N, deterministic=1, n_params=n_params)) == [n_params * 8]
    assert L.workspace("mli_hash_bwd", L.HashBwdArgs(R, N, n_params=n_params)) == [0]
    # wgrad: the stage-b jobs (engine._wgrad_plan shapes): partial slabs only in deterministic mode
    for frag in (False, True):   # rows and (ABI 15) fragment-image operands
        jobs = []
        for name, k_in, k_out in layout.HEADS:
            for m, k in [(256, layout.K0), (256, 256), (256, 256), (256, 256), (k_out, 256)]:
                if frag:
                    jobs.append(L.frag_job(None, None, m, k, None, None, k, (m + 15) // 16, (k + 15) // 16))
                else:
                    jobs.append(L.WgradJob(None, None, m, k, None, None, k))
        arr = (L.WgradJob * len(jobs))(*jobs)
        q = L.WgradArgs(S, len(jobs), C.cast(arr, C.c_void_p), 7, 0, None)
        assert L.workspace("mli_wgrad", q) == [0]
        q.deterministic = 1
        ws = L.workspace("mli_wgrad", q)[0]
        assert 16 * 2 ** 20 < ws < 512 * 2 ** 20, ws   # tens of MiB of fp32 partial slabs
        q.S = 100   # not a multiple of the 64-sample k-step
        with pytest.raises(RuntimeError):
            L.workspace("mli_wgrad", q)
    # invalid fragment jobs: one operand a fragment image and the other not; too few k-steps per tile
    # ABI 16 split B: b2 only with fragment images, b2_q within B's k-steps, enough k-steps in all
    x = C.c_void_p(16)
    for bad in (L.WgradJob(None, None, 256, 256, None, None, 256, L.FRAG_ACC, L.ROWS, 16, 0),
                L.frag_job(None, None, 256, 304, None, None, 304, 16, 16),
                L.WgradJob(None, None, 256, 131, None, None, 131, L.ROWS, L.ROWS, 0, 0, x, 8, 1),
                L.frag_job(None, None, 256, 131, None, None, 131, 16, 8, b2=x, b2_q=9, b2_kst=1),
                L.frag_job(None, None, 256, 160, None, None, 160, 16, 8, b2=x, b2_q=8, b2_kst=1)):
        arr = (L.WgradJob * 1)(bad)
        with pytest.raises(RuntimeError):
            L.workspace("mli_wgrad", L.WgradArgs(S, 1, C.cast(arr, C.c_void_p), 7, 1, None))
    good = (L.WgradJob * 1)(L.frag_job(None, None, 256, 131, None, None, 131, 16, 8, b_order=L.FRAG_NAT, b2=x, b2_q=8,
                                       b2_kst=1))
    assert L.workspace("mli_wgrad", L.WgradArgs(5 * S, 1, C.cast(good, C.c_void_p), 7, 1, None))[0] > 0


def test_source_hash_detects_stale_library(tmp_path, monkeypatch):
    """build() trusts a library only if the source hash compiled into it (read from the file,
    not loaded) equals the hash of the in-tree sources + flags; the hash does not depend on the
    checkout path (the GPU box runs a copy of the tree elsewhere)."""
    from mli_nerf_amd import build as B
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libmli_hip.so not built")
    want = B.source_hash()
    assert B.built_hash(L.LIB_PATH) == want and len(want) == 16
    fake = tmp_path / "libfake.so"
    fake.write_bytes(b"\0" * 64 + B.HASH_MARK + b"0123456789abcdef" + b"\0" * 8)
    assert B.built_hash(str(fake)) == "0123456789abcdef" != want
    assert B.built_hash(str(tmp_path / "missing.so")) is None
    # another checkout path, same sources: same hash
    deps = B._deps()
    monkeypatch.setattr(B, "_deps", lambda: deps)   # the same files, read from here
    monkeypatch.setattr(B, "REPO", "/elsewhere/repo")
    monkeypatch.setattr(B, "FLAGS", [f.replace(ROOT, "/elsewhere/repo") for f in B.FLAGS])
    assert B.source_hash() == want


def test_untile_inverts_the_tile_blocked_layout():
    """layout.untile (the host's view of the ABI 14 tile-blocked images) against the index rule
    include/mli_hip.h states: sample m of row r at (m / 256) * rows * 256 + r * 256 + m % 256."""
    import torch
    from mli_nerf_amd import layout
    rows, S = 5, 768
    out = layout.untile(torch.arange(rows * S, dtype=torch.int64), rows)
    assert out.shape == (rows, S)
    for r, m in ((0, 0), (3, 517), (4, 767), (1, 255), (2, 256)):
        assert out[r, m].item() == (m // 256) * rows * 256 + r * 256 + m % 256


def test_unfrag_inverts_the_fragment_layout():
    """layout.unfrag (the host's view of the ABI 15 fragment images) against the index rule
    include/mli_hip.h states, ACC and NAT order, with a tile stride above rows / 16."""
    import torch
    from mli_nerf_amd import layout
    for order in ("acc", "nat"):
        rows, kst, S = 40, 4, 96
        img = torch.arange(S * kst * 16, dtype=torch.int64)
        out = layout.unfrag(img, rows, kst, order)
        assert out.shape == (rows, S)
        for f in range(rows):
            for m in (0, 5, 31, 32, 63, 95):
                assert out[f, m].item() == layout.frag_index(m, f, kst, order), (order, f, m)
        assert torch.equal(layout.unfrag(layout.to_frag(out, kst, order), rows, kst, order), out)
    t = torch.arange(3 * 512).view(3, 512)
    assert torch.equal(layout.untile(layout.to_tiled(t), 3), t)
    # ACC order is what acc_to_frag() stores: element j of lane half h is accumulator row
    # acc_row(8 s + j, h) of k-step 2t + s (mlp_core.h / common.h)
    acc_row = lambda i, h: (i & 3) + 8 * (i >> 2) + 4 * h  # noqa: E731
    for s in (0, 1):
        for h in (0, 1):
            for j in range(8):
                f = acc_row(8 * s + j, h)
                assert layout.frag_index(0, f, 2) == (s * 512 + 32 * h * 8 + j), (s, h, j)
