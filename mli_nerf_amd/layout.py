"""Packing plans shared by the host and the kernels (see include/mli_hip.h).

Packed-k order of the head layer-0 input (MLI_HEAD_K0 = 304 rows):
    0..255   feat (SDF layer-1 softplus output), accumulator order
    256..258 p, 259..261 normal, 262..271 zero pad          (k-step 16, NAT order)
    272..287 SH16(light position)                           (k-step 17, NAT order)
    288..303 SH16(view direction)                           (k-step 18, NAT order)
Reference column order of each head's first Linear (NeuralLumen/utils/modules.py:149-151):
    mlp   (rgb): [p 3, view 16, n 3, feat 256, light 16] = 294
    mlp_r (o_r): [p 3, n 3, feat 256]                    = 262
    mlp_s (o_s): [p 3, n 3, feat 256, light 16]          = 278
"""
import numpy as np

HEADS = (("mlp", 294, 3), ("mlp_r", 262, 3), ("mlp_s", 278, 1))
HEADS_A = HEADS[:1]   # LumenRGB mode 'rgb' (stage a): the single 294 -> 3 head, input order as 'mlp'
SDF_K0 = 131          # neural_sdf.mlp.linears.0 input: p 3 + hash encoding 128
HIDDEN = 256
K0 = 304
KS0 = 19
NAT, ACC = 0, 1


def chunk_bytes(k_steps):
    return k_steps * 1024 + 128


def head_kmap(name):
    """Packed k (0..303) -> reference input column (-1 = zero)."""
    km = -np.ones(K0, dtype=np.int16)
    feat0 = {"mlp": 22, "mlp_r": 6, "mlp_s": 6}[name]
    n0 = {"mlp": 19, "mlp_r": 3, "mlp_s": 3}[name]
    light0 = {"mlp": 278, "mlp_r": None, "mlp_s": 262}[name]
    view0 = {"mlp": 3, "mlp_r": None, "mlp_s": None}[name]
    km[0:256] = feat0 + np.arange(256)
    km[256:259] = np.arange(3)
    km[259:262] = n0 + np.arange(3)
    if light0 is not None:
        km[272:288] = light0 + np.arange(16)
    if view0 is not None:
        km[288:304] = view0 + np.arange(16)
    return km


def head_kinv(name, k_ref):
    km = head_kmap(name)
    inv = np.zeros(k_ref, dtype=np.int16)
    for kk, c in enumerate(km):
        if c >= 0:
            inv[c] = kk
    return inv


def ident_kmap(n, pad_to):
    km = -np.ones(pad_to, dtype=np.int16)
    km[:n] = np.arange(n)
    return km


def param_prefix(head, layer):
    return "neural_rgb.%s.linears.%d" % (head, layer)


def trainable_layout(stage="b"):
    """Flat fp32 buffer layout of the trainable parameters: [(name, shape, offset)].
    Stage b (partial_grad neural_rgb, NeuralLumen/trainer.py:44-54): the three heads.
    Stage a (every parameter, NeuralLumen/model.py:422-438): the SDF MLP, the single head and
    s_var -- the hash table is a separate buffer (``neural_sdf.tcnn_encoding.params``)."""
    out, off = [], 0
    if stage == "a":
        for li, k_in in enumerate((SDF_K0, HIDDEN)):
            pre = "neural_sdf.mlp.linears.%d" % li
            for suffix, shape in (("weight_v", (HIDDEN, k_in)), ("weight_g", (HIDDEN, 1)), ("bias", (HIDDEN,))):
                out.append((pre + "." + suffix, shape, off))
                off += int(np.prod(shape))
        for suffix, shape in (("weight", (1, HIDDEN)), ("bias", (1,))):
            out.append(("neural_sdf.mlp.linear_sdf." + suffix, shape, off))
            off += int(np.prod(shape))
    for head, k_in, k_out in (HEADS_A if stage == "a" else HEADS):
        dims = [k_in] + [HIDDEN] * 4 + [k_out]
        for li in range(5):
            pre = param_prefix(head, li)
            for suffix, shape in (("weight_v", (dims[li + 1], dims[li])), ("weight_g", (dims[li + 1], 1)),
                                  ("bias", (dims[li + 1],))):
                out.append((pre + "." + suffix, shape, off))
                off += int(np.prod(shape))
    if stage == "a":
        out.append(("s_var", (), off))
        off += 1
    return out, off


def fwd_plan(heads=HEADS):
    """Chunk sequence of the forward weight image, in kernel consumption order.
    Each entry: dict(param prefix, n_out, k_ref, transpose, n_tiles, k_steps, kmap, kmode)."""
    plan = [dict(prefix="neural_sdf.mlp.linears.1", n_out=256, k_ref=256, transpose=0, n_tiles=8,
                 k_steps=16, kmap=ident_kmap(256, 256), kmode=np.full(16, ACC, np.uint8))]
    for head, k_in, k_out in heads:
        kmode0 = np.array([ACC] * 16 + [NAT] * 3, np.uint8)
        plan.append(dict(prefix=param_prefix(head, 0), n_out=256, k_ref=k_in, transpose=0, n_tiles=8,
                         k_steps=KS0, kmap=head_kmap(head), kmode=kmode0))
        for li in (1, 2, 3):
            plan.append(dict(prefix=param_prefix(head, li), n_out=256, k_ref=256, transpose=0,
                             n_tiles=8, k_steps=16, kmap=ident_kmap(256, 256),
                             kmode=np.full(16, ACC, np.uint8)))
        plan.append(dict(prefix=param_prefix(head, 4), n_out=k_out, k_ref=256, transpose=0, n_tiles=1,
                         k_steps=16, kmap=ident_kmap(256, 256), kmode=np.full(16, ACC, np.uint8)))
    return _with_offsets(plan)


def bwd_plan():
    """Transposed weights of the dX chain: per head W4^T (k over the outputs, 1 k-step),
    W3^T, W2^T, W1^T."""
    plan = []
    for head, k_in, k_out in HEADS:
        plan.append(dict(prefix=param_prefix(head, 4), n_out=k_out, k_ref=256, transpose=1, n_tiles=8,
                         k_steps=1, kmap=ident_kmap(k_out, 16), kmode=np.full(1, ACC, np.uint8)))
        for li in (3, 2, 1):
            plan.append(dict(prefix=param_prefix(head, li), n_out=256, k_ref=256, transpose=1,
                             n_tiles=8, k_steps=16, kmap=ident_kmap(256, 256),
                             kmode=np.full(16, ACC, np.uint8)))
    return _with_offsets(plan)


def geo_plan():
    """Stage-a backward image (mli_geo_bwd): the single head's W4^T, W3^T, W2^T, W1^T, then
    W0^T over the packed input rows 0..287 (feat in ACC order, p, normal; row map = head_kmap),
    then SDF layer 1 transposed (rows = h0 index, k = its outputs in ACC order)."""
    head, k_in, k_out = HEADS_A[0]
    plan = [dict(prefix=param_prefix(head, 4), n_out=k_out, k_ref=256, transpose=1, n_tiles=8,
                 k_steps=1, kmap=ident_kmap(k_out, 16), kmode=np.full(1, ACC, np.uint8))]
    for li in (3, 2, 1):
        plan.append(dict(prefix=param_prefix(head, li), n_out=256, k_ref=256, transpose=1, n_tiles=8,
                         k_steps=16, kmap=ident_kmap(256, 256), kmode=np.full(16, ACC, np.uint8)))
    plan.append(dict(prefix=param_prefix(head, 0), n_out=256, k_ref=k_in, transpose=1, n_tiles=9,
                     k_steps=16, kmap=ident_kmap(256, 256), kmode=np.full(16, ACC, np.uint8),
                     nmap=head_kmap(head)[:288]))
    plan.append(dict(prefix="neural_sdf.mlp.linears.1", n_out=256, k_ref=256, transpose=1, n_tiles=8,
                     k_steps=16, kmap=ident_kmap(256, 256), kmode=np.full(16, ACC, np.uint8)))
    return _with_offsets(plan)


def _with_offsets(plan):
    off = 0
    for p in plan:
        p["chunk_stride"] = chunk_bytes(p["k_steps"])
        p["dst_offset"] = off
        off += p["n_tiles"] * p["chunk_stride"]
    return plan, off


def u_fine(n_fine):
    """Midpoint quantiles exactly as nerf_util.sample_dists_from_pdf builds them (:55-56)."""
    import torch
    grid = torch.linspace(0, 1, n_fine + 1)
    return (0.5 * (grid[:-1] + grid[1:])).tolist()


def fastmod_magic(d):
    return ((1 << 64) // d + 1) & ((1 << 64) - 1)


def q4_segs(N):
    """MLI_Q4_SEGS (include/mli_hip.h): ray segments per 256-sample workgroup of the PQ partials."""
    if 256 % N == 0:
        return 256 // N
    return 1 if N % 256 == 0 else 256 // N + 2


def untile(img, rows):
    """A tile-blocked activation image ([S/256][rows][256], include/mli_hip.h ABI 14) as
    feature-major rows [rows][S] (a view copy, for inspection and tests)."""
    flat = img.reshape(-1)
    S = flat.numel() // rows
    return flat.view(S // 256, rows, 256).permute(1, 0, 2).reshape(rows, S)


def unfrag(img, rows, kst=None, order="acc"):
    """A fragment image ([S/32][kst][64 lanes][8 halves], include/mli_hip.h ABI 15; ``kst`` k-steps
    per 32-sample tile, default rows / 16) as feature-major rows [rows][S] (a copy, for
    inspection and tests).  Element j of lane c + 32 h of k-step q is sample c of the tile and
    feature 16 q + 8 (j >> 2) + 4 h + (j & 3) (ACC order) or 16 q + 8 h + j (NAT order)."""
    kst = kst or (rows + 15) // 16
    flat = img.reshape(-1)
    S = flat.numel() // (kst * 16)
    x = flat.view(S // 32, kst, 2, 32, 2, 4) if order == "acc" else flat.view(S // 32, kst, 2, 32, 8)
    if order == "acc":
        # dims (tile, q, h, c, j>>2, j&3) -> feature 16 q + 8 (j>>2) + 4 h + (j&3)
        x = x.permute(1, 4, 2, 5, 0, 3)       # (q, j>>2, h, j&3, tile, c)
    else:
        x = x.permute(1, 2, 4, 0, 3)          # (q, h, j, tile, c)
    return x.reshape(kst * 16, S)[:rows]


def frag_index(m, f, kst, order="acc"):
    """Element offset of (sample m, feature f) in a fragment image with kst k-steps per tile
    (the index rule of include/mli_hip.h, for tests)."""
    q, r = divmod(f, 16)
    if order == "acc":
        h, j = (r >> 2) & 1, ((r >> 3) << 2) | (r & 3)
    else:
        h, j = r >> 3, r & 7
    return ((m // 32) * kst + q) * 512 + ((m % 32) + 32 * h) * 8 + j


def to_frag(rows, kst=None, order="acc"):
    """Feature-major rows [rows][S] (S % 32 == 0) as a fragment image with ``kst`` k-steps per
    tile (rows past the matrix zero): the inverse of unfrag (tests)."""
    import torch
    n, S = rows.shape
    kst = kst or (n + 15) // 16
    full = torch.zeros(kst * 16, S, dtype=rows.dtype, device=rows.device)
    full[:n] = rows
    if order == "acc":
        x = full.view(kst, 2, 2, 4, S // 32, 32).permute(4, 0, 2, 5, 1, 3)   # (tile, q, h, c, j>>2, j&3)
    else:
        x = full.view(kst, 2, 8, S // 32, 32).permute(3, 0, 1, 4, 2)         # (tile, q, h, c, j)
    return x.contiguous().reshape(-1)


def to_tiled(rows):
    """Feature-major rows [rows][S] (S % 256 == 0) as a tile-blocked image: inverse of untile."""
    n, S = rows.shape
    return rows.view(n, S // 256, 256).permute(1, 0, 2).contiguous().reshape(-1)
