"""Oracle of the on-device training-ray draw (TEST INFRASTRUCTURE ONLY; never imported by the
product package).

Reference behaviour (``projects/NeuralLumen/data.py:120-132``, ``data_blender.py:179-195``,
``projects/neuralangelo/data.py:84-92``): ``ray_idx = torch.randperm(H*W)[:R]`` -- R
distinct pixels drawn uniformly -- then ``image.flatten(1, 2)[:, ray_idx].t()`` and the
same gather for the pseudo labels ``[C,H,W] -> [R,C]``.

``mli_ray_batch`` replaces the host randperm by a seeded bijection of [0, 2^bits)
(4-round Feistel network, round function = a 32-bit integer mixer) walked until it lands
in [0, n_pixels) (cycle walking), so ray r's pixel is perm(r) of a permutation of the pixel
range: distinct by construction, no host round trip.  This file restates the kernel's
integer arithmetic bit for bit (numpy uint32/uint64), so the GPU draw is checked EXACTLY;
the gather is checked against the reference's own flatten/index expression.
"""
import numpy as np

M32 = 0xFFFFFFFF


def _mix32_int(x):
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def _mix32(x):
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def n_bits(n_pixels):
    bits = 1
    while (1 << bits) < n_pixels:
        bits += 1
    return bits


def feistel(x, bits, seed):
    """x: uint64 array in [0, 2^bits) -> its image under the keyed bijection."""
    lb = bits >> 1
    hb = bits - lb
    lmask, hmask = np.uint64((1 << lb) - 1), np.uint64((1 << hb) - 1)
    x = x.astype(np.uint64)
    Lh, Rr = x >> np.uint64(lb), x & lmask
    for k in range(4):
        key = _mix32_int(((seed >> (8 * k)) & M32) + ((0x9E3779B9 * (k + 1)) & M32))
        f = _mix32((Rr & np.uint64(M32)).astype(np.uint32) ^ np.uint32(key) ^ np.uint32((seed >> 32) & M32))
        nL, nR = Rr, (Lh ^ f.astype(np.uint64)) & hmask
        comb = (nL << np.uint64(hb)) | nR
        Lh, Rr = comb >> np.uint64(lb), comb & lmask
    return (Lh << np.uint64(lb)) | Rr


def ray_indices(seed, n_pixels, R):
    """The R pixel indices mli_ray_batch draws (int64 [R])."""
    seed = int(seed) & ((1 << 64) - 1)
    bits = n_bits(n_pixels)
    x = np.arange(R, dtype=np.uint64)
    x = feistel(x, bits, seed)
    todo = x >= np.uint64(n_pixels)
    while todo.any():  # cycle walking
        x[todo] = feistel(x[todo], bits, seed)
        todo = x >= np.uint64(n_pixels)
    return x.astype(np.int64)


def gather(image_chw, ray_idx):
    """The reference's ``image.flatten(1, 2)[:, ray_idx].t()`` (numpy)."""
    c = image_chw.shape[0]
    return image_chw.reshape(c, -1)[:, ray_idx].T
