"""Build libmli_hip.so (gfx950) in-tree with hipcc.  ``python -m mli_nerf_amd.build``."""
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmli_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["rays.hip", "sdf.hip", "mlp_fwd.hip", "mlp_fwd_pq.hip", "mlp_fwd_train.hip", "mlp_bwd.hip", "mlp_geo.hip",
           "wgrad.hip", "params.hip", "loss.hip"]
# sdf.hip: no SLP packing, so fma(fp16 -> fp32 feature, w, acc) selects v_fma_mix_f32 (one
# instruction) instead of v_cvt_f32_f16 x2 + v_pk_fma_f32
PER_FILE = {"sdf.hip": ["-fno-slp-vectorize"]}
FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-I", os.path.join(REPO, "include"), "-I", CSRC]


HASH_MARK = b"MLI_SOURCE_HASH="


def _deps():
    return [os.path.join(CSRC, s) for s in SOURCES] + sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")) + [
        os.path.join(REPO, "include", "mli_hip.h")]


def source_hash():
    """sha256 (16 hex digits) of every source, header and compile flag of the library; compiled
    into it (mli_source_hash) so a stale or foreign libmli_hip.so is detected, not trusted by mtime."""
    h = hashlib.sha256()
    for d in _deps():
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    rel = [os.path.relpath(f, REPO) if os.path.isabs(f) else f for f in FLAGS]  # the same on any checkout path
    h.update(repr((rel, sorted(PER_FILE.items()))).encode())
    return h.hexdigest()[:16]


def built_hash(path):
    """The source hash embedded in a built library (read from the file, not loaded), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(HASH_MARK)
    return None if i < 0 else data[i + len(HASH_MARK):i + len(HASH_MARK) + 16].decode("ascii", "replace")


def _compile(src, extra, tag="", digest=""):
    obj = os.path.join(CSRC, "build" + tag, os.path.splitext(src)[0] + ".o")
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    cmd = [HIPCC] + FLAGS + PER_FILE.get(src, []) + list(extra) + ['-DMLI_SOURCE_HASH="%s"' % digest,
                                                                   "-c", os.path.join(CSRC, src), "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, res.stderr))
    return obj, res.stderr


def build(verbose=False, extra=(), out=None):
    """Compile + link; ``out``/``extra`` build an experiment variant (tools/, not the product)."""
    out = out or OUT
    tag = "" if out == OUT else "_" + os.path.splitext(os.path.basename(out))[0]
    digest = source_hash()
    if not extra and built_hash(out) == digest:  # built from exactly these sources and flags
        return out
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        results = list(ex.map(lambda s: _compile(s, extra, tag, digest), SOURCES))
    if verbose:
        for _, log in results:
            if log:
                print(log)
    objs = [o for o, _ in results]
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("link failed:\n" + res.stderr)
    return out


if __name__ == "__main__":
    extra = sys.argv[1:]
    print(build(verbose=True, extra=extra))
