"""Build libmli_hip.so (gfx950) in-tree with hipcc.  ``python -m mli_nerf_amd.build``."""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmli_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["rays.hip", "sdf.hip", "mlp.hip", "heads_bwd.hip", "wgrad.hip", "params.hip", "loss.hip"]
# sdf.hip: no SLP packing, so fma(fp16 -> fp32 feature, w, acc) selects v_fma_mix_f32 (one
# instruction) instead of v_cvt_f32_f16 x2 + v_pk_fma_f32
# heads_bwd.hip: the dW accumulators live in AGPRs through asm constraints; the compiler's own
# (chain) MFMAs must then take the VGPR form
PER_FILE = {"sdf.hip": ["-fno-slp-vectorize"], "heads_bwd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}
FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-I", os.path.join(REPO, "include"), "-I", CSRC]


def _compile(src, extra, tag=""):
    obj = os.path.join(CSRC, "build" + tag, os.path.splitext(src)[0] + ".o")
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    cmd = [HIPCC] + FLAGS + PER_FILE.get(src, []) + list(extra) + ["-c", os.path.join(CSRC, src), "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, res.stderr))
    return obj, res.stderr


def build(verbose=False, extra=(), out=None):
    """Compile + link; ``out``/``extra`` build an experiment variant (tools/, not the product)."""
    out = out or OUT
    tag = "" if out == OUT else "_" + os.path.splitext(os.path.basename(out))[0]
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [
        os.path.join(REPO, "include", "mli_hip.h")]
    if os.path.exists(out) and not extra and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        results = list(ex.map(lambda s: _compile(s, extra, tag), SOURCES))
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
