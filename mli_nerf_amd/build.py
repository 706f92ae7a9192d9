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
# No SLP packing of scalar fp32 math in the MFMA and geometry kernels: v_pk_*_f32 beside MFMAs
# costs more than the two scalar ops it replaces (MI355X_MICROARCH.md, 'price of one filler') and
# its even-aligned register pairs raise the VGPR count (field_mlp 167 -> 118).
# rays.hip / params.hip (VALU-only sampling, AdamW) keep it.
PER_FILE = {s: ["-fno-slp-vectorize"] for s in ("sdf.hip", "mlp_fwd.hip", "mlp_fwd_pq.hip", "mlp_fwd_train.hip",
                                                 "mlp_bwd.hip", "mlp_geo.hip", "wgrad.hip", "loss.hip")}
FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-I", os.path.join(REPO, "include"), "-I", CSRC]
# the device assembly of every file stays next to its object (-save-temps=obj), so that build()
# can audit the inline-asm memory operations of the library it just built (tools/asm_audit.py)
TEMPS = ["-save-temps=obj"]


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
    h.update(repr((rel, TEMPS, sorted(PER_FILE.items()))).encode())
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


def _object_key(src, cmd):
    """What one object is built from: its source, every header of the library (a header change
    rebuilds every object) and its compile command (params.hip's embeds the library hash)."""
    h = hashlib.sha256()
    for d in [os.path.join(CSRC, src)] + [d for d in _deps() if d.endswith(".h")]:
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(repr([os.path.relpath(c, REPO) if os.path.isabs(c) else c for c in cmd]).encode())
    return h.hexdigest()


def _compile(src, extra, tag="", digest=""):
    obj = os.path.join(CSRC, "build" + tag, os.path.splitext(src)[0] + ".o")
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    cmd = [HIPCC] + FLAGS + TEMPS + PER_FILE.get(src, []) + list(extra) + [
        '-DMLI_SOURCE_HASH="%s"' % digest, "-c", os.path.join(CSRC, src), "-o", obj]
    key = _object_key(src, cmd)
    stamp = obj + ".key"
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == key:
        return obj, ""   # built from exactly this source, these headers and this command
    res = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.dirname(obj))
    if res.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, res.stderr))
    with open(stamp, "w") as f:
        f.write(key)
    return obj, res.stderr


def build(verbose=False, extra=(), out=None):
    """Compile + link; ``out``/``extra`` build an experiment variant (tools/, not the product)."""
    out = out or OUT
    tag = "" if out == OUT else "_" + os.path.splitext(os.path.basename(out))[0]
    digest = source_hash()
    if not extra and built_hash(out) == digest:  # built from exactly these sources and flags
        findings = audit_asm(os.path.join(CSRC, "build")) if os.path.isdir(os.path.join(CSRC, "build")) else []
        if findings:
            raise RuntimeError("asm audit of the device assembly found %d hazard(s):\n%s" % (
                len(findings), "\n".join(findings[:20])))
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
    findings = audit_asm(os.path.dirname(objs[0]))
    if findings and not extra:
        os.remove(out)   # never leave a library whose counted waits do not hold
        raise RuntimeError("asm audit of the device assembly found %d hazard(s):\n%s" % (
            len(findings), "\n".join(findings[:20])))
    return out


def audit_asm(build_dir):
    """tools/asm_audit.py over the device assembly of a build directory: a compiler instruction
    naming an inline-asm load's destination while that load may be in flight, or an asm 16 B store
    without its s_nop.  Returns the findings (empty: clean)."""
    import importlib.util
    import io
    spec = importlib.util.spec_from_file_location("asm_audit", os.path.join(REPO, "tools", "asm_audit.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    found = []
    for f in sorted(os.listdir(build_dir)):
        if f.endswith("-hip-amdgcn-amd-amdhsa-gfx950.s"):
            buf = io.StringIO()
            if mod.audit(os.path.join(build_dir, f), out=buf):
                found += buf.getvalue().strip().split("\n")
    return found


if __name__ == "__main__":
    extra = sys.argv[1:]
    print(build(verbose=True, extra=extra))
