"""Knock-out variants of the fused heads backward (experiment tooling, not the product).

Builds libmli_hip.so variants into xlib/ from text patches of mli_nerf_amd/csrc/heads_bwd.hip
(the product source stays free of experiment branches), then -- on the GPU box -- times
mli_heads_bwd in bench.py with each (MLI_HIP_LIB=...).

    python tools/hb_variants.py build [names...]     # here (hipcc cross-compiles)
    python tools/hb_variants.py run [names...]       # on the GPU box (gpurun)
"""
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from mli_nerf_amd import build as B  # noqa: E402

SRC = "heads_bwd.hip"

# name -> list of (old, new) text patches of heads_bwd.hip
VARIANTS = {
    "base": [],
    # no dW MFMAs: the chain, DMA and staging alone
    "no_dw": [('  asm("s_nop 1\\n\\t"\n      "v_mfma_f32_32x32x16_f16 %0, %2, %4, %0\\n\\t"',
               '  if (0) asm("s_nop 1\\n\\t"\n      "v_mfma_f32_32x32x16_f16 %0, %2, %4, %0\\n\\t"')],
    # no chain MFMAs (zeros): DMA, staging and dW
    "no_chain": [("    for (int i = 0; i < PF; ++i) acc = mfma32(buf[g & 1][i], in[g * PF + i], acc);",
                  "    for (int i = 0; i < PF; ++i) if (i > 99) acc = mfma32(buf[g & 1][i], in[g * PF + i], acc);")],
    # no weight-chunk DMAs at all (stale weights; DMA issue-cost probe)
    "no_ringdma": [("  for (int u = 0; u < RING_OPS; ++u) glds16(src + (2 * u + rw) * 1024 + k.lane * 16, dst + (2 * u + rw) * 1024);",
                    "  for (int u = 0; u < RING_OPS; ++u) if (rw > 7) glds16(src + (2 * u + rw) * 1024 + k.lane * 16, dst + (2 * u + rw) * 1024);")],
    # no dZ^T staging writes to LDS
    "no_stage": [("    *reinterpret_cast<uint16_t*>(sb + ((i & 3) + 8 * (i >> 2)) * SROW) = __builtin_bit_cast(uint16_t, x);",
                  "    if (i > 99) *reinterpret_cast<uint16_t*>(sb + ((i & 3) + 8 * (i >> 2)) * SROW) = __builtin_bit_cast(uint16_t, x);")],
    # no X DMAs (stale X)
    "no_xdma": [("    glds16(base + (size_t)(64 * ws + 4 * u) * k.S + lo[u & 3], k.lds + M.x + ws * XW + u * 1024);",
                 "    if (ii > 99) glds16(base + (size_t)(64 * ws + 4 * u) * k.S + lo[u & 3], k.lds + M.x + ws * XW + u * 1024);")],
    # no chain AND no dW MFMAs
    "no_mfma": [("    for (int i = 0; i < PF; ++i) acc = mfma32(buf[g & 1][i], in[g * PF + i], acc);",
                 "    for (int i = 0; i < PF; ++i) if (i > 99) acc = mfma32(buf[g & 1][i], in[g * PF + i], acc);"),
                ('  asm("s_nop 1\\n\\t"\n      "v_mfma_f32_32x32x16_f16 %0, %2, %4, %0\\n\\t"',
                 '  if (0) asm("s_nop 1\\n\\t"\n      "v_mfma_f32_32x32x16_f16 %0, %2, %4, %0\\n\\t"')],
    # only one layer's workgroups do work (the others return at once): per-layer timing
    "only_l1": [("  const bool load = k.wave >= 2;\n", "  const bool load = k.wave >= 2;\n  if (L != 1) return;\n")],
    "only_l2": [("  const bool load = k.wave >= 2;\n", "  const bool load = k.wave >= 2;\n  if (L != 2) return;\n")],
    "only_l3": [("  const bool load = k.wave >= 2;\n", "  const bool load = k.wave >= 2;\n  if (L != 3) return;\n")],
    # every wave drains its queue at the end of every phase (counted-wait check)
    "wait0": [("MLI_FI void vm_wait63(int n) {\n  switch (n) {", "MLI_FI void vm_wait63(int n) {\n  n = 0;\n  switch (n) {")],
    # weight chunks DMA'd by waves 0-1 only (8 pieces each), every wave drains every phase
    "ring2_wait0": [("MLI_FI void vm_wait63(int n) {\n  switch (n) {", "MLI_FI void vm_wait63(int n) {\n  n = 0;\n  switch (n) {"),
                    ("constexpr int RING_OPS = WCH / 1024 / 4; ", "constexpr int RING_OPS = WCH / 1024 / 2; "),
                    ("    const int piece = 4 * u + k.wave;\n    glds16(", "    const int piece = 2 * u + k.wave;\n    if (k.wave < 2) glds16(")],
    # mlp.hip stager: no LDS staging writes / no flush (heads forward + rgb_bwd; timing only)
    "mlp_no_stagew": [("mlp.hip", "    *reinterpret_cast<uint16_t*>(sb + ((i & 3) + 8 * (i >> 2)) * SROW) = __builtin_bit_cast(uint16_t, x);",
                       "    if (i > 99) *reinterpret_cast<uint16_t*>(sb + ((i & 3) + 8 * (i >> 2)) * SROW) = __builtin_bit_cast(uint16_t, x);")],
    "mlp_no_flush": [("mlp.hip", "    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(g + u * step));",
                      "    if (u > 99) __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(g + u * step));")],
    # transposed stager: no b64 staging writes / no tr reads in the flush (timing only)
    "tst_no_w": [("mlp.hip", "    *reinterpret_cast<half4*>(row + (((2 * g + h) ^ sswz(s)) << 3)) = x;",
                  "    if (g > 99) *reinterpret_cast<half4*>(row + (((2 * g + h) ^ sswz(s)) << 3)) = x;")],
    "tst_no_r": [("mlp.hip", "    const half4 a = ds_read_tr16(sb + 1024 * NW * u + l0);\n    const half4 b = ds_read_tr16(sb + 1024 * NW * u + l1);",
                  "    const half4 a = {}; const half4 b = {};")],
    "tst_no_wr": [("mlp.hip", "    *reinterpret_cast<half4*>(row + (((2 * g + h) ^ sswz(s)) << 3)) = x;",
                   "    if (g > 99) *reinterpret_cast<half4*>(row + (((2 * g + h) ^ sswz(s)) << 3)) = x;"),
                  ("mlp.hip", "    const half4 a = ds_read_tr16(sb + 1024 * NW * u + l0);\n    const half4 b = ds_read_tr16(sb + 1024 * NW * u + l1);",
                   "    const half4 a = {}; const half4 b = {};")],
    "tst_no_flush": [("mlp.hip", "    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, x),",
                      "    if (u > 99) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, x),")],
    # mlp.hip flush: plain (write-back) stores instead of non-temporal
    "flush_plain": [("mlp.hip", "    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(g + u * step));",
                     "    *reinterpret_cast<u32x4*>(g + u * step) = x;")],
    # the RING waves do not wait for the next weight chunk (wrong results; latency probe)
    "no_ringwait": [("        if (ROLE == RING) vm_wait63(RING_OPS * (DIST - 1));",
                     "        if (ROLE == RING) {}")],
    # no s_barrier in the phase loop (wrong results; synchronisation probe)
    "no_barrier": [("        block_sync();\n        cur++;", "        asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");\n        cur++;")],
}


def build_variant(name):
    src_dir = os.path.join(REPO, "xlib", name, "csrc")
    if os.path.exists(src_dir):
        shutil.rmtree(src_dir)
    shutil.copytree(B.CSRC, src_dir, ignore=shutil.ignore_patterns("build*"))
    for patch in VARIANTS[name]:
        fname, old, new = patch if len(patch) == 3 else (SRC,) + tuple(patch)
        p = os.path.join(src_dir, fname)
        s = open(p).read()
        if s.count(old) == 0:
            raise SystemExit("%s: patch not found: %r" % (name, old[:60]))
        open(p, "w").write(s.replace(old, new))
    objs = []
    for f in B.SOURCES:
        obj = os.path.join(src_dir, os.path.splitext(f)[0] + ".o")
        cmd = [B.HIPCC] + B.FLAGS[:-2] + ["-I", src_dir] + B.PER_FILE.get(f, []) + ["-c", os.path.join(src_dir, f),
                                                                                  "-o", obj]
        subprocess.run(cmd, check=True, capture_output=True)
        objs.append(obj)
    out = os.path.join(REPO, "xlib", name, "libmli_hip.so")
    subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
    for o in objs:
        os.remove(o)
    print("built", out)


def run_variant(name, extra):
    env = dict(os.environ, MLI_HIP_LIB=os.path.join(REPO, "xlib", name, "libmli_hip.so"))
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "30", "--warmup", "3", "--no-cpu",
           "--pipeline", "off"] + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(name, "FAILED", r.stderr[-2000:])
        return None
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ks = {n: round(v["ms_per_launch"], 4) for n, v in d["kernels"].items()
          if n in ("mli_heads_bwd", "mli_rgb_fwd", "mli_rgb_bwd", "mli_wgrad:big")}
    print(json.dumps({"variant": name, "extra": " ".join(extra), "ms_step": d["ms_per_step"], "kernels": ks}), flush=True)
    return d


if __name__ == "__main__":
    what = sys.argv[1]
    names = [a for a in sys.argv[2:] if not a.startswith("--")] or list(VARIANTS)
    extra = [a for a in sys.argv[2:] if a.startswith("--")]
    extra = [x for e in extra for x in e.split("=", 1)]
    for n in names:
        if what == "build":
            build_variant(n)
        else:
            run_variant(n, extra)
