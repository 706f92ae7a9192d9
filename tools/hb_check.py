import os, sys, subprocess
for v in sys.argv[1:]:
    env = dict(os.environ, MLI_HIP_LIB="xlib/%s/libmli_hip.so" % v)
    r = subprocess.run([sys.executable, "-m", "pytest", "tests/test_gpu_heads_bwd.py", "-x", "-q", "-s", "-k", "float64",
                        "--timeout", "200"], env=env, capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if "layer" in l or "bit-id" in l or "passed" in l or "failed" in l]
    print(v, "\n  " + "\n  ".join(lines))
