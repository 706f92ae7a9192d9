#!/bin/bash
# EXPERIMENT: stage-b bench with the W64 heads forward (env MLI_W64 on an experiment library),
# alternating with the library's product kernel.  bash tools/w64_sweep.sh <tag> <lib> [bench args]
set -o pipefail
OUT=gpurun_out/$1
LIB=$2
shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  for arm in base 2 1 22 21; do
    case $arm in
      base) E="MLI_AB_NONE=1" ;;
      2|1) E="MLI_W64=$arm" ;;
      22) E="MLI_W64=2 MLI_W64B=2" ;;
      21) E="MLI_W64=2 MLI_W64B=1" ;;
    esac
    env $E timeout -k 10 150 python tools/ab_run.py "$LIB" --no-cpu --steps 300 "$@" > "$OUT/${arm}_$rep.json" 2> "$OUT/${arm}_$rep.err" || { echo "$arm failed"; tail -3 "$OUT/${arm}_$rep.err"; exit 1; }
    python - "$OUT/${arm}_$rep.json" "$arm" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d.get("kernels", {})
ks = " ".join("%s=%.3f" % (n.replace("mli_", ""), v["ms_per_launch"]) for n, v in k.items() if n in
              ("mli_rgb_fwd", "mli_rgb_bwd", "mli_wgrad"))
print("W64=%-5s %12.1f %s  %8.3f ms  %s" % (sys.argv[2], d["value"], d["unit"], d["ms_per_step"], ks))
PY
  done
done
