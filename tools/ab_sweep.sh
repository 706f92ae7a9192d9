#!/bin/bash
# A/B sweep (run on the box): bench.py against experiment libraries, alternating with the
# product build.  bash tools/ab_sweep.sh <tag> <mode: train|infer|a> <lib|base> ...
set -o pipefail
OUT=gpurun_out/$1
MODE=$2
shift 2
mkdir -p "$OUT"
case $MODE in
  train) ARGS="--no-cpu --steps 300" ;;
  infer) ARGS="--no-cpu --mode infer --frames 2 --warmup 1" ;;
  a) ARGS="--no-cpu --config syn_hotdog_a --steps 100" ;;
esac
i=0
for lib in "$@"; do
  i=$((i + 1))
  name="${i}_$(basename "$lib" .so)_$MODE"
  if [ "$lib" = base ]; then
    timeout -k 10 150 python bench.py $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  else
    timeout -k 10 150 python tools/ab_run.py "$lib" $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  fi
  rc=$?
  [ $rc -ne 0 ] && { echo "$name failed rc=$rc"; tail -3 "$OUT/$name.err"; exit 1; }
  python - "$OUT/$name.json" "$name" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
k = d.get("kernels", {})
ks = " ".join("%s=%.3f" % (n.replace("mli_", ""), v["ms_per_launch"]) for n, v in k.items() if n in
              ("mli_rgb_fwd", "mli_rgb_bwd", "mli_wgrad:big", "mli_wgrad:wide", "mli_wgrad"))
print("%-24s %12.1f %s  %8.3f ms  %s" % (sys.argv[2], d["value"], d["unit"], d["ms_per_step"], ks))
EOF
done
