#!/bin/bash
# Prefetch-depth A/B (run on the box): bash tools/depth_sweep.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
for d in 1 2 1 2; do
  timeout -k 10 120 python bench.py --no-cpu --steps 300 --prefetch-depth $d > "$OUT/depth_$d.json" 2> "$OUT/depth_$d.err" || { echo "depth $d failed"; tail -3 "$OUT/depth_$d.err"; exit 1; }
  echo "depth $d: $(python -c "import json; d=json.load(open('$OUT/depth_$d.json')); print(d['value'], d['ms_per_step'])")"
done
