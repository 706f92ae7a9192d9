#!/bin/bash
# Prefetch-gate sweep (run on the box): bash tools/gate_sweep.sh <tag>; alternates the gates.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
for g in heads wgrad call off heads wgrad call off; do
  timeout -k 10 120 python bench.py --no-cpu --steps 300 --pipeline $g > "$OUT/gate_$g.json" 2> "$OUT/gate_$g.err" || { echo "gate $g failed"; exit 1; }
  echo "gate $g: $(python -c "import json; d=json.load(open('$OUT/gate_$g.json')); print(d['value'], d['ms_per_step'])")"
done
