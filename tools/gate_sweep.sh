#!/bin/bash
# Prefetch-gate sweep (run on the box): bash tools/gate_sweep.sh <tag> [depth] [gates...]; alternates.
set -o pipefail
OUT=gpurun_out/$1
D=${2:-1}
shift 2
G="${*:-heads wgrad call off}"
mkdir -p "$OUT"
for rep in 1 2; do
  for g in $G; do
    timeout -k 10 120 python bench.py --no-cpu --steps 300 --pipeline $g --prefetch-depth $D > "$OUT/gate_${g}_d$D.json" 2> "$OUT/gate_${g}_d$D.err" || { echo "gate $g failed"; exit 1; }
    echo "gate $g depth $D: $(python -c "import json; d=json.load(open('$OUT/gate_${g}_d$D.json')); print(d['value'], d['ms_per_step'])")"
  done
done
