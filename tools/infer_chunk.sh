#!/bin/bash
# Inference chunk-size sweep (run on the box): bash tools/infer_chunk.sh <tag> <chunk> ...
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for c in "$@"; do
  timeout -k 10 150 python bench.py --no-cpu --mode infer --frames 2 --warmup 1 --chunk "$c" > "$OUT/infer_$c.json" 2> "$OUT/infer_$c.err" || { echo "chunk $c failed"; tail -3 "$OUT/infer_$c.err"; exit 1; }
  echo "chunk $c: $(python -c "import json; d=json.load(open('$OUT/infer_$c.json')); print(d['value'], d['ms_per_step'])")"
done
