#!/bin/bash
# One GPU measurement pass (run on the box): bench lines + rocprofv3 kernel stats.
#   bash tools/measure.sh <tag> [b|a|infer|all]
# Outputs under gpurun_out/<tag>/ (copy the summaries to profiles/ afterwards).
set -o pipefail
TAG=${1:-run}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed rc=$?"; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['unit'], d['ms_per_step'], 'ms/step', 'roof', d['roofline']['kernel'], d['roofline']['frac'])")"
}
prof() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$name" -o run -- python bench.py --no-cpu "$@" \
    > "$OUT/prof_$name.log" 2>&1 || { echo "prof $name failed rc=$?"; return 1; }
  find "$OUT/prof_$name" -name "*kernel_stats.csv" -exec cp {} "$OUT/${name}_kernel_stats.csv" \;
  find "$OUT/prof_$name" -name "*kernel_trace.csv" -exec cp {} "$OUT/${name}_kernel_trace.csv" \;
  echo "prof $name ok"
}
if [ "$WHAT" = b ] || [ "$WHAT" = all ]; then
  run bench_b 300 && prof b 200 --steps 10 --warmup 3 || exit 1
fi
if [ "$WHAT" = a ] || [ "$WHAT" = all ]; then
  run bench_a 400 --config syn_hotdog_a --cpu-rays 256 --cpu-steps 3 && prof a 200 --config syn_hotdog_a --steps 10 --warmup 3 || exit 1
fi
if [ "$WHAT" = infer ] || [ "$WHAT" = all ]; then
  run bench_infer 400 --mode infer --frames 3 --warmup 1 || exit 1
fi
if [ "$WHAT" = vis ] || [ "$WHAT" = all ]; then
  run bench_infer_vis 400 --mode infer --vis --frames 3 --warmup 1 --no-cpu || exit 1
fi
if [ "$WHAT" = pikachu ] || [ "$WHAT" = all ]; then
  run bench_pikachu 300 --config NRHints_Pikachu_b --rays 8192 --fine 32 --no-cpu || exit 1
fi
