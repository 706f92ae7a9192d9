#!/bin/bash
# CU-mask experiment (run on the box): the stage-b step with the prefetch stream (and optionally
# the step's stream) restricted to CU subsets.  bash tools/cu_sweep.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-cu}
shift
mkdir -p "$OUT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 120 python bench.py --no-cpu --steps 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed rc=$?"; tail -3 "$OUT/$name.err"; return 1; }
  echo "$name: $(python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'])")"
}
run base0 || exit 1
for spec in "$@"; do
  [ -z "$spec" ] && continue
  name=$(echo "$spec" | tr ' :-' '___')
  run "$name" $spec || exit 1
done
run base1 || exit 1
