#!/bin/bash
# A/B of an environment switch (run on the box): bash tools/env_ab.sh <tag> <VAR=value> [bench args]
set -o pipefail
OUT=gpurun_out/$1
SW=$2
shift 2
mkdir -p "$OUT"
for rep in 1 2; do
  for arm in base switch; do
    if [ $arm = switch ]; then E="$SW"; else E="MLI_AB_NONE=1"; fi
    env $E timeout -k 10 120 python bench.py --no-cpu --steps 300 "$@" > "$OUT/${arm}_$rep.json" 2> "$OUT/${arm}_$rep.err" || { echo "$arm failed"; tail -3 "$OUT/${arm}_$rep.err"; exit 1; }
    echo "$arm ($E): $(python -c "import json; d=json.load(open('$OUT/${arm}_$rep.json')); print(d['value'], d['ms_per_step'], d['kernels'].get('mli_dw4', {}).get('ms_per_launch'))")"
  done
done
