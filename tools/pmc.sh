#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, per MI355X_MICROARCH.md "rocprofv3 PMC
# slots"): HBM bytes (FETCH_SIZE, WRITE_SIZE in separate passes) and L2 hit/miss, over a
# short training bench.  Usage (GPU box): bash tools/pmc.sh [outdir] [extra bench.py args]
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu --no-kernel-timing --steps 3 --warmup 2 ${2:-}"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- python bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- python bench.py $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d "$OUT/l2" -o run -- python bench.py $ARGS > "$OUT/l2.log" 2>&1
