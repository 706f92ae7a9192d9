#!/bin/bash
# Stream-priority A/B on the current step (the small critical-path kernels dw4 / wgrad_reduce
# stretch 4x beside the prefetched geometry in the round-6 timeline).  bash tools/r6/prio_ab.sh
set -o pipefail
O=gpurun_out/r6/prio; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for p in none main; do
    timeout -k 10 150 python bench.py --no-cpu --steps 300 --priority $p > $O/$p$i.json 2> $O/$p$i.err || { echo "$p failed"; tail -3 $O/$p$i.err; exit 1; }
    echo "$p $i $(python -c "import json; d=json.load(open('$O/$p$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/prof_main -o run -- python bench.py --no-cpu --steps 10 --warmup 3 --priority main --no-kernel-timing > $O/prof_main.log 2>&1 || { echo prof failed; exit 1; }
find $O/prof_main -name "*kernel_trace.csv" -exec cp {} $O/main_kernel_trace.csv \;
