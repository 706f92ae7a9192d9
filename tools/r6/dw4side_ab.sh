#!/bin/bash
# mli_dw4 on a side stream beside rgb_bwd (MLI_DW4_SIDE=1) against in line between rgb_bwd and
# BIG (0): the PQ / dW tests, the step alternating, one kernel trace.  bash tools/r6/dw4side_ab.sh
set -o pipefail
O=gpurun_out/r6/dw4side; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pq.py tests/test_gpu_dropin.py tests/test_gpu_determinism.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for i in 1 2 3; do
  for v in 0 1; do
    MLI_DW4_SIDE=$v timeout -k 10 150 python bench.py --no-cpu --steps 300 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { echo "bench $v failed"; tail -3 $O/bench_${v}_$i.err; exit 1; }
    echo "bench $i side=$v $(python -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
MLI_DW4_SIDE=1 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/prof -o run -- python bench.py --no-cpu --steps 10 --warmup 3 --no-kernel-timing > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/side_kernel_trace.csv \;
