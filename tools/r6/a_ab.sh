#!/bin/bash
# Stage-a A/B: experiment library X against the product -- stage-a GPU tests on the product, then
# the stage-a bench line alternating.   X=hbold bash tools/r6/a_ab.sh
set -o pipefail
O=gpurun_out/r6/a_ab_$X; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_stage_a.py tests/test_gpu_determinism.py} > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for i in 1 2 3; do
  for v in prod $X; do
    if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
    timeout -k 10 200 python bench.py --no-cpu --config syn_hotdog_a --steps 100 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { echo "bench $v failed"; tail -3 $O/bench_${v}_$i.err; exit 1; }
    echo "bench a $i $v $(python -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); k=d['kernels']; print(d['value'], d['ms_per_step'])")"
  done
done
