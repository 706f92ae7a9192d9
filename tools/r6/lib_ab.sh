#!/bin/bash
# Experiment library against the product: bit-identity of the sampler / field outputs (dumps in
# /tmp on the box), GPU tests on the experiment library, kbench and the step alternating.
#   X=pk0 TESTS="tests/test_gpu_field.py ..." bash tools/r6/lib_ab.sh
set -o pipefail
O=gpurun_out/r6/ab_$X; mkdir -p $O
export TMPDIR=/tmp
run_lib() { if [ "$1" = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$1.so; fi; }
for v in prod $X; do
  run_lib $v
  timeout -k 10 200 python tools/kbench.py --reps 3 --dump /tmp/dump_$v.pt > $O/dump_$v.txt 2>&1 || { echo "dump $v failed"; tail -5 $O/dump_$v.txt; exit 1; }
done
python - <<PY || exit 1
import torch
a, b = torch.load("/tmp/dump_prod.pt"), torch.load("/tmp/dump_$X.pt")
print("bit-identical:", {k: bool(torch.equal(a[k], b[k])) for k in a})
PY
run_lib $X
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_field.py} > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for i in 1 2; do
  for v in prod $X; do
    run_lib $v
    timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_${v}_$i.txt 2>&1 || { echo "kbench $v failed"; exit 1; }
    echo "== $i $v $(grep -E "field|sample|heads fwd|backward" $O/kbench_${v}_$i.txt | tr -s ' ' | tr '\n' ' ')"
  done
done
for i in 1 2 3; do
  for v in prod $X; do
    run_lib $v
    timeout -k 10 150 python bench.py --no-cpu --steps 300 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { echo "bench $v failed"; tail -3 $O/bench_${v}_$i.err; exit 1; }
    echo "bench $i $v $(python -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
for v in prod $X; do
  run_lib $v
  timeout -k 10 200 python bench.py --no-cpu --config syn_hotdog_a > $O/bench_a_$v.json 2> $O/bench_a_$v.err || { echo "bench a $v failed"; tail -3 $O/bench_a_$v.err; exit 1; }
  echo "bench a $v $(python -c "import json; d=json.load(open('$O/bench_a_$v.json')); print(d['value'], d['ms_per_step'])")"
done
