#!/bin/bash
# Round 6, hash-grid gathers: parity of the x-paired product kernels, then kbench and the
# TA / TCP counter passes of the product library against xlib/base.so (the round-5 kernels).
set -o pipefail
O=gpurun_out/r6/gather_ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_field.py tests/test_gpu_parity.py tests/test_gpu_pq.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests ok: $(grep -c PASSED $O/tests.log) passed"
for v in base prod; do
  if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
  timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_$v.txt 2>&1 || { echo "kbench $v failed"; tail -5 $O/kbench_$v.txt; exit 1; }
  echo "== kbench $v"; grep -E "field|sample" $O/kbench_$v.txt
done
for v in base prod; do
  if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
  bash tools/r6/pmc_gather.sh $O/pmc_$v || exit 1
done
unset MLI_HIP_LIB
