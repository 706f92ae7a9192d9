#!/bin/bash
# Gather variants: encoding parity of each experiment library, then kbench FIELD / sampling and
# the TCP / TA counter passes, alternating.  AB_LIBS="v2 v4" bash tools/r6/gather_ab2.sh
set -o pipefail
O=gpurun_out/r6/${AB_TAG:-gather_ab2}
mkdir -p $O
for v in $AB_LIBS; do
  MLI_HIP_LIB=xlib/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_field.py > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $O/tests_$v.log)"
done
for i in 1 2; do
for v in base prod $AB_LIBS; do
  if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
  timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_${v}_$i.txt 2>&1 || { echo "kbench $v failed"; tail -5 $O/kbench_${v}_$i.txt; exit 1; }
  echo "== $i $v $(grep -E "field|sample" $O/kbench_${v}_$i.txt | tr -s ' ' | tr '\n' ' ')"
done
done
for v in $AB_LIBS; do
  export MLI_HIP_LIB=xlib/$v.so
  bash tools/r6/pmc_gather.sh $O/pmc_$v || exit 1
done
unset MLI_HIP_LIB
