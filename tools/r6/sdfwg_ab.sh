#!/bin/bash
# sdf_kernel at 2 workgroups per CU (225 VGPRs, no AGPRs) against 1 (252 + 16 AGPRs: one wave
# per SIMD): bit-identity of the sampler / field outputs, the field parity tests, then kbench
# alternating.  bash tools/r6/sdfwg_ab.sh
set -o pipefail
O=gpurun_out/r6/sdfwg; mkdir -p $O
export TMPDIR=/tmp
for v in sdfwg1 sdfwg2; do
  MLI_HIP_LIB=xlib/$v.so timeout -k 10 200 python tools/kbench.py --reps 3 --dump $O/$v.pt > $O/dump_$v.txt 2>&1 || { echo "dump $v failed"; tail -5 $O/dump_$v.txt; exit 1; }
done
python - <<PY || exit 1
import torch
a, b = torch.load("$O/sdfwg1.pt"), torch.load("$O/sdfwg2.pt")
print("bit-identical:", {k: bool(torch.equal(a[k], b[k])) for k in a})
PY
MLI_HIP_LIB=xlib/sdfwg2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_field.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for i in 1 2; do
  for v in sdfwg1 sdfwg2; do
    MLI_HIP_LIB=xlib/$v.so timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_${v}_$i.txt 2>&1 || { echo "kbench $v failed"; exit 1; }
    echo "== $i $v $(grep -E "field|sample" $O/kbench_${v}_$i.txt | tr -s ' ' | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for v in sdfwg1 sdfwg2; do
    MLI_HIP_LIB=xlib/$v.so timeout -k 10 150 python bench.py --no-cpu --steps 300 > $O/bench_${v}_$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    echo "bench $i $v $(python -c "import json; d=json.load(open('$O/bench_${v}_$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
