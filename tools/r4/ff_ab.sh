set -o pipefail
mkdir -p gpurun_out/r4/ff
O=gpurun_out/r4/ff
MLI_MARGINS_OUT=$O/field_margins.json timeout -k 10 300 python -u -m pytest tests/test_gpu_field.py -v -s --timeout 200 --timeout-method thread > $O/field_test.log 2>&1
rc=$?
echo field tests rc=$rc; grep -E "passed|failed" $O/field_test.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { echo PARITY_FAIL; tail -30 $O/parity.log; exit 1; }
echo parity ok
for i in 1 2; do
  for f in one two; do
    timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 10 --field $f > $O/train_${f}_$i.json 2> $O/train_${f}_$i.err || { echo BENCH_FAIL $f; tail $O/train_${f}_$i.err; exit 1; }
    echo train $f $i $(python -c "import json;d=json.load(open('$O/train_${f}_$i.json'));print(d['value'],d['ms_per_step'],d.get('kernels',{}).get('mli_sdf:field',{}))")
  done
done
for f in one two; do
  timeout -k 10 300 python bench.py --no-cpu --mode infer --frames 2 --warmup 1 --field $f > $O/infer_${f}.json 2> $O/infer_${f}.err || { echo INFER_FAIL $f; tail $O/infer_${f}.err; exit 1; }
  echo infer $f $(python -c "import json;d=json.load(open('$O/infer_${f}.json'));print(d['value'],d['ms_per_step'],d.get('kernels',{}).get('mli_sdf:field',{}))")
done
