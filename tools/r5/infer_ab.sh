# Inference bench A/B of experiment libraries against the in-tree library, alternating on one box.
#   AB_LIBS="v1 v2" [AB_ROUNDS=2] bash tools/r5/infer_ab.sh
set -o pipefail
O=gpurun_out/r5/${AB_TAG:-infer_ab}
mkdir -p $O
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in prod $AB_LIBS; do
    if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
    timeout -k 10 300 python bench.py --mode infer --frames 2 --warmup 1 --no-cpu > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v failed"; tail -3 $O/${v}_$i.err; exit 1; }
    echo "$v $i $(python -c "import json;d=json.load(open('$O/${v}_$i.json'));k=d.get('kernels',{});print(d['value'],d['ms_per_step'],{n:round(v['ms_per_launch'],3) for n,v in k.items() if 'rgb' in n or 'field' in n})")"
  done
done
unset MLI_HIP_LIB
