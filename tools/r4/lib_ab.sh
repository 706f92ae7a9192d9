# Alternating bench A/B of experiment libraries (MLI_HIP_LIB) against the in-tree library.
#   AB_TAG=name AB_LIBS="v1 v2" AB_ARGS="..." bash tools/r4/lib_ab.sh
set -o pipefail
O=gpurun_out/r4/${AB_TAG:-lib_ab}
mkdir -p $O
ROUNDS=${AB_ROUNDS:-2}
for i in $(seq 1 $ROUNDS); do
  for v in prod $AB_LIBS; do
    if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu ${AB_ARGS:---steps 40 --warmup 10} > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v failed"; tail -3 $O/${v}_$i.err; exit 1; }
    echo "$v $i $(python -c "import json;d=json.load(open('$O/${v}_$i.json'));k=d.get('kernels',{});print(d['value'],d['ms_per_step'],{n:round(v['ms_per_launch'],3) for n,v in k.items() if 'wgrad' in n or 'rgb' in n or 'sdf' in n})")"
  done
done
unset MLI_HIP_LIB
