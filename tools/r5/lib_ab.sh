# Alternating kernel + bench A/B of experiment libraries (MLI_HIP_LIB=xlib/<v>.so) against the
# in-tree library, one box.   AB_TAG=name AB_LIBS="v1 v2" [AB_ARGS="..."] bash tools/r5/lib_ab.sh
set -o pipefail
O=gpurun_out/r5/${AB_TAG:-lib_ab}
mkdir -p $O
ROUNDS=${AB_ROUNDS:-2}
for v in prod $AB_LIBS; do
  if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
  timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_$v.txt 2>&1 || { echo "kbench $v failed"; tail -5 $O/kbench_$v.txt; exit 1; }
  echo "== kbench $v"; grep -E "heads|backward|bwd|field|sample" $O/kbench_$v.txt
done
for i in $(seq 1 $ROUNDS); do
  for v in prod $AB_LIBS; do
    if [ $v = prod ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu ${AB_ARGS:---steps 40 --warmup 10} > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "$v failed"; tail -3 $O/${v}_$i.err; exit 1; }
    echo "$v $i $(python -c "import json;d=json.load(open('$O/${v}_$i.json'));k=d.get('kernels',{});print(d['value'],d['ms_per_step'],{n:round(v['ms_per_launch'],3) for n,v in k.items() if 'wgrad' in n or 'rgb' in n or 'sdf' in n})")"
  done
done
unset MLI_HIP_LIB
