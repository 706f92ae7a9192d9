# Alternating bench A/B of an environment switch on one box (the in-tree library):
#   AB_TAG=name AB_VAR=MLI_X AB_VALS="0 1" [AB_ROUNDS=2] [AB_A=1] bash tools/r5/env_ab.sh
set -o pipefail
O=gpurun_out/r5/${AB_TAG:-env_ab}
mkdir -p $O
for v in $AB_VALS; do
  env $AB_VAR=$v timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_$v.txt 2>&1 || { echo "kbench $v failed"; tail -5 $O/kbench_$v.txt; exit 1; }
  echo "== kbench $AB_VAR=$v"; grep -E "heads|backward|wgrad" $O/kbench_$v.txt
done
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in $AB_VALS; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 10 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { echo "b $v failed"; tail -3 $O/b_${v}_$i.err; exit 1; }
    echo "b $v $i $(python -c "import json;d=json.load(open('$O/b_${v}_$i.json'));k=d.get('kernels',{});print(d['value'],d['ms_per_step'],{n:round(v['ms_per_launch'],3) for n,v in k.items() if 'wgrad' in n})")"
    if [ "${AB_A:-0}" = 1 ]; then
      env $AB_VAR=$v timeout -k 10 300 python bench.py --config syn_hotdog_a --no-cpu --steps 40 --warmup 5 > $O/a_${v}_$i.json 2> $O/a_${v}_$i.err || { echo "a $v failed"; tail -3 $O/a_${v}_$i.err; exit 1; }
      echo "a $v $i $(python -c "import json;d=json.load(open('$O/a_${v}_$i.json'));print(d['value'],d['ms_per_step'])")"
    fi
  done
done
