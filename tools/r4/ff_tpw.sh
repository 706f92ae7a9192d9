set -o pipefail
O=gpurun_out/r4/ff_tpw
mkdir -p $O
timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_8.txt 2>&1 || { tail $O/kbench_8.txt; exit 1; }
grep "sdf field" $O/kbench_8.txt | sed 's/^/tpw8 /'
for t in 2 4 32; do
  MLI_HIP_LIB=xlib/ff$t.so timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_$t.txt 2>&1 || { tail $O/kbench_$t.txt; exit 1; }
  grep "sdf field" $O/kbench_$t.txt | sed "s/^/tpw$t /"
done
for t in 2 32; do
  MLI_HIP_LIB=xlib/ff$t.so timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 10 --field one > $O/train_$t.json 2> $O/train_$t.err || exit 1
  echo train tpw$t $(python -c "import json;d=json.load(open('$O/train_$t.json'));print(d['value'],d['ms_per_step'])")
done
timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 10 --field two > $O/train_two.json 2> $O/train_two.err || exit 1
echo train two $(python -c "import json;d=json.load(open('$O/train_two.json'));print(d['value'],d['ms_per_step'])")
