set -o pipefail
O=gpurun_out/r4/${AB_TAG:-pair}
mkdir -p $O
MLI_HIP_LIB=xlib/base.so timeout -k 10 120 python tools/r4/field_dump.py $O/base.pt > $O/dump_base.log 2>&1 || { tail $O/dump_base.log; exit 1; }
timeout -k 10 120 python tools/r4/field_dump.py $O/new.pt > $O/dump_new.log 2>&1 || { tail $O/dump_new.log; exit 1; }
python tools/r4/cmp_dump.py $O/base.pt $O/new.pt | tee $O/cmp.txt
rm -f $O/base.pt $O/new.pt
timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_new.txt 2>&1 || { tail $O/kbench_new.txt; exit 1; }
MLI_HIP_LIB=xlib/base.so timeout -k 10 200 python tools/kbench.py --reps 10 > $O/kbench_base.txt 2>&1 || exit 1
grep -E "sdf field|sample" $O/kbench_new.txt | sed 's/^/new  /'; grep -E "sdf field|sample" $O/kbench_base.txt | sed 's/^/base /'
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export MLI_HIP_LIB=xlib/base.so; else unset MLI_HIP_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 10 > $O/train_${v}_$i.json 2> $O/train_${v}_$i.err || { tail $O/train_${v}_$i.err; exit 1; }
    echo train $v $i $(python -c "import json;d=json.load(open('$O/train_${v}_$i.json'));print(d['value'],d['ms_per_step'],d['kernels']['mli_sdf:field']['ms_per_launch'])")
  done
done
unset MLI_HIP_LIB
for v in new base; do
  if [ $v = new ]; then unset MLI_HIP_LIB; else export MLI_HIP_LIB=xlib/$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu --mode infer --frames 2 --warmup 1 > $O/infer_$v.json 2> $O/infer_$v.err || { tail $O/infer_$v.err; exit 1; }
  echo infer $v $(python -c "import json;d=json.load(open('$O/infer_$v.json'));print(d['value'],d['ms_per_step'],d['kernels']['mli_sdf:field']['ms_per_unit'])")
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_new -o run -- python bench.py --no-cpu --no-kernel-timing --steps 10 --warmup 3 > $O/prof_new.log 2>&1 || { tail $O/prof_new.log; exit 1; }
MLI_HIP_LIB=xlib/base.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_base -o run -- python bench.py --no-cpu --no-kernel-timing --steps 10 --warmup 3 > $O/prof_base.log 2>&1 || { tail $O/prof_base.log; exit 1; }
for v in new base; do f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -E "encode5|field_mlp|sdf_kernel|rgb_fwd|rgb_bwd|wgrad_dma" $f | cut -d, -f1-4 | cut -c1-150; done
