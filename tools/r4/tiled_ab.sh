# GPU suite (margins recorded) on the tree, then the step / inference / stage-a bench A/B against
# the previous commit's tree exported to xbase/ (alternating on one box).
set -o pipefail
O=gpurun_out/r4/${AB_TAG:-tiled}
mkdir -p $O
export TMPDIR=/tmp
MLI_MARGINS_OUT=$O/margins.json timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python tools/act_report.py > $O/act_report.txt 2>&1; tail -8 $O/act_report.txt
b() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python bench.py --no-cpu "$@") > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -3 $O/$tag.err; return 1; }
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));k=d.get('kernels',{});print(d['value'],d['ms_per_step'],{n:round(v['ms_per_launch'],3) for n,v in k.items() if 'wgrad' in n or 'rgb' in n})")"
}
for i in 1 2; do
  b train_new_$i . --steps 40 --warmup 10 || exit 1
  b train_base_$i xbase --steps 40 --warmup 10 || exit 1
done
b a_new . --config syn_hotdog_a --steps 20 --warmup 5 || exit 1
b a_base xbase --config syn_hotdog_a --steps 20 --warmup 5 || exit 1
