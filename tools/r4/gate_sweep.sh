# Prefetch gate / depth sweep on the current tree (bench flags only), alternating.
set -o pipefail
O=gpurun_out/r4/gate
mkdir -p $O
for i in 1 2; do
  for cfg in "heads 2" "wgrad 2" "call 2" "heads 1"; do
    set -- $cfg
    tag=${1}_d${2}_$i
    timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 10 --pipeline $1 --prefetch-depth $2 > $O/$tag.json 2> $O/$tag.err || { tail -3 $O/$tag.err; exit 1; }
    echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['ms_per_step'])")"
  done
done
