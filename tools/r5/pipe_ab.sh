# Prefetch pipeline / gate / depth configurations of the stage-b step, alternating on one box.
set -o pipefail
O=gpurun_out/r5/pipe
mkdir -p $O
for i in 1 2; do
  for cfg in "heads 2" "wgrad 2" "heads 1" "wgrad 1" "call 2"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 10 --pipeline $1 --prefetch-depth $2 > $O/${1}_${2}_$i.json 2> $O/${1}_${2}_$i.err || { echo "$cfg failed"; tail -3 $O/${1}_${2}_$i.err; exit 1; }
    echo "$1 $2 $i $(python -c "import json;d=json.load(open('$O/${1}_${2}_$i.json'));print(d['value'],d['ms_per_step'])")"
  done
done
