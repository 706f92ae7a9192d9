set -o pipefail
mkdir -p gpurun_out/r5/c
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5/c/suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r5/c/suite.log; exit 1; }
tail -2 gpurun_out/r5/c/suite.log
AB_TAG=c AB_LIBS="oldheads" AB_ROUNDS=2 bash tools/r5/lib_ab.sh || exit 1
O=gpurun_out/r5/c
for i in 1 2; do
  for z in 1 0; do
    MLI_TABLE_ZERO_OVERLAP=$z timeout -k 10 300 python bench.py --config syn_hotdog_a --no-cpu --steps 40 --warmup 5 \
      > $O/a_z${z}_$i.json 2> $O/a_z${z}_$i.err || { echo "bench a z$z failed"; tail -3 $O/a_z${z}_$i.err; exit 1; }
    echo "a z$z $i $(python -c "import json;d=json.load(open('$O/a_z${z}_$i.json'));print(d['value'],d['ms_per_step'])")"
  done
done
