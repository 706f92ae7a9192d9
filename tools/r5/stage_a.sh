# Stage-a checks + measurement on one box: the stage-a / wgrad / parity GPU tests, then bench a
# with and without the side-stream table-gradient zeroing (alternating), then a kernel profile.
#   TAG=name bash tools/r5/stage_a.sh
set -o pipefail
O=gpurun_out/r5/${TAG:-stage_a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stage_a.py \
  tests/test_gpu_kernels.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for z in 1 0; do
    MLI_TABLE_ZERO_OVERLAP=$z timeout -k 10 300 python bench.py --config syn_hotdog_a --no-cpu --steps 40 --warmup 5 \
      > $O/a_z${z}_$i.json 2> $O/a_z${z}_$i.err || { echo "bench a z$z failed"; tail -3 $O/a_z${z}_$i.err; exit 1; }
    echo "z$z $i $(python -c "import json;d=json.load(open('$O/a_z${z}_$i.json'));print(d['value'],d['ms_per_step'])")"
  done
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_a -o run -- python bench.py --no-cpu --config syn_hotdog_a \
  --steps 10 --warmup 3 > $O/prof_a.log 2>&1 || { echo "prof a failed"; exit 1; }
find $O/prof_a -name "*kernel_stats.csv" -exec cp {} $O/a_kernel_stats.csv \;
python - <<PY
import csv
rows = list(csv.DictReader(open("$O/a_kernel_stats.csv")))
for r in rows[:16]:
    print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6 / 13, 3), "ms/step (13 steps)")
PY
