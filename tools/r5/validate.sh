# Suite + smoke + bench on the tree, then the SQ/HBM trio and a kernel-trace profile of the step.
set -o pipefail
T=${TAG:-validate}
TAG=$T bash tools/r5/suite_bench.sh || exit 1
O=gpurun_out/r5/$T/trio
bash tools/pmc_trio.sh $O > $O.log 2>&1 && python tools/sq_summary.py $O $O/summary.json > $O/summary.txt 2>&1
echo "trio rc=$?"; head -8 $O/summary.txt
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r5/$T/prof_b -o run -- python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/r5/$T/prof_b.log 2>&1 || { echo prof failed; exit 1; }
f=$(find gpurun_out/r5/$T/prof_b -name "*kernel_trace.csv" | head -1); python tools/timeline.py $f 8 > gpurun_out/r5/$T/timeline.txt; tail -40 gpurun_out/r5/$T/timeline.txt
