# Round-5 final, part 1: GPU suite + smoke + bench (suite_bench.sh), the HBM PMC passes and the SQ trio.
set -o pipefail
export TMPDIR=/tmp
TAG=final bash tools/r5/suite_bench.sh || exit 1
O=gpurun_out/r5/final
bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
python tools/pmc_summary.py $O/pmc $O/pmc_summary.json > $O/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
head -12 $O/pmc_summary.txt
bash tools/pmc_trio.sh $O/trio > $O/trio.log 2>&1 && python tools/sq_summary.py $O/trio $O/trio/summary.json > $O/trio/summary.txt 2>&1
echo "trio rc=$?"; head -8 $O/trio/summary.txt
