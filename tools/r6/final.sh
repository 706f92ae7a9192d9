#!/bin/bash
# Round-6 final records on the committed tree: GPU suite (margins) + smoke + the training bench
# lines (suite_bench.sh), then the HBM PMC passes, the SQ trio and the kernel --stats of the
# stage-b, stage-a and inference lines.  Outputs under gpurun_out/r6/final (copy to profiles/r6/final).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/final
TAG=final bash tools/r6/suite_bench.sh || exit 1
bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
python tools/pmc_summary.py $O/pmc $O/pmc_summary.json > $O/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
head -16 $O/pmc_summary.txt
bash tools/pmc_trio.sh $O/trio > $O/trio.log 2>&1 && python tools/sq_summary.py $O/trio $O/trio/summary.json > $O/trio/summary.txt 2>&1
echo "trio rc=$?"; head -8 $O/trio/summary.txt
bash tools/measure.sh r6/final/m all || exit 1
