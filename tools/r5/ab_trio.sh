# wgrad DMA variants A/B, then the SQ / HBM counters of the step's kernels on the product tree.
set -o pipefail
AB_TAG=wgrad_dma AB_LIBS="noswz porder" AB_ROUNDS=1 bash tools/r5/lib_ab.sh || exit 1
O=gpurun_out/r5/trio
bash tools/pmc_trio.sh $O > $O.log 2>&1 && python tools/sq_summary.py $O $O/summary.json > $O/summary.txt 2>&1
echo "trio rc=$?"; head -8 $O/summary.txt
