# Round-4 final measurement on one box: smoke, PMC HBM traffic (first, so the bench lines carry
# it), bench lines + rocprofv3 kernel stats (tools/measure.sh all), SQ counters of the step.
set -o pipefail
T=${FINAL_TAG:-r4/final}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
bash tools/pmc.sh $O/pmc || { echo pmc failed; exit 1; }
python tools/pmc_summary.py $O/pmc $O/pmc_summary.json > $O/pmc_summary.txt 2>&1 || { tail $O/pmc_summary.txt; exit 1; }
echo pmc ok
export MLI_PMC_SUMMARY=$O/pmc_summary.json
bash tools/measure.sh $T all || exit 1
bash tools/pmc_trio.sh $O/pmc_trio && python tools/sq_summary.py $O/pmc_trio $O/pmc_trio/summary.json > $O/pmc_trio/summary.txt 2>&1
echo final done
