# The GPU suite with every parity bar's measured margin recorded (MLI_MARGINS_OUT).
set -o pipefail
O=gpurun_out/r4/${SUITE_TAG:-suite}
mkdir -p $O
MLI_MARGINS_OUT=$O/margins.json timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | tail -6
exit $rc
