set -o pipefail
O=gpurun_out/r5/decomp
mkdir -p $O
MLI_MARGINS_OUT=$O/margins.json timeout -k 10 300 python -u -m pytest tests/test_gpu_grad_decomp.py -v -s --timeout 200 --timeout-method thread > $O/decomp.log 2>&1
echo "decomp rc=$?"; grep -E "leg|passed|failed|Error|assert" $O/decomp.log | tail -12
bash tools/r5/ab_trio.sh
