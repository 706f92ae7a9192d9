# GPU suite (margins recorded), smoke, and the default bench line on the current tree.
#   TAG=name bash tools/r5/suite_bench.sh
set -o pipefail
O=gpurun_out/r5/${TAG:-suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -x -v -s --timeout 100 --timeout-method thread > $O/kernels.log 2>&1
rc=$?
echo "kernels rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/kernels.log | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
MLI_MARGINS_OUT=$O/margins.json timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d.get('hbm_peak_gib'),{n:round(v['ms_per_launch'],3) for n,v in d.get('kernels',{}).items()})"
