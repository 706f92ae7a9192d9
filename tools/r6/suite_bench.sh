#!/bin/bash
# GPU suite (margins recorded), smoke, the default bench line and the stage-a line on the tree.
#   TAG=name [PRE="cmd"] bash tools/r6/suite_bench.sh
set -o pipefail
O=gpurun_out/r6/${TAG:-suite}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$PRE" ]; then bash -c "$PRE" || { echo "pre failed"; exit 1; }; fi
MLI_MARGINS_OUT=$O/margins.json timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $O/suite.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d.get('hbm_peak_gib'),{n:round(v['ms_per_launch'],3) for n,v in d.get('kernels',{}).items()})"
timeout -k 10 300 python bench.py --config syn_hotdog_a --no-cpu > $O/bench_a.json 2> $O/bench_a.err || { echo bench a failed; tail $O/bench_a.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_a.json'));print('stage a', d['value'],d['ms_per_step'])"
