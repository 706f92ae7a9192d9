# GPU suite, smoke, the inference and default training bench lines on the current tree.
set -o pipefail
O=gpurun_out/r5/${TAG:-final4}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/suite.log 2>&1 || { echo "suite failed"; tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py --mode infer --frames 3 --warmup 1 --no-cpu > $O/bench_infer.json 2> $O/bench_infer.err || { echo "infer failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_infer.json'));print('infer', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('train', d['value'], d['ms_per_step'])"
