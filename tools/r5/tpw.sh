# Two tiles per wave in the heads forward: micro-benchmark, the forward's GPU tests on the
# product (MLI_FWD_TPW=2), then the A/B against xlib/tpw1 (one tile per wave).
set -o pipefail
O=gpurun_out/r5/tpw
mkdir -p $O
timeout -k 10 120 ./tools/r5/heads_proto > $O/proto.txt 2>&1 || { echo "proto failed"; cat $O/proto.txt; exit 1; }
cat $O/proto.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_pq.py tests/test_gpu_activations.py tests/test_gpu_stage_a.py tests/test_gpu_grad_decomp.py > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TAG=tpw AB_LIBS="tpw1" AB_ROUNDS=2 bash tools/r5/lib_ab.sh
