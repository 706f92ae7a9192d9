#!/bin/bash
# the weights-stationary heads prototype against the product's chain pattern.
set -o pipefail
O=gpurun_out/r6/heads_ws
mkdir -p $O
timeout -k 10 120 ./tools/r6/heads_ws_proto > $O/proto.txt 2>&1 || { echo "proto failed"; cat $O/proto.txt; exit 1; }
cat $O/proto.txt
