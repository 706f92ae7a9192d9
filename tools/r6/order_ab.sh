#!/bin/bash
# FIELD / sampling kernel times against the order of the batch's rays (tools/kbench.py --ray-order).
set -o pipefail
O=gpurun_out/r6/order_ab
mkdir -p $O
export MLI_HIP_LIB=xlib/base.so
for i in 1 2; do
for o in random sorted xcd; do
  timeout -k 10 200 python tools/kbench.py --reps 10 --ray-order $o > $O/kbench_${o}_$i.txt 2>&1 || { echo "kbench $o failed"; tail -5 $O/kbench_${o}_$i.txt; exit 1; }
  echo "== $i $o $(grep -E "field|sample|heads fwd train" $O/kbench_${o}_$i.txt | tr -s ' ' | tr '\n' ' ')"
done
done
