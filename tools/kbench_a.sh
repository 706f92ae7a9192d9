#!/bin/bash
# A/B of mli_hash_bwd variants (build here first: python tools/kbench_a.sh build; then on the
# GPU box: bash tools/kbench_a.sh run).
set -e
V=(base "" laneatom "-DMLI_EXP_LANE_ATOMICS" notap "-DMLI_EXP_NO_TAP_SCATTER" noatom "-DMLI_EXP_NO_ATOMICS" dense "-DMLI_EXP_LEVELS_LO=0 -DMLI_EXP_LEVELS_HI=6" hashed "-DMLI_EXP_LEVELS_LO=6 -DMLI_EXP_LEVELS_HI=16")
if [ "$1" = build ]; then
  for ((i = 0; i < ${#V[@]}; i += 2)); do
    python -c "from mli_nerf_amd.build import build; build(extra='${V[i+1]}'.split() or ['-DMLI_EXP_NONE'], out='exp/lib_${V[i]}.so')"
  done
else
  for ((i = 0; i < ${#V[@]}; i += 2)); do
    MLI_HIP_LIB=exp/lib_${V[i]}.so timeout -k 10 120 python tools/kbench_a.py
  done
fi
