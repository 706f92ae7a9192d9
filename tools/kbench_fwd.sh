#!/bin/bash
# Knockout A/B of rgb_fwd_kernel (build here: bash tools/kbench_fwd.sh build; on the GPU box:
# bash tools/kbench_fwd.sh run).
set -e
V=(fbase "-DMLI_EXP_NONE" fnodma "-DMLI_EXP_NODMA" fnosync "-DMLI_EXP_NOSYNC" fnomfma "-DMLI_EXP_NOMFMA" fnostage "-DMLI_EXP_NOSTAGE" fnosyncdma "-DMLI_EXP_NOSYNC -DMLI_EXP_NODMA")
if [ "$1" = build ]; then
  for ((i = 0; i < ${#V[@]}; i += 2)); do
    python -c "from mli_nerf_amd.build import build; build(extra='${V[i+1]}'.split(), out='xlib/lib_${V[i]}.so')"
  done
else
  for ((i = 0; i < ${#V[@]}; i += 2)); do
    MLI_HIP_LIB=xlib/lib_${V[i]}.so timeout -k 10 120 python tools/kbench_fwd.py
  done
fi
