#!/bin/bash
# PMC passes over tools/field_probe.py (one counter group per pass).  Run on the GPU box.
set -o pipefail
OUT=gpurun_out/pmc_field
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run -f csv -- python tools/field_probe.py > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok"
done
