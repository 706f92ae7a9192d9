#!/bin/bash
# SQ stall / pipe counters over a short training bench (one counter group per pass).
set -e
OUT=${1:-gpurun_out/pmc_sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu --no-kernel-timing --steps 3 --warmup 2"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS -f csv -d "$OUT/a" -o run -- python bench.py $ARGS > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_LDS -f csv -d "$OUT/b" -o run -- python bench.py $ARGS > "$OUT/b.log" 2>&1
