#!/bin/bash
# TA / TCP / TD counter passes over tools/field_probe.py (the geometry kernels alone):
# what bounds the hash-grid gathers.  One counter group per pass
# (MI355X_MICROARCH.md: 4 TCP, 2 TA, 2 TD, 8 SQ, 2 GRBM per pass).  GPU box only.
#   bash tools/r6/pmc_gather.sh <outdir> [field_probe args]
set -o pipefail
OUT=${1:-gpurun_out/r6/pmc_gather}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run -f csv -- python tools/field_probe.py "${@:2}" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
