#!/bin/bash
# SQ / MFMA counters of the stage-b step's kernels (heads trio first), one counter group per
# rocprofv3 pass (MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ, 2 GRBM per pass).
# Usage (GPU box): bash tools/pmc_trio.sh [outdir]; then python tools/sq_summary.py <outdir> <json>
set -o pipefail
OUT=${1:-gpurun_out/pmc_trio}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu --no-kernel-timing --steps 3 --warmup 2 --pipeline off ${TRIO_ARGS:-}"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "counter list failed rc=$?"
have() { grep -qw "$1" "$OUT/counters.txt"; }
P2=""
for c in SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
         SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU; do
  if have $c && [ $(echo $P2 | wc -w) -lt 8 ]; then P2="$P2 $c"; fi
done
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp -f csv -d "$OUT/p$i" -o run -- python bench.py $ARGS \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo "pmc_trio done"
