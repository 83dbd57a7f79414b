#!/bin/bash
# Round-3 diagnostics: phase stamps of the persistent rollout kernels (stamps build) and the two SQ
# counter passes of the metric-config bench (k_upd / rollout utilisation).
#   bash scripts/gpu_diag_r03.sh <tag>
set -o pipefail
TAG=${1:-diag}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 scripts/roll_stamps.py > $OUT/roll_stamps.txt 2>&1 || { echo "roll stamps failed"; tail -20 $OUT/roll_stamps.txt; exit 1; }
cat $OUT/roll_stamps.txt
bash scripts/gpu_counters.sh $TAG \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
  > $OUT/sq_counters.txt 2>&1 || { echo "counters failed"; tail -20 $OUT/sq_counters.txt; exit 1; }
grep -E "^(fwdbwd|rollout|values|dw) " $OUT/sq_counters.txt
