#!/bin/bash
# SQ counters of the late-round-3 build: cfg2 (k_upd2, k_dw2_dma) and the metric config (k_dwf_dma).
#   bash scripts/gpu_sq_r03b.sh <tag>
set -o pipefail
TAG=${1:-sq3b}
R=$GRAFT_REPO_ROOT
cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
CTR_CMD="scripts/bench_configs.py --only cfg2 --iters 1 --warmup 1" timeout -k 10 700 bash scripts/gpu_counters.sh ${TAG}_cfg2 "$P1" "$P2" > gpurun_out/${TAG}_cfg2.txt 2>&1 || { echo "cfg2 counters failed"; tail -20 gpurun_out/${TAG}_cfg2.txt; exit 1; }
grep -E "^(fwdbwd|dw) " gpurun_out/${TAG}_cfg2.txt
timeout -k 10 700 bash scripts/gpu_counters.sh ${TAG}_metric "$P1" "$P2" > gpurun_out/${TAG}_metric.txt 2>&1 || { echo "metric counters failed"; tail -20 gpurun_out/${TAG}_metric.txt; exit 1; }
grep -E "^(fwdbwd|dw) " gpurun_out/${TAG}_metric.txt
